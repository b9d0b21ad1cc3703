"""CPU ORACLE for RAFT's frequency-domain response solve -- TEST INFRASTRUCTURE ONLY.

This module is a plain-NumPy restatement of the reference algorithm
(lucas-carmo/RAFT-testStuff @ 2024-10-16, RAFT v1.3.1 fork) for the hot path:
Z(w) assembly + per-bin complex solve, the Borgman drag-linearisation fixed point,
strip-theory inertial/drag excitation and the motion outputs.  Every function cites
the reference file:line it restates.

It is the CHECKER, never the product: only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import it.  The product path
(raft-teststuff_amd/raft) runs on the HIP library and fails loudly without it.

Parity pin: the restatement is checked against golden vectors produced by running
the reference itself in the build container (tests/golden/make_golden.py) -- see
tests/test_oracle.py.

Inputs are the per-design tables (`T`, a dict with the keys written by
make_golden.design_tables / produced by raft.prep), restricted here to submerged
nodes.  Two flavours of the hot loops exist:
  * vectorised over frequency bins (fast; used for parity checks), and
  * `loop=True`: the reference's own per-node / per-bin Python loop structure
    (used only as the timed CPU baseline in bench.py, kind = "port").
"""
import numpy as np

SQRT_8_PI = np.sqrt(8 / np.pi)
RAD2DEG = 57.29577951308232   # raft/helpers.py:25-26
DEG2RAD = 0.017453292519943295


# ----------------------------------------------------------------------------------
# helpers (raft/helpers.py)
# ----------------------------------------------------------------------------------
def wave_number(omega, h, e=0.001):
    """Fixed-point dispersion iteration, relative tolerance 1e-3 (raft/helpers.py:295-310)."""
    g = 9.81
    k1 = omega * omega / g
    k2 = omega * omega / (np.tanh(k1 * h) * g)
    while np.abs(k2 - k1) / k1 > e:
        k1 = k2
        k2 = omega * omega / (np.tanh(k1 * h) * g)
    return k2


def jonswap(ws, Hs, Tp, Gamma=None):
    """JONSWAP spectrum with IEC 61400-3 automatic gamma (raft/helpers.py:606-663)."""
    if not Gamma:
        t = Tp / np.sqrt(Hs)
        if t <= 3.6:
            Gamma = 5.0
        elif t >= 5.0:
            Gamma = 1.0
        else:
            Gamma = np.exp(5.75 - 1.15 * t)
    ws = np.atleast_1d(np.array(ws, dtype=float))
    f = 0.5 / np.pi * ws
    fpOvrf4 = pow((Tp * f), -4.0)
    C = 1.0 - (0.287 * np.log(Gamma))
    Sigma = 0.07 * (f <= 1.0 / Tp) + 0.09 * (f > 1.0 / Tp)
    Alpha = np.exp(-0.5 * ((f * Tp - 1.0) / Sigma) ** 2)
    return 0.5 / np.pi * C * 0.3125 * Hs * Hs * fpOvrf4 / f * np.exp(-1.25 * fpOvrf4) * Gamma ** Alpha


def get_rms(x):
    """raft/helpers.py:581-587"""
    return np.sqrt(0.5 * np.sum(np.abs(x) ** 2))


def get_psd(x, dw):
    """raft/helpers.py:590-603"""
    if x.ndim == 1:
        return 0.5 * np.abs(x) ** 2 / dw
    return np.sum(0.5 * np.abs(x) ** 2 / dw, axis=0)


def get_rao(Xi, zeta):
    """raft/helpers.py:665-684"""
    idx = np.where(np.abs(zeta) > 1e-6)
    out = np.zeros_like(Xi, dtype=complex)
    out[..., idx] = Xi[..., idx] / zeta[idx]
    return out


def small_rotate(r, th):
    """th x r for small rotations (raft/helpers.py:314-326); th may carry a bin axis."""
    return np.array([-th[2] * r[1] + th[1] * r[2],
                     th[2] * r[0] - th[0] * r[2],
                     -th[1] * r[0] + th[0] * r[1]])


def kinematics(r, Xi, w):
    """Node displacement/velocity/acceleration from 6-DOF amplitudes (raft/helpers.py:66-101)."""
    dr = Xi[:3] + small_rotate(r, Xi[3:])
    v = 1j * w * dr
    a = 1j * w * v
    return dr, v, a


def wave_kin(zeta0, beta, w, k, h, r, rho=1025.0, g=9.81):
    """Airy kinematics at a point, vectorised over bins (raft/helpers.py:105-154).

    Branches per bin on k*h (> 89.4 -> deep-water exponentials).  k == 0 is a
    breakpoint() in the reference and is rejected here."""
    zeta0 = np.asarray(zeta0)
    nw = len(w)
    zeta = zeta0 * np.exp(-1j * (k * (np.cos(beta) * r[0] + np.sin(beta) * r[1])))
    u = np.zeros([3, nw], dtype=complex)
    ud = np.zeros([3, nw], dtype=complex)
    pDyn = np.zeros(nw, dtype=complex)
    z = r[2]
    if z <= 0:
        if np.any(k == 0.0):
            raise ValueError("wave number 0 (reference raft/helpers.py:128-132 stops here)")
        deep = k * h > 89.4
        with np.errstate(over="ignore", invalid="ignore"):
            s_sh = np.where(deep, np.exp(k * z), np.sinh(k * (z + h)) / np.sinh(k * h))
            c_sh = np.where(deep, np.exp(k * z), np.cosh(k * (z + h)) / np.sinh(k * h))
            c_ch = np.where(deep, np.exp(k * z) + np.exp(-k * (z + 2.0 * h)),
                            np.real(np.cosh(k * (z + h))) / np.cosh(k * h))
        u[0] = w * zeta * c_sh * np.cos(beta)
        u[1] = w * zeta * c_sh * np.sin(beta)
        u[2] = 1j * w * zeta * s_sh
        ud[:] = 1j * w * u
        pDyn[:] = rho * g * zeta * c_ch
    return u, ud, pDyn


def get_h(r):
    """Alternator matrix (raft/helpers.py:346-355)."""
    return np.array([[0, r[2], -r[1]], [-r[2], 0, r[0]], [r[1], -r[0], 0]])


def translate_matrix_3to6(Min, r):
    """raft/helpers.py:455-478"""
    H = get_h(r)
    out = np.zeros([6, 6])
    out[:3, :3] = Min
    out[:3, 3:] = Min @ H
    out[3:, :3] = out[:3, 3:].T
    out[3:, 3:] = H @ Min @ H.T
    return out


def translate_matrix_6to6(Min, r):
    """6x6 matrix about a translated reference point (raft/helpers.py:481-503)."""
    H = get_h(r)
    Mout = np.zeros([6, 6])
    Mout[:3, :3] = Min[:3, :3]
    Mout[:3, 3:] = np.matmul(Min[:3, :3], H) + Min[:3, 3:]
    Mout[3:, :3] = Mout[:3, 3:].T
    Mout[3:, 3:] = (np.matmul(np.matmul(H, Min[:3, :3]), H.T) + np.matmul(Min[3:, :3], H) + np.matmul(H.T, Min[:3, 3:])
                    + Min[3:, 3:])
    return Mout


def translate_force_3to6(F, r):
    """[F; r x F] with a trailing bin axis allowed (raft/helpers.py:386-401)."""
    F = np.asarray(F)
    m = np.array([r[1] * F[2] - r[2] * F[1],
                  r[2] * F[0] - r[0] * F[2],
                  r[0] * F[1] - r[1] * F[0]])
    return np.concatenate([F, m], axis=0)


# ----------------------------------------------------------------------------------
# per-design node view
# ----------------------------------------------------------------------------------
def imat_mcf(T):
    """MacCamy-Fuchs inertia matrices Imat_MCF[node,3,3,nw] of the MCF nodes
    (raft/raft_member.py:972-1088), rebuilt from the node tables with scipy's hankel1."""
    from scipy.special import hankel1
    rho = float(T["rho"])
    k = T["k"]
    n = len(T["node_sub"])
    out = np.zeros([n, 3, 3, len(k)], dtype=complex)
    for i in range(n):
        if not (T["node_mcf"][i] and T["node_sub"][i]):
            continue
        ds, drs, dls, z = T["node_ds"][i], T["node_drs"][i], T["node_dls"][i], T["node_r"][i, 2]
        circ = bool(T["node_circ"][i])
        v = 0.25 * np.pi * ds[0] ** 2 * dls if circ else ds[0] * ds[1] * dls
        if z + 0.5 * dls > 0:
            v = v * (0.5 * dls - z) / dls
        ve = np.pi / 12.0 * abs((ds[0] + drs[0]) ** 3 - (ds[0] - drs[0]) ** 3)
        q, p1, p2 = T["node_q"][i], T["node_p1"][i], T["node_p2"][i]
        Iend = rho * ve * T["node_Ca_End"][i] * np.outer(q, q)
        c10, c20 = 1. + T["node_Ca_p1"][i], 1. + T["node_Ca_p2"][i]
        R = ds[0] / 2
        Tr = np.pi / 5 / R
        for ik, kk in enumerate(k):
            Hp1 = 0.5 * (hankel1(0, kk * R) - hankel1(2, kk * R))
            Cm = 4j / (np.pi * (kk * R) ** 2 * Hp1)
            ramp = 0.5 * (1 - np.cos(np.pi * (kk - 0) / Tr)) if kk < Tr else 1
            ramp = 0 if kk <= 0 else ramp
            c1, c2 = Cm * ramp + c10 * (1 - ramp), Cm * ramp + c20 * (1 - ramp)
            out[i, :, :, ik] = rho * v * (c1 * np.outer(p1, p1) + c2 * np.outer(p2, p2)) + Iend
    return out


class Nodes:
    """Submerged-node view of the design tables (order = reference member/node order)."""

    def __init__(self, T):
        sub = np.asarray(T["node_sub"]).astype(bool)
        self.idx = np.nonzero(sub)[0]
        g = lambda k: np.asarray(T[k])[sub]
        self.r, self.r_rel = g("node_r"), g("node_r_rel")
        self.q, self.p1, self.p2 = g("node_q"), g("node_p1"), g("node_p2")
        self.circ = g("node_circ").astype(bool)
        self.ds, self.drs, self.dls = g("node_ds"), g("node_drs"), g("node_dls")
        self.Cd_q, self.Cd_p1, self.Cd_p2, self.Cd_End = g("node_Cd_q"), g("node_Cd_p1"), g("node_Cd_p2"), g("node_Cd_End")
        self.a_i = g("node_a_i")
        self.mcf = g("node_mcf").astype(bool)
        self.Imat = g("node_Imat")
        if "node_Imat_MCF" in T:
            self.Imat_MCF = np.asarray(T["node_Imat_MCF"])[sub]
        elif np.any(np.asarray(T["node_mcf"])[sub]):
            self.Imat_MCF = imat_mcf(T)[sub]
        else:
            self.Imat_MCF = None
        self.n = len(self.idx)
        self.r_rel_dry = np.asarray(T["node_r_rel"])[~sub]   # only for the loop flavour's cost shape


def sea_state(case, w, dw):
    """beta, S, zeta per heading (raft/raft_fowt.py:982-1014)."""
    hd = case["wave_heading"]
    nH = 1 if np.isscalar(hd) else len(hd)

    def arr(key, default=None, dtype=float):
        v = case.get(key, default)
        if v is None:
            raise ValueError(f"Key '{key}' not found in input file...")
        if np.isscalar(v):
            return [dtype(v)] * nH
        return [dtype(x) for x in v]

    heading = arr("wave_heading", 0)
    spectrum = arr("wave_spectrum", "JONSWAP", str)
    period = arr("wave_period", None)
    height = arr("wave_height", None)
    gamma = arr("wave_gamma", 0)
    beta = np.array(heading) * DEG2RAD
    nw = len(w)
    S = np.zeros([nH, nw])
    zeta = np.zeros([nH, nw], dtype=complex)
    for ih in range(nH):
        sp = spectrum[ih]
        if sp == "unit":
            S[ih] = 1.0
        elif sp == "constant":
            S[ih] = height[ih]
        elif sp == "JONSWAP":
            S[ih] = jonswap(w, height[ih], period[ih], Gamma=gamma[ih])
        elif sp in ("none", "still"):
            S[ih] = 0.0
        else:
            raise ValueError(f"Wave spectrum input '{sp}' not recognized.")
        zeta[ih] = np.sqrt(2 * S[ih] * dw)
    return beta, S, zeta


def hydro_excitation(T, nodes, beta, zeta):
    """Strip-theory wave kinematics + inertial excitation (raft/raft_fowt.py:1098-1124).

    pDyn uses getWaveKin's DEFAULT rho=1025, g=9.81: calcHydroExcitation does not pass
    the site values (raft/raft_fowt.py:1109-1110)."""
    w, k, h = T["w"], T["k"], float(T["depth"])
    nH, nw = zeta.shape
    u = np.zeros([nH, nodes.n, 3, nw], dtype=complex)
    ud = np.zeros_like(u)
    pDyn = np.zeros([nH, nodes.n, nw], dtype=complex)
    F = np.zeros([nH, 6, nw], dtype=complex)
    for j in range(nodes.n):
        for ih in range(nH):
            u[ih, j], ud[ih, j], pDyn[ih, j] = wave_kin(zeta[ih], beta[ih], w, k, h, nodes.r[j])
        for ih in range(nH):
            if nodes.mcf[j]:
                Im = nodes.Imat_MCF[j]                       # [3,3,nw]
                f = np.einsum("ijb,jb->ib", Im, ud[ih, j])
            else:
                f = nodes.Imat[j] @ ud[ih, j]
            f = f + pDyn[ih, j] * nodes.a_i[j] * nodes.q[j][:, None]
            F[ih] += translate_force_3to6(f, nodes.r_rel[j])
    return u, ud, pDyn, F


def drag_coefficients(T, nodes, j):
    """Per-node constant factors of the Borgman coefficients (raft/raft_fowt.py:1199-1240):
    returns (area*Cd) for q, p1, p2, end."""
    ds, dls, drs = nodes.ds[j], nodes.dls[j], nodes.drs[j]
    if nodes.circ[j]:
        a_q = np.pi * ds[0] * dls
        a_p1 = ds[0] * dls
        a_p2 = ds[0] * dls
        a_end = np.abs(np.pi * ds[0] * drs[0])
    else:
        a_q = 2 * (ds[0] + ds[0]) * dls              # ds[0] twice, as the reference
        a_p1 = ds[0] * dls
        a_p2 = ds[1] * dls
        a_end = np.abs((ds[0] + drs[0]) * (ds[1] + drs[1]) - (ds[0] - drs[0]) * (ds[1] - drs[1]))
    return a_q, a_p1, a_p2, a_end


def hydro_linearization(T, nodes, Xi, u0):
    """Borgman linearised drag (raft/raft_fowt.py:1152-1266).

    Xi: [6,nw] complex; u0: [nodes,3,nw] wave velocity of sea state 0.
    Returns B_drag [6,6], Bmat [nodes,3,3], F_drag [6,nw]."""
    w = T["w"]
    rho = float(T["rho"])
    B = np.zeros([6, 6])
    F = np.zeros([6, len(w)], dtype=complex)
    Bmat = np.zeros([nodes.n, 3, 3])
    for j in range(nodes.n):
        _, vnode, _ = kinematics(nodes.r_rel[j], Xi, w)
        q, p1, p2 = nodes.q[j], nodes.p1[j], nodes.p2[j]
        vrel = u0[j] - vnode
        vrel_q = np.sum(vrel * q[:, None], axis=0) * q[:, None]
        vrel_p = vrel - vrel_q
        vrel_p1 = np.sum(vrel * p1[:, None], axis=0) * p1[:, None]
        vrel_p2 = np.sum(vrel * p2[:, None], axis=0) * p2[:, None]
        vq = get_rms(vrel_q)
        if nodes.circ[j]:
            vp1 = get_rms(vrel_p)
            vp2 = vp1
        else:
            vp1 = get_rms(vrel_p1)
            vp2 = get_rms(vrel_p2)
        a_q, a_p1, a_p2, a_end = drag_coefficients(T, nodes, j)
        Bq = SQRT_8_PI * vq * 0.5 * rho * a_q * nodes.Cd_q[j]
        Bp1 = SQRT_8_PI * vp1 * 0.5 * rho * a_p1 * nodes.Cd_p1[j]
        Bp2 = SQRT_8_PI * vp2 * 0.5 * rho * a_p2 * nodes.Cd_p2[j]
        Bend = SQRT_8_PI * vq * 0.5 * rho * a_end * nodes.Cd_End[j]
        sides = Bq * np.outer(q, q) + Bp1 * np.outer(p1, p1) + Bp2 * np.outer(p2, p2)
        Bmat[j] = sides + Bend * np.outer(q, q)
        B += translate_matrix_3to6(Bmat[j], nodes.r_rel[j])
        F += translate_force_3to6(Bmat[j] @ u0[j], nodes.r_rel[j])
    return B, Bmat, F


def drag_excitation(nodes, Bmat, u_ih):
    """raft/raft_fowt.py:1270-1293"""
    F = np.zeros([6, u_ih.shape[-1]], dtype=complex)
    for j in range(nodes.n):
        F += translate_force_3to6(Bmat[j] @ u_ih[j], nodes.r_rel[j])
    return F


def linear_matrices(T):
    """M_lin, B_lin, C_lin for one FOWT without rotor aero (raft/raft_model.py:911-913)."""
    nw = len(T["w"])
    M = T["M_struc"][:, :, None] + np.asarray(T["A_BEM"]) + T["A_hydro_morison"][:, :, None]
    B = T["B_struc"][:, :, None] + np.asarray(T["B_BEM"]) + np.zeros([6, 6, nw])
    C = T["C_struc"] + T["C_moor"] + T["C_hydro"]
    return M, B, C


def solve_dynamics(T, case, nIter, XiStart=0.0, tol=0.01, loop=False, second_order=None):
    """Single-FOWT Model.solveDynamics (raft/raft_model.py:852-1146).

    second_order: None (potSecOrder = 0) or dict(w1_2nd, k1_2nd) for potSecOrder = 1
    (raft/raft_model.py:966-989): at the first convergence the RAO feeds the slender-body
    QTF, its difference-frequency force is added to F_lin (Q5) and the loop continues with
    iiter reset to 0 then incremented and XiLast NOT relaxed (Q6).
    Returns dict(Xi=[nH+1,6,nw], iters, converged, B_drag, Bmat, Z, F_iner, zeta, S, ...)."""
    nodes = Nodes(T)
    w = T["w"]
    nw = len(w)
    dw = float(T["dw"])
    beta, S, zeta = sea_state(case, w, dw)
    nH = len(beta)
    exc = _hydro_excitation_loop if loop else hydro_excitation
    u, ud, pDyn, F_iner = exc(T, nodes, beta, zeta)
    M_lin, B_lin, C_lin = linear_matrices(T)
    F_lin = F_iner[0]
    nloop = int(nIter) + 1
    XiLast = np.zeros([6, nw], dtype=complex) + XiStart
    lin = _linearize_loop if loop else hydro_linearization
    solve = _solve_bins_loop if loop else _solve_bins
    iiter = 0
    converged = False
    F2 = np.zeros([6, nw], dtype=complex)
    qtf_done = second_order is None
    pair = []
    extra = {}
    while iiter < nloop:
        B_drag, Bmat, F_drag = lin(T, nodes, XiLast, u[0])
        F_drag = (_drag_excitation_loop if loop else drag_excitation)(nodes, Bmat, u[0])
        B_tot = B_lin + B_drag[:, :, None]
        F_tot = F_lin + F_drag
        Z, Xi = solve(w, M_lin, B_tot, C_lin, F_tot)
        if np.any(np.isnan(Xi).ravel()):
            raise Exception("Nan detected in response vector Xi.")
        tolCheck = np.abs(Xi - XiLast) / ((np.abs(Xi) + tol))
        if (tolCheck < tol).all():
            pair.append(iiter + 1)
            if qtf_done:
                converged = True
                break
            from .qtf_oracle import hydro_force_2nd, qtf_slender
            Xi0 = get_rao(Xi, zeta[0])
            qtf = qtf_slender(T, Xi0, second_order["w1_2nd"], second_order["k1_2nd"], beta[0])
            fm, f = hydro_force_2nd(qtf, second_order["w1_2nd"], w, S[0], dw)
            F2 = f.astype(complex)
            F_lin = F_lin + F2                                   # Q5: F_lin[0] += Fhydro_2nd
            extra.update(Xi0=Xi0, qtf=qtf, Fhydro_2nd=F2, Fhydro_2nd_mean=fm)
            qtf_done = True
            iiter = 0
        else:
            XiLast = 0.2 * XiLast + 0.8 * Xi
        iiter += 1
    iters = iiter + 1 if converged else nloop
    # system solve (raft/raft_model.py:1021-1065): Zinv = inv(Z) per bin; Xi[ih] = Zinv F_wave
    XiOut = np.zeros([nH + 1, 6, nw], dtype=complex)
    if loop:
        Zinv = np.zeros([6, 6, nw], dtype=complex)
        for iw in range(nw):
            Zinv[:, :, iw] = np.linalg.inv(Z[:, :, iw])
        for ih in range(nH):
            _, _, _, F_again = _hydro_excitation_loop(T, nodes, beta, zeta)   # the reference recomputes it (:1057)
            F_wave = F_again[ih] + _drag_excitation_loop(nodes, Bmat, u[ih])
            for iw in range(nw):
                XiOut[ih, :, iw] = np.matmul(Zinv[:, :, iw], F_wave[:, iw])
    else:
        Zinv = np.linalg.inv(np.moveaxis(Z, 2, 0))
        for ih in range(nH):
            F_wave = F_iner[ih] + drag_excitation(nodes, Bmat, u[ih]) + (F2 if ih == 0 else 0)
            XiOut[ih] = np.einsum("bij,jb->ib", Zinv, F_wave)
    return dict(Xi=XiOut, iters=iters, converged=converged, B_drag=B_drag, Bmat=Bmat, Z=Z,
                F_iner=F_iner, F_drag=F_drag, zeta=zeta, S=S, beta=beta, iters_pair=pair, **extra)


def solve_farm(Ts, case, nIter, K_array=None, XiStart=0.0, tol=0.01):
    """Multi-FOWT Model.solveDynamics (raft/raft_model.py:852-1146 with nFOWT > 1): each
    FOWT runs its own drag fixed point (:869-1013, no coupling inside the loop); then
    Z_sys = blockdiag(fowt.Z) + array stiffness (:1021-1031), Zinv per bin (:1037-1040) and
    Xi[ih] = Zinv F_wave with F_wave = F_BEM + F_hydro_iner + drag excitation (:1049-1065).
    Returns dict(Xi=[nH+1,6N,nw], iters=[N], fowts=[per-FOWT solve_dynamics results])."""
    per = [solve_dynamics(T, case, nIter, XiStart, tol) for T in Ts]
    nf = len(Ts)
    nw = len(Ts[0]["w"])
    nD = 6 * nf
    Zsys = np.zeros([nw, nD, nD], dtype=complex)
    for i, r in enumerate(per):
        Zsys[:, 6 * i:6 * i + 6, 6 * i:6 * i + 6] += np.moveaxis(r["Z"], 2, 0)
    if K_array is not None:
        Zsys += np.asarray(K_array, dtype=float)[None, :, :]
    Zinv = np.linalg.inv(Zsys)
    nH = len(per[-1]["beta"])                          # Q11: the last FOWT's nWaves
    Xi = np.zeros([nH + 1, nD, nw], dtype=complex)
    for ih in range(nH):
        F_wave = np.zeros([nD, nw], dtype=complex)
        for i, (T, r) in enumerate(zip(Ts, per)):
            nodes = Nodes(T)
            u, _, _, F_iner = hydro_excitation(T, nodes, r["beta"], r["zeta"])
            F_wave[6 * i:6 * i + 6] = F_iner[ih] + drag_excitation(nodes, r["Bmat"], u[ih])
        Xi[ih] = np.einsum("bij,jb->ib", Zinv, F_wave)
    return dict(Xi=Xi, iters=[r["iters"] for r in per], converged=[r["converged"] for r in per], fowts=per)


def _solve_bins(w, M, B, C, F):
    """Per-bin Z assembly + LAPACK zgesv (raft/raft_model.py:942-947), batched."""
    Zb = (-w[:, None, None] ** 2 * np.moveaxis(M, 2, 0) + 1j * w[:, None, None] * np.moveaxis(B, 2, 0)
          + C[None, :, :])
    Xi = np.linalg.solve(Zb, F.T[:, :, None])[:, :, 0].T
    return np.moveaxis(Zb, 0, 2), Xi


def motion_outputs(Xi, dw):
    """std and PSD per DOF, rotations in degrees (raft/raft_fowt.py:1831-1875)."""
    out = {}
    for i, dof in enumerate(["surge", "sway", "heave", "roll", "pitch", "yaw"]):
        x = Xi[:, i, :] * RAD2DEG if i >= 3 else Xi[:, i, :]
        out[dof + "_std"] = get_rms(x)
        out[dof + "_PSD"] = get_psd(x, dw)
    return out


def rotor_outputs(Xi, w, dw, rot, Xi0_pitch=0.0, g=9.81):
    """Nacelle-acceleration and tower-base-moment channels of saveTurbineOutputs with zero
    aero loads (raft/raft_fowt.py:1900-1970), in the reference's arithmetic order.
    rot: dict of per-rotor arrays r_rel_z (RNA reference height), mRNA, IrRNA, mtower,
    zCG_tow (tower CG height), zBase (tower member rA z), Mtow [nrot, 6, 6] (tower M_struc)."""
    nr = len(rot["mRNA"])
    nw = len(w)
    out = {k: np.zeros(nr) for k in ["AxRNA_std", "AxRNA_avg", "AxRNA_max", "AxRNA_min",
                                      "Mbase_avg", "Mbase_std", "Mbase_max", "Mbase_min"]}
    out["AxRNA_PSD"] = np.zeros([nw, nr])
    out["Mbase_PSD"] = np.zeros([nw, nr])
    for ir in range(nr):
        XiHub = Xi[:, 0, :] + rot["r_rel_z"][ir] * Xi[:, 4, :]                         # :1909
        out["AxRNA_std"][ir] = get_rms(XiHub * w ** 2)                                 # :1912
        out["AxRNA_PSD"][:, ir] = get_psd(XiHub * w ** 2, dw)
        out["AxRNA_avg"][ir] = abs(np.sin(Xi0_pitch) * 9.81)
        out["AxRNA_max"][ir] = out["AxRNA_avg"][ir] + 3 * out["AxRNA_std"][ir]
        out["AxRNA_min"][ir] = out["AxRNA_avg"][ir] - 3 * out["AxRNA_std"][ir]
        m_t = rot["mtower"][ir] + rot["mRNA"][ir]                                       # :1941
        zCG = (rot["zCG_tow"][ir] * rot["mtower"][ir] + rot["r_rel_z"][ir] * rot["mRNA"][ir]) / m_t
        hArm = zCG - rot["zBase"][ir]
        aCG = -w ** 2 * (Xi[:, 0, :] + zCG * Xi[:, 4, :])                               # :1947
        Mtr = translate_matrix_6to6(np.asarray(rot["Mtow"][ir], dtype=float), [0, 0, -zCG])
        ICG = Mtr[4, 4] + rot["mRNA"][ir] * (rot["r_rel_z"][ir] - zCG) ** 2 + rot["IrRNA"][ir]
        M_I = -m_t * aCG * hArm - ICG * (-w ** 2 * Xi[:, 4, :])                        # :1953
        M_w = m_t * g * hArm * Xi[:, 4]                                                 # :1954
        dyn = M_I + M_w                                                                  # :1960, aero terms 0
        out["Mbase_avg"][ir] = m_t * g * hArm * np.sin(Xi0_pitch)                       # :1965, f_aero0 = 0
        out["Mbase_std"][ir] = get_rms(dyn)
        out["Mbase_PSD"][:, ir] = get_psd(dyn, dw)
        out["Mbase_max"][ir] = out["Mbase_avg"][ir] + 3 * out["Mbase_std"][ir]
        out["Mbase_min"][ir] = out["Mbase_avg"][ir] - 3 * out["Mbase_std"][ir]
    return out


# ----------------------------------------------------------------------------------
# reference-structured loops (CPU baseline timing only; same arithmetic)
# ----------------------------------------------------------------------------------
def _linearize_loop(T, nodes, Xi, u0):
    """calcHydroLinearization with the reference's per-node x per-bin loop shape
    (raft/raft_fowt.py:1176-1259): per-bin 3x3 matvec + translate with np.cross."""
    w = T["w"]
    rho = float(T["rho"])
    nw = len(w)
    B = np.zeros([6, 6])
    F = np.zeros([6, nw], dtype=complex)
    Bmat = np.zeros([nodes.n, 3, 3])
    for r_dry in nodes.r_rel_dry:                # evaluated for dry nodes too
        dr = np.zeros([3, nw], dtype=complex)
        for i in range(nw):
            dr[:, i] = Xi[:3, i] + small_rotate(r_dry, Xi[3:, i])
    for j in range(nodes.n):
        dr = np.zeros([3, nw], dtype=complex)
        for i in range(nw):                      # getKinematics per bin (helpers.py:95-98)
            dr[:, i] = Xi[:3, i] + small_rotate(nodes.r_rel[j], Xi[3:, i])
        vnode = 1j * w * dr
        q, p1, p2 = nodes.q[j], nodes.p1[j], nodes.p2[j]
        vrel = u0[j] - vnode
        vrel_q = np.sum(vrel * q[:, None], axis=0) * q[:, None]
        vrel_p = vrel - vrel_q
        vrel_p1 = np.sum(vrel * p1[:, None], axis=0) * p1[:, None]
        vrel_p2 = np.sum(vrel * p2[:, None], axis=0) * p2[:, None]
        vq = get_rms(vrel_q)
        vp1, vp2 = (get_rms(vrel_p),) * 2 if nodes.circ[j] else (get_rms(vrel_p1), get_rms(vrel_p2))
        a_q, a_p1, a_p2, a_end = drag_coefficients(T, nodes, j)
        Bq = SQRT_8_PI * vq * 0.5 * rho * a_q * nodes.Cd_q[j]
        Bp1 = SQRT_8_PI * vp1 * 0.5 * rho * a_p1 * nodes.Cd_p1[j]
        Bp2 = SQRT_8_PI * vp2 * 0.5 * rho * a_p2 * nodes.Cd_p2[j]
        Bend = SQRT_8_PI * vq * 0.5 * rho * a_end * nodes.Cd_End[j]
        Bmat[j] = Bq * np.outer(q, q) + Bp1 * np.outer(p1, p1) + Bp2 * np.outer(p2, p2) + Bend * np.outer(q, q)
        B += translate_matrix_3to6(Bmat[j], nodes.r_rel[j])
        for i in range(nw):
            f = np.matmul(Bmat[j], u0[j, :, i])
            F[:, i] += np.concatenate([f, np.cross(nodes.r_rel[j], f)])
    return B, Bmat, F


def _wave_kin_loop(zeta0, beta, w, k, h, r, rho=1025.0, g=9.81):
    """getWaveKin with the reference's per-bin scalar loop (raft/helpers.py:114-152)."""
    nw = len(w)
    u = np.zeros([3, nw], dtype=complex)
    ud = np.zeros([3, nw], dtype=complex)
    pDyn = np.zeros(nw, dtype=complex)
    z = r[2]
    for i in range(nw):
        zeta = zeta0[i] * np.exp(-1j * (k[i] * (np.cos(beta) * r[0] + np.sin(beta) * r[1])))
        if z <= 0:
            if k[i] * h > 89.4:
                s_sh = np.exp(k[i] * z)
                c_sh = np.exp(k[i] * z)
                c_ch = np.exp(k[i] * z) + np.exp(-k[i] * (z + 2.0 * h))
            else:
                s_sh = np.sinh(k[i] * (z + h)) / np.sinh(k[i] * h)
                c_sh = np.cosh(k[i] * (z + h)) / np.sinh(k[i] * h)
                c_ch = np.real(np.cosh(k[i] * (z + h))) / np.cosh(k[i] * h)
            u[0, i] = w[i] * zeta * c_sh * np.cos(beta)
            u[1, i] = w[i] * zeta * c_sh * np.sin(beta)
            u[2, i] = 1j * w[i] * zeta * s_sh
            ud[:, i] = 1j * w[i] * u[:, i]
            pDyn[i] = rho * g * zeta * c_ch
    return u, ud, pDyn


def _hydro_excitation_loop(T, nodes, beta, zeta):
    """calcHydroExcitation with the reference's loop shape (raft/raft_fowt.py:1098-1124)."""
    w, k, h = T["w"], T["k"], float(T["depth"])
    nH, nw = zeta.shape
    u = np.zeros([nH, nodes.n, 3, nw], dtype=complex)
    ud = np.zeros_like(u)
    pDyn = np.zeros([nH, nodes.n, nw], dtype=complex)
    F = np.zeros([nH, 6, nw], dtype=complex)
    for j in range(nodes.n):
        for ih in range(nH):
            u[ih, j], ud[ih, j], pDyn[ih, j] = _wave_kin_loop(zeta[ih], beta[ih], w, k, h, nodes.r[j])
        for ih in range(nH):
            for i in range(nw):
                Im = nodes.Imat_MCF[j][:, :, i] if nodes.mcf[j] else nodes.Imat[j]
                f = np.matmul(Im, ud[ih, j, :, i]) + pDyn[ih, j, i] * nodes.a_i[j] * nodes.q[j]
                F[ih, :, i] += np.concatenate([f, np.cross(nodes.r_rel[j], f)])
    return u, ud, pDyn, F


def _drag_excitation_loop(nodes, Bmat, u_ih):
    nw = u_ih.shape[-1]
    F = np.zeros([6, nw], dtype=complex)
    for j in range(nodes.n):
        for i in range(nw):
            f = np.matmul(Bmat[j], u_ih[j, :, i])
            F[:, i] += np.concatenate([f, np.cross(nodes.r_rel[j], f)])
    return F


def _solve_bins_loop(w, M, B, C, F):
    nw = len(w)
    Z = np.zeros([6, 6, nw], dtype=complex)
    Xi = np.zeros([6, nw], dtype=complex)
    for ii in range(nw):
        Z[:, :, ii] = -w[ii] ** 2 * M[:, :, ii] + 1j * w[ii] * B[:, :, ii] + C
        Xi[:, ii] = np.linalg.solve(Z[:, :, ii], F[:, ii])
    return Z, Xi
