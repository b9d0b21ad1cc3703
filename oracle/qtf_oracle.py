"""CPU ORACLE for the slender-body second-order QTF -- TEST INFRASTRUCTURE ONLY.

NumPy restatement of FOWT.calcQTF_slenderBody (raft/raft_fowt.py:1385-1648), its wave
helpers (raft/helpers.py:157-291), Member.correction_KAY (raft/raft_member.py:1090-1205)
and FOWT.calcHydroForce_2ndOrd (raft/raft_fowt.py:1728-1818, 'qtf' mode with the
interp2d restatement of SURVEY.md Q13).  The pair loop is vectorised over all (i1 <= i2)
pairs; every per-node / per-pair formula keeps the reference's operand order, including
the quirks of SURVEY.md §8.Q (Q1 degree conversion of an angle already in radians, Q2
grad[2,1] = grad[0,1], Q3 in-place projection of the node velocity, Q9 KAY radius and
conjugation, Q12 partly-submerged volume).  Pinned by tests/golden/c3_qtf.npz (reference
run in the build container); only tests/ and bench.py's cpu_baseline may import it.
"""
import numpy as np
from scipy.special import hankel1

from .raft_oracle import DEG2RAD, kinematics, translate_force_3to6, wave_kin


def grad_u1(w, k, beta, h, r):
    """raft/helpers.py:157-195, vectorised over (w, k) -> [n,3,3]."""
    w = np.atleast_1d(w).astype(float)
    k = np.atleast_1d(k).astype(float)
    n = len(w)
    g = np.zeros([n, 3, 3], dtype=complex)
    x, y, z = r
    cb, sb = np.cos(beta * DEG2RAD), np.sin(beta * DEG2RAD)      # Q1
    if z > 0:
        return g
    ok = k > 0
    deep = k * h >= 10
    with np.errstate(over="ignore", invalid="ignore"):
        kxy = np.where(deep, np.exp(k * z), np.cosh(k * (z + h)) / np.sinh(k * h))
        kz = np.where(deep, np.exp(k * z), np.sinh(k * (z + h)) / np.sinh(k * h))
    ph = np.exp(-1j * (k * (np.cos(beta) * x + np.sin(beta) * y)))
    aux = w * cb * ph
    g[:, 0, 0] = -1j * aux * kxy * k * cb
    g[:, 0, 1] = -1j * aux * kxy * k * sb
    g[:, 0, 2] = aux * k * kz
    aux = w * sb * ph
    g[:, 1, 0] = g[:, 0, 1]
    g[:, 1, 1] = -1j * aux * kxy * k * sb
    g[:, 1, 2] = aux * k * kz
    aux = 1j * w * ph
    g[:, 2, 0] = g[:, 0, 2]
    g[:, 2, 1] = g[:, 0, 1]                                         # Q2
    g[:, 2, 2] = aux * k * kxy
    g[~ok] = 0
    return g


def grad_pres1st(k, beta, h, r, rho, g):
    """raft/helpers.py:202-225 -> [n,3]"""
    k = np.atleast_1d(k).astype(float)
    out = np.zeros([len(k), 3], dtype=complex)
    x, y, z = r
    cb, sb = np.cos(beta * DEG2RAD), np.sin(beta * DEG2RAD)
    if z > 0:
        return out
    deep = k * h >= 10
    with np.errstate(over="ignore", invalid="ignore"):
        kxy = np.where(deep, np.exp(k * z), np.cosh(k * (z + h)) / np.cosh(k * h))
        kz = np.where(deep, np.exp(k * z), np.sinh(k * (z + h)) / np.cosh(k * h))
    ph = np.exp(-1j * (k * (cb * x + sb * y)))
    out[:, 0] = rho * g * kxy * ph * (-1j * k * cb)
    out[:, 1] = rho * g * kxy * ph * (-1j * k * sb)
    out[:, 2] = rho * g * kz * ph * k
    out[~(k > 0)] = 0
    return out


def pot2nd(w1, w2, k1, k2, beta, h, r, g, rho):
    """Second-order potential acceleration and pressure (raft/helpers.py:254-291),
    vectorised over pairs; zero on the diagonal w1 == w2."""
    n = len(w1)
    acc = np.zeros([n, 3], dtype=complex)
    p = np.zeros(n, dtype=complex)
    z = r[2]
    b = beta * DEG2RAD                                             # Q1
    cb, sb = np.cos(b), np.sin(b)
    m = (w1 != w2) & (k1 > 0) & (k2 > 0)
    if z > 0 or not m.any():
        return acc, p
    w1, w2, k1, k2 = w1[m], w2[m], k1[m], k2[m]
    kx = k1 * cb - k2 * cb
    ky = k1 * sb - k2 * sb
    nk = np.sqrt(kx * kx + ky * ky)                                # np.linalg.norm of [kx, ky, 0]
    t1, t2 = np.tanh(k1 * h), np.tanh(k2 * h)
    g12 = (-1j * g / (2 * w1)) * ((k1 ** 2) * (1 - t1 ** 2) - 2 * k1 * k2 * (1 + t1 * t2)) / \
        ((w1 - w2) ** 2 / g - nk * np.tanh(nk * h))
    g21 = (-1j * g / (2 * w2)) * ((k2 ** 2) * (1 - t2 ** 2) - 2 * k2 * k1 * (1 + t2 * t1)) / \
        ((w2 - w1) ** 2 / g - nk * np.tanh(nk * h))
    aux = 0.5 * (g21 + np.conj(g12))
    kxy = np.cosh(nk * (z + h)) / np.cosh(nk * h)
    kz = np.sinh(nk * (z + h)) / np.cosh(nk * h)
    ph = np.exp(-1j * (kx * r[0] + ky * r[1] + 0 * r[2]))
    a = np.zeros([len(w1), 3], dtype=complex)
    a[:, 0] = aux * kxy * ph * ((w1 - w2) * kx)
    a[:, 1] = aux * kxy * ph * ((w1 - w2) * ky)
    a[:, 2] = aux * kz * ph * (1j * (w1 - w2) * nk)
    acc[m] = a
    p[m] = aux * kxy * ph * (-1j * rho * (w1 - w2))
    return acc, p


def _hank_d(n, x):
    """0.5 (H_{n-1}(x) - H_{n+1}(x)) (raft/raft_member.py:1104-1107)."""
    return 0.5 * (hankel1(n - 1, x) - hankel1(n + 1, x))


def kay_omega(k1R, k2R, n):
    """omega() of raft/raft_member.py:1102-1109, vectorised."""
    H_N_ii = _hank_d(n, k1R)
    H_N_jj = np.conj(_hank_d(n, k2R))
    H_Nm1_ii = _hank_d(n + 1, k1R)
    H_Nm1_jj = np.conj(_hank_d(n + 1, k2R))
    return 1 / (H_Nm1_ii * H_N_jj) - 1 / (H_N_ii * H_Nm1_jj)


class MemberView:
    """All strip nodes of one member from the design tables (reference order)."""

    def __init__(self, T, im):
        sel = np.nonzero(np.asarray(T["node_member"]) == im)[0]
        self.r = T["node_r"][sel]
        self.q, self.p1, self.p2 = T["node_q"][sel[0]], T["node_p1"][sel[0]], T["node_p2"][sel[0]]
        self.ds, self.drs, self.dls = T["node_ds"][sel], T["node_drs"][sel], T["node_dls"][sel]
        self.Ca_p1, self.Ca_p2, self.Ca_End = T["node_Ca_p1"][sel], T["node_Ca_p2"][sel], T["node_Ca_End"][sel]
        self.a_i = T["node_a_i"][sel]
        self.circ = bool(T["member_circ"][im])
        self.mcf = bool(T["member_mcf"][im])
        self.rA, self.rB = T["member_rA"][im], T["member_rB"][im]
        self.qMat, self.p1Mat, self.p2Mat = np.outer(self.q, self.q), np.outer(self.p1, self.p1), np.outer(self.p2, self.p2)
        self.ns = len(sel)


def correction_kay(mem, h, w1, w2, k1, k2, beta, rho, g, Nm=10):
    """Kim & Yue second-order diffraction correction (raft/raft_member.py:1090-1205),
    vectorised over pairs -> [np, 6]."""
    npair = len(w1)
    F = np.zeros([npair, 6], dtype=complex)
    if not mem.mcf:
        return F
    cb, sb = np.cos(beta), np.sin(beta)
    kk = np.stack([k1 * cb - k2 * cb, k1 * sb - k2 * sb, 0 * k1], axis=1)
    bv = np.array([cb, sb, 0])
    pf = np.dot(bv, mem.p1) * mem.p1 + np.dot(bv, mem.p2) * mem.p2
    pf = pf / np.linalg.norm(pf)
    if not (mem.rA[2] * mem.rB[2] < 0):
        return F
    rwl = mem.rA + (mem.rB - mem.rA) * (0 - mem.rA[2]) / (mem.rB[2] - mem.rA[2])
    radii = 0.5 * mem.ds[:, 0]
    R = np.interp(0, mem.r[:, 2], radii)
    k1R, k2R = k1 * R, k2 * R
    Fwl = 0 + 0j
    for nn in range(Nm + 1):
        Fwl = Fwl + -rho * g * R * 2j / np.pi / (k1R * k2R) * kay_omega(k1R, k2R, nn)
    Fwl = np.real(Fwl) * np.exp(-1j * (kk @ rwl))
    F += translate_force_3to6(Fwl[None, :] * pf[:, None], rwl).T
    for il in range(mem.ns - 1):
        z1 = mem.r[il, 2]
        if z1 > 0:
            continue
        z2 = mem.r[il + 1, 2]
        z2 = 0 if z2 > 0 else z2
        R1 = mem.ds[il, 0] / 2
        if mem.dls[il] == 0:
            R1 = mem.ds[il, 0]
        R2 = mem.ds[il + 1, 0] / 2
        if mem.dls[il + 1] == 0:
            R2 = mem.ds[il, 0]                                    # Q9
        Rm = 0.5 * (R1 + R2)
        k1R, k2R = k1 * Rm, k2 * Rm
        H = h / Rm
        k1h, k2h = k1R * H, k2R * H
        eq = w1 == w2
        with np.errstate(divide="ignore", invalid="ignore"):
            a2 = np.sinh((k1 + k2) * (z2 + h)) / (k1h + k2h)
            a1 = np.sinh((k1 + k2) * (z1 + h)) / (k1h + k2h)
            d2 = np.sinh((k1 - k2) * (z2 + h)) / (k1h - k2h)
            d1 = np.sinh((k1 - k2) * (z1 + h)) / (k1h - k2h)
        Im = np.where(eq, 0.5 * (a2 - (z2 + h) / h - a1 + (z1 + h) / h), 0.5 * (a2 - d2 - a1 + d1))
        Ip = np.where(eq, 0.5 * (a2 + (z2 + h) / h - a1 - (z1 + h) / h), 0.5 * (a2 + d2 - a1 - d1))
        ch1, ch2 = np.cosh(k1h), np.cosh(k2h)
        dF = 0 + 0j
        for nn in range(Nm + 1):
            dF = dF + rho * g * Rm * 2j / np.pi / (k1R * k2R) * kay_omega(k1R, k2R, nn) * (
                k1h * k2h / np.sqrt(k1h * np.tanh(k1h)) / np.sqrt(k2h * np.tanh(k2h))
                * (Im + Ip * nn * (nn + 1) / k1R / k2R) / ch1 / ch2)
        rr = 0.5 * (mem.r[il] + mem.r[il + 1])
        dF = np.real(dF) * np.exp(-1j * (kk @ rwl))
        F += translate_force_3to6(dF[None, :] * pf[:, None], rr).T
    F = np.where((k1 < k2)[:, None], np.conj(F), F)
    return F


def _mv(A, x):
    """3x3 real/complex matrix (or [np,3,3]) times [np,3]."""
    if A.ndim == 2:
        return x @ A.T
    return np.einsum("nij,nj->ni", A, x)


def qtf_slender(T, Xi0, w1_2nd, k1_2nd, beta, rho=None, g=None):
    """FOWT.calcQTF_slenderBody (raft/raft_fowt.py:1385-1640) -> qtf [n2, n2, 1, 6]."""
    rho = float(T["rho"]) if rho is None else rho
    g = float(T["g"]) if g is None else g
    h = float(T["depth"])
    w = T["w"]
    n2 = len(w1_2nd)
    Xi = np.zeros([6, n2], dtype=complex)
    for d in range(6):
        Xi[d] = np.interp(w1_2nd, w, Xi0[d], left=0, right=0)
    M = T["M_struc"]
    F1 = np.zeros([6, n2], dtype=complex)
    F1[0:3] = M[0, 0] * (-w1_2nd ** 2 * Xi[0:3])
    F1[3:6] = M[3:, 3:] @ (-w1_2nd ** 2 * Xi[3:])
    i1, i2 = np.triu_indices(n2)
    keep = w1_2nd[i2] >= w1_2nd[i1]
    i1, i2 = i1[keep], i2[keep]
    W1, W2, K1, K2 = w1_2nd[i1], w1_2nd[i2], k1_2nd[i1], k1_2nd[i2]
    npair = len(i1)
    Q = np.zeros([npair, 6], dtype=complex)
    # Pinkster IV rotation term (:1449-1456)
    th1, th2 = Xi[3:, i1].T, Xi[3:, i2].T
    Q[:, 0:3] = 0.25 * (np.cross(th1, np.conj(F1[0:3, i2].T)) + np.cross(np.conj(th2), F1[0:3, i1].T))
    Q[:, 3:6] = 0.25 * (np.cross(th1, np.conj(F1[3:, i2].T)) + np.cross(np.conj(th2), F1[3:, i1].T))
    nmem = len(T["member_rA"])
    for im in range(nmem):
        mem = MemberView(T, im)
        if mem.rA[2] > 0 and mem.rB[2] > 0:
            continue
        Q += _member_terms(mem, Xi, w1_2nd, k1_2nd, i1, i2, beta, h, rho, g)
        Q += correction_kay(mem, h, W1, W2, K1, K2, beta, rho, g)
    qtf = np.zeros([n2, n2, 1, 6], dtype=complex)
    qtf[i1, i2, 0, :] = Q
    for d in range(6):
        q = qtf[:, :, 0, d]
        qtf[:, :, 0, d] = q + np.conj(q).T - np.diag(np.diag(np.conj(q)))
    return qtf


def _member_terms(mem, Xi, w1_2nd, k1_2nd, i1, i2, beta, h, rho, g):
    """Node and waterline force terms of one member for all pairs (:1467-1633)."""
    n2 = len(w1_2nd)
    npair = len(i1)
    W1, W2, K1, K2 = w1_2nd[i1], w1_2nd[i2], k1_2nd[i1], k1_2nd[i2]
    Q = np.zeros([npair, 6], dtype=complex)
    q, p1Mat, p2Mat, qMat = mem.q, mem.p1Mat, mem.p2Mat, mem.qMat
    # per-(frequency, node) tables (:1468-1483)
    nodeV = np.zeros([mem.ns, n2, 3], dtype=complex)
    dr = np.zeros_like(nodeV)
    u = np.zeros_like(nodeV)
    gu = np.zeros([mem.ns, n2, 3, 3], dtype=complex)
    gp = np.zeros([mem.ns, n2, 3], dtype=complex)
    var = np.zeros([mem.ns, n2], dtype=complex)
    for il in range(mem.ns):
        r = mem.r[il]
        d_, v_, _ = kinematics(r, Xi, w1_2nd)
        dr[il], nodeV[il] = d_.T, v_.T
        u[il] = wave_kin(np.ones(n2), beta, w1_2nd, k1_2nd, h, r, rho=rho, g=g)[0].T
        gu[il] = grad_u1(w1_2nd, k1_2nd, beta, h, r)
        var[il] = (u[il] - nodeV[il]) @ q
        gp[il] = grad_pres1st(k1_2nd, beta, h, r, rho=rho, g=g)
    gdudt = 1j * w1_2nd[None, :, None, None] * gu
    # waterline tables (:1486-1502)
    cross_wl = mem.r[-1, 2] * mem.r[0, 2] < 0
    eta = np.zeros(n2, dtype=complex)
    ud_wl = np.zeros([n2, 3], dtype=complex)
    dr_wl = np.zeros([n2, 3], dtype=complex)
    a_wl = np.zeros([n2, 3], dtype=complex)
    r_int = None
    if cross_wl:
        r_int = mem.r[0] + (mem.r[-1] - mem.r[0]) * (0. - mem.r[0, 2]) / (mem.r[-1, 2] - mem.r[0, 2])
        _, udw, et = wave_kin(np.ones(n2), beta, w1_2nd, k1_2nd, h, r_int, rho=1, g=1)
        ud_wl, eta = udw.T, et
        d_, _, a_ = kinematics(r_int, Xi, w1_2nd)
        dr_wl, a_wl = d_.T, a_.T
    ge1 = np.zeros([n2, 3], dtype=complex)
    for iw in range(n2):
        ge1[iw] = -g * (np.cross(Xi[3:, iw], mem.p1)[2] * mem.p1 + np.cross(Xi[3:, iw], mem.p2)[2] * mem.p2)
    eta_r = eta - dr_wl[:, 2]
    O1 = _omega_mat(1j * W1[:, None] * Xi[3:, i1].T)
    O2 = _omega_mat(1j * W2[:, None] * Xi[3:, i2].T)
    Ca_p1 = Ca_p2 = None
    for il in range(mem.ns):
        r = mem.r[il]
        if r[2] >= 0:
            continue
        Ca_p1, Ca_p2, Ca_End = mem.Ca_p1[il], mem.Ca_p2[il], mem.Ca_End[il]
        CmM = (1. + Ca_p1) * p1Mat + (1. + Ca_p2) * p2Mat
        CaM = Ca_p1 * p1Mat + Ca_p2 * p2Mat
        ds, drs, dls = mem.ds[il], mem.drs[il], mem.dls[il]
        v_i = 0.25 * np.pi * ds[0] ** 2 * dls if mem.circ else ds[0] * ds[1] * dls
        if r[2] + 0.5 * dls > 0:                                   # Q12
            v_i = v_i * (0.5 * dls - r[2]) / dls
        acc2, p2 = pot2nd(W1, W2, K1, K2, beta, h, r, g, rho)
        f_2nd = rho * v_i * _mv(CmM, acc2)
        conv = 0.25 * (_mv(gu[il, i1], np.conj(u[il, i2])) + _mv(np.conj(gu[il, i2]), u[il, i1]))
        f_conv = rho * v_i * _mv(CmM, conv)
        # Rainey axial divergence (helpers.py:228-251); node velocities projected in place (Q3)
        dwdz1 = np.einsum("nij,j->ni", gu[il, i1], q) @ q
        dwdz2 = np.einsum("nij,j->ni", gu[il, i2], q) @ q
        vel1 = nodeV[il, i1] - np.outer(nodeV[il, i1] @ q, q)
        vel2 = nodeV[il, i2] - np.outer(nodeV[il, i2] @ q, q)
        u1 = u[il, i1] - np.outer(u[il, i1] @ q, q)
        u2 = u[il, i2] - np.outer(u[il, i2] @ q, q)
        acc = 0.25 * (dwdz1[:, None] * np.conj(u2 - vel2) + np.conj(dwdz2)[:, None] * (u1 - vel1))
        acc = acc - np.outer(acc @ q, q)
        f_axdv = rho * v_i * _mv(CaM, acc)
        acc_n = 0.25 * _mv(gdudt[il, i1], np.conj(dr[il, i2])) + 0.25 * _mv(np.conj(gdudt[il, i2]), dr[il, i1])
        f_nabla = rho * v_i * _mv(CmM, acc_n)
        va1 = var[il, i1][:, None] * q[None, :]
        va2 = var[il, i2][:, None] * q[None, :]
        f_rslb = -0.25 * 2 * _mv(CaM, _mv(O1, np.conj(va2)) + _mv(np.conj(O2), va1))
        f_rslb = f_rslb * (rho * v_i)
        u1a = u[il, i1] - vel1                       # uses the projected node velocity (Q3)
        u2a = u[il, i2] - vel2
        V1 = gu[il, i1] + O1
        V2 = gu[il, i2] + O2
        aux = 0.25 * (_mv(V1, np.conj(_mv(CaM, u2a))) + _mv(np.conj(V2), _mv(CaM, u1a)))
        aux = aux - _mv(qMat, aux)
        f_rslb = f_rslb + rho * v_i * aux
        u1a = u1a - _mv(qMat, u1a)
        u2a = u2a - _mv(qMat, u2a)
        aux = 0.25 * (_mv(CaM, _mv(V1, np.conj(u2a))) + _mv(CaM, _mv(np.conj(V2), u1a)))
        f_rslb = f_rslb + -rho * v_i * aux
        # axial / end effects (:1580-1594)
        if mem.circ:
            ve = np.pi / 12.0 * abs((ds[0] + drs[0]) ** 3 - (ds[0] - drs[0]) ** 3)
        else:
            ve = np.pi / 12.0 * ((np.mean(ds + drs)) ** 3 - (np.mean(ds - drs)) ** 3)
        ai = mem.a_i[il]
        f_2nd = f_2nd + ai * p2[:, None] * q[None, :]
        f_2nd = f_2nd + rho * ve * Ca_End * _mv(qMat, acc2)
        f_conv = f_conv + rho * ve * Ca_End * _mv(qMat, conv)
        f_nabla = f_nabla + rho * ve * Ca_End * _mv(qMat, acc_n)
        pn = 0.25 * np.sum(gp[il, i1] * np.conj(dr[il, i2]), axis=1) + 0.25 * np.sum(np.conj(gp[il, i2]) * dr[il, i1], axis=1)
        f_nabla = f_nabla + ai * pn[:, None] * q[None, :]
        # node velocities here are the ones projected in place by _axdivAcc (Q3)
        pdrop = -2 * 0.25 * 0.5 * rho * np.sum(_mv(p1Mat + p2Mat, u[il, i1] - vel1) *
                                               np.conj(_mv(CaM, u[il, i2] - vel2)), axis=1)
        f_conv = f_conv + ai * pdrop[:, None] * q[None, :]
        for f in (f_2nd, f_conv, f_axdv, f_nabla, f_rslb):
            Q += translate_force_3to6(f.T, r).T
    if cross_wl:
        i_wl = np.where(mem.r[:, 2] < 0)[0][-1]
        if mem.circ:
            d_wl = 0.5 * (mem.ds[i_wl, 0] + mem.ds[i_wl + 1, 0]) if i_wl != mem.ns - 1 else mem.ds[i_wl, 0]
            a_wl_area = 0.25 * np.pi * d_wl ** 2
        else:
            if i_wl != mem.ns - 1:
                d1 = 0.5 * (mem.ds[i_wl, 0] + mem.ds[i_wl + 1, 0])
                d2 = 0.5 * (mem.ds[i_wl, 1] + mem.ds[i_wl + 1, 1])
            else:
                d1, d2 = mem.ds[i_wl, 0], mem.ds[i_wl, 1]
            a_wl_area = d1 * d2
        # Ca_p1 / Ca_p2 are those of the LAST submerged node of the loop above (:1625-1627)
        CmM = (1. + Ca_p1) * p1Mat + (1. + Ca_p2) * p2Mat
        CaM = Ca_p1 * p1Mat + Ca_p2 * p2Mat
        fe = 0.25 * (ud_wl[i1] * np.conj(eta_r[i2])[:, None] + np.conj(ud_wl[i2]) * eta_r[i1][:, None])
        fe = rho * a_wl_area * _mv(CmM, fe)
        ae = 0.25 * (a_wl[i1] * np.conj(eta_r[i2])[:, None] + np.conj(a_wl[i2]) * eta_r[i1][:, None])
        fe = fe - rho * a_wl_area * _mv(CaM, ae)
        fe = fe - 0.25 * rho * a_wl_area * (ge1[i1] * np.conj(eta_r[i2])[:, None] + np.conj(ge1[i2]) * eta_r[i1][:, None])
        Q += translate_force_3to6(fe.T, r_int).T
    return Q


def _omega_mat(v):
    """-getH(v) for a stack of vectors (raft/raft_fowt.py:1556-1557)."""
    n = len(v)
    H = np.zeros([n, 3, 3], dtype=complex)
    H[:, 0, 1], H[:, 0, 2] = v[:, 2], -v[:, 1]
    H[:, 1, 0], H[:, 1, 2] = -v[:, 2], v[:, 0]
    H[:, 2, 0], H[:, 2, 1] = v[:, 1], -v[:, 0]
    return -H


def hydro_force_2nd(qtf, w1_2nd, w, S0, dw):
    """calcHydroForce_2ndOrd 'qtf' mode (raft/raft_fowt.py:1788-1810): bilinear resample of
    the QTF to (w, w) with 0 outside the QTF grid (Q13), difference-frequency diagonals."""
    from scipy.interpolate import RegularGridInterpolator
    nw = len(w)
    f = np.zeros([6, nw])
    fm = np.zeros(6)
    X, Y = np.meshgrid(w, w)
    pts = np.stack([Y.ravel(), X.ravel()], axis=-1)
    for d in range(6):
        re = RegularGridInterpolator((w1_2nd, w1_2nd), qtf[:, :, 0, d].real, bounds_error=False, fill_value=0)(pts)
        im = RegularGridInterpolator((w1_2nd, w1_2nd), qtf[:, :, 0, d].imag, bounds_error=False, fill_value=0)(pts)
        Qi = (re + 1j * im).reshape(nw, nw)
        for mu in range(1, nw):
            Saux = np.zeros(nw)
            Saux[0:nw - mu] = S0[mu:]
            Qaux = np.zeros(nw, dtype=complex)
            Qaux[0:nw - mu] = np.diag(Qi, mu)
            f[d, mu] = 4 * np.sqrt(np.sum(S0 * Saux * np.abs(Qaux) ** 2)) * dw
        fm[d] = 2 * np.sum(S0 * np.diag(Qi.real, 0)) * dw
    f[:, 0:-1] = f[:, 1:]
    f[:, -1] = 0
    return fm, f


def hydro_force_2nd_spectrum(qtf, w1_2nd, w, S0, dw):
    """calcHydroForce_2ndOrd 'spectrum' mode (raft/raft_fowt.py:1760-1784, 1809-1810): the
    force spectrum on the QTF grid from the resampled wave spectrum, then resampled to w."""
    nw1 = len(w1_2nd)
    nw = len(w)
    S = np.interp(w1_2nd, w, S0, left=0, right=0)
    mu = w1_2nd - w1_2nd[0]
    d1 = w1_2nd[1] - w1_2nd[0]
    f = np.zeros([6, nw], dtype=complex)
    fm = np.zeros(6)
    for d in range(6):
        Q = qtf[:, :, 0, d]
        Sf = np.zeros(nw1)
        for imu in range(1, nw1):
            Saux = np.zeros(nw1)
            Saux[0:nw1 - imu] = S[imu:]
            Qaux = np.zeros(nw1, dtype=complex)
            Qaux[0:nw1 - imu] = np.diag(Q, imu)
            Sf[imu] = 8 * np.sum(S * Saux * np.abs(Qaux) ** 2) * d1
        fm[d] = 2 * np.sum(S * np.diag(Q.real, 0)) * d1
        f[d, :] = np.sqrt(2 * np.interp(w - w[0], mu, Sf, left=0, right=0) * dw)
    f[:, 0:-1] = f[:, 1:]
    f[:, -1] = 0
    return fm, f
