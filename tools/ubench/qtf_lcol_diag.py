"""Check the MFMA QTF path's global-motion L columns (lcoef_block, y < 18) against a NumPy
restatement of node_force_z / wl_probe evaluated on the same device tables (read back from the
workspace after the call): VolturnUS-S, 24 frequencies, a random RAO in one DOF, M66 = 0 (no
Pinkster column).  Prints, per probe g, the relative difference of the column."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

QT = dict(U=0, VP=3, VA=6, DR=7, GU=10, GP=19, DWDZ=22, COUNT=23)
WT = dict(ETAR=0, UD=1, A=4, GE=7, COUNT=10)
FT_OM, FT_COUNT = 12, 15
KKAYT = 8


def skew(o):   # o [..., 3] -> [..., 3, 3], O x = o x x
    O = np.zeros(o.shape[:-1] + (3, 3), dtype=complex)
    O[..., 0, 1], O[..., 0, 2] = -o[..., 2], o[..., 1]
    O[..., 1, 0], O[..., 1, 2] = o[..., 2], -o[..., 0]
    O[..., 2, 0], O[..., 2, 1] = -o[..., 1], o[..., 0]
    return O


def mv(M, x):
    return np.einsum("...ij,...j->...i", M, x)


def dlin(j, x, y, z):
    return [np.array([1., 0, 0]), np.array([0, 1., 0]), np.array([0, 0, 1.]), np.array([0, -z, y]),
            np.array([z, 0, -x]), np.array([-y, x, 0])][j]


def main():
    import torch
    import raft
    from conftest import load_design, load_golden, statics_of
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    T = load_golden("c2_nw200")
    d = load_design("VolturnUS-S_example")
    d["platform"]["outFolderQTF"] = None
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    dd = f.device_design()
    w2 = np.linspace(0.3, 1.8, 24)
    k2 = wave_numbers(w2, f.depth)
    rng = np.random.default_rng(9)
    beta = np.deg2rad(20.0)
    for jx in (3, 5):
        X = np.zeros((6, f.nw), dtype=complex)
        X[jx] = (rng.normal(size=f.nw) + 1j * rng.normal(size=f.nw)) * 0.5
        Xt = torch.tensor(X, dtype=torch.complex128, device=dd.device)
        MM = torch.zeros([6, 6], dtype=torch.float64, device=dd.device)
        qd = QtfDevice(f, w2, k2, beta, 0)
        qd.qtf(dd.w, Xt, MM)
        torch.cuda.synchronize()
        W = qd.work.cpu().numpy()
        n2, nq, nmq, nkr = qd.n2, qd.nq, qd.nmq, qd.nkr
        n2p = (n2 + 15) & ~15
        kb = 8 * nq + 3 * nmq + 18
        kp = (kb + 15) & ~15
        o = 0
        node = W[o:o + nq * QT["COUNT"] * n2].reshape(nq, QT["COUNT"], n2); o += nq * QT["COUNT"] * n2
        wl = W[o:o + nmq * WT["COUNT"] * n2].reshape(nmq, WT["COUNT"], n2); o += nmq * WT["COUNT"] * n2
        freq = W[o:o + FT_COUNT * n2].reshape(FT_COUNT, n2); o += FT_COUNT * n2
        o += nkr * n2 * 12 + (nkr * n2 * KKAYT + 1) // 2
        o += kp * n2p                                   # R
        L = W[o:o + 6 * kp * n2p].reshape(6, kp, n2p)[:, :, :n2]
        qn = np.asarray(qd.host["qnode"])
        qmt = np.asarray(qd.host["qmemb"])
        rho, g = qd.rho, qd.g
        w = w2
        om1 = freq[FT_OM:FT_OM + 3].T                   # [n2, 3]
        ref = np.zeros([18, n2, 6], dtype=complex)
        alt = {k: np.zeros([n2, 6], dtype=complex) for k in ("no_om", "om_only", "D_neg", "om_x", "om_y", "om_pos")}
        for n in range(nq):
            x, y, z = qn[0:3, n]
            qv = qn[3:6, n]
            rv, rve, ai = rho * qn[6, n], rho * qn[7, n] * qn[9, n], qn[8, n]
            CM, CA, P12, QM = (qn[b:b + 9, n].reshape(3, 3) for b in (10, 19, 28, 37))
            T_ = node[n]
            u1, vp1, dr1, gp1 = (T_[QT[k]:QT[k] + 3].T for k in ("U", "VP", "DR", "GP"))
            G1 = T_[QT["GU"]:QT["GU"] + 9].T.reshape(n2, 3, 3)
            dz1, va1 = T_[QT["DWDZ"]], T_[QT["VA"]]
            ur1 = u1 - vp1
            O1 = skew(om1)
            for gg, var in [(gg, None) for gg in range(12)] + [(11, k) for k in alt]:
                j = gg % 6
                D = dlin(j, x, y, z)
                if var == "om_only":
                    D = 0 * D
                if var == "D_neg":
                    D = -D
                zdr = zvp = zom = None
                zva = 0
                if gg < 6:
                    zdr = np.broadcast_to(D.astype(complex), (n2, 3))
                else:
                    v = -1j * D
                    vq = v @ qv
                    zvp = np.broadcast_to(v - vq * qv, (n2, 3))
                    zva = -vq
                    if j >= 3:
                        e = np.zeros(3, complex); e[j - 3] = -1j
                        if var == "om_x":
                            e = np.array([-1j, 0, 0])
                        if var == "om_y":
                            e = np.array([0, -1j, 0])
                        if var == "om_pos":
                            e = -e
                        if var == "no_om":
                            e = 0 * e
                        zom = np.broadcast_to(e, (n2, 3))
                Z3 = np.zeros((n2, 3), complex)
                zdr_ = Z3 if zdr is None else zdr
                zvp_ = Z3 if zvp is None else zvp
                vM = 0.25 * mv(G1, 1j * w[:, None] * zdr_)
                ur2 = -zvp_
                sq = -0.25 * rho * np.sum(mv(P12, ur1) * mv(CA, ur2), axis=1)
                sq = sq + 0.25 * np.sum(gp1 * zdr_, axis=1)
                v3 = 0.25 * dz1[:, None] * (-zvp_)
                vA = v3 - (v3 @ qv)[:, None] * qv
                vA = vA - 0.5 * mv(O1, zva * np.broadcast_to(qv, (n2, 3)))
                O2c = skew(Z3 if zom is None else zom)
                vA = vA - 0.5 * mv(O2c, va1[:, None] * qv)
                V1 = G1 + O1
                ax = 0.25 * mv(V1, mv(CA, ur2))
                vA = vA - 0.25 * mv(V1, ur2 - mv(QM, ur2))
                ax = ax + 0.25 * mv(O2c, mv(CA, ur1))
                vA = vA - 0.25 * mv(O2c, ur1 - mv(QM, ur1))
                fr = ax - mv(QM, ax) + mv(CA, vA)
                fo = mv(rv * CM + rve * QM, vM) + rv * fr + ai * sq[:, None] * qv
                if zdr is None and zvp is None:
                    continue
                tgt = ref[gg] if var is None else alt[var]
                tgt[:, :3] += fo
                tgt[:, 3:] += np.cross([x, y, z], fo)
        for mm in range(nmq):
            if qmt[0, mm] == 0:
                continue
            x, y, z = qmt[1:4, mm]
            ra = rho * qmt[4, mm]
            CM, CA = qmt[5:14, mm].reshape(3, 3), qmt[14:23, mm].reshape(3, 3)
            p1, p2 = qmt[23:26, mm], qmt[26:29, mm]
            Wm = wl[mm]
            e1, ud1, a1, ge1 = Wm[WT["ETAR"]], Wm[WT["UD"]:WT["UD"] + 3].T, Wm[WT["A"]:WT["A"] + 3].T, Wm[WT["GE"]:WT["GE"] + 3].T
            for gg in list(range(6)) + list(range(12, 18)):
                j = gg % 6
                D = dlin(j, x, y, z)
                ze = 0.0
                zge = np.zeros(3)
                za = np.zeros(3, complex)
                if gg < 6:
                    ze = -D[2]
                    e3, e4 = float(j == 3), float(j == 4)
                    c1, c2 = e3 * p1[1] - e4 * p1[0], e3 * p2[1] - e4 * p2[0]
                    zge = -g * (c1 * p1 + c2 * p2)
                else:
                    za = -D
                fe = 0.25 * (ud1 * ze)
                ae = 0.25 * (a1 * ze + za[None, :] * e1[:, None])
                gt = ge1 * ze + zge[None, :] * e1[:, None]
                fo = ra * mv(CM, fe) - ra * mv(CA, ae) - 0.25 * ra * gt
                ref[gg, :, :3] += fo
                ref[gg, :, 3:] += np.cross([x, y, z], fo)
        c0 = 8 * nq + 3 * nmq
        wl11 = 0.0                                      # no waterline column for g = 11
        print(f"RAO DOF {jx}:", flush=True)
        for gg in range(18):
            got = L[:, c0 + gg, :].T
            den = max(np.abs(ref[gg]).max(), 1e-300)
            if gg == 11:
                for k, A in alt.items():
                    B = A.copy()
                    B += ref[11] - ref11_nodes if False else 0
                    print(f"     alt {k:8s}: node part rel diff vs device {np.abs(got - wl11 - A).max() / den:.2e}", flush=True)
            print(f"  g {gg:2d}: |ref| {np.abs(ref[gg]).max():.3e}  rel diff {np.abs(got - ref[gg]).max() / den:.2e}", flush=True)


if __name__ == "__main__":
    main()
