"""Diagnose the MFMA QTF path for RAOs with one DOF at a time:
VolturnUS-S (c2_nw200 tables) and OC4semi (c3_qtf tables), a 24-frequency sorted grid; per
motion DOF j of the RAO (all others zero), the relative difference of the MFMA
path against the per-pair kernel, the whole QTF and two blocks: w1 with no motion x w2 moving,
and both moving (the RAO is zero below 1 rad/s).  Optionally with Ca = 0 (no Rainey terms).
This is how the wrong yaw coefficient column (g = 11) was cornered; tools/ubench/
qtf_lcol_diag.py then checks the columns themselves."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import raft
    from conftest import load_design, load_golden, statics_of
    from oracle import qtf_oracle as QO
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    for tag, dname, ca0 in (("c2_nw200", "VolturnUS-S_example", None), ("c3_qtf", "OC4semi-RAFT_QTF", None),
                            ("c2_nw200", "VolturnUS-S_example", "Ca")):
        T = load_golden(tag)
        d = load_design(dname)
        d["platform"]["outFolderQTF"] = None
        if ca0:      # no added mass (Ca = 0): the Rainey (CaM) terms vanish
            for mm in d["platform"]["members"]:
                mm[ca0] = 0.0
        m = raft.Model(d, statics=[statics_of(T)])
        f = m.fowtList[0]
        f.setPosition(T["r6"])
        f.calcStatics()
        f.calcHydroConstants()
        dd = f.device_design()
        w2 = np.linspace(0.3, 1.8, 24)
        k2 = wave_numbers(w2, f.depth)
        rng = np.random.default_rng(9)
        M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
        beta = np.deg2rad(20.0)
        for j, zeroM in [(j, False) for j in range(6)] + [(5, True)]:
            X = np.zeros((6, f.nw), dtype=complex)
            if j >= 0:
                X[j] = (rng.normal(size=f.nw) + 1j * rng.normal(size=f.nw)) * 0.5
                X[j, np.asarray(f.w) < 1.0] = 0.0     # X(w2) = 0 below ~1 rad/s: the blocks below
            Xt = torch.tensor(X, dtype=torch.complex128, device=dd.device)
            MM = torch.zeros_like(M66) if zeroM else M66
            qd = QtfDevice(f, w2, k2, beta, 0)
            a = qd.qtf(dd.w, Xt, MM).cpu().numpy()
            N.check(N.lib().rh_set_qtf_path(N.context(0), 1), "path")
            p = QtfDevice(f, w2, k2, beta, 0).qtf(dd.w, Xt, MM).cpu().numpy()
            N.check(N.lib().rh_set_qtf_path(N.context(0), 0), "path")
            e = np.linalg.norm(a - p) / np.linalg.norm(p)
            per = [np.linalg.norm(a[..., d] - p[..., d]) / np.linalg.norm(p) for d in range(6)]
            # by frequency: the error's share along i1 (rows) and i2 (columns)
            er = np.linalg.norm(a - p, axis=(1, 2)); ec = np.linalg.norm(a - p, axis=(0, 2))
            lo, hi = w2 < 0.95, w2 > 1.05
            blk = lambda A, r, c: np.linalg.norm(A[np.ix_(r, c)])
            print(f"  incident(i1) x motion(i2): {blk(a - p, lo, hi) / blk(p, lo, hi):.2e}   motion x motion: "
                  f"{blk(a - p, hi, hi) / blk(p, hi, hi):.2e}", flush=True)
            print(f"{dname:22s} Ca0 {ca0} RAO DOF {j} M66 {'zero' if zeroM else 'kept'}: mfma vs pairs {e:.2e}; per DOF "
                  + " ".join(f"{x:.1e}" for x in per) + "; rows " + " ".join(f"{x:.0e}" for x in er[::4])
                  + "; cols " + " ".join(f"{x:.0e}" for x in ec[::4]), flush=True)


if __name__ == "__main__":
    main()
