"""Time the READ-ONLY reference's FOWT.calcQTF_slenderBody on the 24-frequency C3 subset of the
400 grid (tests/golden/c3_qtf.npz sub400_*: 300 pairs, the RAO of the reference's first
convergence), one core, and print one JSON line.  Build container only (the reference is not on
the GPU box); run by tools/calibrate_cpu.py --qtf with the reference environment of
make_golden.py:

    PYTHONPATH=tests/golden/refshim:/root/reference:tests/golden OPENBLAS_NUM_THREADS=1 \\
        python tools/ref_time_qtf.py
"""
import json
import os
import time

import numpy as np

import make_golden as G   # tests/golden/make_golden.py (imports the reference as `raft`)


def main():
    import raft.raft_fowt as rf
    rf.interp2d = G.bilinear_interp2d
    T = dict(np.load(os.path.join(G.HERE, "c3_qtf.npz")))
    design = G.load_design(os.path.join(G.REF, "examples", "OC4semi-RAFT_QTF.yaml"))
    design["platform"].pop("outFolderQTF", None)
    model = G.raft.Model(design)
    fowt = model.fowtList[0]
    case = dict(zip(design["cases"]["keys"], design["cases"]["data"][0]))
    case["wind_speed"] = 0
    G.prepare_fowt(fowt, case)
    fowt.calcHydroExcitation(case, memberList=fowt.memberList)
    fowt.w1_2nd, fowt.k1_2nd = T["sub400_w"].copy(), T["sub400_k"].copy()
    fowt.w2_2nd, fowt.k2_2nd = fowt.w1_2nd.copy(), fowt.k1_2nd.copy()
    t0 = time.perf_counter()
    fowt.calcQTF_slenderBody(0, Xi0=T["out_Xi0"], verbose=False)
    dt = time.perf_counter() - t0
    err = float(np.linalg.norm(fowt.qtf - T["sub400_qtf"]) / np.linalg.norm(T["sub400_qtf"]))
    n2 = len(fowt.w1_2nd)
    print(json.dumps({"reference_s": dt, "pairs": n2 * (n2 + 1) // 2, "rel_err_vs_fixture": err}))


if __name__ == "__main__":
    main()
