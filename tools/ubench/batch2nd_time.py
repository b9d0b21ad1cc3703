"""Time Model.analyzeCasesBatch for N potSecOrder = 1 cases of OC4semi-RAFT_QTF (one heading):
first pass, a slender-body QTF per converged case (its RAO), its force, the second pass.  With
the incident-wave cache (a design's QTFs after the first keep the Kim & Yue / basis parts) and
without it (every QTF whole).  usage: batch2nd_time.py [N]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main(n):
    import torch
    import raft
    from raft import qtf as Q
    from conftest import load_design, load_golden, statics_of
    T = load_golden("c3_qtf")
    d = load_design("OC4semi-RAFT_QTF")
    d["platform"]["outFolderQTF"] = None
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    rng = np.random.default_rng(3)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(7, 16)), wave_height=float(rng.uniform(2, 8)),
                  wave_heading=0.0, wave_gamma=0.0, wind_speed=0) for _ in range(n)]
    full = Q.QtfDevice.qtf
    res = {}
    for mode in ("cached", "whole", "cached", "whole"):
        if mode == "whole":
            Q.QtfDevice.qtf = lambda self, *a, incident_cached=False, **k: full(self, *a, **k)
        else:
            Q.QtfDevice.qtf = full
        m.analyzeCasesBatch(cases[:4])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = m.analyzeCasesBatch(cases)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res.setdefault(mode, []).append(dt)
        print(f"{mode:6s}: {n} potSecOrder=1 cases in {dt * 1e3:8.2f} ms ({dt / n * 1e3:.3f} ms per case), "
              f"second passes {int((np.asarray(r['iters_pair'])[:, 1] > 0).sum())}", flush=True)
    Q.QtfDevice.qtf = full


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 64)
