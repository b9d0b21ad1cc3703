"""Where a QTF of a new (design, grid, heading) spends its time: the native host tables
(raft/qtf.py native_tables), the whole QtfDevice construction (tables, one pinned upload,
device Hankel table, workspace) and the QTF launches.  Then 50 new QTFs end to end (the
bench's end_to_end_ms) and a cProfile of 50 QtfDevice constructions.
Run on the GPU box: python tools/ubench/qtf_cold.py [PROFILE_OUT]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from raft import qtf as Q  # noqa: E402


def main():
    T, f, dd, X, M66, w2, k2 = bench.build_qtf(0)
    for rep in range(4):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        Q.native_tables(f, 0.0)
        t.append(time.perf_counter())
        qd = Q.QtfDevice(f, w2, k2, 0.0, 0)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        print(f"rep {rep}: native_tables {d[0]:.3f} ms, QtfDevice {d[1]:.3f} ms (+ sync {d[2]:.3f}), first qtf "
              f"{d[3]:.3f} ms, warm qtf {d[4]:.3f} ms", flush=True)
    e2e, ctor = [], []
    for rep in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        qd = Q.QtfDevice(f, w2, k2, 0.0, 0)
        t1 = time.perf_counter()
        q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        e2e.append(time.perf_counter() - t0)
        ctor.append(t1 - t0)
    print("50 new QTFs: end to end median %.3f ms (min %.3f), QtfDevice median %.3f ms (min %.3f)"
          % (np.median(e2e) * 1e3, np.min(e2e) * 1e3, np.median(ctor) * 1e3, np.min(ctor) * 1e3), flush=True)
    if len(sys.argv) > 1:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for rep in range(50):
            qd = Q.QtfDevice(f, w2, k2, 0.0, 0)
        pr.disable()
        torch.cuda.synchronize()
        with open(sys.argv[1], "w") as fh:
            pstats.Stats(pr, stream=fh).sort_stats("tottime").print_stats(30)
    del q


if __name__ == "__main__":
    main()
