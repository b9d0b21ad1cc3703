"""Where a cold C3 QTF spends its time: host tables, uploads, device Hankel table, workspace,
first launch.  Run on the GPU box: python tools/ubench/qtf_cold.py"""
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
        tab = Q.build_tables(f, w2, k2, 0.0)
        t.append(time.perf_counter())
        qd = Q.QtfDevice(f, w2, k2, 0.0, 0)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        d = np.diff(t) * 1e3
        print(f"rep {rep}: build_tables {d[0]:.3f} ms, QtfDevice {d[1]:.3f} ms, first qtf {d[2]:.3f} ms, "
              f"warm qtf {d[3]:.3f} ms", flush=True)
    del tab, q


if __name__ == "__main__":
    main()
