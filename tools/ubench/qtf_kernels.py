"""Time the C3 QTF (400x400, OC4semi) on the default path; run under rocprofv3 --stats for
per-kernel times.  argv[1]: path (0 = MFMA GEMMs, 1 = per-pair kernel), argv[2]: repetitions."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main(path, reps):
    import torch
    import bench
    from raft import _native as N
    from raft.qtf import QtfDevice
    T, f, dd, X, M66, w2, k2 = bench.build_qtf(0)
    qd = QtfDevice(f, w2, k2, 0.0, 0)
    N.check(N.lib().rh_set_qtf_path(N.context(0), path), "rh_set_qtf_path")
    for _ in range(3):
        qd.qtf(dd.w, X, M66)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        qd.qtf(dd.w, X, M66)
    torch.cuda.synchronize()
    print(f"path {path}: {(time.perf_counter() - t0) / reps * 1e3:.4f} ms per QTF", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 0, int(sys.argv[2]) if len(sys.argv) > 2 else 50)
