"""Time the C3 QTF (400x400, OC4semi, MFMA path) with the library named by RAFTHIP_LIB (default:
the in-tree librafthip.so): HIP-event time per QTF over 50 back-to-back QTFs after 5 warm-up
ones; with --save/--check, the QTF is saved to / compared with an .npy file (max relative
difference over the matrix)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--save")
    ap.add_argument("--check")
    ap.add_argument("--n", type=int, default=50)
    ap.add_argument("--path", type=int, default=0, help="rh_set_qtf_path (0 default, 2 = 32 x 32 GEMM tiles, 3 = coefficients and Kim & Yue as two launches)")
    a = ap.parse_args()
    import torch
    import bench
    from raft.qtf import QtfDevice
    T, f, dd, X, M66, w2, k2 = bench.build_qtf(0)
    qd = QtfDevice(f, w2, k2, 0.0, 0)
    from raft import _native as N
    N.check(N.lib().rh_set_qtf_path(N.context(0), a.path), "rh_set_qtf_path")
    for _ in range(5):
        q = qd.qtf(dd.w, X, M66)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.n):
        q = qd.qtf(dd.w, X, M66)
    e1.record()
    torch.cuda.synchronize()
    qh = q.cpu().numpy()
    msg = f"{a.tag:12s} QTF {e0.elapsed_time(e1) / a.n * 1e3:8.1f} us"
    if a.save:
        np.save(a.save, qh)
    if a.check:
        ref = np.load(a.check)
        msg += f"  max rel diff vs {os.path.basename(a.check)} {np.abs(qh - ref).max() / np.abs(ref).max():.2e}"
    print(msg, flush=True)


if __name__ == "__main__":
    main()
