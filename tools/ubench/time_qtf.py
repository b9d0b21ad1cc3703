"""Time the C3 QTF (400x400, OC4semi) with the library named by RAFTHIP_LIB."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main(tag):
    import torch
    import bench
    T, f, qd, dd, X, M66, w2, k2, nkay, nwl = bench.build_qtf(0)
    for _ in range(2):
        qd.qtf(dd.w, X, M66)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        qd.qtf(dd.w, X, M66)
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag:10s} QTF {e0.elapsed_time(e1) / 10:8.3f} ms", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "default")
