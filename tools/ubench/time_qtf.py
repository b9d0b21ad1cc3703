"""Time the C3 QTF (400x400, OC4semi) with the library named by RAFTHIP_LIB."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def time_ranks(qd, dd, X, M66, world, reps=50):
    """Each rank's share of a QTF sharded over `world` GPUs (rh_qtf_slender_rows), timed alone
    on this GPU with HIP events around `reps` back-to-back calls: one line per rank, then the
    whole QTF (rh_qtf_slender) for comparison."""
    import torch
    out = torch.zeros([qd.n2, qd.n2, 6], dtype=torch.complex128, device=dd.device)
    for r in list(range(world)) + [None]:
        call = (lambda: qd.qtf(dd.w, X, M66)) if r is None else (lambda: qd.qtf_rows(dd.w, X, M66, out, r, world))
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        print(f"{'whole QTF' if r is None else f'rank {r} of {world}':>14s}: {us:8.1f} us per call", flush=True)


def main(tag):
    import torch
    import bench
    from raft import _native as N
    from raft.qtf import QtfDevice
    T, f, dd, X, M66, w2, k2 = bench.build_qtf(0)
    qd = QtfDevice(f, w2, k2, 0.0, 0)
    if tag == "ranks":
        time_ranks(qd, dd, X, M66, int(sys.argv[2]) if len(sys.argv) > 2 else 8)
        return
    if tag == "pmc_cached":     # one whole QTF, then 20 of new RAOs with the incident parts kept
        q = qd.qtf(dd.w, X, M66)
        Xb = (X * 0.9).contiguous()
        for i in range(20):
            q = qd.qtf(dd.w, Xb if i % 2 else X, M66, incident_cached=True)
        torch.cuda.synchronize()
        print("pmc_cached: 1 + 20 QTFs", flush=True)
        return
    ref = None
    # PMC passes: the default path only (MFMA GEMMs on this sorted grid); otherwise the
    # per-pair kernel at 1, 2 and 4 waves per tile
    for waves in ((0,) if tag == "pmc" else (1, 2, 4)):
        N.check(N.lib().rh_set_qtf_path(N.context(0), 0 if tag == "pmc" else 1), "rh_set_qtf_path")
        N.check(N.lib().rh_set_qtf_waves(N.context(0), waves), "rh_set_qtf_waves")
        for _ in range(2):
            q = qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            q = qd.qtf(dd.w, X, M66)
        e1.record()
        torch.cuda.synchronize()
        qh = q.cpu().numpy()
        if ref is None:
            ref = qh
        d = np.abs(qh - ref).max() / np.abs(ref).max()
        print(f"{tag:10s} waves={waves} QTF {e0.elapsed_time(e1) / 10:8.3f} ms  maxrel vs waves=1 {d:.2e}", flush=True)
    N.check(N.lib().rh_set_qtf_waves(N.context(0), 0), "rh_set_qtf_waves")
    N.check(N.lib().rh_set_qtf_path(N.context(0), 0), "rh_set_qtf_path")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "default")
