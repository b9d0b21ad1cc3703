"""Launch-tail analysis of the C2 batch (512 cases, nw = 1000) with an RH_WGTIME build
(RAFTHIP_LIB): per-workgroup start / end of the fixed point (s_memrealtime, 100 MHz), the
makespan against the busy time summed over workgroups (one workgroup per CU at a time:
k_solve_lds<2, 512> holds ~100 KB of LDS)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main():
    import torch
    import bench
    from raft import _native as N
    from raft.solver import CaseSet, prepare_batch, solve_batch
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    L = N.lib()
    buf = (ctypes.c_ulonglong * (2 * 512))()
    for rep in range(50):
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("std",), prepared=prep)
    torch.cuda.synchronize()
    N.check(L.rh_wgt_read(buf, 512), "rh_wgt_read")
    t = np.array(buf, dtype=np.float64).reshape(512, 2) * 10e-3   # us
    t -= t[:, 0].min()
    dur = t[:, 1] - t[:, 0]
    span = t[:, 1].max()
    ncu = 256
    print(f"makespan {span:.1f} us  busy/CU {dur.sum() / ncu:.1f} us  utilisation {dur.sum() / (ncu * span):.3f}")
    print(f"workgroup duration: min {dur.min():.1f} median {np.median(dur):.1f} max {dur.max():.1f} us")
    st = np.sort(t[:, 0])
    print(f"start times: first 256 within {st[255]:.1f} us; 257th at {st[256]:.1f}; last at {st[-1]:.1f} us")
    en = np.sort(t[:, 1])
    print(f"end times: 50% {en[255]:.1f}  90% {en[460]:.1f}  99% {en[506]:.1f}  max {en[-1]:.1f} us")

if __name__ == "__main__":
    main()
