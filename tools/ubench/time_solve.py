"""Time the C2 bench batch (512 cases, nw=1000) with the library named by RAFTHIP_LIB;
prints ms per launch, mean iterations and ms per executed iteration."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main(tag):
    import torch
    import bench
    from raft.solver import CaseSet, prepare_batch, solve_batch
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    for _ in range(3):
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("psd", "std", "zeta", "rao"), prepared=prep)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("psd", "std", "zeta", "rao"), prepared=prep)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    it = res["iters"].float().mean().item()
    print(f"{tag:10s} {ms:8.3f} ms/launch  iters {it:5.2f}  {ms / it:7.3f} ms/iter", flush=True)
    from raft import _native as N
    L = N.lib()
    if hasattr(L, "rh_prof_read"):
        import ctypes
        buf = (ctypes.c_ulonglong * 8)()
        L.rh_prof_read(buf, 1)
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("psd", "std", "zeta", "rao"), prepared=prep)
        torch.cuda.synchronize()
        L.rh_prof_read(buf, 1)
        v = list(buf)
        nwg, nit = 512, max(v[7], 1)
        names = ["prologue/WG", "A/iter", "B/iter", "C-exc/iter", "C-solve/iter", "flags/iter", "epilogue/WG"]
        per = [v[0] / nwg, v[1] / nit, v[2] / nit, v[3] / nit, v[4] / nit, v[5] / nit, v[6] / nwg]
        print("  cycles (s_memtime, wave 0): " + "  ".join(f"{n}={x:,.0f}" for n, x in zip(names, per)), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.environ.get("RAFTHIP_LIB", "default"))
