"""Host cost of one C2 bench step: time to enqueue K steps (no synchronisation) against the
time until they finish, and the GPU time between events around them.  If the enqueue rate is
close to the finish rate, the step is host-bound."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main():
    import torch
    import bench
    from raft.solver import CaseSet, prepare_batch, solve_batch
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    want = ("psd", "std", "zeta", "rao")

    def step():
        dd.retabulate()
        return solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    K = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(K):
        step()
    e1.record()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e3 * (t1 - t0) / K:.3f} ms/step  finish {1e3 * (t2 - t0) / K:.3f} ms/step  "
          f"gpu {e0.elapsed_time(e1) / K:.3f} ms/step", flush=True)
    # the bench's per-step timing events: wall time per step with 0, 2 and 3 events per step
    for nev in (0, 2, 3):
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
        torch.cuda.synchronize()
        a = time.perf_counter()
        for i in range(K):
            if nev == 3:
                evs[i][0].record()
            dd.retabulate()
            if nev >= 2:
                evs[i][1].record()
            solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
            if nev >= 2:
                evs[i][2].record()
        torch.cuda.synchronize()
        print(f"  {nev} timing events per step: {1e3 * (time.perf_counter() - a) / K:.3f} ms/step wall", flush=True)
    # host cost alone: the same calls with the GPU idle are not possible (they launch), so time
    # a few pieces with a synchronisation in front of each
    for name, fn in (("retabulate", lambda: dd.retabulate()),
                     ("solve_batch", lambda: solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep))):
        ts = []
        for _ in range(10):
            torch.cuda.synchronize()
            a = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - a)
        print(f"  host {name}: {1e3 * np.median(ts):.3f} ms (call returns, GPU idle before)", flush=True)


if __name__ == "__main__":
    main()
