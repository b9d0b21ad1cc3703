"""C2 batch (512 cases, nw = 1000) timed with rh_solve_cases in two passes (default) and in one
(rh_set_solver 5 / 4), alternating; HIP events over 20 launches each."""
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
    want = ("psd", "std", "zeta", "rao")
    for _ in range(200):
        solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
    for rep in range(3):
        for mode in (5, 4):
            N.check(N.lib().rh_set_solver(N.context(0), mode), "rh_set_solver")
            for _ in range(5):
                solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
            e1.record()
            torch.cuda.synchronize()
            print(f"{'two-pass' if mode == 5 else 'one-pass'} {e0.elapsed_time(e1) / 20:.3f} ms/launch", flush=True)
    N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")


if __name__ == "__main__":
    main()
