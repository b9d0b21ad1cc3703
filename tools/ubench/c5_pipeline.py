"""C5 end to end with raft/batch.py solve_sweep at several block counts (1 = no overlap of
host preparation and solve).  Three passes each; the last is reported."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))

if __name__ == "__main__":
    import bench
    pool, P = bench.c5_pool(1)
    import torch
    from raft.batch import solve_sweep, sweep_cases
    from raft.sweep import sea_state_grid, sweep_multipliers, sweep_variant
    base, C_moor = bench.c5_base()
    mult = sweep_multipliers(250)
    variants = [sweep_variant(base, mult[i]) for i in range(250)]
    grid = sea_state_grid()
    idx, _ = sweep_cases(250, grid)
    sidx = np.arange(len(idx)) % len(grid)
    torch.zeros(1, device="cuda")
    ref = None
    for chunks in [int(x) for x in (sys.argv[1:] or ["1", "3", "5", "8"])]:
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out, keep = solve_sweep(variants, {"C_moor": C_moor}, idx, sidx, grid, device=0, pool=pool, chunks=chunks)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        std = out["std"].cpu().numpy()
        if ref is None:
            ref = std
        print(f"chunks {chunks}: {dt * 1e3:.1f} ms = {len(idx) / dt:.3e} cases/s; std identical to chunks=first: "
              f"{np.array_equal(std, ref)}", flush=True)
        del out, keep
    pool.close()
    pool.join()
