"""Per-block host timings of the pipelined C5 sweep (raft/batch.py solve_sweep, timings=):
where the host spends the time between blocks, and when the device finishes."""
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
    chunks = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for rep in range(3):
        tm = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if os.environ.get("C5_SPECS", "1") == "1":    # the bench's path: spec records from the multipliers
            from raft.native_prep import sweep_specs
            st = {"C_moor": C_moor}
            out, keep = solve_sweep([base] * 250, st, idx, sidx, grid, device=0, chunks=chunks, timings=tm,
                                    specs=lambda a, b: sweep_specs(base, mult[a:b], statics=st), threads=P)
        else:
            out, keep = solve_sweep(variants, {"C_moor": C_moor}, idx, sidx, grid, device=0, pool=pool,
                                    chunks=chunks, timings=tm)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"rep {rep}: {dt * 1e3:.1f} ms total ({len(idx) / dt:.3e} cases/s), host done enqueuing at "
              f"{t_enq * 1e3:.1f} ms", flush=True)
        for k, t in enumerate(tm):
            print("   block %d: DesignBatch %.1f ms (host %.1f, upload %.1f), case set + tables %.1f ms, solve enqueue %.1f ms"
                  % (k, t[0] * 1e3, t[3] * 1e3, t[4] * 1e3, t[1] * 1e3, t[2] * 1e3), flush=True)
        del out, keep
    pool.close()
    pool.join()          # the workers exit before the interpreter does (no SIGTERM at exit)
