"""Stage times of the C5 preparation (bench.py bench_c5) on one GPU: pooled host work,
device tables per design, wave tables per (design, heading), solve."""
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
    from raft.batch import DesignBatch, sweep_cases
    from raft.solver import prepare_batch
    from raft.sweep import sea_state_grid, sweep_multipliers, sweep_variant
    base, C_moor = bench.c5_base()
    mult = sweep_multipliers(250)
    variants = [sweep_variant(base, mult[i]) for i in range(250)]
    idx, cases = sweep_cases(250, sea_state_grid())
    torch.zeros(1, device="cuda")
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        B = DesignBatch(variants, statics={"C_moor": C_moor}, device=0, pool=pool,
                        native=os.environ.get("C5_NATIVE", "1") == "1", light=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        grid = sea_state_grid()
        cs = B.case_set_grid(idx, np.arange(len(idx)) % len(grid), grid)
        t2 = time.perf_counter()
        prep = prepare_batch(B.dds, cs)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        res = B.solve(None, cs, want=("psd", "std"), prepared=prep)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        print(f"rep {rep}: host pool {B.host_seconds*1e3:.1f} ms, device tables {B.upload_seconds*1e3:.1f} ms, "
              f"case_set {(t2-t1)*1e3:.1f} ms, prepare_batch {(t3-t2)*1e3:.1f} ms, solve {(t4-t3)*1e3:.1f} ms, "
              f"total {(t4-t0)*1e3:.1f} ms", flush=True)
    pool.close()
    pool.join()
