"""C5 as one rank of an N-rank launch sees it, on one GPU: rank r's contiguous case block of the
250-design x 40-sea-state sweep (raft/batch.py sweep_shard), its design blocks prepared natively
with the host threads that rank gets (bench.py: min(16, host cores // N)), pipelined against the
solve (solve_sweep), then the same launches again alone (solve only).  Three passes; the last is
reported with its per-block host timings.
usage: c5_rank.py WORLD [RANK] [THREADS] [CHUNKS] [PROFILE_OUT]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))

if __name__ == "__main__":
    import bench
    import torch
    from raft.batch import solve_sweep, sweep_cases, sweep_shard
    from raft.native_prep import SweepSpecs
    from raft.sweep import sea_state_grid, sweep_multipliers
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    threads = int(sys.argv[3]) if len(sys.argv) > 3 and int(sys.argv[3]) > 0 else max(1, min(16, bench.host_cores()[0] // world))
    chunks = int(sys.argv[4]) if len(sys.argv) > 4 and int(sys.argv[4]) > 0 else bench.c5_chunks(world)
    prof_out = sys.argv[5] if len(sys.argv) > 5 else None
    base, C_moor = bench.c5_base()
    mult = sweep_multipliers(bench.C5_DESIGNS)
    grid = sea_state_grid()
    idx_all, _ = sweep_cases(bench.C5_DESIGNS, grid)
    lo, hi, dlo, dhi = sweep_shard(idx_all, rank, world)
    st = {"C_moor": C_moor}
    local = idx_all[lo:hi] - dlo
    sidx = np.arange(lo, hi) % len(grid)
    ss = SweepSpecs(base, statics=st)
    torch.zeros(1, device="cuda")
    import gc
    gc_mode = os.environ.get("C5_GC", "")
    if gc_mode == "off":
        gc.disable()
    for rep in range(3):
        if gc_mode == "freeze":
            gc.collect()
            gc.freeze()
        tm = []
        torch.cuda.synchronize()
        if prof_out and rep == 2:
            import cProfile
            pr = cProfile.Profile()
            pr.enable()
        t0 = time.perf_counter()
        out, keep = solve_sweep([base] * (dhi - dlo), st, local, sidx, grid, device=0, chunks=chunks,
                                timings=tm, want=("psd", "std"),
                                specs=lambda a, b: SweepSpecs(base, statics=st).records(mult[dlo + a:dlo + b]) if a == 0
                                else ss.records(mult[dlo + a:dlo + b]),
                                threads=threads, first=float(os.environ.get("C5_FIRST", "1")),
                                last=float(os.environ.get("C5_LAST", "1")))
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if prof_out and rep == 2:
            pr.disable()
            import pstats
            with open(prof_out, "w") as fh:
                pstats.Stats(pr, stream=fh).sort_stats("cumulative").print_stats(45)
        if rep < 2:
            del out, keep
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        for B, cs, prep, _ in keep:
            B.solve(None, cs, want=("psd", "std"), prepared=prep)
    torch.cuda.synchronize()
    solve = (time.perf_counter() - t1) / 3
    n = hi - lo
    print(f"[first {os.environ.get('C5_FIRST', '1')} last {os.environ.get('C5_LAST', '1')}] world {world} rank {rank}: {n} cases, {dhi - dlo} designs, {threads} host threads, {chunks} blocks: end to end "
          f"{dt * 1e3:.2f} ms ({n / dt:.3e} cases/s), solve only {solve * 1e3:.2f} ms ({n / solve:.3e} cases/s), "
          f"ratio {solve / dt:.2f}; host done enqueuing at {t_enq * 1e3:.2f} ms", flush=True)
    for k, t in enumerate(tm):
        print("   block %d: DesignBatch %.2f ms (waiting for the prefetched native prep %.2f, host %.2f, upload %.2f), "
              "case set + tables %.2f ms, solve enqueue %.2f ms"
              % (k, t[0] * 1e3, t[5] * 1e3, t[3] * 1e3, t[4] * 1e3, t[1] * 1e3, t[2] * 1e3), flush=True)
