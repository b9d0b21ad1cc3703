"""C2-shaped batches on other frequency grids: VolturnUS-S_example with min_freq = 0.2 / nw
(max 0.2 Hz), 512 seeded JONSWAP cases, the default dispatch (k_solve_lds: one pass for
nw <= 1024, two passes with XiLast in the Xi_last block up to 2048).  Prints the kernel that ran, ms per launch (HIP events
over 10 launches), mean iterations and the SURVEY.md §8(d) roofline fraction.
usage: python tools/ubench/time_grid.py NW[:a0|:gen] [...]   (":a0": rh_set_a0(ctx, 1) for that run,
the opt-in batch GEMM of the iteration-0 phase-A sums; ":gen": the general kernel k_solve_cases,
rh_set_solver(ctx, 1))"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def run(nw, a0=True, gen=False):
    import json
    import torch
    import bench
    import raft
    from raft.solver import CaseSet, prepare_batch, solve_batch
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz")))
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_example.json")) as fh:
        design = json.load(fh)
    design["settings"]["min_freq"] = 0.2 / nw
    m = raft.Model(design, statics=[{k: T[k] for k in ["M_struc", "B_struc", "C_struc", "C_hydro", "C_moor"]}], device=0)
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    from raft import _native as N
    N.check(N.lib().rh_set_a0(N.context(0), int(a0)), "rh_set_a0")
    N.check(N.lib().rh_set_solver(N.context(0), int(gen)), "rh_set_solver")
    want = ("psd", "std", "zeta", "rao")
    for _ in range(3):
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    iters = res["iters"].cpu().numpy()
    circ = dd.node[bench.N_CIRC()].cpu().numpy()
    nc, nr = int((circ != 0).sum()), int((circ == 0).sum())
    flops = float(sum(bench.flops_per_case(int(n), dd.nw, nc, nr, dd.nn) for n in iters))
    frac = flops / (ms * 1e-3) / bench.PEAK_FP64
    N.check(N.lib().rh_set_a0(N.context(0), 0), "rh_set_a0")
    N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")
    kname = "rh::k_solve_cases (general)" if gen else bench.solve_kernel_name(dd.nw)
    print(f"nw={dd.nw:5d} a0={int(a0)} {kname:36s} {ms:8.3f} ms/launch  iters {iters.mean():.2f}  "
          f"{512 / (ms * 1e-3):.3e} cases/s  frac {frac:.3f}", flush=True)


if __name__ == "__main__":
    for a in sys.argv[1:]:
        run(int(a.split(":")[0]), a.endswith(":a0"), a.endswith(":gen"))
