"""A/B of the C2 bench batch (argv[2] cases, default 512; nw=1000) across solver modes:
0 = lock-step grouped kernel (k_solve_grp, two cases per workgroup), 2 = one case per
workgroup (k_solve_lds), 1 = general kernel.  Prints ms per launch and the agreement of
mode 0 with mode 2.  AB_SYNC=1 times isolated launches."""
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
    nc = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    cases = bench.sea_states(nc, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    os.environ["RAFT_GROUP_WIDTH"] = "2"
    prep = prepare_batch([dd], cs)             # carries group_start; mode 2 ignores it
    want = ("psd", "std", "zeta", "rao")
    out = {}
    modes = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["2", "0"])]
    for mode in modes:
        N.check(N.lib().rh_set_solver(N.context(0), mode), "rh_set_solver")
        for _ in range(3):
            res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if os.environ.get("AB_SYNC"):   # isolated launches: no overlap with the previous one
            ms = 0.0
            for _ in range(10):
                e0.record()
                res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
                e1.record()
                torch.cuda.synchronize()
                ms += e0.elapsed_time(e1) / 10
        else:
            e0.record()
            for _ in range(10):
                res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
        h = res.host()
        out[mode] = h
        it = h["iters"]
        print(f"mode {mode} n {nc} width {os.environ.get('RAFT_GROUP_WIDTH', '-')}: {ms:8.3f} ms/launch  {nc / ms * 1e3:10.0f} cases/s  iters mean {it.mean():.3f}", flush=True)
    N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")
    if 0 in out and 2 in out:
        a, b = out[0], out[2]
        same = np.array_equal(a["iters"], b["iters"]) and np.array_equal(a["status"], b["status"])
        rel = max(np.linalg.norm(a["Xi"][i] - b["Xi"][i]) / np.linalg.norm(b["Xi"][i]) for i in range(nc))
        # lock-step waste: iterations executed by groups vs by cases
        g = prep["group_start"].cpu().numpy()
        order = prep["order"].cpu().numpy()
        itg = sum(a["iters"][order[g[k]:g[k + 1]]].max() * (g[k + 1] - g[k]) for k in range(len(g) - 1))
        print(f"grouped vs ungrouped: iters/status identical {same}, max rel Xi diff {rel:.2e}, "
              f"lock-step iterations {itg} vs {a['iters'].sum()} ({itg / a['iters'].sum():.3f}x)", flush=True)


if __name__ == "__main__":
    main()
