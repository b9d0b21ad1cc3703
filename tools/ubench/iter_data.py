"""Per-case drag-iteration counts of the C2 bench batch (512 seeded JONSWAP sea states on
VolturnUS-S_example, nw = 1000) with the sea-state parameters and the closest convergence call:
the data behind the launch-order heuristic (solver.balanced_order).  Writes gpurun_out/iter_data.json."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main():
    import torch
    import bench
    from raft.solver import CaseSet, prepare_batch, solve_batch
    torch.cuda.set_device(0)
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    out = {}
    for seed in (20241016, 20241017, 20241018):
        cases = bench.sea_states(512, seed)
        cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases],
                     ["JONSWAP"] * len(cases), [c["wave_height"] for c in cases], [c["wave_period"] for c in cases],
                     [0.0] * len(cases))
        prep = prepare_batch([dd], cs)
        r = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("std", "margin"), prepared=prep)
        torch.cuda.synchronize()
        out[str(seed)] = {"Hs": [c["wave_height"] for c in cases], "Tp": [c["wave_period"] for c in cases],
                          "heading": [c["wave_heading"] for c in cases],
                          "iters": r["iters"].cpu().numpy().tolist(), "margin": r["margin"].cpu().numpy().tolist(),
                          "std": r["std"].cpu().numpy().tolist(), "order": prep["order"].cpu().numpy().tolist()}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "iter_data.json"), "w") as fh:
        json.dump(out, fh)
    print("ok", {k: float(np.mean(v["iters"])) for k, v in out.items()})


if __name__ == "__main__":
    main()
