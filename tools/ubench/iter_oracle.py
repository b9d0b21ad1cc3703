"""Drag-iteration counts of the C2 bench batches from the oracle on the CPU (no GPU): the
data for the launch-order heuristic (solver.balanced_order).  usage: iter_oracle.py OUT.json [seeds]"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _one(case):
    os.environ["OPENBLAS_NUM_THREADS"] = os.environ["OMP_NUM_THREADS"] = "1"
    from conftest import load_golden
    from oracle import raft_oracle as O
    T = load_golden("c2_nw1000")
    r = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
    return int(r["iters"])


def main():
    import bench
    seeds = [int(s) for s in sys.argv[2:]] or [20241016]
    out = {}
    with ProcessPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        for seed in seeds:
            cases = bench.sea_states(512, seed)
            it = list(ex.map(_one, cases, chunksize=8))
            out[str(seed)] = {"Hs": [c["wave_height"] for c in cases], "Tp": [c["wave_period"] for c in cases],
                              "heading": [c["wave_heading"] for c in cases], "iters": it}
            print(seed, np.bincount(it), flush=True)
    with open(sys.argv[1], "w") as fh:
        json.dump(out, fh)


if __name__ == "__main__":
    main()
