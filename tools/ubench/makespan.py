"""Iteration counts of the C2 bench batch and the dispatch makespan they imply: blocks go to
XCD b % 8 (xcd_remap gives each XCD a contiguous slice of the case order), the first 32 per XCD
start at once, later ones take the first CU that frees up.  Compares the bench's order with a
longest-first order inside each XCD slice."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def makespan(cost_of_slot, G, ncu_xcd=32):
    import heapq
    worst = 0.0
    for x in range(8):
        q, r = G >> 3, G & 7
        lo = x * q + min(x, r)
        n = q + (1 if x < r else 0)
        costs = cost_of_slot[lo:lo + n]
        cus = [0.0] * ncu_xcd
        heapq.heapify(cus)
        for c in costs:
            t = heapq.heappop(cus)
            heapq.heappush(cus, t + c)
        worst = max(worst, max(cus))
    return worst


def main():
    import bench
    from raft.solver import CaseSet, prepare_batch, solve_batch
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("std",), prepared=prep).host()
    it = res["iters"].astype(float)
    order = prep["order"].cpu().numpy()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "c2_iters.npz"), iters=res["iters"], order=order,
             Hs=[c["wave_height"] for c in cases], Tp=[c["wave_period"] for c in cases],
             head=[c["wave_heading"] for c in cases])
    print("iteration histogram:", {int(k): int(v) for k, v in zip(*np.unique(it, return_counts=True))})
    cost = it[order] + 0.25          # + prologue/epilogue in iteration units (phase profile)
    ideal = cost.sum() / 256
    ms = makespan(cost, len(cost))
    print(f"ideal {ideal:.2f}  bench order {ms:.2f} ({ms / ideal:.3f}x)")
    hs = np.asarray([c["wave_height"] for c in cases])
    tp = np.asarray([c["wave_period"] for c in cases])
    for name, key in (("Hs", hs), ("Tp", tp), ("iters(oracle)", it)):
        o2 = order.copy()
        for x in range(8):
            q, r = len(o2) >> 3, len(o2) & 7
            lo = x * q + min(x, r)
            n = q + (1 if x < r else 0)
            seg = o2[lo:lo + n]
            o2[lo:lo + n] = seg[np.argsort(-key[seg], kind="stable")]
        print(f"longest-first by {name}: {makespan(it[o2] + 0.25, len(o2)):.2f}")
    print("corr(iters, Hs) %.2f corr(iters, Tp) %.2f" % (np.corrcoef(it, hs)[0, 1], np.corrcoef(it, tp)[0, 1]))


if __name__ == "__main__":
    main()
