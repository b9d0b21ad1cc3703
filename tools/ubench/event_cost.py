"""Cost of per-step timing events: wall-clock time per bench step (C2: wave tables + batched
solve of 512 cases; C4: Model.analyzeArrayBatch of 512 farm cases) over 100 back-to-back steps,
with no events in the loop and with the bench's per-step events (C2: 3, C4: 4)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def timeit(torch, fn, K, nev):
    stream = torch.cuda.current_stream()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(nev)] for _ in range(K)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        fn(ev[i], stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


def main():
    import torch
    import bench
    from raft.solver import CaseSet, prepare_batch, solve_batch
    torch.cuda.set_device(0)
    m, f, T = bench.build_model(0)
    dd = f.device_design()
    cases = bench.sea_states(512, 20241016)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    want = ("psd", "std", "zeta", "rao")

    def c2(ev, stream):
        if ev:
            ev[0].record(stream)
        dd.retabulate()
        if ev:
            ev[1].record(stream)
        solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
        if ev:
            ev[2].record(stream)

    m4, P = bench.build_c4(0)

    def c4(ev, stream):
        if ev:
            ev[0].record(stream)
        m4.analyzeArrayBatch(prepared=P, host=False, marks=(ev[1], ev[2]) if ev else None)
        if ev:
            ev[3].record(stream)

    for fn, nev, tag in ((c2, 3, "C2"), (c4, 4, "C4")):
        timeit(torch, fn, 50, 0)
        for rep in range(2):
            a = timeit(torch, fn, 100, 0)
            b = timeit(torch, fn, 100, nev)
            print(f"{tag} ms/step: no events {a:.4f}, {nev} events per step {b:.4f}", flush=True)


if __name__ == "__main__":
    main()
