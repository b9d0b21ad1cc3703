"""Host cost of one C4 bench step (Model.analyzeArrayBatch on 512 farm sea states): time to
enqueue K steps without synchronising against the time until they finish, then a cProfile of
the enqueue loop (top functions by own time).  If the enqueue rate is the finish rate, the step
is host-bound and the GPU waits between launches."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))


def main():
    import torch
    import bench
    torch.cuda.set_device(0)
    m, P = bench.build_c4(0)
    for _ in range(20):
        m.analyzeArrayBatch(prepared=P, host=False)
    torch.cuda.synchronize()
    K = 100
    t0 = time.perf_counter()
    for _ in range(K):
        m.analyzeArrayBatch(prepared=P, host=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {(t1 - t0) / K * 1e3:.3f} ms/step, finish {(t2 - t0) / K * 1e3:.3f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(K):
        m.analyzeArrayBatch(prepared=P, host=False)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(14)


if __name__ == "__main__":
    main()
