"""The C4 leg of bench.py alone (2-FOWT farm, 512 sea states per step): run under
rocprofv3 --kernel-trace --stats to split the step into kernels and host gaps."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))

if __name__ == "__main__":
    import torch
    import bench
    torch.cuda.set_device(0)
    r = bench.bench_c4(0, int(sys.argv[1]) if len(sys.argv) > 1 else 10, 1, 0, None)
    print(json.dumps({k: r[k] for k in ("value", "ms_per_step", "device_ms_per_step")} | {"kernel_ms": r["roofline"]["kernel_ms"]}))
    from raft import _native as N
    L = N.lib()
    if hasattr(L, "rh_prof_read"):      # RH_PROF builds: phase cycles of the fixed-point launches
        import ctypes
        buf = (ctypes.c_ulonglong * 12)()
        L.rh_prof_read(buf, 0)
        v = list(buf)
        nit = max(v[7], 1)
        names = ["A/iter", "B/iter", "C-exc/iter", "C-solve/iter", "flags/iter"]
        print("  cycles (s_memtime, wave 0, all launches): " + "  ".join(
            f"{n}={x / nit:,.0f}" for n, x in zip(names, v[1:6])) + f"  (Z/iter={v[8] / nit:,.0f}  LU/iter={v[9] / nit:,.0f})"
            f"  prologue+epilogue total/iter={(v[0] + v[6]) / nit:,.0f}", flush=True)
