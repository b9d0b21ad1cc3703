"""Phase cycle counters (RH_PROF build: RAFTHIP_LIB=tools/ubench/var_prof.so) of the C2 bench
batch for solver modes given as argv[1] (2 = k_solve_lds, 0 = grouped k_solve_grp), plus the
plain ms per launch of each mode.  Counters are per workgroup-iteration (wave 0)."""
import ctypes
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
    prep = prepare_batch([dd], cs)
    want = ("psd", "std", "zeta", "rao")
    L = N.lib()
    for mode in [int(x) for x in sys.argv[1].split(",")]:
        N.check(L.rh_set_solver(N.context(0), mode), "rh_set_solver")
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
        line = f"mode {mode}: {ms:8.3f} ms/launch  {nc / ms * 1e3:10.0f} cases/s"
        if hasattr(L, "rh_prof_read"):
            buf = (ctypes.c_ulonglong * 12)()
            L.rh_prof_read(buf, 1)
            res = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=prep)
            torch.cuda.synchronize()
            L.rh_prof_read(buf, 1)
            v = list(buf)
            nwg = int(prep["ngroup"]) or nc
            nit = max(v[7], 1)
            names = ["prologue/WG", "A/it", "B/it", "Cexc/it", "Csolve/it", "(Z/it", "LU/it)", "flags/it", "epilogue/WG"]
            per = [v[0] / nwg, v[1] / nit, v[2] / nit, v[3] / nit, v[4] / nit, v[8] / nit, v[9] / nit, v[5] / nit,
                   v[6] / nwg]
            line += f"  WG-iterations {nit}  " + "  ".join(f"{n}={x:,.0f}" for n, x in zip(names, per))
        print(line, flush=True)


if __name__ == "__main__":
    main()
