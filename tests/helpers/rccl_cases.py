"""The workloads of tests/test_gpu_rccl.py, run once through a process group (the child,
helpers/rccl_world1.py) and once without (the parent): the case-sharded C2 batch with its
output gather, the tile-sharded QTF exchange of C3 and the bin-sharded drag fixed point."""
import numpy as np

from conftest import golden_cases, load_golden


def run_all(group=None):
    import torch
    from raft.parallel import assemble_qtf, gather_cases, solve_bins_sharded
    from raft.solver import CaseSet, solve_batch
    from test_gpu_parity import make_model, random_cases
    out = {}
    # C2-shaped batch (nw = 200 golden design): solve, then the all-gather of its outputs
    T = load_golden("c2_nw200")
    m, f = make_model("VolturnUS-S_example", T)
    cases = random_cases(40, 11)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    r = solve_batch([f.device_design()], cs, m.nIter, m.XiStart, 0.01, want=("psd", "std"))
    g = gather_cases({"Xi": r["Xi"], "psd": r["psd"], "std": r["std"], "iters": r["iters"]}, cs.n, group)
    for k, v in g.items():
        out["cases_" + k] = v.cpu().numpy()
    # C3 QTF at the golden grid: the packed-pair exchange and the Hermitian fill
    from test_gpu_qtf import _case, make
    Tq = load_golden("c3_qtf")
    mq, fq = make(Tq)
    fq.calcHydroExcitation(_case(Tq), memberList=fq.memberList)
    fq.calcQTF_slenderBody(0, Xi0=Tq["out_Xi0"])
    qd = fq._qtf_qd
    dd = fq.device_design()
    X = torch.tensor(Tq["out_Xi0"], dtype=torch.complex128, device=dd.device)
    M66 = torch.tensor(fq.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    q = assemble_qtf(lambda o, rk, n: qd.qtf_rows(dd.w, X, M66, o, rk, n), qd.hermitian_fill, qd.n2,
                     device=dd.device, group=group)
    out["qtf"] = q.cpu().numpy()
    # one case, bins split in two shards per rank: per-iteration all-reduces of the RMS sums and flags
    T1 = load_golden("c1_OC3spar")
    m1, f1 = make_model("OC3spar", T1)
    case = golden_cases(T1)[0]
    Xi, iters, status, B = solve_bins_sharded(f1, case, m1.nIter, m1.XiStart, group=group,
                                              shards=[(0, m1.nw // 2), (m1.nw // 2, m1.nw)])
    out.update(bins_Xi=Xi, bins_iters=np.array(iters), bins_status=np.array(status), bins_B=B)
    return out
