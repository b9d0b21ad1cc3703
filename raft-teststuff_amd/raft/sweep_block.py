"""One design block of a pipelined sweep (raft/batch.py solve_sweep) without a Python object per
design: the block's natively prepared tables (native_prep.PreparedDesigns, pinned) go up in
one copy, the rh_design descriptors of all its designs are written column-wise into one
record array from the preparation's layout, the wave tables of every (design, heading) pair
come from one rh_wave_tables_batch launch (kproj and finer only: the fixed point reads no
velocity table), and the solve takes the same array.  The
descriptors, tables and launches are the ones DesignBatch + prepare_batch + solve_batch make
for the same block (the same bits: tests/test_gpu_sweep.py); the host cost per block no
longer grows with a per-design object, which is what paced the first block of a sweep and a
rank's share at N > 1."""
import ctypes

import numpy as np

from . import _native as N
from .hydro_math import DEG2RAD, get_from_dict


class BlockDesigns:
    """The designs of a block as solver.solve_batch sees them: one rh_design array."""

    def __init__(self, torch, device, dev_index, arr, n, nw, nnmax, nIter, XiStart, keep):
        self.torch, self.device, self.dev_index = torch, device, dev_index
        self.arr, self.n, self.nw, self.nnmax = arr, n, nw, nnmax
        self.nIter, self.XiStart = nIter, XiStart
        self._keep = keep
        self.host_seconds = 0.0       # the block's native preparation (set by prepare_block)

    def __len__(self):
        return self.n

    def solve(self, design_idx, cases, tol=0.01, want=("psd", "std"), prepared=None, out=None):
        """solver.solve_batch of a CaseSet over the block (as DesignBatch.solve; first order)."""
        from .solver import solve_batch
        return solve_batch(self, cases, self.nIter, self.XiStart, tol, want=want, prepared=prepared, out=out)


def table_plan(design_idx, betas):
    """The wave tables a batch needs (prep.tabulate_batch's plan): per case its heading index
    in its design's tables; the designs involved (sorted) with their heading counts and the
    [len(di), hstride] heading table (rad) of the launch."""
    n = len(design_idx)
    order = np.lexsort((betas, design_idx))
    ds, bs = design_idx[order], betas[order]
    new = np.ones(n, dtype=bool)
    new[1:] = (ds[1:] != ds[:-1]) | (bs[1:] != bs[:-1])
    grp = np.cumsum(new) - 1                       # unique (design, heading) pair per sorted case
    ud, ub = ds[new], bs[new]
    first = np.ones(len(ud), dtype=bool)
    first[1:] = ud[1:] != ud[:-1]
    start = np.maximum.accumulate(np.where(first, np.arange(len(ud)), 0))
    head = np.empty(n, dtype=np.int32)
    head[order] = (np.arange(len(ud)) - start)[grp]
    di = ud[first]                                 # designs involved, with their heading runs
    bounds = np.append(np.nonzero(first)[0], len(ud))
    nh = np.diff(bounds)
    hstride = int(nh.max())
    bm = np.zeros([len(di), hstride])
    for j in range(len(di)):
        bm[j, :nh[j]] = ub[bounds[j]:bounds[j + 1]]
    return head, di, nh, hstride, bm


def prepare_block(P, designs, cases, device, compute):
    """Upload block P's tables (current stream: the caller's upload stream), write its
    descriptors, launch its wave tables on `compute` after the uploads, and upload the case
    columns.  Returns (BlockDesigns, the prepared case columns of solver.prepare_batch), or None
    when the block needs the per-design path (tables not pinned, MacCamy-Fuchs inertia tables,
    or a design without cases)."""
    import os
    from .prep import _torch
    from .solver import balanced_order
    if getattr(P, "pinned", None) is None or P.imat or cases.n == 0 or len(designs) != len(P.info):
        return None
    if any(get_from_dict((d or {}).get("platform") or {}, "potSecOrder", dtype=int, default=0) > 0
           for d in {id(d): d for d in designs}.values()):
        return None
    if int(os.environ.get("RAFT_GROUP_WIDTH", "1") or 1) > 1 and N.lib().rh_group_cases() > 1:
        return None                                        # lock-step groups: solver.prepare_batch
    torch = _torch()
    dev = torch.device("cuda", device)
    info = P.info
    nd, nw = len(info), P.nw
    head, di, nh, hstride, bm = table_plan(cases.design_idx, cases.heading * DEG2RAD)
    if len(di) != nd:
        return None
    flat = P.pinned.to(dev, non_blocking=True)
    base = flat.data_ptr()
    o, n, mo, nn, nm = (info[:, c].astype(np.int64) for c in range(5))
    nnc, nmc = np.maximum(nn, 1), np.maximum(nm, 1)
    if np.any(2 * nw + N.NF_COUNT * nnc + N.MF_COUNT * nmc + 108 != n):
        raise ValueError("prepare_block: the packed tables do not have the host_tables layout")
    rec = np.zeros(nd, dtype=np.dtype(N.RhDesign))
    p = base + 8 * o
    rec["w"] = p
    rec["k"] = p + 8 * nw
    rec["node"] = p + 16 * nw
    rec["memb"] = rec["node"] + 8 * N.NF_COUNT * nnc
    rec["M"] = rec["memb"] + 8 * N.MF_COUNT * nmc
    rec["B"] = rec["M"] + 8 * 36
    rec["C"] = rec["B"] + 8 * 36
    rec["mstart"] = base + 8 * P.packed.size + 4 * mo
    rec["nw"], rec["nn"], rec["nm"], rec["nhead"] = nw, nn, nm, nh
    rec["dw"] = float(P.w[1] - P.w[0])
    rec["depth"] = float(P.depth)
    sites = {}
    for d in designs:                                      # the site scalars once per distinct site
        if id(d["site"]) not in sites:
            sites[id(d["site"])] = (float(get_from_dict(d["site"], "rho_water", default=1025.0)),
                                    float(get_from_dict(d["site"], "g", default=9.81)))
    rg = np.array([sites[id(d["site"])] for d in designs])
    rec["rho"], rec["g"] = rg[:, 0], rg[:, 1]
    rec["pdyn_rho_g"] = 1025.0 * 9.81                      # getWaveKin defaults (prep.DeviceDesign._make_struct)
    # the block's wave tables: kproj and finer, each design's slices back to back; no velocity
    # table uhat (NULL): the fixed point reads only these two, and the sweep solves nothing else
    rows = nh * nnc * 3 * nw
    c128 = dict(dtype=torch.complex128, device=dev)
    K = torch.empty([int(rows.sum())], **c128)
    Fi = torch.empty([int(nh.sum()) * 6 * nw], **c128)
    ou = np.concatenate([[0], np.cumsum(rows)[:-1]])
    of = np.concatenate([[0], np.cumsum(nh * 6 * nw)[:-1]])
    rec["uhat"] = 0
    rec["kproj"] = K.data_ptr() + 16 * ou
    rec["finer"] = Fi.data_ptr() + 16 * of
    arr = (N.RhDesign * nd).from_buffer(rec)
    arr._rec = rec
    # case columns (solver.prepare_batch's two uploads) and the headings, on the upload stream
    order = balanced_order(cases, head)
    ncase = cases.n
    ints = torch.from_numpy(np.concatenate([cases.design_idx, head, cases.spectrum, order]).astype(np.int32, copy=False)).to(dev)
    flts = torch.from_numpy(np.concatenate([cases.Hs, cases.Tp, cases.gamma]).astype(np.float64, copy=False)).to(dev)
    beta_t = torch.from_numpy(bm).to(dev)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    compute.wait_event(ev)
    N.check(N.lib().rh_wave_tables_batch(N.context(device), arr, nd, N.ptr(beta_t), hstride,
                                         ctypes.c_void_p(compute.cuda_stream)), "rh_wave_tables_batch")
    prep = dict(design=ints[:ncase], head=ints[ncase:2 * ncase], spectrum=ints[2 * ncase:3 * ncase],
                order=ints[3 * ncase:4 * ncase], Hs=flts[:ncase], Tp=flts[ncase:2 * ncase], gamma=flts[2 * ncase:],
                head_host=head, group_start=None, ngroup=0)
    st0 = designs[0].get("settings", {})
    blk = BlockDesigns(torch, dev, device, arr, nd, nw, int(nn.max()), get_from_dict(st0, "nIter", default=15, dtype=int),
                       get_from_dict(st0, "XiStart", default=0.1, dtype=float), (flat, K, Fi, beta_t, rec))
    blk.host_seconds = getattr(P, "host_seconds", 0.0)
    return blk, prep
