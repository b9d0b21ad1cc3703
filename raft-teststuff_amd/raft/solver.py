"""Batched response solve on the device: the throughput path behind Model.solveDynamics /
analyzeCases and bench.py.

A batch is any number of sea-state cases over one or more DeviceDesigns that share a
frequency grid.  One C-ABI call (rh_solve_cases) runs the full drag fixed point of every
case, one workgroup per case; cases are launched sorted by (design, heading) so the
blocks an XCD receives stream the same wave tables out of its L2.
"""
import ctypes
import os

import numpy as np

from . import _native as N
from .hydro_math import DEG2RAD


class CaseSet:
    """Host description of a batch of cases, all with a single sea state (nWaves = 1).

    design_idx : index into the design list, per case
    heading    : wave heading [deg]
    spectrum   : 'JONSWAP' | 'unit' | 'constant' | 'none' (or integer codes)
    Hs, Tp, gamma : wave_height, wave_period, wave_gamma (0 -> IEC automatic)
    """

    def __init__(self, design_idx, heading, spectrum, Hs, Tp, gamma):
        n = len(heading)
        self.n = n
        self.design_idx = np.broadcast_to(np.asarray(design_idx, dtype=np.int32), (n,)).copy()
        self.heading = np.asarray(heading, dtype=float)
        spa = np.asarray(spectrum)
        if spa.dtype.kind in "iu":     # integer codes already
            self.spectrum = np.broadcast_to(spa.astype(np.int32), (n,)).copy()
        else:
            sp = np.broadcast_to(np.asarray(spectrum, dtype=object), (n,))
            self.spectrum = np.array([s if isinstance(s, (int, np.integer)) else N.SPECTRUM_CODES[str(s)] for s in sp],
                                     dtype=np.int32)
        self.Hs = np.broadcast_to(np.asarray(Hs, dtype=float), (n,)).copy()
        self.Tp = np.broadcast_to(np.asarray(Tp, dtype=float), (n,)).copy()
        self.gamma = np.broadcast_to(np.asarray(gamma, dtype=float), (n,)).copy()


class BatchResult(dict):
    """Device tensors of one batched solve (keys: Xi, iters, status, zeta, B_drag, psd, std,
    Bmat, rao, Z when requested)."""

    def host(self):
        return {k: v.cpu().numpy() for k, v in self.items()}


def solve_batch(designs, cases, nIter, XiStart=0.0, tol=0.01, want=("psd", "std", "zeta", "B_drag"),
                fext=None, stream=None, prepared=None, Xi_init=None, first_iter=0, F_wave=None, out=None):
    """Run rh_solve_cases.  `designs`: list of DeviceDesign (same nw); `cases`: CaseSet.
    Returns a BatchResult of device tensors (stream-ordered; caller synchronises).
    want may include "Xi_prev" (the un-relaxed XiLast of the final iteration), "margin"
    (the closest call of the convergence test per case, rh_solve_out.margin) and "noXi" (no
    response output: the linearisation only, for callers that form the response themselves,
    Model.analyzeArrayBatch; then no psd / std / rao either); Xi_init /
    first_iter restart a fixed point from such a state (potSecOrder=1 second pass).  F_wave: a
    contiguous complex128 [ncase, 6, nw] tensor that receives each case's wave excitation with
    its final linearisation (rh_solve_out.F_wave; the F of an array solve, Model.analyzeArrayBatch).
    out: optional dict of preallocated contiguous output tensors (e.g. slices of a whole sweep's
    outputs, raft/batch.py solve_sweep) used instead of fresh ones for the keys it holds."""
    from .sweep_block import BlockDesigns
    if isinstance(designs, BlockDesigns):     # a sweep block: its descriptors already written (sweep_block.py)
        if prepared is None:
            raise ValueError("solve_batch: a BlockDesigns batch comes with its prepared case columns")
        torch, dev, nw, dev_index = designs.torch, designs.device, designs.nw, designs.dev_index
    else:
        d0 = designs[0]
        torch, dev, nw, dev_index = d0.torch, d0.device, d0.nw, d0.dev_index
        for d in designs:
            if d.nw != nw:
                raise ValueError("all designs in a batch must share the frequency grid")
    prep = prepared if prepared is not None else prepare_batch(designs, cases)
    ncase = cases.n
    given = out or {}
    out = BatchResult()
    c128 = dict(dtype=torch.complex128, device=dev)
    f64 = dict(dtype=torch.float64, device=dev)
    i32 = dict(dtype=torch.int32, device=dev)

    def put(key, shape, kw):
        t = given.get(key)
        if t is None:
            t = torch.empty(shape, **kw)
        elif list(t.shape) != shape or t.dtype != kw["dtype"] or not t.is_contiguous():
            raise ValueError(f"out[{key!r}]: expected a contiguous {kw['dtype']} tensor of shape {shape}")
        out[key] = t

    if "noXi" not in want or nw > N.lib().rh_solve_noxi_max_bins():   # "noXi": the linearisation only (zeta / Bmat / B_drag);
        put("Xi", [ncase, 6, nw], c128)                                # the two-pass grids store it regardless
    xl = torch.empty([ncase, 6, nw], **c128)
    put("iters", [ncase], i32)
    put("status", [ncase], i32)
    nnmax = designs.nnmax if isinstance(designs, BlockDesigns) else max(d.nn for d in designs)
    for key, shape, kw in (("zeta", [ncase, nw], f64), ("B_drag", [ncase, 6, 6], f64),
                           ("Bmat", [ncase, nnmax, 3, 3], f64), ("psd", [ncase, 6, nw], f64), ("std", [ncase, 6], f64),
                           ("rao", [ncase, 6, nw], c128), ("Z", [ncase, nw, 6, 6], c128),
                           ("Xi_prev", [ncase, 6, nw], c128), ("margin", [ncase], f64)):
        if key in want:
            put(key, shape, kw)
    for t, shape in ((fext, [ncase, 6, nw]), (Xi_init, [ncase, 6, nw]), (F_wave, [ncase, 6, nw])):
        if t is not None and (list(t.shape) != shape or t.dtype != torch.complex128 or not t.is_contiguous()):
            raise ValueError(f"expected a contiguous complex128 tensor of shape {shape}")
    cs = N.RhCases()
    cs.ncase = ncase
    cs.design, cs.head, cs.spectrum = N.ptr(prep["design"]), N.ptr(prep["head"]), N.ptr(prep["spectrum"])
    cs.Hs, cs.Tp, cs.gamma = N.ptr(prep["Hs"]), N.ptr(prep["Tp"]), N.ptr(prep["gamma"])
    cs.nIter, cs.XiStart, cs.tol = int(nIter), float(XiStart), float(tol)
    cs.fext = N.ptr(fext)
    cs.order = N.ptr(prep["order"])
    cs.Xi_init, cs.first_iter = N.ptr(Xi_init), int(first_iter)
    cs.group_start, cs.ngroup = N.ptr(prep["group_start"]), int(prep["ngroup"])
    o = N.RhSolveOut()
    o.Xi, o.Xi_last, o.iters, o.status = N.ptr(out.get("Xi")), N.ptr(xl), N.ptr(out["iters"]), N.ptr(out["status"])
    for k in ["zeta", "B_drag", "Bmat", "psd", "std", "rao", "Z", "Xi_prev", "margin"]:
        setattr(o, k, N.ptr(out.get(k)))
    o.F_wave = N.ptr(F_wave)
    arr = designs.arr if isinstance(designs, BlockDesigns) else (N.RhDesign * len(designs))(*[d.struct() for d in designs])
    s = stream if stream is not None else N.stream_handle(torch, dev)
    N.check(N.lib().rh_solve_cases(N.context(dev_index), arr, len(designs), ctypes.byref(cs), ctypes.byref(o), s),
            "rh_solve_cases")
    out._keep = (xl, prep, arr, fext, Xi_init, F_wave)
    return out


def prepare_batch(designs, cases, tables_stream=None):
    """Upload per-case parameters and make sure every design has the wave tables its cases
    need.  Reusable across repeated solves of the same batch (bench steady state).
    tables_stream: launch a fresh sweep's batched wave tables on that stream (the uploads
    stay on the current one; raft/batch.py solve_sweep)."""
    torch = designs[0].torch
    dev = designs[0].device
    if cases.n and (cases.design_idx.min() < 0 or cases.design_idx.max() >= len(designs)):
        raise ValueError("design index out of range")
    used = np.unique(cases.design_idx)
    if len(used) > 1 and all(designs[int(i)].uhat is None for i in used):
        # a fresh multi-design batch (a sweep): every table in one launch
        from .prep import tabulate_batch
        head = tabulate_batch(designs, cases.design_idx, cases.heading * DEG2RAD, launch_stream=tables_stream)
    else:
        head = np.zeros(cases.n, dtype=np.int32)
        for di in used:
            d = designs[int(di)]
            sel = np.nonzero(cases.design_idx == di)[0]
            head[sel] = d.ensure_headings(cases.heading[sel] * DEG2RAD)
    # Lock-step groups (k_solve_grp) exist only in tools/ubench variant builds of the library
    # (rh_group_cases() > 1 there) and are opt-in even then: RAFT_GROUP_WIDTH=2.  Measured on
    # the C2 batch they halve the wave-table stream but not the time per case.
    width = min(N.lib().rh_group_cases(), int(os.environ.get("RAFT_GROUP_WIDTH", "1") or 1))
    if width > 1:
        # design-major, then heading; within a (design, heading) run by sea state, so that
        # the cases solved in lock-step by one workgroup tend to need the same iterations
        order = np.lexsort((cases.Tp, cases.Hs, head, cases.design_idx)).astype(np.int32)
        gstart = case_groups(cases.design_idx[order], head[order], width)
    else:
        order = balanced_order(cases, head)
        gstart = None
    # two uploads (the int and the float case columns), each column a view
    n = cases.n
    ints = torch.from_numpy(np.concatenate([cases.design_idx, np.asarray(head, dtype=np.int32), cases.spectrum,
                                            order]).astype(np.int32, copy=False)).to(dev)
    flts = torch.from_numpy(np.concatenate([cases.Hs, cases.Tp, cases.gamma]).astype(np.float64, copy=False)).to(dev)
    return dict(design=ints[:n], head=ints[n:2 * n], spectrum=ints[2 * n:3 * n], order=ints[3 * n:4 * n],
                Hs=flts[:n], Tp=flts[n:2 * n], gamma=flts[2 * n:3 * n], head_host=head,
                group_start=None if gstart is None else torch.tensor(gstart, dtype=torch.int32, device=dev),
                ngroup=0 if gstart is None else len(gstart) - 1)


def balanced_order(cases, head, nxcd=8):
    """Launch order of one-case-per-workgroup batches.  Design-major, then heading, so an
    XCD's contiguous slice of the order (xcd_remap) streams few tables out of its L2; then
    the longest peak period first.  Each pair of adjacent XCD slices is re-dealt so both get
    the same mix of periods.  Longer periods tend to need more drag iterations, so no XCD
    collects the long cases, and within a slice the long ones are dispatched first.  The
    order changes placement only, never results.  Measured on the C2 bench batch (512
    cases, 2 per CU): the last CU finishes after 9.5 instead of 10.5 case-iterations
    (tools/ubench/makespan.py).  A pair whose cases span more than two wave tables is not
    re-dealt: its slices already hold whole tables with their full period mix.  Sorting such
    a pair by period had put the cases of ~12 designs (12 wave
    tables of 2.5 MB) on an XCD at once in the C5 sweep: its L2 hit rate fell to 47 % and a
    2000-case launch fetched 25 GB (profiles/r05_v9/c5_order.txt)."""
    order = np.lexsort((-cases.Tp, head, cases.design_idx))
    G = len(order)
    q, r = G // nxcd, G % nxcd
    bounds = [x * q + min(x, r) for x in range(nxcd + 1)]
    out = order.copy()
    for x in range(0, nxcd - 1, 2):
        a0, a1, a2 = bounds[x], bounds[x + 1], bounds[x + 2]
        seg = order[a0:a2]
        tables = np.unique(cases.design_idx[seg].astype(np.int64) * (int(np.max(head)) + 1) + head[seg])
        if len(tables) > 2:
            continue
        seg = seg[np.argsort(-cases.Tp[seg], kind="stable")]
        na, nb = a1 - a0, a2 - a1
        m = min(na, nb)
        to_a = np.zeros(na + nb, dtype=bool)
        to_a[0:2 * m:2] = True          # dealt alternately ...
        if na > nb:
            to_a[2 * m:] = True          # ... and the larger slice takes what is left
        out[a0:a1] = seg[to_a]
        out[a1:a2] = seg[~to_a]
    return out.astype(np.int32)


def case_groups(design, head, width):
    """Offsets of the lock-step groups of rh_cases.group_start: consecutive (already sorted)
    cases with equal design and heading index, at most `width` per group."""
    n = len(design)
    if n == 0:
        return np.zeros(1, dtype=np.int32)
    starts = [0]
    for i in range(1, n):
        if design[i] != design[i - 1] or head[i] != head[i - 1] or i - starts[-1] >= width:
            starts.append(i)
    starts.append(n)
    return np.asarray(starts, dtype=np.int32)
