"""Multi-GPU partitioning of the response solve.

One process per GPU, torch.distributed with backend "nccl" (RCCL over xGMI).  Two shardings:

* sea-state cases -- contiguous balanced blocks of the case list.  Each rank runs its block
  through rh_solve_cases with no collective inside the drag fixed point (cases are
  independent); the responses are gathered once at the end (all_gather), the "final
  response-spectrum gather" of the north star.  Weak scaling in bench.py.
* QTF (w1, w2) pairs -- the upper triangle in 16 x 16 pair tiles (the MFMA tile of
  rh_qtf_mfma.hip), numbered row-major and cut into contiguous blocks at the pair-count quantiles
  (row blocks balanced by pair count, to within a tile).  A rank's block spans a few w1 tile rows,
  so it computes the w1-side coefficients of those rows only and the frequency tables from its
  first row on (rh_qtf_slender_rows), not the whole grid's.  The disjoint tile shards are
  exchanged with one all_gather of each rank's packed upper-triangle pairs (exact copies),
  then the Hermitian lower triangle is filled on every rank.

The collective helpers take any process group; tests run them with gloo on the CPU.
"""
import numpy as np


def _dist():
    import torch.distributed as dist
    return dist


def world_of(group=None):
    dist = _dist()
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _collective():
    """True when a process group is initialised: the exchanges below then run through it even
    at world size 1 (an identity exchange, but through the backend -- RCCL on the GPU box:
    tests/test_gpu_rccl.py), and never without one."""
    dist = _dist()
    return dist.is_available() and dist.is_initialized()


def case_shard(n, rank, world):
    """[lo, hi) of rank's contiguous block; sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


QTF_TILE = 16


def qtf_tile_block(n2, rank, world):
    """[t0, t1) of rank's contiguous block of the row-major upper-triangle tiles, cut at the
    pair-count quantiles: t_r is the first tile whose preceding tiles hold at least r / world of
    the pairs (rh_abi.hip qtf_tile_block, the same integer arithmetic)."""
    nt = -(-n2 // QTF_TILE)
    cum = [0]
    for a in range(nt):
        ra = min(QTF_TILE * a + QTF_TILE, n2) - QTF_TILE * a
        for b in range(a, nt):
            cb = min(QTF_TILE * b + QTF_TILE, n2) - QTF_TILE * b
            cum.append(cum[-1] + (ra * (ra + 1) // 2 if a == b else ra * cb))
    total = cum[-1]

    def first(r):
        t = 0
        while cum[t] * world < r * total:
            t += 1
        return t
    return first(rank), (len(cum) - 1 if rank + 1 == world else first(rank + 1))


def qtf_tiles(n2, rank, world):
    """16 x 16 upper-triangle pair tiles (T1 <= T2) of rank, as rh_qtf_slender_rows deals
    them: tiles numbered row-major, rank's contiguous block qtf_tile_block."""
    nt = -(-n2 // QTF_TILE)
    allt = [(a, b) for a in range(nt) for b in range(a, nt)]
    t0, t1 = qtf_tile_block(n2, rank, world)
    return allt[t0:t1]


def qtf_pair_flat(n2, tiles):
    """Flat indices i1 * n2 + i2 of the pairs (i1 <= i2 < n2) of `tiles`, tile by tile."""
    out = []
    for a, b in tiles:
        i1 = np.arange(QTF_TILE * a, min(QTF_TILE * (a + 1), n2))
        i2 = np.arange(QTF_TILE * b, min(QTF_TILE * (b + 1), n2))
        I1, I2 = np.meshgrid(i1, i2, indexing="ij")
        keep = I2 >= I1
        out.append((I1 * n2 + I2)[keep])
    return np.concatenate(out) if out else np.zeros(0, int)


def qtf_pairs_of(n2, rank, world):
    """Number of (i1 <= i2) pairs rank computes."""
    return int(len(qtf_pair_flat(n2, qtf_tiles(n2, rank, world))))


def gather_cases(local, n_total, group=None, dst=None):
    """All-gather per-case tensors ([n_local, ...]) of contiguous case blocks into
    [n_total, ...] on every rank.  `local`: dict name -> tensor.  dst: gather to that rank only
    (the other ranks return their `local` block unchanged): each block crosses one xGMI link
    once instead of reaching every rank (DESIGN.md §6 byte budget)."""
    import torch
    dist = _dist()
    rank, world = world_of(group)
    if not _collective():
        return dict(local)
    m = -(-n_total // world)
    out = {}
    gdst = None if dst is None else (dist.get_global_rank(group, dst) if group is not None else dst)
    for k, t in local.items():
        cplx = t.is_complex()
        x = torch.view_as_real(t) if cplx else t
        pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        pad[:x.shape[0]] = x
        if dst is not None:
            parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
            dist.gather(pad, gather_list=parts, dst=gdst, group=group)
            if rank != dst:
                out[k] = t
                continue
        else:
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad, group=group)
        blocks = []
        for r in range(world):
            lo, hi = case_shard(n_total, r, world)
            blocks.append(parts[r][:hi - lo])
        y = torch.cat(blocks, 0)
        out[k] = torch.view_as_complex(y.contiguous()) if cplx else y
    return out


_PAIR_INDEX = {}


def qtf_pair_index(n2, rank, world, device=None):
    """Flat indices i1 * n2 + i2 of the upper-triangle pairs (i2 >= i1) of rank's tiles
    (cached per device)."""
    import torch
    key = (n2, rank, world, str(device))
    if key not in _PAIR_INDEX:
        flat = qtf_pair_flat(n2, qtf_tiles(n2, rank, world))
        _PAIR_INDEX[key] = torch.tensor(flat, dtype=torch.long, device=device)
    return _PAIR_INDEX[key]


def assemble_qtf(compute_rows, hermitian_fill, n2, device=None, group=None, on_computed=None):
    """Tile-sharded QTF: compute_rows(out, rank, world) writes the upper-triangle pairs of
    `rank`'s tiles (qtf_tiles) into the zeroed [n2, n2, 6] complex128 tensor `out`.  The shards are exchanged by
    ONE all_gather of each rank's packed upper-triangle pairs (about n2^2/2 / world pairs x
    96 B, padded to the largest shard) and scattered into place; hermitian_fill(out) then
    mirrors the lower triangle.  Pure copies, so the result is bitwise the single-device
    matrix; a rank moves ~4x fewer bytes than an all-reduce of the full matrix would."""
    import torch
    dist = _dist()
    rank, world = world_of(group)
    out = torch.zeros([n2, n2, 6], dtype=torch.complex128, device=device)
    compute_rows(out, rank, world)
    if on_computed is not None:
        on_computed()
    if _collective():
        flat = out.view(n2 * n2, 6)
        idx = [qtf_pair_index(n2, r, world, device) for r in range(world)]
        m = max(int(i.numel()) for i in idx)
        buf = torch.zeros([m, 6], dtype=torch.complex128, device=device)
        buf[:idx[rank].numel()] = flat.index_select(0, idx[rank])
        parts = [torch.empty_like(torch.view_as_real(buf)) for _ in range(world)]
        dist.all_gather(parts, torch.view_as_real(buf), group=group)
        for r in range(world):   # own shard too: the matrix is what the exchange delivered
            flat.index_copy_(0, idx[r], torch.view_as_complex(parts[r])[:idx[r].numel()])
    hermitian_fill(out)
    return out


def solve_cases_sharded(designs, cases, nIter, XiStart=0.0, tol=0.01, want=("psd", "std", "zeta"), group=None,
                        gather=True):
    """Case-sharded batch solve: this rank solves its contiguous block of `cases`
    (solver.CaseSet); with gather=True every rank receives all cases' outputs."""
    from .solver import CaseSet, solve_batch
    rank, world = world_of(group)
    if gather and cases.n < world:   # decided identically on every rank, before any collective
        raise ValueError(f"solve_cases_sharded: {cases.n} cases for {world} ranks (every rank needs one)")
    lo, hi = case_shard(cases.n, rank, world)
    sub = CaseSet(cases.design_idx[lo:hi], cases.heading[lo:hi], cases.spectrum[lo:hi], cases.Hs[lo:hi],
                  cases.Tp[lo:hi], cases.gamma[lo:hi])
    res = solve_batch(designs, sub, nIter, XiStart, tol, want=want) if sub.n else None
    if not gather:
        return res, (lo, hi)
    return gather_cases(dict(res), cases.n, group), (0, cases.n)


# ------------------------------------------------------------------------------------------
# bin sharding of ONE case
# ------------------------------------------------------------------------------------------
def bin_shard(nw, rank, world):
    """[lo, hi) of rank's contiguous block of frequency bins."""
    return case_shard(nw, rank, world)


def _all_reduce(t, op, group):
    dist = _dist()
    if t.is_cuda and dist.get_backend(group) == "gloo":     # gloo reduces host tensors
        c = t.cpu()
        dist.all_reduce(c, op=op, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=op, group=group)


def bin_fixed_point(partial, step, nn, nIter, nw, device=None, group=None, shards=None):
    """The collective skeleton of the bin-sharded drag fixed point (raft/raft_model.py:918-1000).
    Per iteration: partial(lo, hi, out) writes this rank's per-node |vrel|^2 sums [3 nn] for
    each of its bin shards (summed in shard order), one all-reduce(sum) of 3 nn doubles,
    step(sums, lo, hi, flags) solves its bins and raises flags [not converged, NaN,
    singular], one all-reduce(max) of the flags.  `shards` overrides this rank's bin ranges
    (several per process, e.g. to exercise the split on one device).
    Returns (iterations, status) with status an RH_CASE_* code."""
    import torch
    from . import _native as N
    dist = _dist()
    rank, world = world_of(group)
    coll = _collective()
    mine = shards if shards is not None else [bin_shard(nw, rank, world)]
    sums = torch.zeros(3 * nn, dtype=torch.float64, device=device)
    part = torch.empty_like(sums)
    flags = torch.zeros(3, dtype=torch.int32, device=device)
    for it in range(nIter + 1):                      # the loop runs nIter+1 times (:861)
        sums.zero_()
        for lo, hi in mine:
            partial(lo, hi, part)
            sums += part
        if coll:
            _all_reduce(sums, dist.ReduceOp.SUM, group)
        flags.zero_()
        for lo, hi in mine:
            step(sums, lo, hi, flags)
        if coll:
            _all_reduce(flags, dist.ReduceOp.MAX, group)
        f = flags.tolist()
        if f[1]:
            return it + 1, N.RH_CASE_NAN
        if f[2]:
            return it + 1, N.RH_CASE_SINGULAR
        if not f[0]:
            return it + 1, N.RH_CASE_CONVERGED
    return nIter + 1, N.RH_CASE_NOT_CONVERGED


def solve_bins_sharded(fowt, case, nIter, XiStart=0.0, tol=0.01, group=None, shards=None):
    """Model.solveDynamics' drag fixed point for one single-FOWT case with the frequency bins
    split over the ranks of `group` (rh_lin_partial_sums / rh_bin_step, include/rafthip.h).
    Every rank ends with the full response: the bin slices are exchanged with one
    all-reduce(sum) of zero-padded [6, nw] arrays (exact: x + 0 == x).
    Returns (Xi [6, nw] complex, iterations, status, B_drag [6, 6])."""
    import ctypes

    import numpy as np
    import torch
    from . import _native as N
    dist = _dist()
    case = dict(case)
    fowt.calcHydroExcitation(case, memberList=fowt.memberList)
    if fowt.nWaves != 1:
        raise NotImplementedError("solve_bins_sharded: one sea state per case")
    dd = fowt.device_design()
    nw, nn, dev = dd.nw, dd.nn, dd.device
    zeta = fowt._zeta_dev[0].contiguous()
    head = int(fowt._heads[0])
    XL = torch.full([6, nw], complex(XiStart, 0.0), dtype=torch.complex128, device=dev)
    Xi = torch.zeros([6, nw], dtype=torch.complex128, device=dev)
    Bmat = torch.empty([max(nn, 1) * 9], dtype=torch.float64, device=dev)
    Bd = torch.empty([36], dtype=torch.float64, device=dev)
    d = dd.struct()
    ctx = N.context(dd.dev_index)
    s = N.stream_handle(torch, dev)
    L = N.lib()

    def partial(lo, hi, out):
        N.check(L.rh_lin_partial_sums(ctx, ctypes.byref(d), head, N.ptr(XL), N.ptr(zeta), lo, hi, N.ptr(out), s),
                "rh_lin_partial_sums")

    def step(sums, lo, hi, flags):
        N.check(L.rh_bin_step(ctx, ctypes.byref(d), head, N.ptr(zeta), None, N.ptr(sums), float(tol), lo, hi,
                              N.ptr(Bmat), N.ptr(Bd), N.ptr(Xi), N.ptr(XL), N.ptr(flags), s), "rh_bin_step")

    iters, status = bin_fixed_point(partial, step, nn, nIter, nw, device=dev, group=group, shards=shards)
    if _collective():
        _all_reduce(torch.view_as_real(Xi), dist.ReduceOp.SUM, group)
    if status == N.RH_CASE_NAN:
        raise Exception("Nan detected in response vector Xi.")       # raft/raft_model.py:957
    if status == N.RH_CASE_SINGULAR:
        raise np.linalg.LinAlgError("Singular matrix")
    return Xi.cpu().numpy(), iters, status, Bd.cpu().numpy().reshape(6, 6)
