"""Multi-GPU partitioning of the response solve.

One process per GPU, torch.distributed with backend "nccl" (RCCL over xGMI).  Two shardings:

* sea-state cases -- contiguous balanced blocks of the case list.  Each rank runs its block
  through rh_solve_cases with no collective inside the drag fixed point (cases are
  independent); the responses are gathered once at the end (all_gather), the "final
  response-spectrum gather" of the north star.  Weak scaling in bench.py.
* QTF (w1, w2) pairs -- upper-triangle rows dealt in snake order (round k gives rank r row
  k world + (r if k even else world-1-r)), so every rank gets n2(n2+1)/(2 world) pairs to
  within one row although rows shorten with i1.  The disjoint
  row shards are exchanged with one all-reduce(sum) of the zero-initialised [n2, n2, 6]
  matrix (x + 0 == x, so the exchange is exact), then the Hermitian lower triangle is
  filled on every rank.

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


def case_shard(n, rank, world):
    """[lo, hi) of rank's contiguous block; sizes differ by at most one."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def qtf_rows(n2, rank, world):
    """Upper-triangle rows i1 owned by rank (snake deal, as k_qtf_pairs)."""
    k = np.arange(-(-n2 // world))
    rows = k * world + np.where(k % 2 == 1, world - 1 - rank, rank)
    return rows[rows < n2]


def qtf_pairs_of(n2, rank, world):
    """Number of (i1 <= i2) pairs rank computes."""
    return int(sum(n2 - i for i in qtf_rows(n2, rank, world)))


def gather_cases(local, n_total, group=None):
    """All-gather per-case tensors ([n_local, ...]) of contiguous case blocks into
    [n_total, ...] on every rank.  `local`: dict name -> tensor."""
    import torch
    dist = _dist()
    rank, world = world_of(group)
    if world == 1:
        return dict(local)
    m = -(-n_total // world)
    out = {}
    for k, t in local.items():
        cplx = t.is_complex()
        x = torch.view_as_real(t) if cplx else t
        pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        pad[:x.shape[0]] = x
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        blocks = []
        for r in range(world):
            lo, hi = case_shard(n_total, r, world)
            blocks.append(parts[r][:hi - lo])
        y = torch.cat(blocks, 0)
        out[k] = torch.view_as_complex(y.contiguous()) if cplx else y
    return out


def assemble_qtf(compute_rows, hermitian_fill, n2, device=None, group=None):
    """Row-sharded QTF: compute_rows(out, rank, world) writes the upper-triangle rows of
    `rank` into the zeroed [n2, n2, 6] complex128 tensor `out`; the shards are summed with
    one all-reduce and hermitian_fill(out) mirrors the lower triangle."""
    import torch
    dist = _dist()
    rank, world = world_of(group)
    out = torch.zeros([n2, n2, 6], dtype=torch.complex128, device=device)
    compute_rows(out, rank, world)
    if world > 1:
        v = torch.view_as_real(out)
        dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
    hermitian_fill(out)
    return out


def solve_cases_sharded(designs, cases, nIter, XiStart=0.0, tol=0.01, want=("psd", "std", "zeta"), group=None,
                        gather=True):
    """Case-sharded batch solve: this rank solves its contiguous block of `cases`
    (solver.CaseSet); with gather=True every rank receives all cases' outputs."""
    from .solver import CaseSet, solve_batch
    rank, world = world_of(group)
    lo, hi = case_shard(cases.n, rank, world)
    sub = CaseSet(cases.design_idx[lo:hi], cases.heading[lo:hi], cases.spectrum[lo:hi], cases.Hs[lo:hi],
                  cases.Tp[lo:hi], cases.gamma[lo:hi])
    res = solve_batch(designs, sub, nIter, XiStart, tol, want=want) if sub.n else None
    if not gather:
        return res, (lo, hi)
    if res is None:
        raise ValueError("every rank needs at least one case")
    return gather_cases(dict(res), cases.n, group), (0, cases.n)
