"""CPU (gloo, world_size 2): the multi-GPU partitioning of raft/parallel.py -- case blocks
and their final gather, the row-sharded QTF exchange (all-gather of packed disjoint rows +
Hermitian fill) and the bin-sharded fixed point -- reproduce the single-process results
bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world=2, *args):
    port = _port()
    mp.spawn(_worker, args=(world, port, fn, args), nprocs=world, join=True)


def _worker(rank, world, port, fn, args):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


def test_case_shard_partitions_every_case_once():
    from raft.parallel import case_shard, qtf_pair_flat, qtf_pairs_of, qtf_tiles
    for n in [1, 7, 512, 10000]:
        for world in [1, 2, 3, 8]:
            blocks = [case_shard(n, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    for n2 in [42, 400, 401]:
        iu = np.triu_indices(n2)
        every = np.sort(iu[0] * n2 + iu[1])
        for world in [1, 2, 8]:
            flat = np.concatenate([qtf_pair_flat(n2, qtf_tiles(n2, r, world)) for r in range(world)])
            np.testing.assert_array_equal(np.sort(flat), every)   # every upper pair exactly once
            pairs = [qtf_pairs_of(n2, r, world) for r in range(world)]
            assert sum(pairs) == n2 * (n2 + 1) // 2
            nt = -(-n2 // 16)
            assert max(pairs) - min(pairs) <= 16 * 16 * -(-nt // world) + 256   # about a tile row


def test_sweep_shard_covers_every_case_and_its_design():
    """C5 sharding (bench.py bench_c5): contiguous blocks of the design-major case list; a
    rank's design range holds every design its cases reference, designs cut by a block
    boundary are prepared by both neighbours and by no other rank."""
    from raft.batch import sweep_cases, sweep_shard
    from raft.sweep import sea_state_grid
    for nd, ns in [(250, 40), (3, 2), (7, 5)]:
        idx, cases = sweep_cases(nd, sea_state_grid()[:ns])
        assert len(cases) == nd * ns and np.all(np.diff(idx) >= 0)
        for world in [1, 2, 3, 8]:
            seen = np.zeros(len(idx), dtype=int)
            prepared = np.zeros(nd, dtype=int)
            for r in range(world):
                lo, hi, dlo, dhi = sweep_shard(idx, r, world)
                seen[lo:hi] += 1
                prepared[dlo:dhi] += 1
                if hi > lo:
                    assert dlo <= idx[lo:hi].min() and idx[lo:hi].max() < dhi
            assert np.all(seen == 1)
            assert prepared.min() >= 1 and prepared.max() <= 2


def test_sharded_sweep_spec_blocks_match_whole_sweep():
    """bench_c5 under --gpus N: each rank builds its pipeline blocks' spec records from the
    multipliers of its own design range (specs(a, b) = sweep_specs(base, mult[dlo + a:dlo + b]))
    over raft/batch.py sweep_cuts; every design a rank solves gets the record the whole sweep
    gives it."""
    from raft.batch import sweep_cases, sweep_cuts, sweep_shard
    from raft.native_prep import sweep_specs
    from raft.sweep import sea_state_grid, sweep_multipliers
    from conftest import load_design
    base = load_design("VolturnUS-S_example")
    st = {"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}
    nd = 23
    mult = sweep_multipliers(nd, seed=3)
    whole = sweep_specs(base, mult, statics=st)
    idx, _ = sweep_cases(nd, sea_state_grid()[:4])
    for world in (1, 3, 8):
        for r in range(world):
            lo, hi, dlo, dhi = sweep_shard(idx, r, world)
            cuts = sweep_cuts(dhi - dlo, 5, 0.25, 0.5)
            for a, b in zip(cuts[:-1], cuts[1:]):
                for i, s in enumerate(sweep_specs(base, mult[dlo + a:dlo + b], statics=st)):
                    np.testing.assert_array_equal(s, whole[dlo + a + i])


def test_sweep_variant_restates_parametersweep():
    """The five variables land where raft/parametersweep.py:56-88 puts them; multipliers of 1
    leave the design unchanged."""
    import json
    import os
    from raft.sweep import sweep_baseline, sweep_variant
    with open(os.path.join(os.path.dirname(__file__), "golden", "designs", "VolturnUS-S_example.json")) as fh:
        base = json.load(fh)
    same = sweep_variant(base, [1, 1, 1, 1, 1])
    for a, b in zip(same["platform"]["members"], base["platform"]["members"]):
        assert np.allclose(np.asarray(a["rA"], float), np.asarray(b["rA"], float))
        assert np.allclose(np.asarray(a["rB"], float), np.asarray(b["rB"], float))
        assert np.allclose(np.asarray(a["d"], float), np.asarray(b["d"], float))
    v = sweep_variant(base, [1.1, 0.9, 1.2, 0.8, 1.05])
    b0, b1 = sweep_baseline(base), sweep_baseline(v)
    for k, f in zip(["ccD", "ocD", "T", "ocR", "pH"], [1.1, 0.9, 1.2, 0.8, 1.05]):
        assert np.isclose(b1[k], b0[k] * f), k
    m = v["platform"]["members"]
    assert np.isclose(m[2]["rB"][0], m[1]["rA"][0] - m[1]["d"] / 2)     # pontoon meets the outer column
    assert base["platform"]["members"][0]["d"] == b0["ccD"]            # the base design is not mutated


def _gather_check(rank, world):
    from raft.parallel import case_shard, gather_cases
    n = 11
    rng = np.random.default_rng(5)
    full_x = rng.standard_normal([n, 6, 7]) + 1j * rng.standard_normal([n, 6, 7])
    full_i = np.arange(n, dtype=np.int32) * 3
    lo, hi = case_shard(n, rank, world)
    got = gather_cases({"Xi": torch.tensor(full_x[lo:hi]), "iters": torch.tensor(full_i[lo:hi])}, n)
    np.testing.assert_array_equal(got["Xi"].numpy(), full_x)
    np.testing.assert_array_equal(got["iters"].numpy(), full_i)
    # gather to one rank: the full arrays there, the rank's own block elsewhere
    got = gather_cases({"Xi": torch.tensor(full_x[lo:hi]), "iters": torch.tensor(full_i[lo:hi])}, n, dst=1)
    want_x, want_i = (full_x, full_i) if rank == 1 else (full_x[lo:hi], full_i[lo:hi])
    np.testing.assert_array_equal(got["Xi"].numpy(), want_x)
    np.testing.assert_array_equal(got["iters"].numpy(), want_i)


def test_case_gather_world2():
    _run(_gather_check)


def _qtf_check(rank, world):
    from oracle import qtf_oracle as Q
    from raft.parallel import assemble_qtf, qtf_pair_flat, qtf_tiles
    T = load_golden("c3_qtf")
    ref = Q.qtf_slender(T, T["out_Xi0"], T["w1_2nd"], T["k1_2nd"], 0.0)[:, :, 0, :]
    n2 = len(T["w1_2nd"])
    iu = np.triu(np.ones([n2, n2], dtype=bool))

    def rows(out, r, w):                      # stand-in for rh_qtf_slender_rows: the pairs of rank r's tiles
        flat = qtf_pair_flat(n2, qtf_tiles(n2, r, w))
        out.view(n2 * n2, 6)[torch.tensor(flat)] = torch.tensor(ref.reshape(n2 * n2, 6)[flat])

    def fill(out):                            # same semantics as k_qtf_fill
        x = out.numpy()
        i, j = np.nonzero(~iu)
        x[i, j] = np.conj(x[j, i])

    q = assemble_qtf(rows, fill, n2).numpy()
    np.testing.assert_array_equal(q, ref)


def test_sharded_qtf_exchange_world2():
    _run(_qtf_check)


# ---- bin sharding of one case (raft/parallel.py bin_fixed_point) -------------------------
def _toy(nw, nn):
    """A small fixed point with the structure of the drag loop: per-node sums over ALL bins
    couple the bins; each bin then updates from the global sums; integer-valued data keep
    every sum exact, so sharded and single-process runs must agree bit for bit."""
    rng = np.random.default_rng(4)
    A = torch.tensor(rng.integers(1, 4, size=[nn, nw]).astype(float))
    state = {"x": torch.ones(nw, dtype=torch.float64), "xi": torch.zeros(nw, dtype=torch.float64)}

    def partial(lo, hi, out):
        out.copy_(torch.stack([(A[:, lo:hi] * state["x"][lo:hi]).sum(1)] * 3, 1).reshape(-1))

    def step(sums, lo, hi, flags):
        s = sums.reshape(-1, 3)[:, 0]
        new = torch.floor((A[:, lo:hi] * s[:, None]).sum(0) / (64.0 * nn))
        state["xi"][lo:hi] = new
        if (new != state["x"][lo:hi]).any():
            flags[0] = 1
        state["x"][lo:hi] = torch.floor(0.5 * (state["x"][lo:hi] + new))
    return partial, step, state


def _bins_check(rank, world):
    from raft.parallel import bin_fixed_point, bin_shard
    nw, nn = 37, 5
    solo = [dist.new_group([r]) for r in range(world)][rank]     # single-process reference run
    partial, step, st = _toy(nw, nn)
    it1, s1 = bin_fixed_point(partial, step, nn, 6, nw, group=solo, shards=[(0, nw)])
    ref = st["xi"].clone()
    partial, step, st = _toy(nw, nn)
    it2, s2 = bin_fixed_point(partial, step, nn, 6, nw)           # this rank's block of bins
    lo, hi = bin_shard(nw, rank, world)
    xi = torch.zeros(nw, dtype=torch.float64)
    xi[lo:hi] = st["xi"][lo:hi]
    dist.all_reduce(xi)
    assert (it1, s1) == (it2, s2)
    np.testing.assert_array_equal(xi.numpy(), ref.numpy())


def test_bin_sharded_fixed_point_world2():
    _run(_bins_check)


def test_bin_shards_cover_every_bin_once():
    from raft.parallel import bin_shard
    for nw in (1, 7, 80, 1000):
        for world in (1, 2, 3, 8):
            seen = np.zeros(nw, dtype=int)
            for r in range(world):
                lo, hi = bin_shard(nw, r, world)
                seen[lo:hi] += 1
            assert (seen == 1).all()


def _too_few_cases_check(rank, world):
    """Fewer cases than ranks: every rank raises the same ValueError before any collective
    (no rank is left waiting in the gather)."""
    from raft.parallel import solve_cases_sharded
    from raft.solver import CaseSet
    cs = CaseSet([0], [0.0], ["JONSWAP"], [2.0], [10.0], [0.0])
    with pytest.raises(ValueError, match="every rank needs one"):
        solve_cases_sharded([object()], cs, 4, group=None, gather=True)
    dist.barrier()          # both ranks got here: nobody hangs


def test_too_few_cases_raises_on_every_rank_world2():
    _run(_too_few_cases_check)


def _qtf_local_check(rank, world):
    """QtfDevice.qtf with group=None stays local under an initialised default group (the
    FOWT.calcQTF_slenderBody path): ranks solving different cases never enter a collective.
    Only an explicit group shards."""
    import raft.parallel as P
    from raft.qtf import QtfDevice
    taken = []
    orig = P.assemble_qtf
    P.assemble_qtf = lambda *a, **kw: taken.append("sharded")
    q = QtfDevice.__new__(QtfDevice)         # no device tables: only the dispatch is exercised
    q.torch, q.n2, q.dev = torch, 3, torch.device("cpu")
    try:
        q.qtf(None, None, None, group=dist.group.WORLD)
        assert taken == ["sharded"]
        with pytest.raises(Exception):       # the local path reaches the device call (no GPU here)
            q.qtf(None, None, None)
        assert taken == ["sharded"]
    finally:
        P.assemble_qtf = orig


def test_qtf_default_group_is_local_world2():
    _run(_qtf_local_check)
