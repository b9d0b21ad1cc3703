"""CPU: the native per-design preparation (rh_prep_designs, csrc/rh_prep.h) against the
Python host path it restates (raft/batch.py prepare_design -> raft/member.py,
raft/statics.py, raft/prep.py, itself pinned to the reference's statics goldens and solves).

Sizes, member ranges and the frequency grid are expected bit for bit, every table field
within 1e-14 of its largest entry (single entries may differ by an ulp where NumPy leaves
the summation order of 3x3 products and norms to BLAS).  No GPU: librafthip loads and runs
its host code only."""
import numpy as np
import pytest

from conftest import load_design

C_MOOR = np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])


def _python_tables(d, st, r6=None):
    from raft.batch import prepare_design
    m = prepare_design((d, st, r6, 0, False))
    f = m.fowtList[0]
    return f.host_tables(), f


def _compare(h, n):
    """Same sizes and member ranges, w and k bit for bit; every table field (node-table rows
    one by one) within 1e-14 of its largest entry: rotated members reach their axes through
    3x3 products and norms whose summation order NumPy leaves to BLAS, so single entries may
    differ by an ulp."""
    assert (h["nn"], h["nm"]) == (n["nn"], n["nm"])
    np.testing.assert_array_equal(h["mstart"], n["mstart"])
    for name, (o, shp) in h["layout"].items():
        a = h["packed"][o:o + int(np.prod(shp))].reshape(shp)
        no = n["layout"][name][0]
        b = n["packed"][no:no + a.size].reshape(shp)
        if name in ("w", "k"):
            np.testing.assert_array_equal(a, b)
            continue
        rows = a if a.ndim == 2 and name in ("node", "memb") else a.reshape(1, -1)
        brow = b if a.ndim == 2 and name in ("node", "memb") else b.reshape(1, -1)
        for i, (x, y) in enumerate(zip(rows, brow)):
            tol = 1e-14 * max(np.abs(x).max(), 1.0)   # unit vectors: rounding zeros (1e-48 vs 3e-33)
            assert np.abs(x - y).max() <= tol, (name, i, np.abs(x - y).max(), tol)


def _native(designs, statics, r6=None):
    from raft.hydro_math import wave_numbers
    from raft.model import Model
    from raft.native_prep import PreparedDesigns, design_spec
    w = Model.frequency_grid(designs[0])
    k = wave_numbers(w, float(designs[0]["site"]["water_depth"]))
    return PreparedDesigns([design_spec(d, r6=r6, statics=s) for d, s in zip(designs, statics)], w, k, nthreads=4)


@pytest.mark.parametrize("name", ["VolturnUS-S_example", "VolturnUS-S_test", "OC3spar", "OC3spar_test"])
def test_native_tables_and_statics_match_python(name):
    d = load_design(name)
    st = {"C_moor": C_MOOR}
    h, f = _python_tables(d, st)
    P = _native([d], [st])
    _compare(h, P.host_tables(0))
    for j, key in enumerate(["M_struc", "B_struc", "C_struc", "C_hydro", "A_hydro_morison"]):
        ref = getattr(f, key)
        assert np.abs(P.statics[0, j] - ref).max() <= 1e-14 * max(np.abs(ref).max(), 1e-300), key


def test_native_sweep_variants_match_python():
    """C5 parametersweep variants (raft/sweep.py), every one prepared natively in one call."""
    from raft.sweep import sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    base["settings"]["min_freq"] = 0.0002
    designs = [sweep_variant(base, m) for m in sweep_multipliers(6, seed=5)]
    st = {"C_moor": C_MOOR}
    P = _native(designs, [st] * len(designs))
    for i, d in enumerate(designs):
        _compare(_python_tables(d, st)[0], P.host_tables(i))


def test_sweep_specs_equal_design_spec_of_variants():
    """native_prep.sweep_specs (the base record with the swept fields rewritten, the C5 bench
    path) equals design_spec of each sweep_variant dict, value for value; the base design is
    left untouched."""
    import copy
    from raft.native_prep import design_spec, sweep_specs
    from raft.sweep import sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    base["settings"]["min_freq"] = 0.0002
    keep = copy.deepcopy(base)
    st = {"C_moor": C_MOOR}
    mult = np.vstack([sweep_multipliers(40, seed=11), np.ones(5), np.full(5, 0.75), np.full(5, 1.25)])
    fast = sweep_specs(base, mult, statics=st)
    assert len(fast) == len(mult)
    for m, s in zip(mult, fast):
        np.testing.assert_array_equal(s, design_spec(sweep_variant(base, m), statics=st))
    assert base == keep


def test_native_pose_and_mooring_stiffness():
    """A displaced, rotated pose (members, RNA and hydrostatics move) and the mooring
    stiffness computed from the design's own mooring system (raft/mooring.py)."""
    d = load_design("VolturnUS-S_example")
    r6 = np.array([3.0, -2.0, 0.5, 0.02, -0.03, 0.1])
    h, f = _python_tables(d, None, r6=r6)
    P = _native([d], [None], r6=r6)
    _compare(h, P.host_tables(0))


def test_native_statics_given_override():
    """Given M_struc / C_struc / C_hydro (setStatics) replace the computed ones."""
    d = load_design("OC3spar")
    rng = np.random.default_rng(3)
    st = {k: rng.normal(size=(6, 6)) for k in ("M_struc", "C_struc", "C_hydro", "C_moor")}
    h, f = _python_tables(d, st)
    P = _native([d], [st])
    _compare(h, P.host_tables(0))


def test_native_maccamy_fuchs_matches_python():
    """OC4semi (MacCamy-Fuchs columns, raft/raft_member.py:1053-1088): the node tables as
    above, and the frequency-dependent inertia table rh_prep_imat against raft/member.py's
    Imat_MCF (scipy's hankel1 there, rh_bessel.h's series / recurrences here: 1e-13 of the
    table's largest entry)."""
    d = load_design("OC4semi-RAFT_QTF")
    st = {"C_moor": C_MOOR}
    h, f = _python_tables(d, st)
    P = _native([d], [st])
    n = P.host_tables(0)
    _compare(h, n)
    assert h["imat"] is not None and n["imat"] is not None
    assert n["imat"].shape == h["imat"].shape
    err = np.abs(n["imat"] - h["imat"]).max()
    assert err <= 1e-13 * np.abs(h["imat"]).max(), err


def test_native_bad_specs():
    from raft import _native as N
    from raft.native_prep import PreparedDesigns, design_spec
    w = np.arange(1, 11) * 0.1
    s = design_spec(load_design("OC3spar"), statics={"C_moor": C_MOOR})
    with pytest.raises(ValueError, match="spec record"):
        PreparedDesigns([s[:-1]], w, w)
    bad = s.copy()
    bad[0] = 1.0
    with pytest.raises(ValueError, match="magic"):
        PreparedDesigns([bad], w, w)
    assert N.lib().rh_prep_layout(None, None) == N.RH_EINVAL
    assert N.lib().rh_prep_imat(None, 0, None) == N.RH_EINVAL


def _pool_specs(n):
    from raft.hydro_math import wave_numbers
    from raft.model import Model
    from raft.native_prep import design_spec
    from raft.sweep import sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    designs = [sweep_variant(base, m) for m in sweep_multipliers(n, seed=7)]
    w = Model.frequency_grid(base)
    k = wave_numbers(w, float(base["site"]["water_depth"]))
    return [design_spec(d, statics={"C_moor": C_MOOR}) for d in designs], w, k


def _pool_child(q, specs, w, k):
    from raft.native_prep import PreparedDesigns
    q.put(PreparedDesigns(specs, w, k, nthreads=3).packed.tobytes())


def test_prep_worker_pool_threads_callers_and_fork():
    """rh_prep_designs runs on worker threads kept across calls (csrc/rh_abi.hip PrepPool):
    every thread count gives the single-thread tables bit for bit, calls from several Python
    threads at once (queued on the pool) too, and a forked child, which has none of its
    parent's workers, gets a pool of its own."""
    import multiprocessing as mp
    import threading
    from raft.native_prep import PreparedDesigns
    specs, w, k = _pool_specs(12)
    ref = PreparedDesigns(specs, w, k, nthreads=1).packed.copy()
    for nt in (2, 5, 16, 3, 16):
        np.testing.assert_array_equal(PreparedDesigns(specs, w, k, nthreads=nt).packed, ref)
    out = [None] * 4
    def call(i):
        out[i] = PreparedDesigns(specs, w, k, nthreads=2 + 3 * i).packed.copy()
    th = [threading.Thread(target=call, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(60)
    for o in out:
        np.testing.assert_array_equal(o, ref)
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_pool_child, args=(q, specs, w, k))
    p.start()
    got = q.get(timeout=120)
    p.join(60)
    assert p.exitcode == 0
    assert got == ref.tobytes()
