"""GPU parity of the batched entry points on second-order designs and multi-sea-state farms.

* potSecOrder=1 (OC4semi-RAFT_QTF, tests/golden/c3_qtf.npz): Model.analyzeCasesBatch solves the
  reference's case and seeded sea states in one batch -- first pass, slender-body QTF of each
  converged RAO, second pass from iteration 1 (raft/raft_model.py:966-989) -- against the
  reference run (1e-9, identical iteration pair) and against Model.solveDynamics per case
  (1e-12, identical pairs).  A second sea state raises the reference's IndexError (Q8).
* potSecOrder=2 (.12d file QTF, tests/golden/qtf12d.npz): the reference's three cases, one
  with two sea states, plus seeded ones, through analyzeCasesBatch; the file QTF's force
  enters the fixed point and every further sea state (:903-904, :1059-1061).
* DesignBatch mixing a potSecOrder=1 design with a first-order design in one launch.
* C4 farm (tests/golden/c4_farm.npz) with two sea states per case through analyzeArrayBatch:
  row 0 and the iteration counts against the reference run, every row against
  Model.solveDynamics (1e-12) and the oracle's solve_farm (1e-9).
"""
import json

import numpy as np
import pytest

from conftest import farm_tables, golden_cases, load_design, load_golden, statics_of
from oracle import raft_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-9
SAME = 1e-12


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def _qtf_model(T):
    import raft
    d = load_design("OC4semi-RAFT_QTF")
    d["platform"]["outFolderQTF"] = None
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    return m, f


def _seeded(rng, k, headings=(0.0,)):
    return [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(7, 16)), wave_height=float(rng.uniform(2, 8)),
                 wave_heading=float(rng.choice(headings)), wave_gamma=float(rng.choice([0.0, 2.0])), wind_speed=0)
            for _ in range(k)]


def test_slender_body_qtf_design_through_the_batch():
    T = load_golden("c3_qtf")
    m, f = _qtf_model(T)
    gold = {k: v[0] for k, v in json.loads(str(T["cases_json"]))[0].items()}
    gold["wind_speed"] = 0
    cases = [dict(gold)] + _seeded(np.random.default_rng(61), 5, headings=(0.0, 30.0))
    r = m.analyzeCasesBatch(cases, want=("psd", "std", "zeta", "B_drag", "Fhydro_2nd"))
    assert list(r["iters_pair"][0]) == list(T["out_iters_pair"]), (r["iters_pair"][0], T["out_iters_pair"])
    assert rel(r["Xi"][0], T["out_Xi"][0]) < RTOL, rel(r["Xi"][0], T["out_Xi"][0])
    assert rel(r["B_drag"][0], T["out_B_drag"]) < RTOL
    assert rel(r["Fhydro_2nd"][0], T["out_Fhydro_2nd"][0]) < RTOL
    np.testing.assert_allclose(r["f2nd_mean"][0], T["out_Fhydro_2nd_mean"][0], rtol=RTOL,
                               atol=RTOL * np.abs(T["out_Fhydro_2nd_mean"]).max())
    for j, c in enumerate(cases):
        Xi = m.solveDynamics(dict(c))
        pair = f.iterations_pair + [0] * (2 - len(f.iterations_pair))
        assert list(r["iters_pair"][j]) == pair, (j, r["iters_pair"][j], f.iterations_pair)
        assert r["iters"][j] == f.iterations
        assert rel(r["Xi"][j], Xi[0]) < SAME, (j, rel(r["Xi"][j], Xi[0]))
        np.testing.assert_allclose(r["f2nd_mean"][j], f.Fhydro_2nd_mean[0], rtol=SAME,
                                   atol=SAME * np.abs(f.Fhydro_2nd_mean[0]).max())
        np.testing.assert_allclose(r["std"][j], f._stats["std"], rtol=SAME)
    with pytest.raises(IndexError, match="out of bounds for axis 2 with size 1"):
        m.analyzeCasesBatch([dict(gold, wave_heading=[0.0, 30.0], wave_period=[12.0, 8.0], wave_height=[6.0, 2.0],
                                  wave_spectrum=["JONSWAP", "JONSWAP"], wave_gamma=[0.0, 0.0])])
    with pytest.raises(IndexError, match="out of bounds for axis 2 with size 1"):
        m.solveDynamics(dict(gold, wave_heading=[0.0, 30.0], wave_period=[12.0, 8.0], wave_height=[6.0, 2.0],
                             wave_spectrum=["JONSWAP", "JONSWAP"], wave_gamma=[0.0, 0.0]))


def test_slender_body_batch_off_axis_headings_match_oracle():
    """potSecOrder=1 at 30 and 60 degrees, where the first-pass RAO has sway, roll and yaw (the
    reference run is at 0 degrees, and solveDynamics shares the batch's QTF kernels): the batch
    against the oracle's whole potSecOrder=1 solve (oracle/raft_oracle.py solve_dynamics with
    its qtf_slender), 1e-9 and the same iteration pair."""
    T = load_golden("c3_qtf")
    m, f = _qtf_model(T)
    cases = _seeded(np.random.default_rng(67), 4, headings=(30.0, 60.0))
    r = m.analyzeCasesBatch(cases)
    for j, c in enumerate(cases):
        o = O.solve_dynamics(T, dict(c), int(T["nIter"]), float(T["XiStart"]),
                             second_order=dict(w1_2nd=T["w1_2nd"], k1_2nd=T["k1_2nd"]))
        assert list(r["iters_pair"][j]) == list(o["iters_pair"]), (j, r["iters_pair"][j], o["iters_pair"])
        assert np.abs(o["Xi"][0, 5]).max() > 1e-3 * np.abs(o["Xi"][0]).max()      # the RAO yaws
        assert rel(r["Xi"][j], o["Xi"][0]) < RTOL, (j, rel(r["Xi"][j], o["Xi"][0]))


def test_slender_body_unconverged_first_pass_keeps_first_order():
    """tol = 1e-13: no case converges in the first pass, so no QTF is formed (the reference
    reaches :966 only on convergence) and the batch equals solveDynamics with first order only."""
    T = load_golden("c3_qtf")
    m, f = _qtf_model(T)
    cases = _seeded(np.random.default_rng(62), 3)
    r = m.analyzeCasesBatch(cases, tol=1e-13)
    assert not np.any(r["status"] == 1)
    for j, c in enumerate(cases):
        Xi = m.solveDynamics(dict(c), tol=1e-13)
        assert len(f.iterations_pair) == 1 and r["iters_pair"][j][1] == 0
        assert r["iters"][j] == f.iterations
        assert not np.any(r["f2nd_mean"][j])
        assert rel(r["Xi"][j], Xi[0]) < SAME


def test_file_qtf_design_through_the_batch(tmp_path):
    import raft
    T = load_golden("qtf12d")
    stem = str(tmp_path / "q")
    np.savetxt(stem + ".12d", T["table12d"], fmt="%.17g")
    d = load_design("OC4semi-RAFT_QTF")
    d["settings"]["min_freq"] = 0.0025
    for k in ("outFolderQTF", "min_freq2nd", "max_freq2nd", "df_freq2nd"):
        d["platform"].pop(k, None)
    d["platform"]["potSecOrder"] = 2
    d["platform"]["hydroPath"] = stem
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    gold = json.loads(str(T["cases_json"]))
    rng = np.random.default_rng(63)
    seeded = _seeded(rng, 4, headings=(0.0, 30.0))
    two = dict(gold[2], wave_period=[10.0, 6.5], wave_height=[4.0, 1.5], wave_heading=[30.0, 0.0])
    cases = gold + seeded + [two]
    r = m.analyzeCasesBatch(cases)
    Xw = r["Xi_waves"]
    for ic in range(len(gold)):
        nW = len(np.atleast_1d(gold[ic]["wave_heading"]))
        assert r["iters"][ic] == int(T["out_iters"][ic])
        assert rel(Xw[ic, :nW + 1], T["out_Xi"][ic][:nW + 1]) < RTOL, (ic, rel(Xw[ic, :nW + 1], T["out_Xi"][ic][:nW + 1]))
        assert rel(r["B_drag"][ic], T["out_B_drag"][ic]) < RTOL
        ref = T["out_Fhydro_2nd_mean"][ic][:nW]
        np.testing.assert_allclose(r["f2nd_mean_waves"][ic, :nW], ref, rtol=RTOL, atol=RTOL * np.abs(ref).max())
    for j, c in enumerate(cases):
        Xi = m.solveDynamics(dict(c))
        nW = f.nWaves
        assert r["iters"][j] == f.iterations and r["nWaves"][j] == nW
        assert rel(Xw[j, :nW + 1], Xi) < SAME, (j, rel(Xw[j, :nW + 1], Xi))
        assert not np.any(Xw[j, nW + 1:])
        np.testing.assert_allclose(r["f2nd_mean_waves"][j, :nW], f.Fhydro_2nd_mean, rtol=SAME,
                                   atol=SAME * np.abs(f.Fhydro_2nd_mean).max())
        np.testing.assert_allclose(r["std"][j], f._stats["std"], rtol=SAME)
        np.testing.assert_allclose(r["psd"][j], f._stats["psd"], rtol=SAME, atol=SAME * np.abs(f._stats["psd"]).max())


def test_design_batch_mixes_second_and_first_order_designs():
    """DesignBatch (full models) with the QTF design and the same platform at potSecOrder=0 in
    one launch: each case equals its own model's analyzeCasesBatch; light / native designs with
    potSecOrder > 0 are refused."""
    from raft.batch import DesignBatch
    T = load_golden("c3_qtf")
    d1 = load_design("OC4semi-RAFT_QTF")
    d1["platform"]["outFolderQTF"] = None
    d0 = json.loads(json.dumps(d1))
    d0["platform"]["potSecOrder"] = 0
    st = statics_of(T)
    B = DesignBatch([d1, d0], statics=[st, st], r6=T["r6"])
    cases = _seeded(np.random.default_rng(64), 4)
    idx = np.array([0, 1, 0, 1, 1, 0, 0, 1], dtype=np.int32)
    allc = [cases[i % 4] for i in range(8)]
    r = B.solve(idx, allc, want=("psd", "std", "zeta", "B_drag")).host()
    for j in range(8):
        ref = B.models[idx[j]].analyzeCasesBatch([allc[j]])
        assert list(r["iters_pair"][j]) == list(ref.get("iters_pair", np.array([[ref["iters"][0], 0]]))[0])
        assert rel(r["Xi"][j], ref["Xi"][0]) < SAME
        assert (r["iters_pair"][j][1] > 0) == (idx[j] == 0 and r["status"][j] == 1)
    with pytest.raises(NotImplementedError, match="potSecOrder"):
        DesignBatch([d1], statics=st, native=True)


def _farm(T):
    import raft
    Ts = farm_tables(T)
    m = raft.Model(load_design("VolturnUS-S_farm"), statics=[statics_of(t) for t in Ts])
    m.K_array = T["K_array"]
    for f, t in zip(m.fowtList, Ts):
        f.setPosition(t["r6"])
        f.calcStatics()
        f.calcHydroConstants()
    return m, Ts


def test_farm_batch_with_several_sea_states():
    T = load_golden("c4_farm")
    m, Ts = _farm(T)
    gold = golden_cases(T)
    rng = np.random.default_rng(65)
    cases = []
    for ic, g in enumerate(gold):         # the reference's sea state first, a seeded one after it
        extra = dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 14)),
                     wave_height=float(rng.uniform(1, 5)), wave_heading=float(rng.choice([0, 45, 135])),
                     wave_gamma=0.0)
        cases.append({k: [g[k], extra[k]] for k in extra} | {"wind_speed": 0})
    cases.append(dict(gold[0]))                                   # one sea state, mixed in
    cases.append(dict(wave_spectrum=["JONSWAP"] * 3, wave_heading=[90.0, 0.0, 270.0], wave_height=[1.68, 3.0, 2.0],
                      wave_period=[8.15, 11.0, 6.0], wave_gamma=[0.0, 2.0, 0.0], wind_speed=0))
    r = m.analyzeCasesBatch(cases)
    Xw = r["Xi_waves"]
    assert Xw.shape == (len(cases), 4, 12, m.nw)
    for ic in range(len(gold)):
        assert list(r["iters"][ic]) == list(T["out_iters"][ic])
        assert rel(Xw[ic, 0], T["out_Xi"][ic][0]) < RTOL
        assert rel(r["Xi"][ic], T["out_Xi"][ic][0]) < RTOL
    for j, c in enumerate(cases):
        Xi = m.solveDynamics(dict(c))
        nW = m.fowtList[-1].nWaves
        assert list(r["iters"][j]) == [f.iterations for f in m.fowtList]
        assert rel(Xw[j, :nW + 1], Xi) < SAME, (j, rel(Xw[j, :nW + 1], Xi))
        for i, f in enumerate(m.fowtList):
            np.testing.assert_allclose(r["std"][j, i], f._stats["std"], rtol=SAME)
            np.testing.assert_allclose(r["psd"][j, i], f._stats["psd"], rtol=SAME,
                                       atol=SAME * np.abs(f._stats["psd"]).max())
    for j in (0, 3):
        o = O.solve_farm(Ts, dict(cases[j]), int(T["nIter"]), T["K_array"], float(T["XiStart"]))
        assert list(r["iters"][j]) == o["iters"]
        nW = len(np.atleast_1d(cases[j]["wave_heading"]))
        assert rel(Xw[j, :nW + 1], o["Xi"]) < RTOL, rel(Xw[j, :nW + 1], o["Xi"])


def test_heading_response_explicit_bmat_stride_and_bad_index():
    """rh_heading_response_ext on a strict subset of the designs of the solve that wrote Bmat
    (designs with different node counts): with the solve's row stride passed explicitly the
    subset call gives the bits of the full call; a stride below the designs' node count is
    refused; a design or heading index out of range leaves NaN rows (no table is read)."""
    import torch
    from raft import _native as N
    from raft.batch import DesignBatch
    from raft.solver import CaseSet, solve_batch
    from raft.sweep import sweep_variant
    base = load_design("VolturnUS-S_example")
    designs = [base, sweep_variant(base, (1.0, 1.0, 1.5, 1.0, 1.0))]
    B = DesignBatch(designs, statics={"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}, native=True)
    dds = B.dds
    nns = [d.nn for d in dds]
    assert nns[0] != nns[1], nns
    small = int(np.argmin(nns))
    for d in dds:
        d.ensure_headings(np.deg2rad([0.0, 30.0]))
    idx = np.array([0, 1, 0, 1], dtype=np.int32)
    cs = CaseSet(idx, [0.0] * 4, ["JONSWAP"] * 4, [2.0, 4.0, 6.0, 3.0], [8.0, 10.0, 12.0, 9.0], [0.0] * 4)
    res = solve_batch(dds, cs, B.nIter, B.XiStart, 0.01, want=("zeta", "B_drag", "Bmat"))
    stride = int(res["Bmat"].shape[1])
    assert stride == max(nns)
    sel = np.nonzero(idx == small)[0]
    st = torch.tensor(sel, dtype=torch.long, device=dds[0].device)
    zeta, bdrag = res["zeta"].index_select(0, st).contiguous(), res["B_drag"].index_select(0, st).contiguous()
    bmat = res["Bmat"].index_select(0, st).contiguous()
    i32 = dict(dtype=torch.int32, device=dds[0].device)
    hidx = torch.tensor([dds[small].ensure_headings([np.deg2rad(30.0)])[0]] * len(sel), **i32)
    ctx, s = N.context(0), N.stream_handle(torch, dds[0].device)

    def call(views, didx, nn):
        arr = (N.RhDesign * len(views))(*[v.struct() for v in views])
        out = torch.zeros([len(sel), 6, dds[0].nw], dtype=torch.complex128, device=dds[0].device)
        di = torch.tensor(didx, **i32)
        rc = N.lib().rh_heading_response_ext(ctx, arr, len(views), len(sel), N.ptr(di), N.ptr(hidx), N.ptr(zeta),
                                             N.ptr(bdrag), N.ptr(bmat), nn, None, N.ptr(out), s)
        torch.cuda.synchronize()
        return rc, out.cpu().numpy()

    rc, full = call(dds, [small] * len(sel), stride)
    assert rc == N.RH_OK
    rc, sub = call([dds[small]], [0] * len(sel), stride)
    assert rc == N.RH_OK
    np.testing.assert_array_equal(sub, full)
    assert np.all(np.isfinite(full))
    rc, _ = call(dds, [small] * len(sel), min(nns))
    assert rc == N.RH_EINVAL
    rc, bad = call(dds, [7] + [small] * (len(sel) - 1), stride)
    assert rc == N.RH_OK and np.all(np.isnan(bad[0])) and np.all(np.isfinite(bad[1:]))
    np.testing.assert_array_equal(bad[1:], full[1:])
