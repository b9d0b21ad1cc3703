"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors and
the CPU oracle on the same seeded inputs.

Tolerance (north_star): FP64, 1e-9 relative (normwise per case) and IDENTICAL drag
iteration counts.  Full-size batches (C2: nw=1000, 512 cases) are checked on a seeded
sample against the oracle plus size-independent properties (determinism, permutation
invariance, status/iteration consistency).
"""
import numpy as np
import pytest

from conftest import golden_cases, load_design, load_golden, statics_of
from oracle import raft_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def make_model(design_name, T, settings=None):
    import raft
    d = load_design(design_name)
    if settings:
        d["settings"].update(settings)
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    return m, f


SOLVES = [("c1_OC3spar", "OC3spar", None), ("c2_nw200", "VolturnUS-S_example", None),
          ("multi_heading", "VolturnUS-S_test", None), ("c2_nw1000", "VolturnUS-S_example", {"min_freq": 0.0002})]


@pytest.mark.parametrize("tag,design,settings", SOLVES)
def test_solve_dynamics_matches_reference(tag, design, settings):
    T = load_golden(tag)
    m, f = make_model(design, T, settings)
    for ic, case in enumerate(golden_cases(T)):
        Xi = m.solveDynamics(dict(case))
        assert f.iterations == T["out_iters"][ic], (ic, f.iterations, T["out_iters"][ic])
        assert int(f.converged) == T["out_conv"][ic]
        assert rel(Xi, T["out_Xi"][ic]) < RTOL, rel(Xi, T["out_Xi"][ic])
        assert rel(f.B_hydro_drag, T["out_B_drag"][ic]) < RTOL
        assert rel(f.F_hydro_iner, T["out_F_iner"][ic]) < RTOL
        res = {}
        f.saveTurbineOutputs(res, case)
        dofs = ["surge", "sway", "heave", "roll", "pitch", "yaw"]
        smax = max(T[f"out_{d}_std"][ic] for d in dofs)
        pmax = max(T[f"out_{d}_PSD"][ic].max() for d in dofs)
        for dof in dofs:
            np.testing.assert_allclose(res[dof + "_std"], T[f"out_{dof}_std"][ic], rtol=RTOL, atol=RTOL * smax)
            np.testing.assert_allclose(res[dof + "_PSD"], T[f"out_{dof}_PSD"][ic], rtol=RTOL, atol=RTOL * pmax)
        if "out_Z" in T:
            assert rel(f.Z, T["out_Z"][ic]) < 1e-12
        check_rotor_channels(res, T, ic)


def check_rotor_channels(res, T, ic):
    """AxRNA_* / Mbase_* (raft/raft_fowt.py:1900-1970, rh_channel_stats) against the
    reference's own saveTurbineOutputs values."""
    if "out_AxRNA_std" not in T:
        return
    for ch in ["AxRNA", "Mbase"]:
        scale = np.abs(T[f"out_{ch}_std"][ic]).max()
        pscale = np.abs(T[f"out_{ch}_PSD"][ic]).max()
        for st in ["avg", "std", "max", "min"]:
            np.testing.assert_allclose(res[f"{ch}_{st}"], T[f"out_{ch}_{st}"][ic], rtol=RTOL, atol=RTOL * scale,
                                       err_msg=f"{ch}_{st}")
        assert res[f"{ch}_PSD"].shape == T[f"out_{ch}_PSD"][ic].shape
        np.testing.assert_allclose(res[f"{ch}_PSD"], T[f"out_{ch}_PSD"][ic], rtol=RTOL, atol=RTOL * pscale)


@pytest.mark.parametrize("tag,design", [("fowt_VolturnUS-S", "VolturnUS-S_test"), ("fowt_OC3spar", "OC3spar_test")])
def test_hydro_excitation_matches_reference(tag, design):
    """72 heading/period/height cases of the reference tests/test_fowt.py:214-250."""
    T = load_golden(tag)
    import raft
    m = raft.Model(load_design(design))
    f = m.fowtList[0]
    f.setPosition(np.zeros(6))
    f.calcHydroConstants()
    for (hd, tp, hs), Fref in zip(T["exc_cases"], T["exc_F_iner"]):
        f.calcHydroExcitation({"wave_heading": hd, "wave_period": tp, "wave_height": hs}, memberList=f.memberList)
        assert rel(f.F_hydro_iner, Fref) < RTOL


@pytest.mark.parametrize("tag,design", [("fowt_VolturnUS-S", "VolturnUS-S_test"), ("fowt_OC3spar", "OC3spar_test")])
def test_hydro_linearization_matches_reference(tag, design):
    """B_hydro_drag and F_hydro_drag of tests/test_fowt.py:252-277."""
    T = load_golden(tag)
    import raft
    m = raft.Model(load_design(design))
    f = m.fowtList[0]
    f.setPosition(np.zeros(6))
    f.calcHydroConstants()
    f.calcHydroExcitation({"wave_spectrum": "unit", "wave_heading": 0, "wave_period": 10, "wave_height": 2},
                          memberList=f.memberList)
    B = f.calcHydroLinearization(T["lin_Xi"])
    F = f.calcDragExcitation(0)
    assert rel(B, T["lin_B_drag"]) < RTOL
    assert rel(F, T["lin_F_drag"]) < RTOL
    assert rel(f.F_hydro_drag, T["lin_F_drag"]) < RTOL


def random_cases(n, seed, headings=(0, 30, 60, 90)):
    rng = np.random.default_rng(seed)
    return [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                 wave_heading=float(rng.choice(headings)), wave_gamma=float(rng.choice([0.0, 0.0, 1.0, 3.3])))
            for _ in range(n)]


def test_batch_matches_oracle_nw200():
    """64 seeded cases in one device call vs the oracle case by case."""
    T = load_golden("c2_nw200")
    m, f = make_model("VolturnUS-S_example", T)
    cases = random_cases(64, 7)
    res = m.analyzeCasesBatch(cases, want=("psd", "std", "zeta", "B_drag", "rao"))
    for ic, case in enumerate(cases):
        r = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
        assert res["iters"][ic] == r["iters"], (ic, res["iters"][ic], r["iters"])
        assert (res["status"][ic] == 1) == r["converged"]
        assert rel(res["Xi"][ic], r["Xi"][0]) < RTOL
        assert rel(res["zeta"][ic], r["zeta"][0].real) < 1e-13
        assert rel(res["B_drag"][ic], r["B_drag"]) < RTOL
        mo = O.motion_outputs(r["Xi"], float(T["dw"]))
        dofs = ["surge", "sway", "heave", "roll", "pitch", "yaw"]
        smax = max(mo[d + "_std"] for d in dofs)
        pmax = max(mo[d + "_PSD"].max() for d in dofs)
        for i, dof in enumerate(dofs):
            np.testing.assert_allclose(res["psd"][ic, i], mo[dof + "_PSD"], rtol=RTOL, atol=RTOL * pmax)
            np.testing.assert_allclose(res["std"][ic, i], mo[dof + "_std"], rtol=RTOL, atol=RTOL * smax)
        np.testing.assert_allclose(res["rao"][ic], O.get_rao(r["Xi"][0], r["zeta"][0]), rtol=1e-8, atol=1e-12)


def test_batch_edge_spectra_and_grids():
    """'unit', 'constant' and 'none' spectra, nw not a multiple of 64 (OC3spar nw=80)."""
    T = load_golden("c1_OC3spar")
    m, f = make_model("OC3spar", T)
    cases = [dict(wave_spectrum="unit", wave_period=9, wave_height=4, wave_heading=0),
             dict(wave_spectrum="constant", wave_period=9, wave_height=0.5, wave_heading=45),
             dict(wave_spectrum="none", wave_period=9, wave_height=4, wave_heading=0),
             dict(wave_spectrum="JONSWAP", wave_period=3.0, wave_height=12.0, wave_heading=180)]
    res = m.analyzeCasesBatch(cases)
    for ic, case in enumerate(cases):
        r = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
        assert res["iters"][ic] == r["iters"]
        assert rel(res["Xi"][ic], r["Xi"][0]) < RTOL
    assert np.all(res["Xi"][2] == 0)           # still water: no response


def test_non_convergence_and_xistart():
    """nIter=0 (a single solve, not converged) and XiStart != 0 follow the reference loop."""
    T = load_golden("c2_nw200")
    for nIter, xs in [(0, 0.0), (1, 0.1), (6, 0.5)]:
        m, f = make_model("VolturnUS-S_example", T, {"nIter": nIter, "XiStart": xs})
        cases = random_cases(8, 11 + nIter)
        res = m.analyzeCasesBatch(cases)
        for ic, case in enumerate(cases):
            r = O.solve_dynamics(T, dict(case), nIter, xs)
            assert res["iters"][ic] == r["iters"]
            assert (res["status"][ic] == 1) == r["converged"]
            assert rel(res["Xi"][ic], r["Xi"][0]) < RTOL


def test_multi_sea_state_cases_through_the_batch():
    """analyzeCasesBatch on cases with several sea states (raft/raft_model.py:918-1065: the drag
    linearisation from the first, the response to each with it frozen): the reference's
    multi-heading golden run (2 sea states) reproduced inside a batch that mixes it with
    single-sea-state cases and a 3-sea-state case -- Xi_waves in the reference's [nW+1, 6, nw]
    layout, iteration counts, and the motion PSD / std summed over the sea states, at 1e-9;
    every case of the batch also equals its own Model.solveDynamics."""
    T = load_golden("multi_heading")
    m, f = make_model("VolturnUS-S_test", T)
    gc = golden_cases(T)[0]
    three = dict(wave_spectrum=["JONSWAP"] * 3, wave_period=[10.0, 7.0, 14.0], wave_height=[4.0, 1.5, 3.0],
                 wave_heading=[30.0, 90.0, 0.0], wave_gamma=[0.0, 3.3, 1.0])
    single = dict(wave_spectrum="JONSWAP", wave_period=9.0, wave_height=3.0, wave_heading=60.0, wave_gamma=0.0)
    cases = [single, dict(gc), three, dict(gc)]
    res = m.analyzeCasesBatch(cases)
    assert res["Xi_waves"].shape == (4, 4, 6, m.nw)
    np.testing.assert_array_equal(res["nWaves"], [1, 2, 3, 2])
    dofs = ["surge", "sway", "heave", "roll", "pitch", "yaw"]
    for ic in (1, 3):
        assert res["iters"][ic] == T["out_iters"][0]
        assert rel(res["Xi_waves"][ic, :3], T["out_Xi"][0]) < RTOL, rel(res["Xi_waves"][ic, :3], T["out_Xi"][0])
        assert np.all(res["Xi_waves"][ic, 3] == 0)
        smax = max(T[f"out_{d}_std"][0] for d in dofs)
        pmax = max(T[f"out_{d}_PSD"][0].max() for d in dofs)
        for k, d in enumerate(dofs):
            np.testing.assert_allclose(res["std"][ic, k], T[f"out_{d}_std"][0], rtol=RTOL, atol=RTOL * smax)
            np.testing.assert_allclose(res["psd"][ic, k], T[f"out_{d}_PSD"][0], rtol=RTOL, atol=RTOL * pmax)
    for ic, case in enumerate(cases):
        Xi = m.solveDynamics(dict(case))
        nW = Xi.shape[0] - 1
        assert res["iters"][ic] == f.iterations
        assert rel(res["Xi_waves"][ic, :nW + 1], Xi) < 1e-12, ic
        assert rel(res["Xi"][ic], Xi[0]) < 1e-12, ic
        np.testing.assert_allclose(res["std"][ic], f._stats["std"], rtol=1e-12, atol=1e-15)


def test_nan_raises_reference_message():
    T = load_golden("c1_OC3spar")
    m, f = make_model("OC3spar", T)
    with pytest.raises(Exception, match="Nan detected in response vector Xi."):
        m.solveDynamics(dict(wave_spectrum="JONSWAP", wave_period=10, wave_height=float("nan"), wave_heading=0))


def test_full_size_c2_batch_properties():
    """C2 at full size: nw=1000, 512 seeded cases in one call.  Sampled cases vs the oracle,
    bitwise determinism across calls, invariance to case order."""
    T = load_golden("c2_nw1000")
    m, f = make_model("VolturnUS-S_example", T, {"min_freq": 0.0002})
    cases = random_cases(512, 20241016)
    a = m.analyzeCasesBatch(cases, want=("psd", "std", "zeta", "B_drag", "margin"))
    b = m.analyzeCasesBatch(cases)
    np.testing.assert_array_equal(a["Xi"], b["Xi"])
    np.testing.assert_array_equal(a["iters"], b["iters"])
    perm = np.random.default_rng(3).permutation(len(cases))
    c = m.analyzeCasesBatch([cases[i] for i in perm])
    np.testing.assert_array_equal(c["Xi"], a["Xi"][perm])
    assert set(np.unique(a["status"])) <= {0, 1}
    assert np.all(a["iters"][a["status"] == 0] == int(T["nIter"]) + 1)
    # a random sample plus the 16 closest calls of the convergence test (the cases whose
    # iteration count is most at risk of flipping, rh_solve_out.margin)
    close = np.argsort(np.abs(a["margin"]))[:16]
    pick = np.unique(np.concatenate([np.random.default_rng(5).choice(len(cases), 6, replace=False), close]))
    print(f"closest calls |margin|/tol: {np.sort(np.abs(a['margin']))[:4] / 0.01}")
    for ic in pick:
        r = O.solve_dynamics(T, dict(cases[ic]), int(T["nIter"]), float(T["XiStart"]))
        assert a["iters"][ic] == r["iters"], (ic, a["margin"][ic])
        assert rel(a["Xi"][ic], r["Xi"][0]) < RTOL


def _oracle_c2_case(args):
    """Worker of test_full_size_c2_every_case_vs_oracle (spawned process: NumPy only)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conftest import load_golden as lg
    from oracle import raft_oracle as Ow
    case, = args
    T = lg("c2_nw1000")
    r = Ow.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
    return int(r["iters"]), np.asarray(r["Xi"][0])


def test_full_size_c2_every_case_vs_oracle():
    """Every one of the 512 full-size C2 cases (nw=1000) against the oracle:
    identical iteration counts and Xi within RTOL (the oracle in a pool of spawned CPU
    processes, about 0.1 s per case)."""
    import multiprocessing as mp
    import os
    from concurrent.futures import ProcessPoolExecutor
    T = load_golden("c2_nw1000")
    m, f = make_model("VolturnUS-S_example", T, {"min_freq": 0.0002})
    cases = random_cases(512, 20241016)
    a = m.analyzeCasesBatch(cases)
    nproc = max(1, min(16, len(os.sched_getaffinity(0)), os.cpu_count() or 1))
    # spawned workers (never forked from this GPU process); a worker that cannot start breaks
    # the executor with an error instead of being respawned
    with ProcessPoolExecutor(nproc, mp_context=mp.get_context("spawn")) as ex:
        refs = list(ex.map(_oracle_c2_case, [(c,) for c in cases], chunksize=8))
    bad = [ic for ic, (it, _) in enumerate(refs) if it != a["iters"][ic]]
    assert not bad, f"iteration counts differ for cases {bad[:10]}"
    worst = max(rel(a["Xi"][ic], X) for ic, (_, X) in enumerate(refs))
    print(f"512 cases: worst rel Xi error vs oracle {worst:.2e}")
    assert worst < RTOL


def test_system_solve_12dof_matches_numpy():
    """rh_system_solve on random well-conditioned 2-FOWT systems (farm path)."""
    import torch
    import raft  # noqa: F401
    from raft import _native as N
    rng = np.random.default_rng(1)
    nw = 100
    Z = (rng.standard_normal([2, nw, 6, 6]) + 1j * rng.standard_normal([2, nw, 6, 6])) + 8 * np.eye(6)
    K = rng.standard_normal([12, 12])
    F = rng.standard_normal([12, nw]) + 1j * rng.standard_normal([12, nw])
    dev = torch.device("cuda", 0)
    Zt = torch.tensor(Z, device=dev)
    Kt = torch.tensor(K, device=dev)
    Ft = torch.tensor(F, device=dev)
    X = torch.empty([12, nw], dtype=torch.complex128, device=dev)
    N.check(N.lib().rh_system_solve(N.context(0), 2, nw, N.ptr(Zt), N.ptr(Kt), N.ptr(Ft), N.ptr(X),
                                    N.stream_handle(torch, dev)))
    X = X.cpu().numpy()
    for b in range(nw):
        Zs = np.zeros([12, 12], dtype=complex)
        Zs[:6, :6] = Z[0, b]
        Zs[6:, 6:] = Z[1, b]
        Zs += K
        np.testing.assert_allclose(X[:, b], np.linalg.solve(Zs, F[:, b]), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("tag,design,settings,ncase", [("c2_nw1000", "VolturnUS-S_example", {"min_freq": 0.0002}, 128),
                                                       ("c2_nw200", "VolturnUS-S_example", None, 64),
                                                       ("c1_OC3spar", "OC3spar", None, 17)])
def test_fast_and_general_kernels_agree(tag, design, settings, ncase):
    """The default path (k_solve_lds: one case per workgroup, XiLast in LDS) against the
    general kernel (k_solve_cases, rh_set_solver(ctx, 1)) on the same batch: identical
    iteration counts and statuses, outputs within 1e-12 (they differ only in the summation
    order of the per-node bin reductions)."""
    from raft import _native as N
    T = load_golden(tag)
    m, f = make_model(design, T, settings)
    cases = random_cases(ncase, 99)
    want = ("psd", "std", "zeta", "B_drag", "rao")
    a = m.analyzeCasesBatch(cases, want=want)
    N.check(N.lib().rh_set_solver(N.context(0), 1), "rh_set_solver")
    try:
        b = m.analyzeCasesBatch(cases, want=want)
    finally:
        N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")
    np.testing.assert_array_equal(a["iters"], b["iters"])
    np.testing.assert_array_equal(a["status"], b["status"])
    for ic in range(ncase):
        assert rel(a["Xi"][ic], b["Xi"][ic]) < 1e-12, ic
        assert rel(a["B_drag"][ic], b["B_drag"][ic]) < 1e-12, ic
    np.testing.assert_array_equal(a["zeta"], b["zeta"])


def _singular_copy(dd):
    """A copy of a DeviceDesign whose M, B, C and node table are zero: no stiffness, no
    inertia, no drag, so Z(w) = 0 in every bin and the LU meets an exactly zero pivot."""
    import copy
    z = copy.copy(dd)
    z.__dict__ = {k: v for k, v in dd.__dict__.items() if k not in dd._layout and k != "_struct"}
    z._packed = dd._packed.clone()
    for name in ("M", "B", "C", "node"):
        getattr(z, name).zero_()
    return z


@pytest.mark.parametrize("tag,design,settings,ncase", [("c2_nw1000", "VolturnUS-S_example", {"min_freq": 0.0002}, 12),
                                                       ("c2_nw200", "VolturnUS-S_example", None, 9)])
def test_failed_cases_fast_and_general_agree(tag, design, settings, ncase):
    """A batch with a NaN sea state and a case on a singular design: both solve kernels stop
    those cases with RH_CASE_NAN / RH_CASE_SINGULAR after the same iteration and report no
    response for them (Xi, F_wave, PSD, RAO and std all NaN -- an array solve of them then gives
    NaN too; the reference raises there, raft/raft_model.py:957), while the other cases of the
    batch are unaffected and agree."""
    import torch
    from raft import _native as N
    from raft.solver import CaseSet, solve_batch
    T = load_golden(tag)
    m, f = make_model(design, T, settings)
    cases = random_cases(ncase, 21)
    cases[2]["wave_height"] = float("nan")
    dd = f.device_design()
    idx = np.zeros(ncase, dtype=np.int32)
    idx[5] = 1
    cs = CaseSet(idx, [c["wave_heading"] for c in cases], [c["wave_spectrum"] for c in cases],
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * ncase)
    want = ("psd", "std", "zeta", "rao")
    out = []
    for solver in (0, 1):
        N.check(N.lib().rh_set_solver(N.context(0), solver), "rh_set_solver")
        try:
            # F_wave starts as stale finite memory: a failed case must overwrite it with NaN
            Fw = torch.ones([ncase, 6, m.nw], dtype=torch.complex128, device=dd.device)
            r = solve_batch([dd, _singular_copy(dd)], cs, m.nIter, m.XiStart, 0.01, want=want, F_wave=Fw).host()
            r["F_wave"] = Fw.cpu().numpy()
            out.append(r)
        finally:
            N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")
        torch.cuda.synchronize()
    a, b = out
    assert a["status"][2] == N.RH_CASE_NAN and a["status"][5] == N.RH_CASE_SINGULAR, a["status"]
    np.testing.assert_array_equal(a["status"], b["status"])
    np.testing.assert_array_equal(a["iters"], b["iters"])
    for r in (a, b):
        for k in ("Xi", "psd", "std", "rao", "F_wave"):
            assert np.all(np.isnan(r[k][[2, 5]])), k
            ok = np.delete(r[k], [2, 5], axis=0)
            assert np.all(np.isfinite(ok)), k
    for ic in set(range(ncase)) - {2, 5}:
        assert rel(a["Xi"][ic], b["Xi"][ic]) < 1e-12, ic


@pytest.mark.parametrize("tag,design,settings,ncase", [("c2_nw1000", "VolturnUS-S_example", {"min_freq": 0.0002}, 160),
                                                       ("c2_nw200", "VolturnUS-S_example", None, 53),
                                                       ("c1_OC3spar", "OC3spar", None, 17)])
def test_a0_gemm_agrees_with_per_case_phase_a(tag, design, settings, ncase):
    """Iteration 0's phase-A sums as one batch GEMM (k_a0_sums, opt-in rh_set_a0(ctx, 1))
    against every workgroup forming them itself (the default, rh_set_a0(ctx, 0)): identical
    iteration counts and statuses, outputs within 1e-12 (only the grouping of the bin sums
    differs).  Random headings, so the 16-case tiles hold several (design, heading) keys; ncase
    not a multiple of 16."""
    from raft import _native as N
    if N.lib().rh_set_a0(N.context(0), 1) != N.RH_OK:
        pytest.skip("k_a0_sums is a variant kernel: run with RAFTHIP_LIB set to a tools/build_variants.sh library")
    N.check(N.lib().rh_set_a0(N.context(0), 0), "rh_set_a0")
    T = load_golden(tag)
    m, f = make_model(design, T, settings)
    cases = random_cases(ncase, 7)
    want = ("psd", "std", "zeta", "B_drag", "margin")
    b = m.analyzeCasesBatch(cases, want=want)
    N.check(N.lib().rh_set_a0(N.context(0), 1), "rh_set_a0")
    try:
        a = m.analyzeCasesBatch(cases, want=want)
    finally:
        N.check(N.lib().rh_set_a0(N.context(0), 0), "rh_set_a0")
    np.testing.assert_array_equal(a["iters"], b["iters"])
    np.testing.assert_array_equal(a["status"], b["status"])
    for ic in range(ncase):
        assert rel(a["Xi"][ic], b["Xi"][ic]) < 1e-12, ic
        assert rel(a["B_drag"][ic], b["B_drag"][ic]) < 1e-12, ic
    np.testing.assert_array_equal(a["zeta"], b["zeta"])
    np.testing.assert_allclose(a["margin"], b["margin"], rtol=1e-9, atol=1e-15)
    assert N.lib().rh_set_a0(N.context(0), 2) == N.RH_EINVAL


@pytest.mark.parametrize("tag,design,settings", [("c2_nw200", "VolturnUS-S_example", None), ("c1_OC3spar", "OC3spar", None)])
def test_solve_with_native_statics(tag, design, settings):
    """The whole per-design preparation on the host (statics from raft/statics.py, only the
    mooring stiffness given, as MoorPy would supply it) and the device solve reproduce the
    reference's golden runs."""
    import raft
    T = load_golden(tag)
    d = load_design(design)
    if settings:
        d["settings"].update(settings)
    m = raft.Model(d, statics=[{"C_moor": T["C_moor"]}])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    for k in ["M_struc", "C_struc", "C_hydro"]:
        assert np.abs(getattr(f, k) - T[k]).max() <= 1e-12 * np.abs(T[k]).max()
    for ic, case in enumerate(golden_cases(T)):
        Xi = m.solveDynamics(dict(case))
        assert f.iterations == T["out_iters"][ic]
        assert rel(Xi, T["out_Xi"][ic]) < RTOL


def test_analyze_cases_c1_every_channel():
    """Model.analyzeCases on OC3spar (C1, the design's own case table, wind 0) with the
    reference's statics and mooring stiffness: results['case_metrics'][iCase][0] carries every
    key the reference's saveTurbineOutputs writes (except the mooring-tension Tmoor_*
    channels, which need a mooring system) and matches its values; the keys the WEIS caller
    reads (raft/omdao_raft.py:767-801) are present."""
    import raft
    T = load_golden("c1_OC3spar")
    d = load_design("OC3spar")
    cases = golden_cases(T)
    d["cases"]["data"] = [[c.get(k, 0) if k not in ("wind_speed",) else 0 for k in d["cases"]["keys"]]
                          for c in cases]
    for row, c in zip(d["cases"]["data"], cases):
        for j, k in enumerate(d["cases"]["keys"]):
            if k in c:
                row[j] = c[k]
    m = raft.Model(d, statics=[statics_of(T)])
    res = m.analyzeCases()
    assert set(res) >= {"properties", "case_metrics", "mean_offsets"}
    ref_keys = set(str(k) for k in T["out_metric_keys"]) - {f"Tmoor_{s}" for s in ["avg", "std", "max", "min", "PSD"]}
    for ic in range(len(cases)):
        cm = res["case_metrics"][ic][0]
        assert set(cm) >= ref_keys, sorted(ref_keys - set(cm))
        assert rel(cm["surge_RA"], T["out_Xi"][ic][:, 0, :]) < RTOL
        assert rel(cm["pitch_RA"], T["out_Xi"][ic][:, 4, :] * 57.29577951308232) < RTOL
        for dof in ["surge", "sway", "heave", "roll", "pitch", "yaw"]:
            np.testing.assert_allclose(cm[dof + "_std"], T[f"out_{dof}_std"][ic], rtol=RTOL, atol=1e-300)
        np.testing.assert_allclose(cm["wave_PSD"], T["out_wave_PSD"][ic], rtol=RTOL)
        check_rotor_channels(cm, T, ic)
        for n in ["surge", "sway", "heave", "roll", "pitch", "yaw", "AxRNA", "Mbase"]:   # omdao_raft.py:767-777
            for st in ["avg", "std", "max", "PSD"]:
                assert f"{n}_{st}" in cm
        assert "omega_max" in cm                                                          # :800


def test_margin_output_and_knobs():
    """rh_solve_out.margin: the closest call of the convergence test is finite, negative for
    cases whose final iteration passed, and independent of the kernel choice (per-context
    knob rh_set_solver)."""
    from raft import _native as N
    from raft.solver import CaseSet, solve_batch
    T = load_golden("c2_nw200")
    m, f = make_model("VolturnUS-S_example", T)
    cases = random_cases(24, 5)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    a = solve_batch([f.device_design()], cs, m.nIter, m.XiStart, 0.01, want=("margin",)).host()
    ctx = N.context(0)
    assert N.lib().rh_set_solver(ctx, 7) == N.RH_EINVAL
    assert N.lib().rh_set_solver(ctx, 3) == N.RH_EINVAL      # the lane-pair kernel is a tools/ubench variant
    N.check(N.lib().rh_set_solver(ctx, 1), "rh_set_solver")
    try:
        b = solve_batch([f.device_design()], cs, m.nIter, m.XiStart, 0.01, want=("margin",)).host()
    finally:
        N.check(N.lib().rh_set_solver(ctx, 0), "rh_set_solver")
    assert np.all(np.isfinite(a["margin"]))
    conv = a["status"] == N.RH_CASE_CONVERGED
    assert np.all(a["margin"][~conv] > 0) or np.all(conv)
    np.testing.assert_array_equal(a["iters"], b["iters"])
    np.testing.assert_allclose(a["margin"], b["margin"], rtol=1e-9, atol=1e-15)


@pytest.mark.parametrize("nw", [77, 255, 256, 333, 513, 1000, 1025, 1500, 2048])
def test_odd_grids(nw):
    """Grids that leave pad lanes: nw not a multiple of 64 (every block size), odd nw, nw just
    past a block size (whole pad waves), and grids beyond 1024 bins (k_solve_lds in two passes
    with XiLast in the Xi_last block).  The default kernel (k_solve_lds, including its 128-thread
    and two-pass forms) against the general kernel k_solve_cases on the same batch: identical
    iteration counts and statuses, Xi within 1e-12."""
    from raft import _native as N
    T = load_golden("c2_nw200")
    m, f = make_model("VolturnUS-S_example", T, {"min_freq": 0.2 / nw})
    assert m.nw == nw
    cases = random_cases(24, nw)
    want = ("psd", "std", "zeta", "B_drag", "rao", "margin")
    a = m.analyzeCasesBatch(cases, want=want)
    for other in (1,):
        N.check(N.lib().rh_set_solver(N.context(0), other), "rh_set_solver")
        try:
            b = m.analyzeCasesBatch(cases, want=want)
        finally:
            N.check(N.lib().rh_set_solver(N.context(0), 0), "rh_set_solver")
        np.testing.assert_array_equal(a["iters"], b["iters"])
        np.testing.assert_array_equal(a["status"], b["status"])
        for ic in range(len(cases)):
            assert rel(a["Xi"][ic], b["Xi"][ic]) < 1e-12, (other, ic)
            assert rel(a["psd"][ic], b["psd"][ic]) < 1e-12, (other, ic)
            assert rel(a["B_drag"][ic], b["B_drag"][ic]) < 1e-12, (other, ic)
        # per case, relative to its largest DOF (a heading-0 case has noise-level sway/roll/yaw)
        smax = np.abs(b["std"]).max(axis=1, keepdims=True)
        assert np.all(np.abs(a["std"] - b["std"]) <= 1e-12 * smax)
        np.testing.assert_allclose(a["margin"], b["margin"], rtol=1e-9, atol=1e-15)


def test_linearisation_only_solve_without_xi():
    """rh_solve_out.Xi = NULL (solver.solve_batch want "noXi", what Model.analyzeArrayBatch asks
    for): the same iteration counts, B_drag, Bmat and zeta bit for bit as with the response
    stored; psd / std / rao without Xi are refused."""
    from raft import _native as N
    from raft.solver import CaseSet, solve_batch
    T = load_golden("c2_nw200")
    m, f = make_model("VolturnUS-S_example", T)
    cases = random_cases(40, 13)
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases], ["JONSWAP"] * len(cases),
                 [c["wave_height"] for c in cases], [c["wave_period"] for c in cases], [0.0] * len(cases))
    dd = f.device_design()
    a = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("zeta", "B_drag", "Bmat")).host()
    b = solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("zeta", "B_drag", "Bmat", "noXi")).host()
    assert "Xi" not in b
    for k in ("iters", "status", "zeta", "B_drag", "Bmat"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    with pytest.raises(Exception, match="need the Xi output"):
        solve_batch([dd], cs, m.nIter, m.XiStart, 0.01, want=("psd", "noXi"))
