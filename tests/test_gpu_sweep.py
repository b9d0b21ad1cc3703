"""GPU parity for the multi-design (C5) and multi-FOWT (C4) paths, against reference runs.

* C5: three parametersweep variants of VolturnUS-S_example (raft/sweep.py restating
  raft/parametersweep.py:56-88) at nw = 1000.  The reference computed the statics of each
  variant itself (tests/golden/make_golden.py golden_sweep); here the product does the whole
  per-design preparation (members, statics, added mass) and solves every case of every
  design in ONE rh_solve_cases launch.
* C4: tests/test_data/VolturnUS-S_farm.yaml, two FOWTs 1600 m apart, coupled through the
  array stiffness fixture (raft/raft_model.py:1021-1065).

Tolerance (north_star): 1e-9 relative (normwise per case), identical iteration counts.
"""
import numpy as np
import pytest

from conftest import farm_tables, fixture_design, golden_cases, load_design, load_golden, statics_of
from oracle import raft_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-9
SWEEP_TAGS = ["c5_sweep0", "c5_sweep1", "c5_sweep2"]


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def _sweep_inputs():
    designs, cmoor, idx, cases, refs = [], [], [], [], []
    for i, tag in enumerate(SWEEP_TAGS):
        d, T, _ = fixture_design(tag, "VolturnUS-S_example")
        d["settings"]["min_freq"] = 0.0002
        designs.append(d)
        cmoor.append({"C_moor": T["C_moor"]})
        for ic, c in enumerate(golden_cases(T)):
            idx.append(i)
            cases.append(c)
            refs.append((T, ic))
    return designs, cmoor, idx, cases, refs


def _check_case(res, j, T, ic):
    assert res["iters"][j] == T["out_iters"][ic], (j, res["iters"][j], T["out_iters"][ic])
    assert res["status"][j] == T["out_conv"][ic]
    assert rel(res["Xi"][j], T["out_Xi"][ic][0]) < RTOL, rel(res["Xi"][j], T["out_Xi"][ic][0])
    assert rel(res["B_drag"][j], T["out_B_drag"][ic]) < RTOL
    dofs = ["surge", "sway", "heave", "roll", "pitch", "yaw"]
    smax = max(T[f"out_{d}_std"][ic] for d in dofs)
    for i, dof in enumerate(dofs):
        np.testing.assert_allclose(res["std"][j, i], T[f"out_{dof}_std"][ic], rtol=RTOL, atol=RTOL * smax)


@pytest.mark.parametrize("native", [False, True])
def test_sweep_variants_one_launch_match_reference(native):
    """The product's per-design preparation (Python host path, or librafthip's
    rh_prep_designs) + one launch over 3 designs x 2 sea states."""
    from raft.batch import DesignBatch
    designs, cmoor, idx, cases, refs = _sweep_inputs()
    B = DesignBatch(designs, statics=cmoor, native=native)
    for i, (T, _) in enumerate([refs[0], refs[2], refs[4]]):
        for j, k in enumerate(["M_struc", "B_struc", "C_struc", "C_hydro"]):
            got = B._prepared.statics[i, j] if native else getattr(B.fowts[i], k)
            if k in T:
                assert np.abs(got - T[k]).max() <= 1e-12 * np.abs(T[k]).max(), k
    res = B.solve(idx, cases).host()
    for j, (T, ic) in enumerate(refs):
        _check_case(res, j, T, ic)


def test_full_size_c5_sweep_properties():
    """C5 at full size: 250 designs x 40 sea states = 10,000 cases, nw = 1000, one launch.
    The three reference-run variants are designs 0-2 of the batch and their golden cases
    are embedded in the case list; the rest is checked by size-independent properties:
    a 64-case sub-batch reproduces its cases bit for bit, every case finishes with a
    finite response and a consistent status/iteration count."""
    import torch
    from raft.batch import DesignBatch, sweep_cases
    from raft.sweep import sea_state_grid, sweep_multipliers, sweep_variant
    designs, cmoor, gidx, gcases, refs = _sweep_inputs()
    base = load_design("VolturnUS-S_example")
    base["settings"]["min_freq"] = 0.0002
    mult = sweep_multipliers(250)
    designs = designs + [sweep_variant(base, m) for m in mult[3:]]
    B = DesignBatch(designs, statics={"C_moor": refs[0][0]["C_moor"]})
    idx, cases = sweep_cases(len(designs), sea_state_grid())
    idx = np.concatenate([idx, np.asarray(gidx, dtype=np.int32)])
    cases = cases + gcases
    assert len(idx) == 10000 + len(gcases)
    res = B.solve(idx, cases, want=("std", "B_drag", "margin"))
    torch.cuda.synchronize()
    h = res.host()
    n0 = 10000
    # the 16 closest calls of the convergence test vs the oracle on the same host-prepared
    # design tables (conftest.oracle_tables_of): identical iteration counts, Xi within 1e-9
    from conftest import oracle_tables_of
    close = np.argsort(np.abs(h["margin"][:n0]))[:16]
    for ic in close:
        Tn = oracle_tables_of(B.fowts[idx[ic]])
        r = O.solve_dynamics(Tn, dict(cases[ic]), int(B.nIter), float(B.XiStart))
        assert h["iters"][ic] == r["iters"], (ic, h["margin"][ic])
        assert rel(h["Xi"][ic], r["Xi"][0]) < 1e-9
    for j, (T, ic) in enumerate(refs):
        _check_case(h, n0 + j, T, ic)
    assert np.all(np.isfinite(h["Xi"]))
    assert set(np.unique(h["status"])) <= {0, 1}
    assert np.all(h["iters"][h["status"] == 0] == B.nIter + 1)
    assert np.all((h["iters"] >= 1) & (h["iters"] <= B.nIter + 1))
    sub = np.sort(np.random.default_rng(9).choice(n0, 64, replace=False))
    s = B.solve(idx[sub], [cases[i] for i in sub], want=("std", "B_drag")).host()
    np.testing.assert_array_equal(s["Xi"], h["Xi"][sub])
    np.testing.assert_array_equal(s["iters"], h["iters"][sub])


def _farm_model(T, native_statics=False):
    import raft
    Ts = farm_tables(T)
    m = raft.Model(load_design("VolturnUS-S_farm"),
                   statics=[{"C_moor": t["C_moor"]} if native_statics else statics_of(t) for t in Ts])
    m.K_array = T["K_array"]
    for f, t in zip(m.fowtList, Ts):
        f.setPosition(t["r6"])
        f.calcStatics()
        f.calcHydroConstants()
    return m, Ts


@pytest.mark.parametrize("native_statics", [False, True])
def test_farm_matches_reference(native_statics):
    """C4: 2 coupled FOWTs, 12-DOF system; per-FOWT drag loops and iteration counts."""
    T = load_golden("c4_farm")
    m, Ts = _farm_model(T, native_statics)
    for ic, case in enumerate(golden_cases(T)):
        Xi = m.solveDynamics(dict(case))
        assert [f.iterations for f in m.fowtList] == list(T["out_iters"][ic])
        assert Xi.shape == T["out_Xi"][ic].shape
        assert rel(Xi, T["out_Xi"][ic]) < RTOL, rel(Xi, T["out_Xi"][ic])
        for i, f in enumerate(m.fowtList):
            assert rel(f.B_hydro_drag, T["out_B_drag"][ic][i]) < RTOL
            assert rel(f.Xi, T["out_Xi"][ic][:, 6 * i:6 * i + 6]) < RTOL


def test_farm_seeded_cases_match_oracle():
    """Seeded sea states (other headings, gamma) beyond the golden set, vs the oracle."""
    T = load_golden("c4_farm")
    m, Ts = _farm_model(T)
    rng = np.random.default_rng(44)
    for _ in range(3):
        case = dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                    wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=float(rng.choice([0.0, 2.0])))
        Xi = m.solveDynamics(dict(case))
        r = O.solve_farm(Ts, dict(case), int(T["nIter"]), T["K_array"], float(T["XiStart"]))
        assert [f.iterations for f in m.fowtList] == r["iters"]
        assert rel(Xi, r["Xi"]) < RTOL


def test_farm_batch_matches_reference_and_oracle():
    """C4 batched (Model.analyzeArrayBatch): the golden sea states plus 40 seeded ones in one
    batch -- every (case, FOWT) drag loop in one launch, the 12-DOF system solves of all cases in
    another.  Golden cases against the reference run, a sample of the seeded ones against the
    oracle; identical iteration counts; per-FOWT statistics against the host formula."""
    T = load_golden("c4_farm")
    m, Ts = _farm_model(T)
    gold = golden_cases(T)
    rng = np.random.default_rng(45)
    seeded = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                   wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=float(rng.choice([0.0, 2.0])))
              for _ in range(40)]
    cases = gold + seeded
    r = m.analyzeCasesBatch(cases)
    assert r["Xi"].shape == (len(cases), 12, m.nw)
    for ic in range(len(gold)):
        assert list(r["iters"][ic]) == list(T["out_iters"][ic])
        assert rel(r["Xi"][ic], T["out_Xi"][ic][0]) < RTOL, rel(r["Xi"][ic], T["out_Xi"][ic][0])
    for j in [0, 7, 23, 39]:
        o = O.solve_farm(Ts, dict(seeded[j]), int(T["nIter"]), T["K_array"], float(T["XiStart"]))
        assert list(r["iters"][len(gold) + j]) == o["iters"]
        assert rel(r["Xi"][len(gold) + j], o["Xi"][0]) < RTOL
    dw = float(m.fowtList[0].dw)
    for i in range(2):
        x = r["Xi"][:, 6 * i:6 * i + 6, :].copy()
        x[:, 3:] *= 57.29577951308232
        np.testing.assert_allclose(r["psd"][:, i], 0.5 * np.abs(x) ** 2 / dw, rtol=1e-12, atol=1e-300)
        np.testing.assert_allclose(r["std"][:, i], np.sqrt(0.5 * np.sum(np.abs(x) ** 2, axis=2)), rtol=1e-12)


def test_heterogeneous_farm_batch_matches_oracle():
    """A 2-FOWT farm whose platforms differ (raft/raft_model.py:137-156 lets each FOWT take its
    own platform): the second is a parametersweep variant with 1.5x pontoons, 61 submerged nodes
    against 53.  analyzeArrayBatch (Bmat rows padded to the larger node count) against
    oracle.solve_farm on the host-prepared tables of both FOWTs: identical iteration counts,
    Xi at 1e-9; and the per-case Model.solveDynamics path against the batch."""
    import raft
    from conftest import oracle_tables_of
    from raft.sweep import sweep_variant
    T = load_golden("c4_farm")
    Ts = farm_tables(T)
    d = load_design("VolturnUS-S_farm")
    d["platforms"] = [d["platform"], sweep_variant({"platform": d["platform"]}, (1.0, 1.0, 1.5, 1.0, 1.0))["platform"]]
    d["array"]["data"][1][1] = 2
    m = raft.Model(d, statics=[{"C_moor": t["C_moor"]} for t in Ts])
    m.K_array = T["K_array"]
    for f, t in zip(m.fowtList, Ts):
        f.setPosition(t["r6"])
        f.calcStatics()
        f.calcHydroConstants()
    nns = [f.device_design().nn for f in m.fowtList]
    assert nns[0] != nns[1], nns
    rng = np.random.default_rng(46)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                  wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=float(rng.choice([0.0, 2.0])))
             for _ in range(12)]
    r = m.analyzeCasesBatch(cases)
    Tor = [oracle_tables_of(f) for f in m.fowtList]
    for j in (0, 5, 11):
        o = O.solve_farm(Tor, dict(cases[j]), int(m.nIter), T["K_array"], float(m.XiStart))
        assert list(r["iters"][j]) == o["iters"]
        assert rel(r["Xi"][j], o["Xi"][0]) < RTOL, rel(r["Xi"][j], o["Xi"][0])
    Xi = m.solveDynamics(dict(cases[3]))
    assert [f.iterations for f in m.fowtList] == list(r["iters"][3])
    assert rel(r["Xi"][3], Xi[0]) < 1e-12


def test_batched_wave_tables_equal_per_design_tables():
    """rh_wave_tables_batch (one launch for a sweep) writes the same bits as rh_wave_tables
    per design, for designs with different node counts and two headings each."""
    import torch
    from raft.batch import DesignBatch
    from raft.hydro_math import DEG2RAD
    from raft.sweep import sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    designs = [sweep_variant(base, m) for m in sweep_multipliers(4, seed=11)]
    st = {"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}
    A = DesignBatch(designs, statics=st, native=True)
    B = DesignBatch(designs, statics=st, native=True)
    cases = [dict(wave_heading=h, wave_height=4.0, wave_period=10.0) for h in (30.0, 0.0)]
    idx = np.repeat(np.arange(4), 2)
    cs = A.case_set(idx, cases * 4)
    from raft.solver import prepare_batch
    pa = prepare_batch(A.dds, cs)                   # batched path (fresh designs)
    for i, d in enumerate(B.dds):                    # per-design launches
        d.ensure_headings(np.array([0.0, 30.0]) * DEG2RAD)
    torch.cuda.synchronize()
    assert len({d.nn for d in A.dds}) > 1
    for i, (a, b) in enumerate(zip(A.dds, B.dds)):
        for h, beta in enumerate(a.headings):
            j = b.headings.index(beta)
            for t in ("uhat", "kproj", "finer"):
                assert torch.equal(getattr(a, t)[h], getattr(b, t)[j]), (i, h, t)
    res_a = A.solve(None, cs, prepared=pa).host()
    res_b = B.solve(None, cs).host()
    np.testing.assert_array_equal(res_a["Xi"], res_b["Xi"])
    np.testing.assert_array_equal(res_a["iters"], res_b["iters"])


def test_pipelined_sweep_equals_one_batch():
    """solve_sweep (design blocks prepared on the host while the previous block solves, uploads
    on a copy stream) gives the same bits as one DesignBatch over the whole sweep."""
    import torch
    from raft.batch import DesignBatch, solve_sweep, sweep_cases
    from raft.sweep import sea_state_grid, sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    designs = [sweep_variant(base, m) for m in sweep_multipliers(7, seed=13)]
    grid = sea_state_grid()[::5]
    st = {"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}
    idx, _ = sweep_cases(len(designs), grid)
    sidx = np.arange(len(idx)) % len(grid)
    out, keep = solve_sweep(designs, st, idx, sidx, grid, chunks=3, want=("std", "psd"))
    B = DesignBatch(designs, statics=st, native=True)
    ref = B.solve(None, B.case_set_grid(idx, sidx, grid), want=("std", "psd"))
    # the bench's path: spec records from the base and the multipliers, built per block
    from raft.native_prep import sweep_specs
    mult = sweep_multipliers(7, seed=13)
    out2, keep2 = solve_sweep([base] * len(designs), st, idx, sidx, grid, chunks=3, want=("std", "psd"),
                              specs=lambda a, b: sweep_specs(base, mult[a:b], statics=st), threads=4)
    # the per-design path of the blocks (DesignBatch objects) against the block descriptor arrays
    out3, keep3 = solve_sweep([base] * len(designs), st, idx, sidx, grid, chunks=3, want=("std", "psd"),
                              specs=lambda a, b: sweep_specs(base, mult[a:b], statics=st), threads=4,
                              block_path=False)
    from raft import _native as N
    from raft.sweep_block import BlockDesigns
    assert all(isinstance(k[0], BlockDesigns) for k in keep2)
    assert not any(isinstance(k[0], BlockDesigns) for k in keep3)
    # a block's designs carry no velocity table: the entry points that read it refuse them
    blk = keep2[0][0]
    one = torch.zeros(1, dtype=torch.int32, device="cuda")
    z = torch.zeros([1, blk.nw], dtype=torch.float64, device="cuda")
    bd = torch.zeros([1, 36], dtype=torch.float64, device="cuda")
    bm = torch.zeros([1, blk.nnmax, 9], dtype=torch.float64, device="cuda")
    xo = torch.empty([1, 6, blk.nw], dtype=torch.complex128, device="cuda")
    rc = N.lib().rh_heading_response_ext(N.context(0), blk.arr, len(blk), 1, N.ptr(one), N.ptr(one), N.ptr(z),
                                         N.ptr(bd), N.ptr(bm), 0, None, N.ptr(xo), N.stream_handle(torch))
    assert rc == N.RH_EINVAL and b"wave tables missing" in N.lib().rh_last_error()
    torch.cuda.synchronize()
    for k in ("Xi", "iters", "status", "std", "psd"):
        assert torch.equal(out[k], ref[k]), k
        assert torch.equal(out2[k], ref[k]), k
        assert torch.equal(out3[k], ref[k]), k


def test_design_batch_with_operating_rotor():
    """Operating rotors in a design batch: two designs (the reference's VolturnUS-S test design
    with its IEA-15MW rotor, and a parametersweep variant of it), each with a wind-wave-current
    case (8 m/s, tests/test_model.py:68) and a calm sea state, in ONE DesignBatch launch, against
    each design's own Model.analyzeCasesBatch (its per-case aero added mass and damping):
    the same bits and iteration counts."""
    from raft.batch import DesignBatch
    from raft.sweep import sweep_variant
    from test_mooring import CASES
    base = load_design("VolturnUS-S_aero")
    designs = [base, sweep_variant(base, [1.1, 0.9, 1.05, 1.0, 0.95])]
    st = {"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}
    wind = dict(CASES["wind_wave_current"])
    calm = dict(wave_spectrum="JONSWAP", wave_period=9.0, wave_height=3.0, wave_heading=0.0, wave_gamma=0.0,
                wind_speed=0)
    B = DesignBatch(designs, statics=st)
    res = B.solve([0, 0, 1, 1], [wind, calm, wind, calm], want=("std",)).host()
    for d in range(2):
        ref = B.models[d].analyzeCasesBatch([wind, calm], want=("std",))     # the same prepared design
        np.testing.assert_array_equal(res["iters"][2 * d:2 * d + 2], ref["iters"])
        np.testing.assert_array_equal(res["Xi"][2 * d:2 * d + 2], ref["Xi"])
    assert not np.array_equal(res["Xi"][0], res["Xi"][2])          # the variant is another design


def _two_step_array_response(m, P, res):
    """The pre-round-4 path of analyzeArrayBatch's response step: rh_wave_excitation (F of
    every (case, FOWT) to HBM) then rh_system_solve_batch on the fixed point's per-bin Z."""
    import torch
    from raft import _native as N
    nf, n, nw, dev = m.nFOWT, P["n"], m.nw, P["dev"]
    s, ctx = N.stream_handle(torch, dev), N.context(m.device)
    F = torch.empty([n * nf, 6, nw], dtype=torch.complex128, device=dev)
    N.check(N.lib().rh_wave_excitation(ctx, P["arr"], nf, n * nf, N.ptr(P["prep"]["design"]), N.ptr(P["prep"]["head"]),
                                       N.ptr(res["zeta"]), N.ptr(res["Bmat"].contiguous()), N.ptr(F), s),
            "rh_wave_excitation")
    X = torch.empty([n, 6 * nf, nw], dtype=torch.complex128, device=dev)
    N.check(N.lib().rh_system_solve_batch(ctx, n, nf, nw, N.ptr(res["Z"]), N.ptr(P["K"]), N.ptr(F), N.ptr(X), s),
            "rh_system_solve_batch")
    return X.cpu().numpy()


@pytest.mark.parametrize("farm", [True, False], ids=["two_fowts", "one_fowt"])
def test_array_response_equals_two_step_path(farm):
    """rh_array_response (one launch: excitation, impedance rebuilt from M / B_lin / C and the
    case's B_drag, block solve) against the two-step path that wrote every (case, bin)
    impedance Z and excitation F to HBM, for two coupled FOWTs (k_array_resp<2>) and for one
    (k_array_resp<1>): the same expressions, so equal to rounding (the compiler contracts the
    products of the two kernels into FMAs in different places: measured 3e-13 at most)."""
    from raft.solver import solve_batch
    from test_gpu_parity import make_model
    if farm:
        m, _ = _farm_model(load_golden("c4_farm"))
    else:
        T = load_golden("c2_nw200")
        m, _ = make_model("VolturnUS-S_example", T)
        assert m.nFOWT == 1
    rng = np.random.default_rng(46)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                  wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=0.0) for _ in range(24)]
    P = m.prepareArrayBatch(cases)
    fused = m.analyzeArrayBatch(prepared=P)["Xi"]
    res = solve_batch(P["dds"], P["cs"], m.nIter, m.XiStart, 0.01, want=("zeta", "Bmat", "Z"), prepared=P["prep"])
    ref = _two_step_array_response(m, P, res)
    for ic in range(len(cases)):
        assert np.linalg.norm(fused[ic] - ref[ic]) <= 1e-12 * np.linalg.norm(ref[ic]), ic


@pytest.mark.parametrize("farm", [True, False], ids=["two_fowts", "one_fowt"])
def test_array_statistics_equal_motion_stats(farm):
    """analyzeArrayBatch's PSD / RMS, formed by k_array_resp from the solution in registers
    (rh_array_solve_stats), equal rh_motion_stats run on its Xi bit for bit, for two coupled
    FOWTs and for one; plain rh_array_response (its own excitation launch, k_array_exc, instead
    of the fixed points' F_wave) gives the same Xi to rounding.  The one-FOWT grid of c2_nw1000
    (1000 bins) runs four bin chunks per workgroup."""
    import torch
    from raft import _native as N
    from test_gpu_parity import make_model
    if farm:
        m, _ = _farm_model(load_golden("c4_farm"))
    else:
        m, _ = make_model("VolturnUS-S_example", load_golden("c2_nw1000"), {"min_freq": 0.0002})
        assert m.nFOWT == 1 and m.nw > 3 * 256
    rng = np.random.default_rng(47)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                  wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=0.0) for _ in range(12)]
    P = m.prepareArrayBatch(cases)
    out = m.analyzeArrayBatch(prepared=P, host=False)
    nf, n, nw = m.nFOWT, len(cases), m.nw
    X = out["Xi"]
    psd = torch.empty([n * nf, 6, nw], dtype=torch.float64, device=X.device)
    std = torch.empty([n * nf, 6], dtype=torch.float64, device=X.device)
    ctx, s = N.context(m.device), N.stream_handle(torch, X.device)
    N.check(N.lib().rh_motion_stats(ctx, n * nf, 1, nw, float(m.fowtList[0].dw), N.ptr(X), N.ptr(psd), N.ptr(std), s),
            "rh_motion_stats")
    np.testing.assert_array_equal(out["psd"].reshape(n * nf, 6, nw).cpu().numpy(), psd.cpu().numpy())
    np.testing.assert_array_equal(out["std"].reshape(n * nf, 6).cpu().numpy(), std.cpu().numpy())
    res, arr, K = out["_keep"]
    prep = P["prep"]
    X2 = torch.empty_like(X)
    N.check(N.lib().rh_array_response(ctx, arr, nf, nf, n, N.ptr(prep["design"]), N.ptr(prep["head"]),
                                      N.ptr(res["zeta"]), N.ptr(res["B_drag"]), N.ptr(res["Bmat"]), N.ptr(K),
                                      N.ptr(X2), s), "rh_array_response")
    a, b = X2.cpu().numpy(), X.cpu().numpy()
    for ic in range(n):
        assert np.linalg.norm(a[ic] - b[ic]) <= 1e-12 * np.linalg.norm(a[ic]), ic


@pytest.mark.parametrize("farm", [True, False], ids=["two_fowts", "one_fowt"])
def test_fixed_point_f_wave_equals_wave_excitation(farm):
    """rh_solve_out.F_wave (the excitation each fixed point forms with its final linearisation,
    the F of the array solve, raft/raft_model.py:1049-1061) against rh_wave_excitation on the
    fixed point's zeta and Bmat: equal to rounding, from the fast kernel and from the general
    one (rh_set_solver(ctx, 1))."""
    import torch
    from raft import _native as N
    from raft.solver import solve_batch
    from test_gpu_parity import make_model
    if farm:
        m, _ = _farm_model(load_golden("c4_farm"))
    else:
        m, _ = make_model("VolturnUS-S_example", load_golden("c2_nw200"))
    rng = np.random.default_rng(48)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                  wave_heading=float(rng.choice([0, 45, 135, 270])), wave_gamma=0.0) for _ in range(10)]
    P = m.prepareArrayBatch(cases)
    nf, n, nw, dev = m.nFOWT, len(cases), m.nw, P["dev"]
    s, ctx = N.stream_handle(torch, dev), N.context(m.device)
    for solver in (0, 1):
        N.check(N.lib().rh_set_solver(ctx, solver), "rh_set_solver")
        try:
            Fw = torch.empty([n * nf, 6, nw], dtype=torch.complex128, device=dev)
            res = solve_batch(P["dds"], P["cs"], m.nIter, m.XiStart, 0.01, want=("zeta", "Bmat"), prepared=P["prep"],
                              F_wave=Fw)
            F = torch.empty_like(Fw)
            N.check(N.lib().rh_wave_excitation(ctx, P["arr"], nf, n * nf, N.ptr(P["prep"]["design"]),
                                               N.ptr(P["prep"]["head"]), N.ptr(res["zeta"]),
                                               N.ptr(res["Bmat"].contiguous()), N.ptr(F), s), "rh_wave_excitation")
            a, b = Fw.cpu().numpy(), F.cpu().numpy()
        finally:
            N.check(N.lib().rh_set_solver(ctx, 0), "rh_set_solver")
        for e in range(n * nf):
            assert np.linalg.norm(a[e] - b[e]) <= 1e-12 * np.linalg.norm(b[e]), (solver, e)


def test_oc4semi_sweep_native_prep_matches_python_prep():
    """An OC4semi sweep (MacCamy-Fuchs columns, raft/raft_member.py:1053-1088: frequency
    dependent inertia tables) prepared by librafthip's rh_prep_designs against the Python
    preparation (raft/member.py, scipy's hankel1): three offset-column diameters x four sea
    states in one launch each; identical iteration counts, responses and RMS within 1e-11
    (the two Bessel implementations differ in the last bits)."""
    import copy
    from raft.batch import DesignBatch
    base = load_design("OC4semi-RAFT_QTF")
    base["platform"]["potSecOrder"] = 0     # first order: native / light designs carry no QTF
    designs = []
    for f in (1.0, 0.9, 1.1):
        d = copy.deepcopy(base)
        d["platform"]["members"][1]["d"] = [float(x) * f for x in base["platform"]["members"][1]["d"]]
        designs.append(d)
    st = {"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}
    rng = np.random.default_rng(23)
    cases = [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(7, 16)), wave_height=float(rng.uniform(2, 9)),
                  wave_heading=float(rng.choice([0.0, 30.0])), wave_gamma=0.0) for _ in range(4)]
    idx = np.repeat(np.arange(3, dtype=np.int32), 4)
    allc = cases * 3
    A = DesignBatch(designs, statics=st, native=True)
    B = DesignBatch(designs, statics=st, native=False)
    assert all(dd.imat is not None for dd in A.dds) and all(dd.imat is not None for dd in B.dds)
    ra = A.solve(idx, allc).host()
    rb = B.solve(idx, allc).host()
    np.testing.assert_array_equal(ra["iters"], rb["iters"])
    np.testing.assert_array_equal(ra["status"], rb["status"])
    for j in range(len(idx)):
        assert rel(ra["Xi"][j], rb["Xi"][j]) < 1e-11, j
        np.testing.assert_allclose(ra["std"][j], rb["std"][j], rtol=1e-11, atol=1e-11 * rb["std"][j].max())


def test_descriptor_block_equals_per_design_descriptors():
    """prep.descriptor_block (a sweep block's rh_design descriptors filled column-wise) writes
    the bytes DeviceDesign._make_struct writes for every design, with the lazily viewed shared
    wave tables (DeviceDesign.set_tables) and after the views are made."""
    from raft.batch import DesignBatch
    from raft.solver import prepare_batch
    from raft.sweep import sweep_multipliers, sweep_variant
    base = load_design("VolturnUS-S_example")
    designs = [sweep_variant(base, m) for m in sweep_multipliers(5, seed=3)]
    B = DesignBatch(designs, statics={"C_moor": np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])}, native=True)
    cases = [dict(wave_heading=h, wave_height=4.0, wave_period=10.0) for h in (0.0, 30.0)]
    cs = B.case_set(np.repeat(np.arange(5), 2), cases * 5)
    prepare_batch(B.dds, cs)
    for d in B.dds:
        assert "uhat" not in d.__dict__                      # not viewed yet
        assert bytes(d.struct()) == bytes(d._make_struct())
        assert d.uhat.shape == (2, d.nn, 3, d.nw) and d.finer.shape == (2, 6, d.nw)
        assert bytes(d.struct()) == bytes(d._make_struct())
