"""GPU: operating-rotor solves (wind > 0) against the reference.

tests/golden/make_golden.py golden_aero ran the reference's Model.solveDynamics and
saveTurbineOutputs on VolturnUS-S_example (nw = 200) with its IEA-15MW rotor, aeroServoMod 1
and 2, two wind/wave cases each, with the scripted CCBlade stand-in (tests/golden/
fake_ccblade.py; CCBlade is a third-party dependency that is not installed).  The same stand-in
drives this build: Rotor.calcAero's added mass and damping enter the device solve as per-bin
M and B (k_solve_lds, mb_per_bin), so Xi, the iteration counts and every output channel,
including the aero tower-base moment and the rotor speed / torque / pitch spectra, are checked."""
import json

import numpy as np
import pytest

from conftest import aero_model, load_golden

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.mark.parametrize("mod", [1, 2])
def test_operating_rotor_solve_matches_reference(mod, monkeypatch):
    T = load_golden(f"aero_mod{mod}")
    m, f = aero_model(T, mod, monkeypatch)
    for ic, case in enumerate(json.loads(str(T["cases_full_json"]))):
        f.calcTurbineConstants(dict(case), ptfm_pitch=0)
        Xi = m.solveDynamics(dict(case))
        assert f.iterations == T["out_iters"][ic], (ic, f.iterations, T["out_iters"][ic])
        assert rel(Xi, T["out_Xi"][ic]) < RTOL, rel(Xi, T["out_Xi"][ic])
        assert rel(f.B_hydro_drag, T["out_B_drag"][ic]) < RTOL
        res = {}
        f.saveTurbineOutputs(res, case)
        for dof in ["surge", "sway", "heave", "roll", "pitch", "yaw"]:
            np.testing.assert_allclose(res[dof + "_std"], T[f"out_{dof}_std"][ic], rtol=RTOL)
        for ch in ["AxRNA", "Mbase"]:
            for st in ["avg", "std", "max", "min", "PSD"]:
                ref = np.asarray(T[f"out_{ch}_{st}"][ic])
                np.testing.assert_allclose(res[f"{ch}_{st}"], ref, rtol=RTOL, atol=RTOL * np.abs(ref).max(),
                                           err_msg=f"{ch}_{st}")
        for ch in ["omega", "torque", "bPitch"]:
            for st in ["avg", "std", "PSD"]:
                ref = np.asarray(T[f"out_{ch}_{st}"][ic])
                np.testing.assert_allclose(res[f"{ch}_{st}"], ref, rtol=RTOL, atol=RTOL * max(np.abs(ref).max(), 1e-300),
                                           err_msg=f"{ch}_{st}")
        for k in ["omega_max", "omega_min", "power_avg", "wind_PSD"]:
            if "out_" + k in T:
                ref = np.asarray(T["out_" + k][ic])
                np.testing.assert_allclose(res[k], ref, rtol=RTOL, atol=RTOL * max(np.abs(ref).max(), 1e-300), err_msg=k)


def test_operating_rotor_cases_in_one_batch(monkeypatch):
    """analyzeCasesBatch with operating rotors: every wind case of both aero goldens and the
    wind-0 cases of c2_nw200 (same design and grid) in one launch; each case has its own
    per-bin M and B (CaseMB) on the shared node and wave tables."""
    cases, refs = [], []
    T0 = None
    for mod in (1, 2):
        T = load_golden(f"aero_mod{mod}")
        T0 = T0 or T
        for ic, c in enumerate(json.loads(str(T["cases_full_json"]))):
            cases.append((mod, c))
            refs.append((T["out_Xi"][ic][0], T["out_iters"][ic]))
    for mod in (1, 2):
        m, f = aero_model(T0, mod, monkeypatch)
        sel = [i for i, (md, _) in enumerate(cases) if md == mod]
        W = load_golden("c2_nw200")
        from conftest import golden_cases
        calm = golden_cases(W)[:3]
        res = m.analyzeCasesBatch([cases[i][1] for i in sel] + calm, want=("psd", "std"))
        for j, i in enumerate(sel):
            assert res["iters"][j] == refs[i][1], (i, res["iters"][j], refs[i][1])
            assert rel(res["Xi"][j], refs[i][0]) < RTOL, rel(res["Xi"][j], refs[i][0])
        for j in range(len(calm)):
            k = len(sel) + j
            assert res["iters"][k] == W["out_iters"][j]
            assert rel(res["Xi"][k], W["out_Xi"][j][0]) < RTOL, rel(res["Xi"][k], W["out_Xi"][j][0])


def test_run_raft_with_operating_rotor(monkeypatch):
    """runRAFT on VolturnUS-S_example with its own wind cases (16 m/s, class and intensity
    turbulence) and the full rotor: mean offsets with the rotor thrust (solveStatics), then the
    device solve with the aero M and B per bin.  MoorPy is absent, so no reference run covers
    the offsets; the last case's response is checked against the CPU oracle on the same offset
    tables, with the aero matrices as its per-bin added mass and damping."""
    import os
    import sys

    import raft
    import raft.rotor as R
    from conftest import GOLDEN, load_design, oracle_tables_of
    from oracle import raft_oracle as O
    sys.path.insert(0, GOLDEN)
    from fake_ccblade import FakeAirfoil, FakeCCBlade
    monkeypatch.setattr(R, "ccblade_classes", lambda: (FakeCCBlade, FakeAirfoil))
    d = load_design("VolturnUS-S_example")
    with open(os.path.join(GOLDEN, "designs", "IEA15MW_turbine.json")) as fh:
        turb = json.load(fh)
    for k in ("blade", "airfoils", "wt_ops", "pitch_control", "torque_control", "gear_ratio", "I_drivetrain",
              "nBlades", "Rhub", "precone"):
        d["turbine"][k] = turb[k]
    m = raft.runRAFT(d)
    f = m.fowtList[0]
    offs = np.array(m.results["mean_offsets"])
    assert offs.shape[0] == 3 and offs[1, 0] > offs[0, 0] + 1.0      # thrust pushes the platform downwind
    case = dict(zip(d["cases"]["keys"], d["cases"]["data"][-1]))
    T = oracle_tables_of(f)
    T["A_BEM"] = np.sum(f.A_aero, axis=3)
    T["B_BEM"] = np.sum(f.B_aero, axis=3) + np.sum(f.B_gyro, axis=2)[:, :, None]
    r = O.solve_dynamics(T, dict(case), int(m.nIter), float(m.XiStart))
    assert f.iterations == r["iters"]
    assert rel(f.Xi, r["Xi"]) < RTOL, rel(f.Xi, r["Xi"])


def test_wind_case_with_bem_restatement():
    """The reference's wind-wave-current load case (tests/test_model.py:68: 8 m/s wind at 30 deg,
    4 m / 10 s JONSWAP waves, 0.6 m/s current) on its VolturnUS-S test design with the IEA-15MW
    blades, through analyzeCases with the CCBlade restatement (raft/ccblade.py; the package is
    absent): the mean offset equals the reference's desired_X0 at its rtol 1e-5 (the rotor's
    thrust, side forces and hub moments all enter it), and the device solve with the aero
    added mass and damping per bin equals the CPU oracle on the same tables (1e-9, same
    iteration count)."""
    import raft
    from conftest import load_design, oracle_tables_of
    from oracle import raft_oracle as O
    from test_mooring import CASES, DESIRED_X0
    d = load_design("VolturnUS-S_aero")
    case = dict(CASES["wind_wave_current"])
    d["cases"]["data"] = [[case[k] for k in d["cases"]["keys"]]]
    m = raft.Model(d)
    m.analyzeCases()
    f = m.fowtList[0]
    np.testing.assert_allclose(m.results["mean_offsets"][0], DESIRED_X0["wind_wave_current"][0], rtol=1e-5,
                               atol=1e-10)
    assert np.abs(f.B_aero).max() > 0          # aero damping per bin (aeroServoMod 1: no added mass)
    T = oracle_tables_of(f)
    T["A_BEM"] = np.sum(f.A_aero, axis=3)
    T["B_BEM"] = np.sum(f.B_aero, axis=3) + np.sum(f.B_gyro, axis=2)[:, :, None]
    r = O.solve_dynamics(T, dict(case), int(m.nIter), float(m.XiStart))
    assert f.iterations == r["iters"]
    assert rel(f.Xi, r["Xi"]) < RTOL, rel(f.Xi, r["Xi"])
