"""CPU: rotor aerodynamics and control linearisation (raft/rotor.py) against the reference's
Rotor (raft/raft_rotor.py) run by tests/golden/make_golden.py golden_rotor.

CCBlade, the BEM solver both call, is a third-party dependency that is not installed; both
sides run with the same scripted stand-in (tests/golden/fake_ccblade.py), so what is pinned is
RAFT's own rotor code: the CCBlade inputs (polars resampled on the angle-of-attack grid, PCHIP
over the span by thickness, blade tables, site fluid properties), the operating schedule and
control gains, the inflow / tilt / yaw angles handed to CCBlade, the IEC Kaimal rotor spectrum,
and calcAero's mean loads, excitation, added mass and damping for aeroServoMod 1 and 2."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)


@pytest.fixture(scope="module")
def G():
    return dict(np.load(os.path.join(GOLD, "rotor_IEA15MW.npz")))


def _turbine(mod):
    with open(os.path.join(GOLD, "designs", "IEA15MW_turbine.json")) as f:
        t = json.load(f)
    t["aeroServoMod"] = mod
    return t


def _rotor(G, mod):
    from fake_ccblade import FakeAirfoil, FakeCCBlade
    from raft.rotor import Rotor
    return Rotor(_turbine(mod), G["w"], 0, ccblade=(FakeCCBlade, FakeAirfoil))


def test_ccblade_inputs_match_reference(G):
    """Every argument the reference hands CCBlade, and the span tables beside them."""
    rot = _rotor(G, 1)
    for k, v in rot.ccblade.args.items():
        np.testing.assert_allclose(v, G["cc_" + k], rtol=1e-14, atol=0, err_msg=k)
    for k in ("Ca_interp", "r_thick_interp", "cpmin_interp"):
        np.testing.assert_allclose(getattr(rot, k), G[k], rtol=1e-14, atol=0, err_msg=k)


@pytest.mark.parametrize("mod", [1, 2])
def test_calc_aero_and_kaimal_match_reference(G, mod):
    rot = _rotor(G, mod)
    cases = json.loads(str(G["cases"]))
    for ic, c in enumerate(cases):
        rot.yaw_mode = c["yaw_mode"]
        case = {k: v for k, v in c.items() if k != "yaw_mode"}
        rot.setPosition(np.array([0.0, 0.0, 0.0, 0.0, 0.02, 0.1]))
        f0, f, a, b = rot.calcAero(dict(case))
        kai = np.array(rot.IECKaimal(dict(case)))
        tag = f"m{mod}_c{ic}"
        np.testing.assert_allclose(np.array(rot.ccblade.calls[-1]), G[tag + "_call"], rtol=1e-14, atol=1e-15)
        np.testing.assert_allclose([rot.yaw, rot.turbine_heading], G[tag + "_yaw"], rtol=1e-14, atol=1e-15)
        for name, x in (("f0", f0), ("f", f), ("a", a), ("b", b), ("kaimal", kai)):
            ref = G[f"{tag}_{name}"]
            scale = max(np.abs(ref).max(), 1e-300)
            assert np.abs(x - ref).max() <= 1e-12 * scale, (tag, name, np.abs(x - ref).max() / scale)
        if mod == 2:
            np.testing.assert_allclose(rot.C, G[tag + "_C"], rtol=1e-12, atol=0)


def test_calc_aero_needs_ccblade():
    """Without CCBlade (not installed here) the aero path raises instead of guessing."""
    from raft.rotor import Rotor
    w = np.arange(1, 11) * 0.05
    rot = Rotor(_turbine(1), w, 0, ccblade=(None, None))
    assert rot.ccblade is None and rot.blade_r.size > 0
    with pytest.raises(NotImplementedError, match="CCBlade"):
        rot.calcAero(dict(wind_speed=10.0, wind_heading=0.0, turbulence=0.1))


@pytest.mark.parametrize("mod", [1, 2])
def test_turbine_constants_match_reference(mod, monkeypatch):
    """FOWT.calcTurbineConstants at wind > 0 (raft/raft_fowt.py:773-845): A_aero, B_aero,
    f_aero0 and B_gyro about the platform reference point, per golden_aero case."""
    from conftest import aero_model, load_golden
    T = load_golden(f"aero_mod{mod}")
    m, f = aero_model(T, mod, monkeypatch)
    for ic, case in enumerate(json.loads(str(T["cases_full_json"]))):
        f.calcTurbineConstants(dict(case), ptfm_pitch=0)
        for k in ("A_aero", "B_aero", "f_aero0", "B_gyro"):
            ref = T["out_" + k][ic]
            x = np.asarray(getattr(f, k))[..., :ref.shape[-1]] if k == "B_gyro" else getattr(f, k)
            scale = max(np.abs(ref).max(), 1e-300)
            assert np.abs(x - ref).max() <= 1e-12 * scale, (ic, k, np.abs(x - ref).max() / scale)
