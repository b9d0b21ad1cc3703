"""CPU: the CCBlade restatement (raft/ccblade.py) on the reference's IEA-15MW rotor.

What pins it to the reference is in tests/test_mooring.py: the wind and wind-wave-current mean
offsets and the loaded natural frequencies of the reference's tests/test_model.py, which depend
on every mean rotor load (thrust, torque, side forces, hub moments).  These tests check the
solver's own consistency: the BEM residual at the solution, the derivatives RAFT consumes
against re-solved finite differences, and the symmetric-inflow limit."""
import numpy as np
import pytest

from conftest import load_design

CASE = {"wind_speed": 8, "wind_heading": 30, "turbulence": 0, "turbine_status": "operating", "yaw_misalign": 0,
        "wave_spectrum": "JONSWAP", "wave_period": 0, "wave_height": 0, "wave_heading": 0,
        "current_speed": 0, "current_heading": 0}


@pytest.fixture(scope="module")
def rotor():
    import raft
    m = raft.Model(load_design("VolturnUS-S_aero"))
    f = m.fowtList[0]
    f.setPosition(np.zeros(6))
    f.calcTurbineConstants(dict(CASE), ptfm_pitch=0)
    return f.rnaList[0]


def test_restatement_is_used_without_the_package(rotor):
    from raft import ccblade
    assert isinstance(rotor.ccblade, ccblade.CCBlade)
    assert rotor.ccblade.nSector == 4          # tilt and shear: at least 4 sectors


def test_bem_residual_vanishes_at_the_solution(rotor):
    cc = rotor.ccblade
    U, Om, pit = rotor.U_case, rotor.Omega_case, rotor.pitch_case
    for az in (0.0, 90.0, 180.0, 270.0):
        out, _ = cc.distributedAeroLoads(U, Om, pit, az)
        for i in range(len(cc.r)):
            args = (cc.r[i], cc.chord[i], cc.theta[i], cc.af[i], cc._Vx[i], cc._Vy[i])
            f = cc._errf(out["phi"][i], *args)
            assert abs(f) < 1e-9, (az, i, f)
        assert np.all(np.isfinite(out["Np"])) and np.all(out["Np"] > 0)


def test_derivatives_match_resolved_differences(rotor):
    """dT and dQ with respect to Uinf, Omega and pitch (raft/raft_rotor.py:826-832) against
    central differences of complete re-solves."""
    cc = rotor.ccblade
    x0 = np.array([rotor.U_case, rotor.Omega_case, rotor.pitch_case])
    loads, d = cc.evaluate([x0[0]], [x0[1]], [x0[2]])
    for k, name in enumerate(("dUinf", "dOmega", "dpitch")):
        h = 1e-4 * max(1.0, abs(x0[k]))
        xp, xm = x0.copy(), x0.copy()
        xp[k] += h
        xm[k] -= h
        lp, _ = cc.evaluate([xp[0]], [xp[1]], [xp[2]])
        lm, _ = cc.evaluate([xm[0]], [xm[1]], [xm[2]])
        for q in ("T", "Q"):
            fd = (lp[q][0] - lm[q][0]) / (2 * h)
            an = np.diag(d["d" + q][name])[0]
            assert abs(an - fd) <= 2e-4 * abs(fd) + 1e-6 * abs(loads[q][0]), (q, name, an, fd)


def test_axisymmetric_inflow_has_no_side_loads(rotor):
    """No tilt, yaw or shear: one sector, and the in-plane forces and hub moments vanish."""
    from raft.ccblade import CCBlade
    cc = rotor.ccblade
    sym = CCBlade(cc.r, cc.chord, np.degrees(cc.theta), cc.af, cc.Rhub, cc.Rtip, cc.B, cc.rho, cc.mu,
                  np.degrees(cc.precone), 0.0, 0.0, 0.0, cc.hubHt, 4, cc.precurve, cc.precurveTip,
                  cc.presweep, cc.presweepTip)
    assert sym.nSector == 1
    loads, _ = sym.evaluate([rotor.U_case], [rotor.Omega_case], [rotor.pitch_case])
    T = loads["T"][0]
    assert T > 0
    for k in ("Y", "Z", "My", "Mz"):
        assert abs(loads[k][0]) < 1e-12 * T * cc.Rtip, (k, loads[k][0])
