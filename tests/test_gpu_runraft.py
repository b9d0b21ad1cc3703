"""GPU: the top-level entry points runRAFT / runRAFTFarm (raft/raft_model.py:2024-2095) with
the mooring restatement in the loop: unloaded equilibrium, per-case mean offsets, the device
response solve and every output channel including the mooring tensions.

No reference run covers these (MoorPy is absent, so the reference's analyzeCases pickles
cannot be regenerated, and its safe loader refuses them): the response is checked against
the CPU oracle on the SAME offset design tables (conftest.oracle_tables_of), the Tmoor
channels against a host evaluation of J_moor Xi, and the result-dict keys against what the
reference writes and the WEIS caller reads (raft/omdao_raft.py:767-801)."""
import numpy as np
import pytest

from conftest import load_design, oracle_tables_of
from oracle import raft_oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def wind0(d):
    j = d["cases"]["keys"].index("wind_speed")
    for row in d["cases"]["data"]:
        row[j] = 0          # rotor aerodynamics (CCBlade) are outside the accelerated path
    return d


def last_case(d):
    c = dict(zip(d["cases"]["keys"], d["cases"]["data"][-1]))
    return c


@pytest.mark.parametrize("name", ["OC3spar", "VolturnUS-S_example"])
def test_run_raft_single(name):
    import raft
    d = wind0(load_design(name))
    m = raft.runRAFT(d)
    res = m.results
    P = res["properties"]          # (analyzeCases resets it after analyzeUnloaded, as the reference does)
    for k in ["tower mass", "substructure mass", "total mass", "C system", "C_lines0",
              "F_lines0", "M support structure", "buoyancy (pgV)"]:
        assert k in P, k
    assert len(res["mean_offsets"]) == len(d["cases"]["data"])
    f = m.fowtList[0]
    for ic in range(len(d["cases"]["data"])):
        cm = res["case_metrics"][ic][0]
        for n in ["surge", "sway", "heave", "roll", "pitch", "yaw", "AxRNA", "Mbase", "Tmoor"]:
            for st in ["avg", "std", "max", "PSD"]:
                assert f"{n}_{st}" in cm, (n, st)
        assert cm["Tmoor_PSD"].shape == (2 * len(f.ms.lines), m.nw)
        assert np.all(cm["Tmoor_avg"] > 0)
    # the last case: device response == oracle on the same offset tables and mooring stiffness
    case = last_case(d)
    T = oracle_tables_of(f)
    r = O.solve_dynamics(T, dict(case), int(m.nIter), float(m.XiStart))
    assert f.iterations == r["iters"]
    assert rel(f.Xi, r["Xi"]) < RTOL
    cm = res["case_metrics"][len(d["cases"]["data"]) - 1][0]
    mo = O.motion_outputs(r["Xi"], float(T["dw"]))
    np.testing.assert_allclose(cm["pitch_std"], mo["pitch_std"], rtol=RTOL)
    # mooring tensions: PSD of J_moor Xi with the reference's w[0] divisor
    _, J = f.ms.coupled_stiffness_fd(tensions=True)
    amps = np.einsum("td,hdw->htw", J, f.Xi)
    psd = np.sum(0.5 * np.abs(amps) ** 2 / m.w[0], axis=0)
    np.testing.assert_allclose(cm["Tmoor_PSD"], psd, rtol=RTOL, atol=RTOL * psd.max())
    np.testing.assert_allclose(cm["Tmoor_std"], np.sqrt(0.5 * np.sum(np.abs(amps) ** 2, axis=(0, 2))), rtol=RTOL)
    np.testing.assert_allclose(cm["Tmoor_avg"], f.ms.tensions(), rtol=1e-12)
    # eigen analysis at the last offset (host), as the WEIS caller runs after calcOutputs
    fns, modes = m.solveEigen()
    assert np.all(fns > 0) and len(fns) == 6


def test_run_raft_farm():
    """Two coupled FOWTs with the shared array mooring (free clump-weight points)."""
    import raft
    d = wind0(load_design("VolturnUS-S_farm"))
    m = raft.runRAFTFarm(d)
    cm = m.results["case_metrics"][0]
    assert set(cm) >= {0, 1, "array_mooring"}
    am = cm["array_mooring"]
    nl = len(m.ms.lines)
    assert am["Tmoor_PSD"].shape == (2 * nl, m.nw) and np.all(am["Tmoor_avg"] > 0)
    Ts = [oracle_tables_of(f) for f in m.fowtList]
    case = last_case(d)
    r = O.solve_farm(Ts, dict(case), int(m.nIter), m.ms.coupled_stiffness_analytic(), float(m.XiStart))
    assert [f.iterations for f in m.fowtList] == r["iters"]
    assert rel(m.Xi, r["Xi"]) < RTOL
    _, J = m.ms.coupled_stiffness_fd(tensions=True)
    amps = np.einsum("td,hdw->htw", J, m.Xi)
    psd = np.sum(0.5 * np.abs(amps) ** 2 / m.w[0], axis=0)
    np.testing.assert_allclose(am["Tmoor_PSD"], psd, rtol=RTOL, atol=RTOL * psd.max())
