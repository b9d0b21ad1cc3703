"""GPU parity of the potSecOrder=2 path: an external WAMIT .12d QTF (the reference's
examples/OC4semi-WAMIT_Coefs/marin_semi.12d, carried as a numeric table in
tests/golden/qtf12d.npz) read on the host and applied by rh_force_2nd inside the drag loop
(raft/raft_model.py:903-904) and for a second sea state (:1059-1061), against the
reference's own solveDynamics on OC4semi-RAFT_QTF (strip-theory first order, nw = 100).
Tolerance (north_star): 1e-9 relative, identical drag-iteration counts."""
import json

import numpy as np
import pytest

from conftest import load_design, load_golden, statics_of

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


@pytest.fixture(scope="module")
def T():
    return load_golden("qtf12d")


def make(T, stem):
    import raft
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
    return m, f


def test_solve_with_file_qtf_matches_reference(T, tmp_path):
    cases = json.loads(str(T["cases_json"]))
    for ic, case in enumerate(cases):
        m, f = make(T, str(tmp_path / f"q{ic}"))
        np.testing.assert_array_equal(f.qtf, T["qtf"])
        Xi = m.solveDynamics(dict(case))
        nW = f.nWaves
        assert f.iterations == int(T["out_iters"][ic]), (ic, f.iterations, T["out_iters"][ic])
        assert rel(Xi, T["out_Xi"][ic][:nW + 1]) < RTOL, (ic, rel(Xi, T["out_Xi"][ic][:nW + 1]))
        for ih in range(nW):
            ref = T["out_Fhydro_2nd"][ic][ih]
            assert rel(f.Fhydro_2nd[ih], ref) < RTOL, (ic, ih, rel(f.Fhydro_2nd[ih], ref))
            np.testing.assert_allclose(f.Fhydro_2nd_mean[ih], T["out_Fhydro_2nd_mean"][ic][ih], rtol=RTOL,
                                       atol=RTOL * np.abs(T["out_Fhydro_2nd_mean"][ic][ih]).max())
        assert rel(f.B_hydro_drag, T["out_B_drag"][ic]) < RTOL


def test_force_spectrum_from_file_qtf(T, tmp_path):
    """calcHydroForce_2ndOrd alone on the reference's sea state of case 0."""
    m, f = make(T, str(tmp_path / "q"))
    case = json.loads(str(T["cases_json"]))[0]
    f.calcHydroExcitation(dict(case), memberList=f.memberList)
    fm, fd = f.calcHydroForce_2ndOrd(f.beta[0], T["out_S"][0][0])
    assert rel(fd, T["out_Fhydro_2nd"][0][0].real) < RTOL
    np.testing.assert_allclose(fm, T["out_Fhydro_2nd_mean"][0][0], rtol=RTOL,
                               atol=RTOL * np.abs(T["out_Fhydro_2nd_mean"][0][0]).max())


@pytest.mark.parametrize("tag", ["q12_b0", "q12_s1"])
def test_force_spectrum_mode_from_file_qtf(T, tmp_path, tag):
    """interpMode='spectrum' on the .12d QTF against the reference method (f2nd_spectrum.npz)."""
    G = load_golden("f2nd_spectrum")
    m, f = make(T, str(tmp_path / "q"))
    case = json.loads(str(T["cases_json"]))[0]
    f.calcHydroExcitation(dict(case), memberList=f.memberList)
    fm, fd = f.calcHydroForce_2ndOrd(0.0, G[f"{tag}_S0"], interpMode="spectrum")
    assert rel(fd, G[f"{tag}_f"]) < RTOL, rel(fd, G[f"{tag}_f"])
    np.testing.assert_allclose(fm, G[f"{tag}_fmean"], rtol=RTOL, atol=RTOL * np.abs(G[f"{tag}_fmean"]).max())
