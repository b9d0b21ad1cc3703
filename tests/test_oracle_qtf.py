"""CPU: pin the QTF oracle (oracle/qtf_oracle.py) against the reference's own outputs
(tests/golden/c3_qtf.npz: OC4semi-RAFT_QTF, potSecOrder=1, run in the build container)."""
import json

import numpy as np
import pytest

from conftest import load_golden
from oracle import qtf_oracle as Q
from oracle import raft_oracle as O


@pytest.fixture(scope="module")
def T():
    return load_golden("c3_qtf")


def _rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def test_oracle_qtf_n42_matches_reference(T):
    q = Q.qtf_slender(T, T["out_Xi0"], T["w1_2nd"], T["k1_2nd"], 0.0)[:, :, 0, :]
    ref = T["out_qtf"][:, :, 0, :]
    assert _rel(q, ref) < 1e-12
    big = np.abs(ref).max()
    np.testing.assert_allclose(q, ref, rtol=1e-11, atol=1e-13 * big)


@pytest.mark.parametrize("key,beta", [("sub400_qtf", 0.0), ("sub400_beta30_qtf", None)])
def test_oracle_qtf_fine_grid_entries(T, key, beta):
    """Entries of the n2=400 grid (df 0.000825 Hz) on a seeded 24-frequency subset, head-on
    and at 30 deg (the degree/radian quirk Q1 of the wave helpers)."""
    b = float(T["sub400_beta30"]) if beta is None else beta
    q = Q.qtf_slender(T, T["out_Xi0"], T["sub400_w"], T["sub400_k"], b)
    assert _rel(q, T[key]) < 1e-12


def test_oracle_qtf_lower_triangle_is_hermitian_fill(T):
    q = Q.qtf_slender(T, T["out_Xi0"], T["w1_2nd"], T["k1_2nd"], 0.0)[:, :, 0, :]
    i, j = np.tril_indices(len(T["w1_2nd"]), -1)
    np.testing.assert_array_equal(q[i, j], np.conj(q[j, i]))


def test_oracle_force_2nd_matches_reference(T):
    fm, f = Q.hydro_force_2nd(T["out_qtf"], T["w1_2nd"], T["w"], T["out_S"][0], float(T["dw"]))
    np.testing.assert_allclose(fm, T["out_Fhydro_2nd_mean"][0], rtol=1e-12, atol=1e-12 * np.abs(fm).max())
    assert _rel(f, T["out_Fhydro_2nd"][0].real) < 1e-12
    assert np.all(T["out_Fhydro_2nd"][0].imag == 0) and np.all(f[:, -1] == 0)


def test_oracle_second_order_solve_matches_reference(T):
    """Full potSecOrder=1 path: first convergence -> RAO -> QTF -> force -> second pass."""
    case = {k: v[0] for k, v in json.loads(str(T["cases_json"]))[0].items()}
    r = O.solve_dynamics(T, case, int(T["nIter"]), float(T["XiStart"]),
                         second_order=dict(w1_2nd=T["w1_2nd"], k1_2nd=T["k1_2nd"]))
    assert list(r["iters_pair"]) == list(T["out_iters_pair"])
    assert _rel(r["Xi"], T["out_Xi"]) < 1e-12
    assert _rel(r["Xi0"], T["out_Xi0"]) < 1e-12


@pytest.mark.parametrize("tag", ["c3", "q12_b0", "q12_s1"])
def test_oracle_force_2nd_spectrum_matches_reference(tag):
    """interpMode='spectrum' (raft/raft_fowt.py:1760-1784) against the reference method run on
    the fixture QTFs (tests/golden/f2nd_spectrum.npz, make_golden.py golden_f2nd_spectrum)."""
    G = load_golden("f2nd_spectrum")
    src = load_golden("c3_qtf") if tag == "c3" else load_golden("qtf12d")
    qtf = src["out_qtf"] if tag == "c3" else src["qtf"]
    fm, f = Q.hydro_force_2nd_spectrum(qtf, src["w1_2nd"], src["w"], G[f"{tag}_S0"], float(src["dw"]))
    np.testing.assert_allclose(fm, G[f"{tag}_fmean"], rtol=1e-12, atol=1e-12 * np.abs(fm).max())
    assert G[f"{tag}_f"].dtype == complex and f.dtype == complex
    assert _rel(f, G[f"{tag}_f"]) < 1e-12
