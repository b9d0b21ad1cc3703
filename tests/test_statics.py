"""Host statics (raft/statics.py) against the reference's own goldens
and against the statics of the reference-generated fixtures.

* Ten single-member designs of the reference's tests/test_member.py: mass/CG/shell/ballast,
  the 6x6 mass matrix, the hydrostatic vector/stiffness/centre of buoyancy/waterplane
  point, at the reference test's tolerances (rtol 1e-5).
* VolturnUS-S and OC3spar of tests/test_fowt.py: rCG, rCG_sub, m_ballast, M_struc,
  M_struc_sub, C_struc, W_struc, rCB, C_hydro, W_hydro (rtol 1e-5, atol 1e-3 as there).
* The designs behind tests/golden/*.npz: M_struc, C_struc, C_hydro, W_struc, W_hydro as the
  reference computed them for the golden runs, to 1e-12.
Fixtures: tests/golden/make_statics_golden.py (reference test data) and make_golden.py.
"""
import json
import os

import numpy as np
import pytest
from numpy.testing import assert_allclose

from conftest import fixture_design, load_design, load_golden

HERE = os.path.dirname(os.path.abspath(__file__))
REF = np.load(os.path.join(HERE, "golden", "statics_ref.npz"))
with open(os.path.join(HERE, "golden", "statics_members.json")) as fh:
    MEMBERS = json.load(fh)


def make_member(i):
    from raft.hydro_math import get_from_dict
    from raft.member import Member
    md = dict(MEMBERS[i]["members"][0])
    heading = get_from_dict(md, "heading", shape=-1, default=0.)
    m = Member(md, 0, heading=heading)
    m.setPosition()
    return m


@pytest.mark.parametrize("i", range(len(MEMBERS)))
def test_member_inertia_matches_reference_goldens(i):
    from raft.statics import member_inertia
    m = make_member(i)
    mass, cg, mshell, mfill, pfill = member_inertia(m)
    assert_allclose([mshell, mfill[0], cg[0], cg[1], cg[2]], REF["member_inertiaBasic"][i], rtol=1e-5, atol=1e-5)
    assert_allclose(m.M_struc, REF["member_inertiaMatrix"][i], rtol=1e-5, atol=0)


@pytest.mark.parametrize("i", range(len(MEMBERS)))
def test_member_hydrostatics_matches_reference_goldens(i):
    from raft.statics import member_hydrostatics
    m = make_member(i)
    F, C, V, rc, AWP, IWP, xWP, yWP = member_hydrostatics(m, rho=1025, g=9.81)
    got = [F[2], F[3], F[4], C[2, 2], C[3, 3], C[4, 4], rc[0], rc[1], rc[2], xWP, yWP]
    assert_allclose(got, REF["member_hydrostatics"][i], rtol=1e-5, atol=1e-5)


def _fowt(design_name, r6=np.zeros(6), w=np.arange(0.05, 1.0, 0.05)):
    from raft.fowt import FOWT
    d = load_design(design_name)
    f = FOWT(d, w, depth=float(d["site"]["water_depth"]))
    f.setPosition(r6)
    f.calcStatics()
    return f


@pytest.mark.parametrize("idx,design", [(0, "VolturnUS-S_test"), (1, "OC3spar_test")])
def test_fowt_statics_matches_reference_goldens(idx, design):
    f = _fowt(design)
    for k in ["rCG", "rCG_sub", "m_ballast", "M_struc", "M_struc_sub", "C_struc", "W_struc", "rCB", "C_hydro",
              "W_hydro"]:
        assert_allclose(getattr(f, k), REF[f"fowt_{k}_{idx}"], rtol=1e-5, atol=1e-3, err_msg=k)


@pytest.mark.parametrize("tag,design", [("c2_nw1000", "VolturnUS-S_example"), ("c1_OC3spar", "OC3spar"),
                                        ("fowt_VolturnUS-S", "VolturnUS-S_test"), ("fowt_OC3spar", "OC3spar_test"),
                                        ("c3_qtf", "OC4semi-RAFT_QTF")])
def test_fowt_statics_match_golden_fixture_runs(tag, design):
    T = load_golden(tag)
    f = _fowt(design, r6=T["r6"] if "r6" in T else np.zeros(6))
    for k in ["M_struc", "C_struc", "C_hydro", "W_struc", "W_hydro"]:
        if k in T:
            ref = T[k]
            assert np.abs(getattr(f, k) - ref).max() <= 1e-12 * max(np.abs(ref).max(), 1.0), k


@pytest.mark.parametrize("tag,design,fi", [("c4_farm", "VolturnUS-S_farm", 0), ("c4_farm", "VolturnUS-S_farm", 1),
                                           ("c5_sweep0", "VolturnUS-S_example", 0),
                                           ("c5_sweep1", "VolturnUS-S_example", 0),
                                           ("c5_sweep2", "VolturnUS-S_example", 0)])
def test_statics_of_farm_and_sweep_variants(tag, design, fi):
    """Each FOWT of the farm (positioned at x = 0 / 1600 m, rotated 180 / 0 deg) and each
    C5 parametersweep variant: the statics the reference computed for those runs, to 1e-12."""
    import raft
    d, T, _ = fixture_design(tag, design, fi)
    m = raft.Model(d)
    f = m.fowtList[fi]
    f.setPosition(T["r6"])
    f.calcStatics()
    for k in ["M_struc", "C_struc", "C_hydro", "W_struc", "W_hydro"]:
        ref = T[k]
        assert np.abs(getattr(f, k) - ref).max() <= 1e-12 * max(np.abs(ref).max(), 1.0), k


def test_member_without_shell_thickness_fails_only_in_statics():
    from raft.member import Member
    from raft.statics import member_inertia
    md = dict(MEMBERS[0]["members"][0])
    md.pop("t")
    m = Member(md, 0)
    m.setPosition()
    with pytest.raises(TypeError):
        member_inertia(m)
