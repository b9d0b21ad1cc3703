"""CPU: the product's per-design preparation (member discretisation, pose, hydrodynamic
constants, node tables) reproduces the reference's tables exactly."""
import numpy as np
import pytest

from conftest import fixture_design, load_golden

# (fixture, design, settings, FOWT index); c4_farm: the two FOWTs of the farm (x = 0 and
# 1600 m, heading_adjust 180 and 0), c5_sweep*: parametersweep variants (raft/sweep.py)
CASES = [("fowt_VolturnUS-S", "VolturnUS-S_test", {}, 0), ("fowt_OC3spar", "OC3spar_test", {}, 0),
         ("c2_nw200", "VolturnUS-S_example", {}, 0), ("c1_OC3spar", "OC3spar", {}, 0),
         ("c2_nw1000", "VolturnUS-S_example", {"min_freq": 0.0002}, 0),
         ("c4_farm", "VolturnUS-S_farm", {}, 0), ("c4_farm", "VolturnUS-S_farm", {}, 1),
         ("c5_sweep0", "VolturnUS-S_example", {"min_freq": 0.0002}, 0),
         ("c5_sweep1", "VolturnUS-S_example", {"min_freq": 0.0002}, 0),
         ("c5_sweep2", "VolturnUS-S_example", {"min_freq": 0.0002}, 0)]
ARGS = "tag,design,settings,fi"


def _model(tag, design_name, settings, fi):
    import raft
    d, T, _ = fixture_design(tag, design_name, fi)
    d["settings"].update(settings)
    m = raft.Model(d)
    f = m.fowtList[fi]
    f.setPosition(T["r6"])
    f.calcHydroConstants()
    return m, f, T


@pytest.mark.parametrize(ARGS, CASES)
def test_grid_and_wave_numbers(tag, design, settings, fi):
    m, f, T = _model(tag, design, settings, fi)
    np.testing.assert_array_equal(m.w, T["w"])
    np.testing.assert_array_equal(f.k, T["k"])          # vectorised waveNumber is bit-identical
    assert f.dw == T["dw"]


@pytest.mark.parametrize(ARGS, CASES)
def test_node_tables_match_reference(tag, design, settings, fi):
    from raft import _native as N
    from raft.prep import node_table
    m, f, T = _model(tag, design, settings, fi)
    assert sum(mm.ns for mm in f.memberList) == len(T["node_sub"])
    tab, imat, _, _ = node_table(f)
    sub = T["node_sub"].astype(bool)
    assert tab.shape == (N.NF_COUNT, sub.sum())
    ref = {"RX": T["node_r"][sub, 0], "RY": T["node_r"][sub, 1], "RZ": T["node_r"][sub, 2],
           "XX": T["node_r_rel"][sub, 0], "XY": T["node_r_rel"][sub, 1], "XZ": T["node_r_rel"][sub, 2],
           "QX": T["node_q"][sub, 0], "QY": T["node_q"][sub, 1], "QZ": T["node_q"][sub, 2],
           "P1X": T["node_p1"][sub, 0], "P1Y": T["node_p1"][sub, 1], "P1Z": T["node_p1"][sub, 2],
           "P2X": T["node_p2"][sub, 0], "P2Y": T["node_p2"][sub, 1], "P2Z": T["node_p2"][sub, 2],
           "CDQ": T["node_Cd_q"][sub], "CDP1": T["node_Cd_p1"][sub], "CDP2": T["node_Cd_p2"][sub],
           "CDEND": T["node_Cd_End"][sub], "AI": T["node_a_i"][sub], "CIRC": T["node_circ"][sub]}
    for k, v in ref.items():
        np.testing.assert_array_equal(tab[N.NF[k]], v, err_msg=k)
    np.testing.assert_array_equal(tab[N.NF["I00"]:N.NF["I22"] + 1], T["node_Imat"][sub].reshape(-1, 9).T)


@pytest.mark.parametrize(ARGS, CASES)
def test_added_mass_matches_reference(tag, design, settings, fi):
    m, f, T = _model(tag, design, settings, fi)
    np.testing.assert_array_equal(f.A_hydro_morison, T["A_hydro_morison"])


def test_drag_areas_follow_reference_formulas():
    """Rectangular axial area uses ds[0] twice; end areas are |.|."""
    from raft import _native as N
    from raft.prep import node_table
    m, f, T = _model("c2_nw200", "VolturnUS-S_example", {}, 0)
    tab, _, _, _ = node_table(f)
    sub = T["node_sub"].astype(bool)
    ds, dls, drs, circ = T["node_ds"][sub], T["node_dls"][sub], T["node_drs"][sub], T["node_circ"][sub].astype(bool)
    aq = np.where(circ, np.pi * ds[:, 0] * dls, 2 * (ds[:, 0] + ds[:, 0]) * dls)
    np.testing.assert_array_equal(tab[N.NF["AQ"]], aq)
    assert np.all(tab[N.NF["AEND"]] >= 0)


def test_get_from_dict_index_rule():
    from raft.hydro_math import get_from_dict
    d = {"Cd": [1.5, 2.2]}
    np.testing.assert_array_equal(get_from_dict(d, "Cd", shape=2, default=0.6, index=0), [1.5, 1.5])
    np.testing.assert_array_equal(get_from_dict(d, "Cd", shape=2, default=0.6, index=1), [2.2, 2.2])
    np.testing.assert_array_equal(get_from_dict({}, "Cd", shape=3, default=0.6, index=1), [0.6, 0.6, 0.6])
    with pytest.raises(ValueError):
        get_from_dict({"Cd": [1, 2, 3]}, "Cd", shape=2)


def test_wave_number_vectorised_equals_scalar_iteration():
    from oracle import raft_oracle as O
    from raft.hydro_math import wave_numbers
    w = np.linspace(0.001, 3.0, 777)
    for h in [20.0, 200.0, 1000.0]:
        np.testing.assert_array_equal(wave_numbers(w, h), [O.wave_number(x, h) for x in w])
