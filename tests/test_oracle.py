"""CPU: pin the oracle (oracle/raft_oracle.py) against the reference's own outputs.

Golden vectors come from running the reference in the build container
(tests/golden/make_golden.py); the helper known-answer values are the literal expected
values of the reference's tests/test_helpers.py (numbers only).
"""
import numpy as np
import pytest

from conftest import farm_tables, golden_cases, load_golden
from oracle import raft_oracle as O

SOLVE_TAGS = ["c1_OC3spar", "c2_nw200", "multi_heading", "c2_nw1000", "c5_sweep0", "c5_sweep1", "c5_sweep2"]


@pytest.mark.parametrize("tag", SOLVE_TAGS)
def test_oracle_solve_dynamics_matches_reference(tag):
    T = load_golden(tag)
    for ic, case in enumerate(golden_cases(T)):
        r = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
        ref = T["out_Xi"][ic]
        assert r["iters"] == T["out_iters"][ic]
        assert int(r["converged"]) == T["out_conv"][ic]
        assert np.linalg.norm(r["Xi"] - ref) <= 1e-12 * np.linalg.norm(ref)
        np.testing.assert_allclose(r["B_drag"], T["out_B_drag"][ic], rtol=1e-12, atol=1e-12 * np.abs(r["B_drag"]).max())
        mo = O.motion_outputs(r["Xi"], float(T["dw"]))
        dofs = ["surge", "sway", "heave", "roll", "pitch", "yaw"]
        smax = max(T[f"out_{d}_std"][ic] for d in dofs)           # scale: largest DOF response
        pmax = max(T[f"out_{d}_PSD"][ic].max() for d in dofs)
        for dof in dofs:
            np.testing.assert_allclose(mo[dof + "_std"], T[f"out_{dof}_std"][ic], rtol=1e-12, atol=1e-12 * smax)
            np.testing.assert_allclose(mo[dof + "_PSD"], T[f"out_{dof}_PSD"][ic], rtol=1e-11, atol=1e-12 * pmax)


ROTOR_TAGS = ["c1_OC3spar", "c2_nw200", "multi_heading", "c2_nw1000"]


def rotor_dict(T):
    return {k[4:]: T[k] for k in T if k.startswith("rot_")}


@pytest.mark.parametrize("tag", ROTOR_TAGS)
def test_oracle_rotor_channels_match_reference(tag):
    """AxRNA_* / Mbase_* of saveTurbineOutputs (raft/raft_fowt.py:1900-1970) from the
    reference's own Xi and rotor statics."""
    T = load_golden(tag)
    if "out_AxRNA_std" not in T:
        pytest.skip("fixture predates the rotor channels (regenerate with make_golden.py)")
    for ic in range(len(T["out_Xi"])):
        r = O.rotor_outputs(T["out_Xi"][ic], T["w"], float(T["dw"]), rotor_dict(T), Xi0_pitch=T["r6"][4],
                            g=float(T["g"]))
        for ch in ["AxRNA", "Mbase"]:
            for st in ["avg", "std", "max", "min", "PSD"]:
                ref = T[f"out_{ch}_{st}"][ic]
                np.testing.assert_allclose(r[f"{ch}_{st}"], ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_oracle_farm_matches_reference():
    """C4: two coupled FOWTs (tests/test_data/VolturnUS-S_farm.yaml) with the array
    stiffness fixture: per-FOWT iteration counts, the 12-DOF system response, B_drag."""
    T = load_golden("c4_farm")
    Ts = farm_tables(T)
    assert len(Ts) == 2
    for ic, case in enumerate(golden_cases(T)):
        r = O.solve_farm(Ts, dict(case), int(T["nIter"]), T["K_array"], float(T["XiStart"]))
        assert r["iters"] == list(T["out_iters"][ic])
        ref = T["out_Xi"][ic]
        assert np.linalg.norm(r["Xi"] - ref) <= 1e-12 * np.linalg.norm(ref)
        for i, f in enumerate(r["fowts"]):
            Bref = T["out_B_drag"][ic][i]
            np.testing.assert_allclose(f["B_drag"], Bref, rtol=1e-12, atol=1e-12 * np.abs(Bref).max())
        # the shared line couples the bodies: FOWT 1 moves under FOWT 0's excitation alone
        assert np.abs(ref[0, 6:]).max() > 0


@pytest.mark.parametrize("tag", ["fowt_VolturnUS-S", "fowt_OC3spar"])
def test_oracle_excitation_matches_reference(tag):
    """F_hydro_iner for the 72 heading/period/height cases of tests/test_fowt.py:214-250."""
    T = load_golden(tag)
    nodes = O.Nodes(T)
    for (hd, tp, hs), Fref in zip(T["exc_cases"], T["exc_F_iner"]):
        case = {"wave_heading": hd, "wave_period": tp, "wave_height": hs}
        beta, S, zeta = O.sea_state(case, T["w"], float(T["dw"]))
        _, _, _, F = O.hydro_excitation(T, nodes, beta, zeta)
        assert np.linalg.norm(F - Fref) <= 1e-12 * np.linalg.norm(Fref)


@pytest.mark.parametrize("tag", ["fowt_VolturnUS-S", "fowt_OC3spar"])
def test_oracle_linearization_matches_reference(tag):
    """B_hydro_drag / F_hydro_drag for tests/test_fowt.py:252-277's synthetic Xi."""
    T = load_golden(tag)
    nodes = O.Nodes(T)
    beta, S, zeta = O.sea_state({"wave_spectrum": "unit", "wave_heading": 0, "wave_period": 10, "wave_height": 2},
                                T["w"], float(T["dw"]))
    u, _, _, _ = O.hydro_excitation(T, nodes, beta, zeta)
    B, Bmat, F = O.hydro_linearization(T, nodes, T["lin_Xi"], u[0])
    np.testing.assert_allclose(B, T["lin_B_drag"], rtol=1e-12, atol=1e-12 * np.abs(B).max())
    assert np.linalg.norm(F - T["lin_F_drag"]) <= 1e-12 * np.linalg.norm(T["lin_F_drag"])
    F2 = O.drag_excitation(nodes, Bmat, u[0])
    assert np.linalg.norm(F2 - T["lin_F_drag"]) <= 1e-12 * np.linalg.norm(T["lin_F_drag"])


def test_oracle_loop_flavour_equals_vectorised():
    """The reference-structured loop flavour (CPU baseline) computes the same numbers."""
    T = load_golden("c1_OC3spar")
    case = golden_cases(T)[0]
    a = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]))
    b = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]), loop=True)
    assert a["iters"] == b["iters"]
    assert np.linalg.norm(a["Xi"] - b["Xi"]) <= 1e-12 * np.linalg.norm(a["Xi"])


# ---- known-answer values of the reference's tests/test_helpers.py ---------------------
def test_kat_wave_number():
    w = np.array([0.1, 0.25, 0.5, 0.75])
    k = np.array([O.wave_number(x, 200) for x in w])
    np.testing.assert_allclose(k, [0.00233623, 0.0071452, 0.02548611, 0.05733945], rtol=1e-5)


def test_kat_wave_kinematics():
    w = np.array([0.1, 0.25, 0.5, 0.75])
    k = np.array([O.wave_number(x, 200) for x in w])
    u, ud, pd = O.wave_kin(np.full(4, 0.2), 30, w, k, 200, [30, 45, -20])
    u_ref = np.array([[0.0069097100 + 0.0006448900j, 0.0073269700 + 0.0021436100j, 0.0048875900 + 0.0078728400j,
                       -0.0048089800 + 0.0055581900j],
                      [-0.0442590100 - 0.0041307200j, -0.0469316700 - 0.0137305200j, -0.0313066500 - 0.0504281200j,
                       0.0308031300 - 0.0356020400j],
                      [-0.0016613100 + 0.0178002300j, -0.0119250300 + 0.0407604200j, -0.0510284000 + 0.0316793100j,
                       -0.0360333000 - 0.0311762500j]])
    p_ref = np.array([1963.730340920 + 183.276331860j, 1703.156386190 + 498.282218140j,
                      637.171137130 + 1026.342526750j, -417.980049950 + 483.098446900j])
    np.testing.assert_allclose(u, u_ref, rtol=1e-5)
    np.testing.assert_allclose(ud, 1j * w * u_ref, rtol=1e-5)
    np.testing.assert_allclose(pd, p_ref, rtol=1e-5)


def test_kat_kinematics():
    r = [2, 2, 2]
    w = np.array([0.5, 0.75])
    Xi = np.array([[1, 2 + 1j], [0.1 + 0.2j, 0.3 + 0.4j], [0.5 + 0.6j, 0.7 + 0.8j], [0.9 + 1.0j, 1.1 + 1.2j],
                   [1.3 + 1.4j, 1.5 + 1.6j], [1.7 + 1.8j, 1.9 + 2.0j]])
    dr, v, a = O.kinematics(r, Xi, w)
    np.testing.assert_allclose(dr, [[0.2 - 0.8j, 1.2 + 0.2j], [1.7 + 1.8j, 1.9 + 2.0j], [-0.3 - 0.2j, -0.1 + 0j]],
                               rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(v, [[0.4 + 0.1j, -0.15 + 0.9j], [-0.9 + 0.85j, -1.5 + 1.425j], [0.1 - 0.15j, -0.075j]],
                               rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(a, [[-0.05 + 0.2j, -0.675 - 0.1125j], [-0.425 - 0.45j, -1.06875 - 1.125j],
                                   [0.075 + 0.05j, 0.05625 + 0j]], rtol=1e-5, atol=1e-12)


def test_kat_small_rotate_and_translate():
    th = np.array([5 + 3j, 3 + 5j, 4 + 3j]) * O.DEG2RAD   # helpers.deg2rad is a plain multiply
    rt = O.small_rotate([1, 2, 3], th)
    np.testing.assert_allclose(rt, [0.01745329 + 0.15707963j, -0.19198622 - 0.10471976j, 0.12217305 + 0.01745329j],
                               rtol=1e-5)
    F = O.translate_force_3to6(np.array([1.0, 2.0, 3.0]), np.array([4.0, 5.0, 6.0]))
    np.testing.assert_allclose(F, [1, 2, 3, 3, -6, 3])
    M = O.translate_matrix_3to6(np.eye(3), np.array([1.0, 2.0, 3.0]))
    np.testing.assert_allclose(M, M.T)
    np.testing.assert_allclose(M[3:, 3:], O.get_h([1, 2, 3]) @ O.get_h([1, 2, 3]).T)


def test_kat_jonswap_auto_gamma_branches():
    w = np.linspace(0.05, 2.0, 50)
    for hs, tp in [(6, 8), (2, 12), (9, 12)]:             # Tp/sqrt(Hs) <= 3.6, >= 5, between
        S = O.jonswap(w, hs, tp, 0)
        m0 = np.trapezoid(S, w) if hasattr(np, "trapezoid") else np.trapz(S, w)
        assert 0.5 < 4 * np.sqrt(m0) / hs < 1.1


@pytest.mark.parametrize("tag", ["c2_nw1000", "c2_nw200", "c1_OC3spar"])
def test_iteration0_sums_separable_form(tag):
    """The algebra of k_solve_lds's iteration-0 shortcut (csrc/rh_a0.hip), on the reference's
    own node tables and sea states: with XiLast = XiStart in every DOF and bin, the node's
    motion displacement dr is real and bin-independent, so per projection e (q, p1, p2)
        sum_b |e.(u_b - i w_b dr)|^2 = sum z^2 |e.u^|^2 - 2 (e.dr) sum z w Im(e.u^) + (e.dr)^2 sum w^2
    (u = z u^, u^ the unit-amplitude kinematics that kproj tabulates).  The direct and the
    separable sums agree to rounding on every node and projection: the expansion cancels
    nothing that matters at the RTOL of the parity tests."""
    T = load_golden(tag)
    nodes = O.Nodes(T)
    w = T["w"]
    xs = float(T["XiStart"]) or 0.1
    cases = list(golden_cases(T))[:2] + [dict(wave_heading=h, wave_period=p, wave_height=hh, wave_spectrum="JONSWAP")
                                        for h, p, hh in [(0, 6.0, 1.0), (60, 17.5, 9.5)]]
    worst = 0.0
    for case in cases:
        beta, S, zeta = O.sea_state(case, w, float(T["dw"]))
        u, _, _, _ = O.hydro_excitation(T, nodes, beta[:1], zeta[:1])
        z = zeta[0].real
        Xi = np.full([6, len(w)], xs, dtype=complex)
        for j in range(nodes.n):
            dr, _, _ = O.kinematics(nodes.r_rel[j], Xi, w)
            vrel = u[0, j] - 1j * w * dr
            uhat = np.divide(u[0, j], z, out=np.zeros_like(u[0, j]), where=z > 0)
            for e in (nodes.q[j], nodes.p1[j], nodes.p2[j]):
                direct = np.sum(np.abs(e @ vrel) ** 2)
                K = e @ uhat
                b = float(np.real(e @ dr[:, 0]))
                sep = np.sum(z * z * np.abs(K) ** 2) - 2 * b * np.sum(z * w * K.imag) + b * b * np.sum(w * w)
                worst = max(worst, abs(sep - direct) / direct)
    print(f"{tag}: worst relative difference {worst:.2e}")
    assert worst < 1e-12, worst
