"""GPU parity of the slender-body QTF path (rh_qtf_slender / rh_force_2nd through the C-ABI)
against the reference's golden vectors (tests/golden/c3_qtf.npz: OC4semi-RAFT_QTF).

Tolerance (north_star): FP64, 1e-9 relative (normwise) and identical drag-iteration
counts of both passes of the potSecOrder=1 solve.  Full size (n2 = 400, 80,200 pairs):
the 24-frequency subset the reference evaluated must equal the matching rows/columns of
the full 400x400 device QTF (per-frequency tables depend on the frequency only)."""
import json

import numpy as np
import pytest

from conftest import load_design, load_golden, statics_of

pytestmark = pytest.mark.gpu
RTOL = 1e-9


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.fixture(scope="module")
def T():
    return load_golden("c3_qtf")


def _case(T):
    c = {k: v[0] for k, v in json.loads(str(T["cases_json"]))[0].items()}
    c["wind_speed"] = 0
    return c


def make(T, out_folder=None):
    import raft
    d = load_design("OC4semi-RAFT_QTF")
    d["platform"]["outFolderQTF"] = out_folder
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    return m, f


def test_second_order_grid_matches_reference(T):
    m, f = make(T)
    np.testing.assert_array_equal(f.w1_2nd, T["w1_2nd"])
    np.testing.assert_array_equal(f.k1_2nd, T["k1_2nd"])


def test_qtf_matches_reference(T):
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    ref = T["out_qtf"]
    assert f.qtf.shape == ref.shape
    assert rel(f.qtf, ref) < RTOL, rel(f.qtf, ref)
    np.testing.assert_allclose(f.qtf, ref, rtol=RTOL, atol=RTOL * np.abs(ref).max())
    fm, fd = f.calcHydroForce_2ndOrd(f.beta[0], T["out_S"][0])
    np.testing.assert_allclose(fm, T["out_Fhydro_2nd_mean"][0], rtol=RTOL, atol=RTOL * np.abs(fm).max())
    assert rel(fd, T["out_Fhydro_2nd"][0].real) < RTOL
    assert np.all(fd[:, -1] == 0)


@pytest.mark.parametrize("key", ["sub400_qtf", "sub400_beta30_qtf"])
def test_qtf_fine_grid_subset(T, key):
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.w1_2nd, f.k1_2nd = T["sub400_w"], T["sub400_k"]
    f.w2_2nd, f.k2_2nd = f.w1_2nd.copy(), f.k1_2nd.copy()
    if key == "sub400_beta30_qtf":
        f.beta = np.array([float(T["sub400_beta30"])])
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    assert rel(f.qtf, T[key]) < RTOL, rel(f.qtf, T[key])


def test_qtf_full_size_400_grid(T):
    """C3 at full size: 400 frequencies (80,200 pairs).  The reference's 24-frequency subset
    is a principal submatrix of the full QTF; the full matrix is Hermitian-filled."""
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    from raft.hydro_math import wave_numbers
    w400 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    assert len(w400) == int(T["sub400_n2"])
    f.w1_2nd, f.k1_2nd = w400, wave_numbers(w400, f.depth)
    np.testing.assert_array_equal(f.k1_2nd[T["sub400_idx"]], T["sub400_k"])
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    idx = T["sub400_idx"]
    sub = f.qtf[np.ix_(idx, idx)]
    assert rel(sub, T["sub400_qtf"]) < RTOL
    q = f.qtf[:, :, 0, :]
    i, j = np.tril_indices(len(w400), -1)
    np.testing.assert_array_equal(q[i, j], np.conj(q[j, i]))
    # deterministic
    q1 = f.qtf.copy()
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    np.testing.assert_array_equal(f.qtf, q1)


@pytest.mark.parametrize("beta_deg", [0.0, 30.0])
def test_full_400_grid_random_pairs_vs_oracle(T, beta_deg):
    """The full 400 x 400 device QTF against the oracle (oracle/qtf_oracle.py) on 2,080 seeded
    random (i1 <= i2) pairs: every entry is pointwise in (w1, w2) (per-frequency tables, the RAO
    interpolated per frequency, Kim & Yue per pair), so the oracle evaluated on a random
    64-frequency sub-grid gives the matching principal submatrix of the full result.  1e-9
    normwise and elementwise to 1e-9 of the largest entry, at 0 and 30 degrees (Q1)."""
    from oracle import qtf_oracle as Q
    from raft.hydro_math import wave_numbers
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    w400 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    k400 = wave_numbers(w400, f.depth)
    f.w1_2nd, f.k1_2nd = w400, k400
    f.w2_2nd, f.k2_2nd = w400.copy(), k400.copy()
    beta = np.deg2rad(beta_deg)
    f.beta = np.array([beta])
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    idx = np.sort(np.random.default_rng(2026 + int(beta_deg)).choice(len(w400), 64, replace=False))
    ref = Q.qtf_slender(T, T["out_Xi0"], w400[idx], k400[idx], beta)
    sub = f.qtf[np.ix_(idx, idx)]
    iu, ju = np.triu_indices(len(idx))
    assert len(iu) >= 2000
    assert rel(sub[iu, ju], ref[iu, ju]) < RTOL, rel(sub[iu, ju], ref[iu, ju])
    np.testing.assert_allclose(sub, ref, rtol=0, atol=RTOL * np.abs(ref).max())


@pytest.mark.parametrize("beta_deg", [0.0, 30.0])
@pytest.mark.parametrize("grid", ["golden42", "full400"])
def test_mfma_path_matches_per_pair_kernel(T, beta_deg, grid):
    """The default QTF path on a sorted grid (the pair sum as FP64 MFMA GEMMs, rh_qtf_mfma.hip)
    against the per-pair kernel k_qtf_pairs (rh_set_qtf_path(ctx, 1)): the same arithmetic
    reassociated, so they agree far inside the 1e-9 parity bar (1e-12 normwise, elementwise
    to 1e-12 of the largest entry), with the moving body and fixed, at 0 and 30 degrees (Q1).
    The RAOs: the reference's (no sway, roll or yaw at 0 degrees), none, and a seeded random
    one in all six DOFs.  In a variant library (tools/build_variants.sh, RAFTHIP_LIB) the 32 x 32 GEMM tiles
    (rh_set_qtf_path(ctx, 2)) and the GEMM coefficients and Kim & Yue sums as two launches
    (rh_set_qtf_path(ctx, 3), one merged launch by default) give the default's bits; the shipped
    library refuses those paths."""
    import torch
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    m, f = make(T)
    dd = f.device_design()
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    if grid == "golden42":
        w2, k2 = T["w1_2nd"], T["k1_2nd"]
    else:
        w2 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
        k2 = wave_numbers(w2, f.depth)
    qd = QtfDevice(f, w2, k2, np.deg2rad(beta_deg), 0)
    assert qd.order == 1
    ctx = N.context(0)
    variants = N.lib().rh_set_qtf_path(ctx, 2) == N.RH_OK
    N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")
    rng = np.random.default_rng(11)
    Xr = (rng.normal(size=T["out_Xi0"].shape) + 1j * rng.normal(size=T["out_Xi0"].shape)) * np.abs(T["out_Xi0"]).max()
    for X0 in (T["out_Xi0"], np.zeros_like(T["out_Xi0"]), Xr):   # Xr: every DOF moving, yaw included
        X = torch.tensor(X0, dtype=torch.complex128, device=dd.device)
        out = []
        try:
            for path in ((0, 1, 2, 3) if variants else (0, 1)):
                N.check(N.lib().rh_set_qtf_path(ctx, path), "rh_set_qtf_path")
                out.append(qd.qtf(dd.w, X, M66).cpu().numpy())
        finally:
            N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")
        a, b = out[:2]
        if variants:
            np.testing.assert_array_equal(out[2], a)   # 32 x 32 tiles: the same bits as 16 x 16
            np.testing.assert_array_equal(out[3], a)   # two launches: the same arithmetic, the same bits
        else:
            assert N.lib().rh_set_qtf_path(ctx, 3) == N.RH_EINVAL
        assert rel(a, b) < 1e-12, rel(a, b)
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-12 * np.abs(b).max())
        i, j = np.tril_indices(len(w2), -1)
        np.testing.assert_array_equal(a[i, j], np.conj(a[j, i]))


def test_device_hankel_table_matches_scipy(T):
    """rh_qtf_hankel against scipy.special.hankel1 (the reference's call, raft_member.py:1104-1107)
    on the C3 400 grid for every Kim & Yue radius of OC4semi, and on a wide argument sweep
    (x = kR from 1e-3 to 40: series, Miller and forward-recurrence ranges): 1e-13 relative."""
    import torch
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice, hank_table
    m, f = make(T)
    w2 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    qd = QtfDevice(f, w2, k2, 0.0, 0)
    R = qd.kray[0].cpu().numpy()
    dev = qd.hank.cpu().numpy()
    for ir, r in enumerate(R):
        ref = hank_table(k2, r)
        err = np.abs(dev[ir] - ref) / np.abs(ref)
        assert err.max() < 1e-13, (ir, r, err.max())
    x = np.geomspace(1e-3, 40.0, 2000)
    kk = torch.tensor(x, dtype=torch.float64, device=qd.dev)
    one = torch.ones(1, dtype=torch.float64, device=qd.dev)
    out = torch.empty([1, len(x), 12], dtype=torch.complex128, device=qd.dev)
    N.check(N.lib().rh_qtf_hankel(N.context(0), len(x), N.ptr(kk), 1, N.ptr(one), N.ptr(out),
                                  N.stream_handle(torch, qd.dev)), "rh_qtf_hankel")
    ref = hank_table(x, 1.0)
    err = np.abs(out[0].cpu().numpy() - ref) / np.abs(ref)
    assert err.max() < 1e-13, err.max()


@pytest.mark.parametrize("beta_deg", [0.0, 30.0])
def test_all_dof_rao_qtf_matches_oracle(T, beta_deg):
    """A seeded random RAO moving in all six DOFs (the reference's golden RAO has no sway, roll
    or yaw) through the default (MFMA) path against the oracle on the golden 42-frequency grid,
    1e-9 normwise and elementwise to 1e-9 of the largest entry.  The yaw column of the GEMM
    coefficients was once wrong while every golden-RAO test passed."""
    from oracle import qtf_oracle as Q
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.beta = np.array([np.deg2rad(beta_deg)])
    rng = np.random.default_rng(12 + int(beta_deg))
    X0 = T["out_Xi0"]
    X = (rng.normal(size=X0.shape) + 1j * rng.normal(size=X0.shape)) * np.abs(X0).max()
    f.calcQTF_slenderBody(0, Xi0=X)
    ref = Q.qtf_slender(T, X, T["w1_2nd"], T["k1_2nd"], np.deg2rad(beta_deg))
    assert rel(f.qtf, ref) < RTOL, rel(f.qtf, ref)
    np.testing.assert_allclose(f.qtf, ref, rtol=0, atol=RTOL * np.abs(ref).max())


def test_fixed_body_qtf_matches_oracle(T):
    """Xi0=None (fixed body) against the oracle at the n2=42 grid."""
    from oracle import qtf_oracle as Q
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.calcQTF_slenderBody(0)
    ref = Q.qtf_slender(T, np.zeros([6, len(T["w"])], dtype=complex), T["w1_2nd"], T["k1_2nd"], 0.0)
    assert rel(f.qtf, ref) < RTOL


def test_second_order_solve_matches_reference(T):
    """potSecOrder=1 through Model.solveDynamics (raft/raft_model.py:966-989)."""
    m, f = make(T)
    Xi = m.solveDynamics(_case(T))
    assert f.iterations_pair == list(T["out_iters_pair"]), (f.iterations_pair, T["out_iters_pair"])
    assert rel(Xi, T["out_Xi"]) < RTOL, rel(Xi, T["out_Xi"])
    assert rel(f.qtf, T["out_qtf"]) < RTOL
    assert rel(f.Fhydro_2nd, T["out_Fhydro_2nd"]) < RTOL
    np.testing.assert_allclose(f.Fhydro_2nd_mean, T["out_Fhydro_2nd_mean"], rtol=RTOL,
                               atol=RTOL * np.abs(T["out_Fhydro_2nd_mean"]).max())
    assert rel(f.B_hydro_drag, T["out_B_drag"]) < RTOL


def test_qtf_text_outputs(T, tmp_path):
    """.4 / .12d / f_2nd files (raft/raft_fowt.py:1416-1432, 1700-1726, 1810-1814)."""
    m, f = make(T, out_folder=str(tmp_path))
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"], verbose=True, iCase=0, iWT=0)
    n2 = len(T["w1_2nd"])
    q12 = np.loadtxt(tmp_path / "qtf-slender_body-total_Head0p00_Case1_WT0.12d")
    assert q12.shape == (6 * n2 * (n2 + 1) // 2, 9)
    iu, ju = np.triu_indices(n2)
    ref = T["out_qtf"][iu, ju, 0, 0] / (1025.0 * 9.81)
    np.testing.assert_allclose(q12[:len(iu), 7], ref.real, rtol=1e-3, atol=1e-4 * np.abs(ref).max())
    np.testing.assert_allclose(q12[:len(iu), 0], 2 * np.pi / T["w1_2nd"][iu], rtol=1e-4)
    r4 = np.loadtxt(tmp_path / "raos-slender_body_Head0p00_Case1_WT0.4")
    assert r4.shape == (6 * n2, 7)
    f.calcHydroForce_2ndOrd(f.beta[0], T["out_S"][0], iCase=0, iWT=0)
    f2 = np.loadtxt(tmp_path / "f_2nd-_Case1_WT0.txt")
    assert f2.shape == (len(T["w"]), 7)


def test_tile_sharded_qtf_equals_single_device(T):
    """rh_qtf_slender_rows over 3 and 8 simulated ranks (contiguous tile blocks, each call
    computing the tables and w1 coefficients of its own rows only) + sum + rh_qtf_hermitian_fill
    reproduces rh_qtf_slender bit for bit (the multi-GPU exchange of raft/parallel.py)."""
    import torch
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    qd = f._qtf_qd
    dd = f.device_design()
    X = torch.tensor(T["out_Xi0"], dtype=torch.complex128, device=dd.device)
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    for world in (3, 8):
        acc = torch.zeros([qd.n2, qd.n2, 6], dtype=torch.complex128, device=dd.device)
        for r in range(world):
            part = torch.zeros_like(acc)
            qd.qtf_rows(dd.w, X, M66, part, r, world)
            acc += part
        qd.hermitian_fill(acc)
        np.testing.assert_array_equal(acc.cpu().numpy(), f.qtf[:, :, 0, :])


def test_tile_sharded_full_grid_equals_single_device(T):
    """The 400-frequency grid over 2 and 8 simulated ranks: a rank's 163 or 40-odd pair tiles
    (at most one per CU) run the Kim & Yue sums with one wave per part of a member's rows
    (k_qtf_lk<kKayP>), the whole QTF's 325 tiles with one wave per member (k_qtf_lk<1>); the
    parts' sums are added in the same order, so the sharded QTF equals the single-device one
    bit for bit."""
    import torch
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    m, f = make(T)
    dd = f.device_design()
    w2 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    qd = QtfDevice(f, w2, k2, np.deg2rad(30.0), 0)
    rng = np.random.default_rng(21)
    X0 = T["out_Xi0"]
    X = torch.tensor((rng.normal(size=X0.shape) + 1j * rng.normal(size=X0.shape)) * np.abs(X0).max(),
                     dtype=torch.complex128, device=dd.device)
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    whole = qd.qtf(dd.w, X, M66).cpu().numpy()
    for world in (2, 8):
        acc = torch.zeros([qd.n2, qd.n2, 6], dtype=torch.complex128, device=dd.device)
        for r in range(world):
            part = torch.zeros_like(acc)
            qd.qtf_rows(dd.w, X, M66, part, r, world)
            acc += part
        qd.hermitian_fill(acc)
        np.testing.assert_array_equal(acc.cpu().numpy(), whole)


def test_force_spectrum_mode_matches_reference(T):
    """calcHydroForce_2ndOrd(interpMode='spectrum') on the device (rh_force_2nd_spectrum)
    against the reference method on the same QTF and spectrum (f2nd_spectrum.npz)."""
    G = load_golden("f2nd_spectrum")
    m, f = make(T)
    f.calcHydroExcitation(_case(T), memberList=f.memberList)
    f.calcQTF_slenderBody(0, Xi0=T["out_Xi0"])
    fm, fd = f.calcHydroForce_2ndOrd(f.beta[0], G["c3_S0"], interpMode="spectrum")
    assert fd.dtype == complex and np.all(fd.imag == 0) and np.all(fd[:, -1] == 0)
    assert rel(fd, G["c3_f"]) < RTOL, rel(fd, G["c3_f"])
    np.testing.assert_allclose(fm, G["c3_fmean"], rtol=RTOL, atol=RTOL * np.abs(G["c3_fmean"]).max())
    with pytest.raises(ValueError):
        f.calcHydroForce_2ndOrd(f.beta[0], G["c3_S0"], interpMode="bogus")


@pytest.mark.gpu
def test_device_tables_are_the_numpy_tables(T):
    """QtfDevice's tables (rh_qtf_tables on the host, one pinned asynchronous upload) on the
    device equal raft/qtf.py build_tables bit for bit, for two QtfDevices built back to back
    through the one staging buffer (the second must not overwrite the first's upload)."""
    import torch
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice, build_tables
    m, f = make(T)
    w2 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    qds = [QtfDevice(f, w2, k2, b, 0) for b in (0.0, np.deg2rad(30.0))]
    torch.cuda.synchronize()
    for qd, b in zip(qds, (0.0, np.deg2rad(30.0))):
        ref = build_tables(f, w2, k2, b)
        np.testing.assert_array_equal(qd.w2.cpu().numpy(), w2)
        np.testing.assert_array_equal(qd.k2.cpu().numpy(), k2)
        for k in ("qnode", "qmemb", "kray", "qmstart", "kstart"):
            np.testing.assert_array_equal(getattr(qd, k).cpu().numpy(), ref[k], err_msg=k)
            np.testing.assert_array_equal(qd.host[k], ref[k], err_msg=k)


@pytest.mark.gpu
def test_incident_cached_qtf_equals_full_qtf(T):
    """rh_qtf_slender_ext with RH_QTF_INCIDENT_CACHED (the Kim & Yue tables and tile sums, the
    node GEMM basis: the parts that do not depend on the RAO, kept in the workspace from an
    earlier call) gives a new RAO's QTF bit for bit as a full call on a fresh workspace; the
    per-pair path refuses the flag."""
    import torch
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    m, f = make(T)
    dd = f.device_design()
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    w2 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    X1 = torch.tensor(T["out_Xi0"], dtype=torch.complex128, device=dd.device)
    rng = np.random.default_rng(5)
    X2 = X1 * torch.tensor(rng.uniform(0.5, 1.5, X1.shape) * np.exp(1j * rng.uniform(-0.3, 0.3, X1.shape)),
                           dtype=torch.complex128, device=dd.device)
    for beta in (0.0, np.deg2rad(30.0)):
        qd = QtfDevice(f, w2, k2, beta, 0)
        with pytest.raises(ValueError, match="earlier whole-QTF call"):
            qd.qtf(dd.w, X1, M66, incident_cached=True)
        a1 = qd.qtf(dd.w, X1, M66).clone()
        a2 = qd.qtf(dd.w, X2, M66, incident_cached=True).clone()
        a1b = qd.qtf(dd.w, X1, M66, incident_cached=True).clone()
        ref2 = QtfDevice(f, w2, k2, beta, 0).qtf(dd.w, X2, M66)
        torch.cuda.synchronize()
        assert torch.equal(a2, ref2)
        assert torch.equal(a1b, a1)
        assert not torch.equal(a1, a2)
    ctx = N.context(0)
    N.check(N.lib().rh_set_qtf_path(ctx, 1), "rh_set_qtf_path")
    try:
        with pytest.raises(ValueError, match="MFMA path"):
            qd.qtf(dd.w, X2, M66, incident_cached=True)
    finally:
        N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")


@pytest.mark.gpu
def test_qtf_of_a_design_without_kim_yue_rows_cached_and_oracle():
    """VolturnUS-S (no MacCamy-Fuchs members: no Kim & Yue rows, nkr = 0; rectangular pontoons)
    on a 24-frequency grid: the native tables equal build_tables, the MFMA QTF agrees with the
    per-pair kernel (1e-12), and a further RAO with the incident parts kept equals a whole QTF
    bit for bit.  (No reference run of this design's QTF exists: the QTF itself is pinned on
    OC4semi above; here the nkr = 0 paths are.)"""
    import torch
    import raft
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice, build_tables
    d = load_design("VolturnUS-S_example")
    m = raft.Model(d)
    f = m.fowtList[0]
    f.setPosition(np.zeros(6))
    f.calcStatics()
    f.calcHydroConstants()
    dd = f.device_design()
    w2 = np.linspace(0.3, 1.8, 24)
    k2 = wave_numbers(w2, f.depth)
    qd = QtfDevice(f, w2, k2, np.deg2rad(20.0), 0)
    assert qd.nkr == 0 and qd.order == 1
    ref_t = build_tables(f, w2, k2, np.deg2rad(20.0))
    for k in ("qnode", "qmemb", "kray", "qmstart", "kstart"):
        np.testing.assert_array_equal(qd.host[k], ref_t[k], err_msg=k)
    rng = np.random.default_rng(9)
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    X1 = (rng.normal(size=(6, f.nw)) + 1j * rng.normal(size=(6, f.nw))) * 0.5
    X2 = X1 * 1.3 + 0.1j
    T1 = torch.tensor(X1, dtype=torch.complex128, device=dd.device)
    T2 = torch.tensor(X2, dtype=torch.complex128, device=dd.device)
    a1 = qd.qtf(dd.w, T1, M66).cpu().numpy()
    a2 = qd.qtf(dd.w, T2, M66, incident_cached=True).cpu().numpy()
    ref2 = QtfDevice(f, w2, k2, np.deg2rad(20.0), 0).qtf(dd.w, T2, M66).cpu().numpy()
    np.testing.assert_array_equal(a2, ref2)
    ctx = N.context(0)
    N.check(N.lib().rh_set_qtf_path(ctx, 1), "rh_set_qtf_path")
    try:
        p1 = QtfDevice(f, w2, k2, np.deg2rad(20.0), 0).qtf(dd.w, T1, M66).cpu().numpy()
    finally:
        N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")
    assert np.abs(a1).max() > 0 and rel(a1, p1) < 1e-12, rel(a1, p1)
