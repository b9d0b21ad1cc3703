"""Generate the committed golden fixtures by running the READ-ONLY reference
(/root/reference/raft, RAFT v1.3.1 fork) inside the build container.

This script is test infrastructure only.  It never ships to the GPU box; what it
writes (tests/golden/*.npz, *.json) are plain data files: reference INPUT tables
and reference OUTPUT vectors.  No reference source text is copied.

Run (from the repo root, in the build container):

    PYTHONDONTWRITEBYTECODE=1 OPENBLAS_NUM_THREADS=1 \
    PYTHONPATH=tests/golden/refshim:/root/reference python tests/golden/make_golden.py [which...]

`tests/golden/refshim` holds inert stand-ins for the two absent third-party
packages the reference imports at module scope (MoorPy, CCBlade).
Neither is on the hot path: mooring stiffness is an INPUT matrix (set explicitly
from C_MOOR below, as SURVEY.md §8(c) prescribes) and every golden case runs with
wind_speed = 0, so rotor aerodynamics are never evaluated
(reference raft/raft_fowt.py:801).

Iteration counts are read from the reference's own display=2 message
"Iteration k, converged" (raft/raft_model.py:963-964).
"""
import contextlib
import io
import json
import os
import re
import sys
import time

import numpy as np
import yaml

import raft  # the reference, from PYTHONPATH

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

# Stand-in mooring stiffness (SURVEY.md §6 / BASELINE.md: diag(7e4,7e4,2e4,1e7,1e7,1e8)).
C_MOOR = np.diag([7e4, 7e4, 2e4, 1e7, 1e7, 1e8])


def load_design(path, **settings):
    with open(path) as f:
        design = yaml.load(f, Loader=yaml.FullLoader)
    for k, v in settings.items():
        design["settings"][k] = v
    return design


def prepare_fowt(fowt, case):
    """Per-case preparation exactly as Model.analyzeCases/solveStatics would leave the
    FOWT for solveDynamics when the platform sits at its reference position
    (raft/raft_model.py:258-260, :286 with zero mean offset)."""
    fowt.setPosition(np.array([fowt.x_ref, fowt.y_ref, 0, 0, 0, 0], dtype=float))
    fowt.calcStatics()
    fowt.calcTurbineConstants(case, ptfm_pitch=0)
    fowt.calcHydroConstants()
    fowt.C_moor = C_MOOR.copy()


def design_tables(fowt):
    """Dump every per-design input the hot path consumes, node by node, in reference
    order (member list order, node order within member).  Only submerged nodes
    (r_z < 0 strictly, raft/raft_fowt.py:1104,1188) carry hydrodynamics."""
    rows = []
    for im, mem in enumerate(fowt.memberList):
        circ = mem.shape == "circular"
        for il in range(mem.ns):
            ls = mem.ls[il]
            row = dict(
                member=im, node=il, circ=int(circ), sub=int(mem.r[il, 2] < 0),
                mcf=int(bool(mem.MCF)),
                r=mem.r[il, :].copy(), r_rel=(mem.r[il, :] - fowt.r6[:3]).copy(),
                q=mem.q.copy(), p1=mem.p1.copy(), p2=mem.p2.copy(),
                ds=np.atleast_1d(mem.ds[il]).astype(float),
                drs=np.atleast_1d(mem.drs[il]).astype(float),
                dls=float(mem.dls[il]),
                Cd_q=np.interp(ls, mem.stations, mem.Cd_q), Cd_p1=np.interp(ls, mem.stations, mem.Cd_p1),
                Cd_p2=np.interp(ls, mem.stations, mem.Cd_p2), Cd_End=np.interp(ls, mem.stations, mem.Cd_End),
                Ca_p1=np.interp(ls, mem.stations, mem.Ca_p1), Ca_p2=np.interp(ls, mem.stations, mem.Ca_p2),
                Ca_End=np.interp(ls, mem.stations, mem.Ca_End),
                a_i=float(mem.a_i[il]),
                Imat=mem.Imat[il].copy(),
            )
            rows.append((row, mem.Imat_MCF[il] if mem.MCF else None))
    n = len(rows)
    out = {}
    for key in ["member", "node", "circ", "sub", "mcf"]:
        out["node_" + key] = np.array([r[0][key] for r in rows], dtype=np.int64)
    for key in ["r", "r_rel", "q", "p1", "p2"]:
        out["node_" + key] = np.array([r[0][key] for r in rows])
    out["node_ds"] = np.array([np.resize(r[0]["ds"], 2) for r in rows])
    out["node_drs"] = np.array([np.resize(r[0]["drs"], 2) for r in rows])
    for key in ["dls", "Cd_q", "Cd_p1", "Cd_p2", "Cd_End", "Ca_p1", "Ca_p2", "Ca_End", "a_i"]:
        out["node_" + key] = np.array([r[0][key] for r in rows], dtype=float)
    out["node_Imat"] = np.array([r[0]["Imat"] for r in rows])
    nw = fowt.nw
    imcf = np.zeros((n, 3, 3, nw), dtype=complex)
    for i, (_, im) in enumerate(rows):
        if im is not None:
            imcf[i] = im
    if out["node_mcf"].any():
        out["node_Imat_MCF"] = imcf
    out["w"] = fowt.w.copy()
    out["k"] = fowt.k.copy()
    out["dw"] = np.float64(fowt.dw)
    out["depth"] = np.float64(fowt.depth)
    out["rho"] = np.float64(fowt.rho_water)
    out["g"] = np.float64(fowt.g)
    out["r6"] = fowt.r6.copy()
    for key in ["M_struc", "B_struc", "C_struc", "C_hydro", "C_moor", "A_hydro_morison", "W_struc", "W_hydro"]:
        out[key] = np.array(getattr(fowt, key), dtype=float)
    out["A_BEM"] = fowt.A_BEM.copy()
    out["B_BEM"] = fowt.B_BEM.copy()
    out["member_names"] = np.array([m.name for m in fowt.memberList])
    out["member_rA"] = np.array([m.rA for m in fowt.memberList])
    out["member_rB"] = np.array([m.rB for m in fowt.memberList])
    out["member_circ"] = np.array([int(m.shape == "circular") for m in fowt.memberList])
    out["member_mcf"] = np.array([int(bool(m.MCF)) for m in fowt.memberList])
    return out


def rotor_inputs(fowt):
    """Per-rotor statics the AxRNA / Mbase channels read (raft/raft_fowt.py:1909-1951)."""
    rl = fowt.rotorList
    return dict(rot_r_rel_z=np.array([r.r_rel[2] for r in rl], dtype=float),
                rot_mRNA=np.array([r.mRNA for r in rl], dtype=float),
                rot_IrRNA=np.array([r.IrRNA for r in rl], dtype=float),
                rot_mtower=np.array(fowt.mtower, dtype=float),
                rot_zCG_tow=np.array([c[2] for c in fowt.rCG_tow], dtype=float),
                rot_zBase=np.array([fowt.memberList[fowt.nplatmems + i].rA[2] for i in range(len(rl))], dtype=float),
                rot_Mtow=np.array([fowt.memberList[fowt.nplatmems + i].M_struc for i in range(len(rl))], dtype=float))


def run_solve(model, case, tol=0.01):
    buf = io.StringIO()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(buf):
        Xi = model.solveDynamics(case, tol=tol, display=2)
    dt = time.perf_counter() - t0
    txt = buf.getvalue()
    m = re.findall(r"Iteration (\d+), converged", txt)
    if m:
        iters, conv = int(m[0]) + 1, 1
    else:
        iters, conv = int(model.nIter) + 1, 0
    return np.array(Xi), iters, conv, dt


def case_dict(design, row):
    c = dict(zip(design["cases"]["keys"], row))
    c["wind_speed"] = 0  # golden cases: no rotor aerodynamics (see module doc)
    return c


def golden_solve(tag, yaml_path, cases, settings=None, keep_Z=False, aero=False):
    settings = settings or {}
    if isinstance(yaml_path, dict):          # an in-memory design (C5 sweep variants)
        design = yaml_path
        design["settings"].update(settings)
    else:
        design = load_design(yaml_path, **settings)
    model = raft.Model(design)
    fowt = model.fowtList[0]
    out = {}
    caseout = {k: [] for k in ["Xi", "iters", "conv", "B_drag", "F_iner", "F_drag", "zeta", "S", "seconds"]}
    if keep_Z:
        caseout["Z"] = []
    if aero:
        for k in ["A_aero", "B_aero", "f_aero0", "B_gyro"]:
            caseout[k] = []
    metrics = []
    for c in cases:
        case = dict(c)
        prepare_fowt(fowt, case)
        if not out:
            out.update(design_tables(fowt))
        Xi, iters, conv, dt = run_solve(model, case)
        caseout["Xi"].append(Xi)
        caseout["iters"].append(iters)
        caseout["conv"].append(conv)
        caseout["B_drag"].append(fowt.B_hydro_drag.copy())
        caseout["F_iner"].append(fowt.F_hydro_iner.copy())
        caseout["F_drag"].append(fowt.F_hydro_drag.copy())
        caseout["zeta"].append(fowt.zeta.copy())
        caseout["S"].append(fowt.S.copy())
        caseout["seconds"].append(dt)
        if keep_Z:
            caseout["Z"].append(fowt.Z.copy())
        if aero:
            for k in ["A_aero", "B_aero", "f_aero0", "B_gyro"]:
                caseout[k].append(np.array(getattr(fowt, k)).copy())
        res = {}
        fowt.saveTurbineOutputs(res, case)
        metrics.append(res)
        print(f"  {tag}: case {c} iters={iters} conv={conv} t={dt:.2f}s", file=sys.stderr)
    for k, v in caseout.items():
        out["out_" + k] = np.array(v)
    # motion outputs of saveTurbineOutputs (raft/raft_fowt.py:1831-1875)
    for dof in ["surge", "sway", "heave", "roll", "pitch", "yaw"]:
        out[f"out_{dof}_std"] = np.array([m[f"{dof}_std"] for m in metrics])
        out[f"out_{dof}_PSD"] = np.array([m[f"{dof}_PSD"] for m in metrics])
    out["out_wave_PSD"] = np.array([m["wave_PSD"] for m in metrics])
    # rotor channels of saveTurbineOutputs (raft/raft_fowt.py:1900-1970) and their inputs
    for ch in ["AxRNA", "Mbase"]:
        for st in ["avg", "std", "max", "min", "PSD"]:
            out[f"out_{ch}_{st}"] = np.array([m[f"{ch}_{st}"] for m in metrics])
    if aero:   # rotor-control channels (raft/raft_fowt.py:1976-2045)
        for ch in ["omega", "torque", "bPitch"]:
            for st in ["avg", "std", "PSD"]:
                out[f"out_{ch}_{st}"] = np.array([m[f"{ch}_{st}"] for m in metrics])
        for k in ["omega_max", "omega_min", "power_avg", "wind_PSD"]:
            if all(k in m for m in metrics):       # wind_PSD only with aeroServoMod > 1
                out["out_" + k] = np.array([m[k] for m in metrics])
    out["out_metric_keys"] = np.array(sorted(metrics[0].keys()))
    out.update(rotor_inputs(fowt))
    out["nIter"] = np.int64(model.nIter)
    out["XiStart"] = np.float64(model.XiStart)
    keys = ["wave_spectrum", "wave_period", "wave_height", "wave_heading", "wave_gamma"]
    meta = [{k: (np.atleast_1d(c[k]).tolist() if k in c else None) for k in keys} for c in cases]
    out["cases_json"] = np.array(json.dumps(meta))
    if aero:
        out["cases_full_json"] = np.array(json.dumps(cases))
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(f"wrote {tag}.npz", file=sys.stderr)


def golden_fowt_unit(tag, yaml_path):
    """The reference test_fowt.py workloads: F_hydro_iner over 9 headings x 4 periods x
    2 heights (tests/test_fowt.py:214-250) and B_hydro_drag/F_hydro_drag for the
    synthetic Xi = 0.1 exp(i linspace(0, 2pi, 6 nw)) (tests/test_fowt.py:252-277)."""
    design = load_design(yaml_path)
    model = raft.Model(design)
    fowt = model.fowtList[0]
    fowt.setPosition(np.zeros(6))
    fowt.calcStatics()
    out = {}
    fowt.calcHydroConstants()
    out.update(design_tables(fowt))
    F = []
    cases = []
    for hd in [0, 45, 90, 135, 180, 225, 270, 315, 360]:
        for tp in [5, 10, 15, 20]:
            for hs in [1, 2]:
                tc = {"wave_heading": hd, "wave_period": tp, "wave_height": hs}
                fowt.calcHydroConstants()
                fowt.calcHydroExcitation(tc, memberList=fowt.memberList)
                F.append(fowt.F_hydro_iner.copy())
                cases.append([hd, tp, hs])
    out["exc_cases"] = np.array(cases, dtype=float)
    out["exc_F_iner"] = np.array(F)
    tc = {"wave_spectrum": "unit", "wave_heading": 0, "wave_period": 10, "wave_height": 2}
    fowt.calcHydroExcitation(tc, memberList=fowt.memberList)
    phase = np.linspace(0, 2 * np.pi, fowt.nw * 6).reshape(6, fowt.nw)
    Xi = 0.1 * np.exp(1j * phase)
    out["lin_Xi"] = Xi
    out["lin_B_drag"] = fowt.calcHydroLinearization(Xi)
    out["lin_F_drag"] = fowt.calcDragExcitation(0)
    np.savez_compressed(os.path.join(HERE, f"{tag}.npz"), **out)
    print(f"wrote {tag}.npz", file=sys.stderr)


def seeded_cases(n, seed, headings=(0, 30, 60, 90), hs=(1.0, 10.0), tp=(6.0, 18.0)):
    """C2 synthetic sea states: Hs~U(1,10), Tp~U(6,18), gamma=0
    (IEC auto), heading from the listed set, wind 0, current 0."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        out.append(dict(wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating",
                        yaw_misalign=0, wave_spectrum="JONSWAP",
                        wave_period=float(rng.uniform(*tp)), wave_height=float(rng.uniform(*hs)),
                        wave_heading=float(rng.choice(headings)), wave_gamma=0.0))
    return out


DESIGNS = {
    "OC3spar": "designs/OC3spar.yaml",
    "VolturnUS-S_example": "examples/VolturnUS-S_example.yaml",
    "VolturnUS-S_test": "tests/test_data/VolturnUS-S.yaml",
    "OC3spar_test": "tests/test_data/OC3spar.yaml",
    "OC4semi-RAFT_QTF": "examples/OC4semi-RAFT_QTF.yaml",
    "VolturnUS-S_farm": "tests/test_data/VolturnUS-S_farm.yaml",
}


def export_designs():
    """Design inputs as JSON fixtures (the GPU box has no /root/reference).  Blade/airfoil
    aero tables are dropped (rotor aero is out of scope); the mooring sections (points,
    lines, line types) are kept for raft/mooring.py, and the farm's MoorDyn-style array
    mooring file (a data file of the reference's tests) is copied next to the JSON."""
    os.makedirs(os.path.join(HERE, "designs"), exist_ok=True)
    for name, rel in DESIGNS.items():
        with open(os.path.join(REF, rel)) as f:
            d = yaml.load(f, Loader=yaml.FullLoader)
        for tk in ("turbine", "turbines"):
            ts = d.get(tk)
            for t in (ts if isinstance(ts, list) else [ts] if ts else []):
                for drop in ("blade", "airfoils", "pitch_control", "torque_control", "wt_ops", "gear_ratio"):
                    t.pop(drop, None)
        if "array_mooring" in d:
            src = os.path.join(os.path.dirname(os.path.join(REF, rel)), d["array_mooring"]["file"])
            base = os.path.basename(src)
            with open(src) as fi, open(os.path.join(HERE, "designs", base), "w") as fo:
                fo.write(fi.read())
            d["array_mooring"] = {"file": base}
        with open(os.path.join(HERE, "designs", name + ".json"), "w") as f:
            json.dump(d, f, indent=1, default=str)
    print("wrote designs/*.json", file=sys.stderr)


def bilinear_interp2d(x, y, z, bounds_error=False, fill_value=0):
    """Restatement of the removed scipy.interpolate.interp2d(kind='linear') as the reference
    uses it (raft/raft_fowt.py:1792-1793): bilinear on the regular grid,
    z[y_i, x_j] orientation, fill_value strictly outside [x0, x1] x [y0, y1]."""
    from scipy.interpolate import RegularGridInterpolator
    x = np.asarray(x, dtype=float)
    y = np.asarray(y, dtype=float)
    rgi = RegularGridInterpolator((y, x), np.asarray(z, dtype=float), method="linear", bounds_error=False,
                                  fill_value=fill_value)

    def f(xn, yn):
        X, Y = np.meshgrid(np.asarray(xn, dtype=float), np.asarray(yn, dtype=float))
        return rgi(np.stack([Y.ravel(), X.ravel()], axis=-1)).reshape(X.shape)
    return f


def golden_qtf():
    """C3: OC4semi-RAFT_QTF with potSecOrder=1 through the reference's full path
    (first convergence -> RAO -> calcQTF_slenderBody -> calcHydroForce_2ndOrd -> second
    pass, raft/raft_model.py:966-989), plus QTF entries of the n2=400 grid (df 0.000825 Hz)
    on a seeded 24-frequency subset (every pair of a frequency subset is an entry of the
    full 400x400 matrix: the per-frequency tables depend only on the frequency)."""
    import raft.raft_fowt as rf
    rf.interp2d = bilinear_interp2d
    design = load_design(os.path.join(REF, "examples", "OC4semi-RAFT_QTF.yaml"))
    design["platform"].pop("outFolderQTF", None)
    model = raft.Model(design)
    fowt = model.fowtList[0]
    case = dict(zip(design["cases"]["keys"], design["cases"]["data"][0]))
    case["wind_speed"] = 0
    prepare_fowt(fowt, case)
    out = design_tables(fowt)
    mcf = out.pop("node_Imat_MCF", None)
    if mcf is not None:                      # keep a sample of bins only (fixture size)
        out["node_Imat_MCF_bins"] = np.arange(0, fowt.nw, 37)
        out["node_Imat_MCF_sample"] = mcf[..., ::37]
    captured = {}
    orig = fowt.calcQTF_slenderBody

    def spy(waveHeadInd, Xi0=None, verbose=False, iCase=None, iWT=None):
        captured["Xi0"] = np.array(Xi0)
        t0 = time.perf_counter()
        r = orig(waveHeadInd, Xi0=Xi0, verbose=False, iCase=iCase, iWT=iWT)
        captured["qtf_seconds"] = time.perf_counter() - t0
        return r
    fowt.calcQTF_slenderBody = spy
    buf = io.StringIO()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(buf):
        Xi = model.solveDynamics(dict(case), display=2)
    dt = time.perf_counter() - t0
    its = [int(m) + 1 for m in re.findall(r"Iteration (\d+), converged", buf.getvalue())]
    out.update(out_Xi=np.array(Xi), out_iters_pair=np.array(its), out_qtf=fowt.qtf.copy(), out_Xi0=captured["Xi0"],
               out_Fhydro_2nd=fowt.Fhydro_2nd.copy(), out_Fhydro_2nd_mean=fowt.Fhydro_2nd_mean.copy(),
               out_zeta=fowt.zeta.copy(), out_S=fowt.S.copy(), out_B_drag=fowt.B_hydro_drag.copy(),
               w1_2nd=fowt.w1_2nd.copy(), k1_2nd=fowt.k1_2nd.copy(), qtf_seconds=captured["qtf_seconds"],
               seconds=dt, nIter=np.int64(model.nIter), XiStart=np.float64(model.XiStart),
               cases_json=np.array(json.dumps([{k: np.atleast_1d(case[k]).tolist() for k in
                                               ["wave_spectrum", "wave_period", "wave_height", "wave_heading"]}])))
    print(f"  qtf: iters {its}, QTF n2={len(fowt.w1_2nd)} {captured['qtf_seconds']:.1f}s, total {dt:.1f}s",
          file=sys.stderr)
    # 400-grid subset
    w400 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    rng = np.random.default_rng(20241016)
    sel = np.sort(rng.choice(len(w400), 24, replace=False))
    fowt.w1_2nd = w400[sel]
    fowt.w2_2nd = fowt.w1_2nd.copy()
    fowt.k1_2nd = np.array([raft.helpers.waveNumber(w, fowt.depth) for w in fowt.w1_2nd])
    fowt.k2_2nd = fowt.k1_2nd.copy()
    t0 = time.perf_counter()
    orig(0, Xi0=captured["Xi0"], verbose=False)
    out.update(sub400_n2=np.int64(len(w400)), sub400_idx=sel, sub400_w=fowt.w1_2nd.copy(), sub400_k=fowt.k1_2nd.copy(),
               sub400_qtf=fowt.qtf.copy(), sub400_seconds=time.perf_counter() - t0)
    # an oblique heading exercises the degree/radian quirk of the wave helpers
    fowt.beta = np.array([np.deg2rad(30.0)])
    orig(0, Xi0=captured["Xi0"], verbose=False)
    out.update(sub400_beta30_qtf=fowt.qtf.copy(), sub400_beta30=np.float64(fowt.beta[0]))
    print(f"  qtf: 400-grid subset ({len(sel)} freqs, {len(sel)*(len(sel)+1)//2} pairs) "
          f"{out['sub400_seconds']:.1f}s", file=sys.stderr)
    np.savez_compressed(os.path.join(HERE, "c3_qtf.npz"), **out)
    print("wrote c3_qtf.npz", file=sys.stderr)


# Stand-in array-level (shared-line) stiffness for the 2-FOWT farm: both bodies anchored
# by C_MOOR at the FOWT level plus a shared surge/sway line between them.
K_SHARED = np.diag([3.0e4, 1.0e4, 0.0, 0.0, 0.0, 0.0])
K_ARRAY = np.block([[K_SHARED, -K_SHARED], [-K_SHARED, K_SHARED]])


def golden_farm():
    """C4: tests/test_data/VolturnUS-S_farm.yaml (2 FOWTs, x = 0 / 1600 m, heading_adjust
    180 / 0, nw = 240, nIter = 10).  Array coupling enters Z_sys through
    ms.getCoupledStiffnessA (raft/raft_model.py:1030-1031), here the K_ARRAY fixture."""
    design = load_design(os.path.join(REF, "tests", "test_data", "VolturnUS-S_farm.yaml"))
    model = raft.Model(design)
    model.ms.getCoupledStiffnessA = lambda *a, **kw: K_ARRAY.copy()
    cases = seeded_cases(3, 20241018)
    out = {"K_array": K_ARRAY, "nIter": np.int64(model.nIter), "XiStart": np.float64(model.XiStart)}
    res = {k: [] for k in ["Xi", "iters", "B_drag", "zeta", "seconds"]}
    for c in cases:
        case = dict(c)
        for i, fowt in enumerate(model.fowtList):
            prepare_fowt(fowt, case)
            if f"f{i}_w" not in out:
                out.update({f"f{i}_{k}": v for k, v in design_tables(fowt).items()})
        buf = io.StringIO()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(buf):
            Xi = model.solveDynamics(case, display=2)
        dt = time.perf_counter() - t0
        # one "Iteration k, converged" line per FOWT drag loop, in FOWT order
        its = [int(m) + 1 for m in re.findall(r"Iteration (\d+), converged", buf.getvalue())]
        assert len(its) == len(model.fowtList), its
        res["Xi"].append(np.array(Xi))
        res["iters"].append(its)
        res["B_drag"].append([f.B_hydro_drag.copy() for f in model.fowtList])
        res["zeta"].append(model.fowtList[0].zeta.copy())
        res["seconds"].append(dt)
        print(f"  farm: case {c} iters={its} t={dt:.1f}s", file=sys.stderr)
    for k, v in res.items():
        out["out_" + k] = np.array(v)
    keys = ["wave_spectrum", "wave_period", "wave_height", "wave_heading", "wave_gamma"]
    out["cases_json"] = np.array(json.dumps([{k: np.atleast_1d(c[k]).tolist() for k in keys} for c in cases]))
    np.savez_compressed(os.path.join(HERE, "c4_farm.npz"), **out)
    print("wrote c4_farm.npz", file=sys.stderr)


def load_sweep_module():
    """raft-teststuff_amd/raft/sweep.py by file path (numpy only; the name `raft` is the
    reference package here)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.dirname(HERE)), "raft-teststuff_amd", "raft", "sweep.py")
    spec = importlib.util.spec_from_file_location("rh_sweep", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def golden_sweep():
    """C5: three parametersweep-style VolturnUS-S_example variants (raft/parametersweep.py
    variables, U(0.75,1.25) draws) at nw = 1000, two sea states each, statics computed by
    the reference for each variant, mooring stiffness C_MOOR."""
    sw = load_sweep_module()
    with open(os.path.join(REF, "examples", "VolturnUS-S_example.yaml")) as f:
        base = yaml.load(f, Loader=yaml.FullLoader)
    mult = sw.sweep_multipliers(3, seed=20241016)
    grid = sw.sea_state_grid()
    rng = np.random.default_rng(20241019)
    for i, m in enumerate(mult):
        d = sw.sweep_variant(base, m)
        pick = rng.choice(len(grid), 2, replace=False)
        cases = [dict(grid[j], wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating", yaw_misalign=0)
                 for j in pick]
        golden_solve(f"c5_sweep{i}", d, cases, settings=dict(min_freq=0.0002))
        T = dict(np.load(os.path.join(HERE, f"c5_sweep{i}.npz")))
        T.pop("node_Imat_MCF", None)
        T["sweep_mult"] = m
        np.savez_compressed(os.path.join(HERE, f"c5_sweep{i}.npz"), **T)


def golden_qtf12d():
    """potSecOrder=2: an external WAMIT .12d QTF (the reference's own
    examples/OC4semi-WAMIT_Coefs/marin_semi.12d) read by FOWT.readQTF
    (raft/raft_fowt.py:1651-1697) and applied through calcHydroForce_2ndOrd before the drag
    loop and for the other sea states (raft/raft_model.py:903-904, :1059-1061).  Design:
    OC4semi-RAFT_QTF with strip-theory first order (potFirstOrder 0) at nw = 100.
    Stored: the file's numeric table (the test rewrites an equivalent .12d from it), the
    parsed QTF, and per case Xi, iterations, the second-order force and mean drift."""
    import raft.raft_fowt as rf
    rf.interp2d = bilinear_interp2d
    path = os.path.join(REF, "examples", "OC4semi-WAMIT_Coefs", "marin_semi")
    design = load_design(os.path.join(REF, "examples", "OC4semi-RAFT_QTF.yaml"), min_freq=0.0025)
    plat = design["platform"]
    for k in ("outFolderQTF", "min_freq2nd", "max_freq2nd", "df_freq2nd"):
        plat.pop(k, None)
    plat["potSecOrder"] = 2
    plat["hydroPath"] = path
    cases = [dict(wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating", yaw_misalign=0,
                  wave_spectrum="JONSWAP", wave_period=12.0, wave_height=6.0, wave_heading=0.0, current_speed=0,
                  wave_gamma=0.0),
             dict(wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating", yaw_misalign=0,
                  wave_spectrum="JONSWAP", wave_period=9.0, wave_height=3.5, wave_heading=0.0, current_speed=0,
                  wave_gamma=2.0),
             dict(wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating", yaw_misalign=0,
                  wave_spectrum=["JONSWAP", "JONSWAP"], wave_period=[12.0, 7.0], wave_height=[6.0, 2.0],
                  wave_heading=[0.0, 30.0], current_speed=0, wave_gamma=[0.0, 0.0])]
    out = dict(table12d=np.loadtxt(path + ".12d"))
    res = {k: [] for k in ["Xi", "iters", "Fhydro_2nd", "Fhydro_2nd_mean", "B_drag", "zeta", "S"]}
    for ic, case in enumerate(cases):
        model = raft.Model(json.loads(json.dumps(design)))
        fowt = model.fowtList[0]
        prepare_fowt(fowt, case)
        if ic == 0:
            out.update(design_tables(fowt))
            out.update(qtf=fowt.qtf.copy(), heads_2nd=np.array(fowt.heads_2nd, dtype=float), w1_2nd=fowt.w1_2nd.copy())
        Xi, iters, conv, dt = run_solve(model, dict(case))
        nW = fowt.nWaves
        pad = lambda a, n: np.concatenate([a, np.zeros((n - len(a),) + a.shape[1:], dtype=a.dtype)])
        res["Xi"].append(pad(np.array(Xi), 3))
        res["iters"].append(iters)
        res["Fhydro_2nd"].append(pad(fowt.Fhydro_2nd.copy(), 2))
        res["Fhydro_2nd_mean"].append(pad(fowt.Fhydro_2nd_mean.copy(), 2))
        res["B_drag"].append(fowt.B_hydro_drag.copy())
        res["zeta"].append(pad(fowt.zeta.copy(), 2))
        res["S"].append(pad(fowt.S.copy(), 2))
        print(f"  qtf12d case {ic}: nWaves {nW}, iters {iters}, {dt:.1f}s", file=sys.stderr)
    out.update({"out_" + k: np.array(v) for k, v in res.items()})
    out.update(nIter=np.int64(design["settings"]["nIter"]), XiStart=np.float64(design["settings"]["XiStart"]),
               cases_json=np.array(json.dumps(cases)))
    np.savez_compressed(os.path.join(HERE, "qtf12d.npz"), **out)
    print("wrote qtf12d.npz", file=sys.stderr)


def golden_f2nd_spectrum():
    """calcHydroForce_2ndOrd(interpMode='spectrum') (raft/raft_fowt.py:1760-1784), the
    non-default mode: the reference method applied to the QTFs already in the fixtures (the
    C3 slender-body QTF at n2=42, and the .12d file QTF with two of its cases' spectra)."""
    from types import SimpleNamespace

    import raft.raft_fowt as rf
    C3 = dict(np.load(os.path.join(HERE, "c3_qtf.npz")))
    Q12 = dict(np.load(os.path.join(HERE, "qtf12d.npz")))
    out = {}
    runs = [("c3", C3["out_qtf"], np.array([0.0]), C3["w1_2nd"], C3["w"], C3["out_S"][0], 0.0),
            ("q12_b0", Q12["qtf"], Q12["heads_2nd"], Q12["w1_2nd"], Q12["w"], Q12["out_S"][0][0], 0.0),
            ("q12_s1", Q12["qtf"], Q12["heads_2nd"], Q12["w1_2nd"], Q12["w"], Q12["out_S"][1][0], 0.0)]
    for tag, qtf, heads, w1, w, S0, beta in runs:
        obj = SimpleNamespace(nDOF=6, nw=len(w), w=w, dw=float(w[1] - w[0]), qtf=qtf, heads_2nd=heads, w1_2nd=w1,
                              outFolderQTF=None)
        fm, f = rf.FOWT.calcHydroForce_2ndOrd(obj, beta, S0, interpMode="spectrum")
        out.update({f"{tag}_beta": np.float64(beta), f"{tag}_S0": S0, f"{tag}_fmean": fm, f"{tag}_f": f})
    np.savez_compressed(os.path.join(HERE, "f2nd_spectrum.npz"), **out)
    print("wrote f2nd_spectrum.npz", file=sys.stderr)


ROTOR_DESIGNS = {"IEA15MW": "tests/test_data/IEA15MW.yaml"}   # VolturnUS-S_example carries the same turbine


def rotor_cases():
    """Wind conditions of the rotor goldens: below / at / above rated and parked-region
    speeds, misaligned inflow, every yaw mode, turbulence as an intensity and as IEC
    class strings (NTM / ETM / EWM)."""
    out = []
    for U in (5.0, 10.59, 15.0, 25.0):
        for hd, th, ym, ti in ((0.0, 0.0, 0, 0.1), (30.0, 0.0, 0, "IB_NTM"), (-20.0, 10.0, 1, "IIC_ETM"),
                               (45.0, 0.0, 2, "IA_EWM"), (10.0, 25.0, 3, 0.14)):
            out.append(dict(wind_speed=U, wind_heading=hd, turbine_heading=th, turbulence=ti, yaw_mode=ym))
    return out


def golden_rotor():
    """Rotor aero-servo linearisation (raft/raft_rotor.py): the reference's Rotor run with the
    scripted CCBlade stand-in of tests/golden/fake_ccblade.py (CCBlade itself is a third-party
    dependency that is not installed).  Pins RAFT's own rotor code: the CCBlade inputs it builds
    (polars on the angle-of-attack grid, PCHIP over the span, blade tables) and Rotor.calcAero /
    IECKaimal for aeroServoMod 1 and 2.  Writes rotor_<design>.npz and the turbine dicts."""
    import raft.raft_rotor as RR
    from raft.helpers import getFromDict
    sys.path.insert(0, HERE)
    from fake_ccblade import FakeAirfoil, FakeCCBlade
    RR.CCBlade, RR.CCAirfoil = FakeCCBlade, FakeAirfoil
    # the reference's calcAero allocates with np.complex_, an alias NumPy 2 removed; it names
    # complex128 (the same dtype), so restore the alias for the run
    if not hasattr(np, "complex_") or np.__dict__.get("complex_") is None:
        np.complex_ = np.complex128
    for name, rel in ROTOR_DESIGNS.items():
        d = load_design(os.path.join(REF, rel))
        turb = d["turbine"]
        turb["nrotors"] = 1
        site = d["site"]
        turb["rho_air"] = getFromDict(site, "rho_air", shape=0, default=1.225)
        turb["mu_air"] = getFromDict(site, "mu_air", shape=0, default=1.81e-05)
        turb["shearExp_air"] = getFromDict(site, "shearExp_air", shape=0, default=0.12)
        turb["rho_water"] = getFromDict(site, "rho_water", shape=0, default=1025.0)
        turb["mu_water"] = getFromDict(site, "mu_water", shape=0, default=1.0e-03)
        turb["shearExp_water"] = getFromDict(site, "shearExp_water", shape=0, default=0.12)
        with open(os.path.join(HERE, "designs", name + "_turbine.json"), "w") as f:
            json.dump(turb, f, indent=1, default=str)
        w = np.arange(0.01, 0.3 + 0.005, 0.01) * 2 * np.pi
        out = {"w": w}
        cases = rotor_cases()
        for mod in (1, 2):
            t = json.loads(json.dumps(turb, default=str))
            t["aeroServoMod"] = mod
            rot = RR.Rotor(t, w, 0)
            if mod == 1:
                for k, v in rot.ccblade.args.items():
                    out["cc_" + k] = np.asarray(v)
                out["Ca_interp"] = rot.Ca_interp
                out["r_thick_interp"] = rot.r_thick_interp
                out["cpmin_interp"] = rot.cpmin_interp
            for ic, c in enumerate(cases):
                rot.yaw_mode = c["yaw_mode"]
                case = {k: v for k, v in c.items() if k != "yaw_mode"}
                rot.setPosition(np.array([0.0, 0.0, 0.0, 0.0, 0.02, 0.1]))
                f0, f, a, b = rot.calcAero(dict(case))
                U, V, W, Rot = rot.IECKaimal(dict(case))
                tag = f"m{mod}_c{ic}"
                out[tag + "_f0"], out[tag + "_f"], out[tag + "_a"], out[tag + "_b"] = f0, f, a, b
                out[tag + "_kaimal"] = np.array([U, V, W, Rot])
                out[tag + "_call"] = np.array(rot.ccblade.calls[-1])
                out[tag + "_yaw"] = np.array([rot.yaw, rot.turbine_heading])
                if mod == 2:
                    out[tag + "_C"] = rot.C
        out["cases"] = np.array(json.dumps(cases))
        np.savez_compressed(os.path.join(HERE, f"rotor_{name}.npz"), **out)
        print(f"wrote rotor_{name}.npz ({len(cases)} cases x 2 modes)", file=sys.stderr)


def golden_aero():
    """Operating-rotor solves (wind > 0) of VolturnUS-S_example at its own nw = 200 grid, for
    aeroServoMod 1 and 2, with the scripted CCBlade stand-in (tests/golden/fake_ccblade.py):
    A_aero / B_aero / f_aero0 / B_gyro, Xi, iteration counts and every output channel."""
    import raft.raft_rotor as RR
    sys.path.insert(0, HERE)
    from fake_ccblade import FakeAirfoil, FakeCCBlade
    RR.CCBlade, RR.CCAirfoil = FakeCCBlade, FakeAirfoil
    if not hasattr(np, "complex_") or np.__dict__.get("complex_") is None:
        np.complex_ = np.complex128
    cases = [dict(wind_speed=10.59, wind_heading=0.0, turbulence=0.1, turbine_status="operating", yaw_misalign=0,
                  wave_spectrum="JONSWAP", wave_period=12.0, wave_height=6.0, wave_heading=0.0, wave_gamma=0.0),
             dict(wind_speed=18.0, wind_heading=20.0, turbulence="IB_NTM", turbine_status="operating", yaw_misalign=0,
                  wave_spectrum="JONSWAP", wave_period=8.0, wave_height=2.0, wave_heading=30.0, wave_gamma=0.0)]
    for mod in (1, 2):
        d = load_design(os.path.join(REF, "examples", "VolturnUS-S_example.yaml"))
        d["turbine"]["aeroServoMod"] = mod
        golden_solve(f"aero_mod{mod}", d, cases, aero=True)


def main(which):
    if "aero" in which:
        golden_aero()
    if "rotor" in which:
        golden_rotor()
    if "spectrum" in which:
        golden_f2nd_spectrum()
    if "qtf12d" in which:
        golden_qtf12d()
    if "qtf" in which:
        golden_qtf()
    if "farm" in which:
        golden_farm()
    if "sweep" in which:
        golden_sweep()
    if "designs" in which:
        export_designs()
    ex = os.path.join(REF, "examples", "VolturnUS-S_example.yaml")
    td = os.path.join(REF, "tests", "test_data")
    if "unit" in which:
        golden_fowt_unit("fowt_VolturnUS-S", os.path.join(td, "VolturnUS-S.yaml"))
        golden_fowt_unit("fowt_OC3spar", os.path.join(td, "OC3spar.yaml"))
    if "c1" in which:
        d = load_design(os.path.join(REF, "designs", "OC3spar.yaml"))
        cases = [case_dict(d, row) for row in d["cases"]["data"]]
        golden_solve("c1_OC3spar", os.path.join(REF, "designs", "OC3spar.yaml"), cases, keep_Z=True)
    if "c2small" in which:
        # VolturnUS-S example at nw=200 (min_freq 0.001 Hz, the example's own grid)
        cases = seeded_cases(8, 20241016)
        golden_solve("c2_nw200", ex, cases, keep_Z=False)
    if "c2" in which:
        # C2 grid: min_freq 0.0002 Hz, max 0.2 Hz -> nw = 1000
        cases = seeded_cases(4, 20241017)
        golden_solve("c2_nw1000", ex, cases, settings=dict(min_freq=0.0002))
    if "multi" in which:
        # two wave headings in one case (nWaves = 2, raft/raft_model.py:1049-1065)
        c = dict(wind_speed=0, wind_heading=0, turbulence=0, turbine_status="operating", yaw_misalign=0,
                 wave_spectrum=["JONSWAP", "JONSWAP"], wave_period=[12.0, 8.0], wave_height=[6.0, 2.0],
                 wave_heading=[0.0, 60.0], wave_gamma=[0.0, 2.0])
        golden_solve("multi_heading", os.path.join(td, "VolturnUS-S.yaml"), [c])


if __name__ == "__main__":
    main(sys.argv[1:] or ["designs", "unit", "c1", "c2small", "multi", "c2"])
