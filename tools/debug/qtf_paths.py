"""MFMA pair path vs the per-pair kernel on the C3 design, with sub-structures switched off
(Kim & Yue rows, body motion, heading) to localise a disagreement.  Prints one line per variant."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    import torch
    import raft
    from raft import _native as N
    from raft.hydro_math import wave_numbers
    from raft.qtf import QtfDevice
    from conftest import load_design, load_golden, statics_of
    T = load_golden("c3_qtf")
    d = load_design("OC4semi-RAFT_QTF")
    d["platform"]["outFolderQTF"] = None
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    dd = f.device_design()
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    ctx = N.context(0)
    grids = {"n2=42": (T["w1_2nd"], T["k1_2nd"])}
    w400 = np.arange(0.04, 0.35 + 0.5 * 0.04, 0.000825) * 2 * np.pi
    grids["n2=400"] = (w400, wave_numbers(w400, f.depth))
    for gname, (w2, k2) in grids.items():
        for beta in [0.0, np.deg2rad(30.0)]:
            qd = QtfDevice(f, w2, k2, beta, 0)
            for xname, X0 in [("Xi0", T["out_Xi0"]), ("fixed", np.zeros_like(T["out_Xi0"]))]:
                X = torch.tensor(X0, dtype=torch.complex128, device=dd.device)
                for kname, nkr in [("kay", qd.nkr), ("nokay", 0)]:
                    s = qd.struct()
                    s.nkr = nkr
                    outs = []
                    for path in (1, 0):
                        N.check(N.lib().rh_set_qtf_path(ctx, path), "rh_set_qtf_path")
                        out = torch.empty([qd.n2, qd.n2, 6], dtype=torch.complex128, device=dd.device)
                        N.check(N.lib().rh_qtf_slender(ctx, ctypes.byref(s), int(dd.w.numel()), N.ptr(dd.w), N.ptr(X),
                                                       N.ptr(M66), N.ptr(out), N.ptr(qd.work),
                                                       ctypes.c_longlong(qd.work_bytes), N.stream_handle(torch, qd.dev)),
                                "rh_qtf_slender")
                        torch.cuda.synchronize()
                        outs.append(out.cpu().numpy())
                    N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")
                    a, b = outs
                    rel = np.linalg.norm(b - a) / np.linalg.norm(a)
                    per = [np.linalg.norm(b[..., k] - a[..., k]) / max(np.linalg.norm(a[..., k]), 1e-300) for k in range(6)]
                    dg = np.abs(np.diagonal(b - a)).max() / max(np.abs(a).max(), 1e-300)
                    iu = np.triu(np.ones(a.shape[:2], bool), 1)
                    up = np.abs((b - a)[iu]).max() / max(np.abs(a).max(), 1e-300)
                    print(f"{gname} beta={np.rad2deg(beta):4.0f} {xname:6s} {kname:6s} order={qd.order} rel={rel:.2e} "
                          f"diag={dg:.2e} upper={up:.2e} perDOF=" + " ".join(f"{p:.1e}" for p in per), flush=True)
    # timing of both paths at n2 = 400
    qd = QtfDevice(f, *grids["n2=400"], 0.0, 0)
    X = torch.tensor(T["out_Xi0"], dtype=torch.complex128, device=dd.device)
    for path in (1, 0):
        N.check(N.lib().rh_set_qtf_path(ctx, path), "rh_set_qtf_path")
        for _ in range(3):
            qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            qd.qtf(dd.w, X, M66)
        torch.cuda.synchronize()
        print(f"path {path}: {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms per 400x400 QTF", flush=True)
    N.check(N.lib().rh_set_qtf_path(ctx, 0), "rh_set_qtf_path")


if __name__ == "__main__":
    main()
