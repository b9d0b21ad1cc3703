"""Debug: iteration counts and convergence margins of given C2 cases through the fast
(k_solve_lds) and general (k_solve_cases) kernels, next to the oracle's per-iteration
tolCheck maxima.  Usage: python tools/debug/flip_cases.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "raft-teststuff_amd"), ROOT]
from conftest import load_design, load_golden, statics_of  # noqa: E402


def random_cases(n, seed, headings=(0, 30, 60, 90)):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        out.append(dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)),
                        wave_height=float(rng.uniform(1, 10)), wave_heading=float(rng.choice(headings)),
                        wave_gamma=float(rng.choice([0.0, 0.0, 1.0, 3.3]))))
    return out


def main():
    import raft
    from raft import _native as N
    T = load_golden("c2_nw1000")
    d = load_design("VolturnUS-S_example")
    d["settings"]["min_freq"] = 0.0002
    m = raft.Model(d, statics=[statics_of(T)])
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    cases = random_cases(128, 99)
    want = ("psd", "std", "zeta", "B_drag", "margin")
    a = m.analyzeCasesBatch(cases, want=want)
    old = os.environ.get("RAFTHIP_OLD_ABI") == "1"     # round-1 library: process-wide knob, no margin
    if old:
        import ctypes
        N.lib().rh_set_solver.argtypes = [ctypes.c_int]
        want = ("psd", "std", "zeta", "B_drag")
        a = m.analyzeCasesBatch(cases, want=want)
        a["margin"] = np.zeros(len(cases))
    N.check(N.lib().rh_set_solver(*(() if old else (N.context(0),)), 1))
    b = m.analyzeCasesBatch(cases, want=want)
    N.check(N.lib().rh_set_solver(*(() if old else (N.context(0),)), 0))
    if old:
        b["margin"] = np.zeros(len(cases))
    diff = np.nonzero(a["iters"] != b["iters"])[0]
    print("differ:", diff.tolist())
    for ic in diff.tolist() + list(np.argsort(np.abs(a["margin"]))[:3]):
        print(ic, "fast", a["iters"][ic], a["margin"][ic], "general", b["iters"][ic], b["margin"][ic],
              "rel Xi", np.linalg.norm(a["Xi"][ic] - b["Xi"][ic]) / np.linalg.norm(a["Xi"][ic]),
              "B_drag", np.abs(a["B_drag"][ic] - b["B_drag"][ic]).max() / np.abs(a["B_drag"][ic]).max())


if __name__ == "__main__":
    main()
