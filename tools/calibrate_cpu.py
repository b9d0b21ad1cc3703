"""§8(d) calibration of the CPU baseline: the port (oracle/raft_oracle.py, loop=True, the
reference's per-node/per-bin loop structure) against the reference itself on the same four C2
golden cases (tests/golden/c2_nw1000.npz: VolturnUS-S, nw = 1000), one core each.  The
reference's per-case seconds were recorded while it generated the fixture (out_seconds,
tests/golden/make_golden.py run_solve).  Prints one line per case and the mean ratio.
--interleave: time the reference again here, case by case beside the port (tools/ref_time_c2.py in
a child process with make_golden.py's reference environment), so both see the same machine load.
--qtf: the same for the QTF port on the reference's 24-frequency C3 subset (tools/ref_time_qtf.py)."""
import json
import os
import subprocess
import sys
import time

os.environ["OPENBLAS_NUM_THREADS"] = os.environ["OMP_NUM_THREADS"] = "1"
import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import golden_cases  # noqa: E402
from oracle import raft_oracle as O  # noqa: E402


def reference_seconds(ic):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "tests", "golden", "refshim"), "/root/reference",
                                           os.path.join(ROOT, "tests", "golden")]))
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ref_time_c2.py"), str(ic)], env=env,
                       capture_output=True, text=True, check=True, cwd=ROOT)
    r = json.loads(p.stdout.strip().splitlines()[-1])
    return float(r["reference_s"]), int(r["iters"])


def calibrate_qtf(reps=3):
    """The QTF port (oracle/qtf_oracle.py, vectorised over pairs) against the reference's
    calcQTF_slenderBody (its per-pair, per-node loops) on the same 24-frequency C3 subset, one
    core each, alternating, so both see the same machine load.  The bench's QTF cpu_baseline
    reports value x mean ratio as the reference-equivalent rate."""
    from oracle import qtf_oracle as Q
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c3_qtf.npz")))
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
               PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "tests", "golden", "refshim"), "/root/reference",
                                           os.path.join(ROOT, "tests", "golden")]))
    out = []
    for rep in range(reps):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ref_time_qtf.py")], env=env,
                           capture_output=True, text=True, check=True, cwd=ROOT)
        ref = json.loads(p.stdout.strip().splitlines()[-1])
        t0 = time.perf_counter()
        q = Q.qtf_slender(T, T["out_Xi0"], T["sub400_w"], T["sub400_k"], 0.0)
        dt = time.perf_counter() - t0
        err = float(np.linalg.norm(q - T["sub400_qtf"]) / np.linalg.norm(T["sub400_qtf"]))
        out.append(dict(port_s=dt, reference_s=ref["reference_s"], ratio=dt / ref["reference_s"], port_err=err))
        print(f"rep {rep}: port {dt:6.2f} s  reference {ref['reference_s']:6.2f} s  ratio {dt / ref['reference_s']:6.3f}"
              f"  (300 pairs; port vs fixture {err:.1e})", flush=True)
    print(json.dumps({"qtf": out, "pairs": 300, "mean_ratio": float(np.mean([o["ratio"] for o in out]))}))


def main():
    if "--qtf" in sys.argv:
        return calibrate_qtf()
    interleave = "--interleave" in sys.argv
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz")))
    out = []
    for ic, case in enumerate(golden_cases(T)):
        if interleave:
            ref, its = reference_seconds(ic)
            assert its == T["out_iters"][ic]
        t0 = time.perf_counter()
        r = O.solve_dynamics(T, dict(case), int(T["nIter"]), float(T["XiStart"]), loop=True)
        dt = time.perf_counter() - t0
        if not interleave:
            ref = float(T["out_seconds"][ic])
        assert r["iters"] == T["out_iters"][ic]
        out.append(dict(case=ic, port_s=dt, reference_s=ref, ratio=dt / ref))
        print(f"case {ic}: port {dt:6.1f} s  reference {ref:6.1f} s  ratio {dt / ref:5.2f}", flush=True)
    print(json.dumps({"cases": out, "interleaved": interleave,
                      "mean_ratio": float(np.mean([o["ratio"] for o in out]))}))


if __name__ == "__main__":
    main()
