"""Throughput benchmark of the RAFT frequency-domain response solve on MI355X.

Workload (BASELINE.json configs[1]): examples/VolturnUS-S_example.yaml
at min_freq 0.0002 Hz -> nw = 1000 bins, 53 submerged strip nodes (20 circular +
33 rectangular), nIter = 4; a step = one batch of 512 synthetic JONSWAP sea states
(Hs~U(1,10) m, Tp~U(6,18) s, gamma 0 = IEC auto, heading in {0,30,60,90} deg), solved to
converged RAO + motion PSD in one device call.  Inputs (design tables, case parameters)
are resident in HBM before the timed region.  Multi-GPU: one process per GPU, every rank
solves its own 512-case shard (weak scaling, no collective inside the drag loop); each
step's per-case outputs (std, PSD, iteration counts) are gathered to rank 0 over RCCL on a second
stream while the next step solves (the final response-spectrum gather of north_star), and
the line also reports the same steps without the gather.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raft-teststuff_amd"))

NCASE = 512
C5_CHUNKS = 5         # C5 design blocks of a whole sweep: block k+1 is prepared on the host while block k solves


def c5_chunks(world):
    """Design blocks per rank of the C5 pipeline: C5_CHUNKS for the whole sweep, fewer for a
    rank's share at N > 1 (each block carries a fixed host cost, profiles/r06_v1/c5_rank_pacing.txt)."""
    return max(1, min(C5_CHUNKS, round(C5_CHUNKS / max(1, world) ** 0.5)))
PEAK_FP64 = 78.6e12   # MI355X FP64 dense peak (vector = matrix rate), FLOP/s
# HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE x2 per the gfx950
# correction of MI355X_MICROARCH.md + WRITE_SIZE), written by tools/pmc_summary.py
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06_v9", "pmc_summary.json")


def pmc_section(workload):
    """The per-kernel PMC records of one workload ("solve", "qtf", "c4") from PMC_SUMMARY
    (a summary with one section per workload, tools/gpu.sh pmc; older flat summaries
    serve every workload), or None."""
    try:
        with open(PMC_SUMMARY) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None
    if all(k in ("solve", "qtf", "c4") for k in d):
        return d.get(workload)
    return d


def pmc_traffic(workload, *kernels):
    """HBM traffic (bytes per call) summed over the kernels named in `kernels` (one launch
    each per call) from the `workload` section of PMC_SUMMARY, or None if any is missing."""
    d = pmc_section(workload)
    if d is None:
        return None
    total = 0.0
    for kernel in kernels:
        hit = [v for name, v in d.items()
               if kernel_name_is(name, kernel) and "hbm_read_bytes_corrected" in v and "hbm_write_bytes" in v]
        if len(hit) != 1:      # exactly one launch of exactly this kernel
            return None
        total += hit[0]["hbm_read_bytes_corrected"] + hit[0]["hbm_write_bytes"]
    return total


# FP64 FLOPs per wave-instruction counter (64 lanes): an FMA is 2 FLOPs per lane, MUL / ADD /
# transcendental 1; one SQ_INSTS_VALU_MFMA_MOPS_F64 unit is 512 FLOPs (the rocprof FLOP metric).
HW_FLOP_WEIGHTS = {"SQ_INSTS_VALU_FMA_F64": 128.0, "SQ_INSTS_VALU_MUL_F64": 64.0, "SQ_INSTS_VALU_ADD_F64": 64.0,
                   "SQ_INSTS_VALU_TRANS_F64": 64.0, "SQ_INSTS_VALU_MFMA_MOPS_F64": 512.0}


def pmc_hw_flops(workload, *kernels):
    """FP64 FLOPs the hardware executed per call (every lane of every issued FP64 VALU and MFMA
    wave-instruction, HW_FLOP_WEIGHTS), summed over `kernels` from the `workload` section of
    PMC_SUMMARY; None if a kernel or counter is missing.  Beside the formula credit of SURVEY
    §8(d): work the kernel really does, padding and recomputation included."""
    d = pmc_section(workload)
    if d is None:
        return None
    total = 0.0
    for kernel in kernels:
        hit = [v.get("counters", {}) for name, v in d.items() if kernel_name_is(name, kernel)]
        if len(hit) != 1 or not all(c in hit[0] for c in HW_FLOP_WEIGHTS):
            return None
        total += sum(w * hit[0][c] for c, w in HW_FLOP_WEIGHTS.items())
    return total


def hw_util(workload, kernels, kernel_ms):
    """{"hw_flops": per call, "hw_achieved": TFLOP/s over the measured launch time, "hw_frac"} or
    Nones when PMC_SUMMARY lacks the FP64 instruction counters."""
    f = pmc_hw_flops(workload, *kernels)
    if f is None or not kernel_ms:
        return {"hw_flops": None, "hw_achieved": None, "hw_frac": None}
    a = f / (kernel_ms * 1e-3)
    return {"hw_flops": f, "hw_achieved": a / 1e12, "hw_frac": a / PEAK_FP64}


def kernel_name_is(name, kernel):
    """Whether the demangled rocprof kernel `name` ("rh::k_qtf_kay(rh_qtf_design, ...)" or
    "void rh::k_solve_lds<2, 512, false, 1>(rh::CaseArgs)") is `kernel` exactly (a namespace-
    qualified or bare name, template arguments included when `kernel` has them): k_qtf_kay
    does not match k_qtf_kay_sum, k_solve_lds<2, 512, false does not match k_solve_lds<2, 512, false, 1>."""
    base = name.split("(")[0].strip()
    if base.startswith("void "):
        base = base[5:]
    if "<" not in kernel:
        base = base.split("<")[0]
    return base == kernel or base.endswith("::" + kernel)


# The L2 -> CU rate of the solve kernel's own kproj access pattern with no arithmetic beside it
# (tools/ubench/l2_stream.hip on the box: 512 one-per-CU workgroups, 2.5 MB per heading, lane =
# bin, buffer loads; profiles/r02_v5/l2_stream.txt): 49.5 TB/s.  The stream's ceiling, measured.
L2_PEAK = 49.5e12


def pmc_l2(kernel, kernel_ms):
    """L2 request traffic of `kernel` per launch from PMC_SUMMARY (C2 section): (TCC_HIT +
    TCC_MISS) x 128 B and its rate over the measured launch time, or None."""
    d = pmc_section("solve")
    if d is None:
        return None
    for name, v in d.items():
        c = v.get("counters", {})
        if kernel_name_is(name, kernel) and "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            b = 128.0 * (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
            rate = b / (kernel_ms * 1e-3)
            return {"bytes": b, "TB_per_s": rate / 1e12, "peak_TB_per_s": L2_PEAK / 1e12, "frac": rate / L2_PEAK,
                    "peak_note": "measured stream ceiling of this access pattern (tools/ubench/l2_stream.hip)",
                    "hit_rate": c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])}
    return None


def solve_kernels(nw):
    """Every kernel one rh_solve_cases call launches for this grid (one: the iteration-0 GEMM
    k_a0_sums of round 4 is a variant-library kernel now)."""
    return (solve_kernel_name(nw),)


def solve_kernel_name(nw):
    """The kernel rh_solve_cases launches for this grid (dispatch in rh_abi.hip)."""
    if nw <= 256:
        return f"rh::k_solve_lds<{1 if nw <= 128 else 2}, 128, true, 1>"
    if nw <= 1024:
        return f"rh::k_solve_lds<{1 if nw <= 512 else 2}, 512, false, 1>"
    return "rh::k_solve_lds<2, 512, false, 2>"      # nw <= 2048 (check_design): two passes, XiLast in Xi_last


def flops_per_case(n_loop, nw, nc, nr, nsub):
    """SURVEY.md §8(d) fixed formula: F_case = n_loop*nw*(142 Nc + 158 Nr + 1340) + nw*(100 Nsub + 1400)."""
    return n_loop * nw * (142 * nc + 158 * nr + 1340) + nw * (100 * nsub + 1400)


def build_model(device):
    import raft
    from raft import _native  # noqa: F401
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz")))
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_example.json")) as f:
        design = json.load(f)
    design["settings"]["min_freq"] = 0.0002
    statics = {k: T[k] for k in ["M_struc", "B_struc", "C_struc", "C_hydro", "C_moor"]}
    m = raft.Model(design, statics=[statics], device=device)
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    return m, f, T


def sea_states(n, seed):
    rng = np.random.default_rng(seed)
    return [dict(wave_spectrum="JONSWAP", wave_period=float(rng.uniform(6, 18)), wave_height=float(rng.uniform(1, 10)),
                 wave_heading=float(rng.choice([0, 30, 60, 90])), wave_gamma=0.0) for _ in range(n)]


def _cpu_worker(job):
    """One host-core worker of the CPU baseline (spawned before the parent touches the GPU):
    ("case", seed) -> one C2 case through oracle/raft_oracle.py loop=True;
    ("qtf", seed, seconds) -> 24-frequency QTF subsets of C3 through oracle/qtf_oracle.py."""
    os.environ["OPENBLAS_NUM_THREADS"] = os.environ["OMP_NUM_THREADS"] = "1"
    sys.path.insert(0, ROOT)
    t0 = time.perf_counter()
    if job[0] == "case":
        from oracle import raft_oracle as O
        T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz")))
        c = sea_states(1, job[1])[0]
        O.solve_dynamics(T, dict(c), int(T["nIter"]), float(T["XiStart"]), loop=True)
        return 1, time.perf_counter() - t0
    from oracle import qtf_oracle as Q
    from raft.hydro_math import wave_numbers
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c3_qtf.npz")))
    w2 = np.arange(W400[0], W400[1] + 0.5 * W400[0], W400[2]) * 2 * np.pi
    k2 = wave_numbers(w2, float(T["depth"]))
    rng = np.random.default_rng(job[1])
    pairs = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < job[2]:
        sel = np.sort(rng.choice(len(w2), 24, replace=False))
        Q.qtf_slender(T, T["out_Xi0"], w2[sel], k2[sel], 0.0)
        pairs += 24 * 25 // 2
    return pairs, time.perf_counter() - t0


def host_cores():
    """(P, note): the host cores this process may run on -- len(os.sched_getaffinity(0)), as
    SURVEY.md §8(d) prescribes -- capped by the cgroup CPU quota when one is set (a GPU box
    shows the whole machine's cores in the affinity mask but grants this job a share of
    them: more single-threaded workers than the quota would only time-slice)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            quota = max(1, int(float(q) // float(per)))
    except (OSError, ValueError):
        pass
    P = aff if quota is None else min(aff, quota)
    return P, f"affinity {aff} cores, cgroup quota {quota if quota is not None else 'none'}"


def cpu_baselines(qtf_seconds=10.0):
    """CPU baseline on the box's host cores: P = host_cores() single-
    threaded worker processes.  C2 leg: P whole cases (one per worker, ~10-20 s wall);
    QTF leg: every worker computes C3 sub-grid QTFs for `qtf_seconds`.  Wall clock."""
    import multiprocessing as mp
    P, cores_note = host_cores()
    try:
        with open("/proc/cpuinfo") as fh:
            model = next((l.split(":", 1)[1].strip() for l in fh if l.startswith("model name")), "unknown")
    except OSError:
        model = "unknown"
    ctx = mp.get_context("spawn")
    with ctx.Pool(P) as pool:
        t0 = time.perf_counter()
        res = pool.map(_cpu_worker, [("case", 99 + i) for i in range(P)], chunksize=1)
        dt = time.perf_counter() - t0
        per_case = float(np.mean([r[1] for r in res]))
        t1 = time.perf_counter()
        qres = pool.map(_cpu_worker, [("qtf", 7 + i, qtf_seconds) for i in range(P)], chunksize=1)
        dq = time.perf_counter() - t1
    npairs = sum(r[0] for r in qres)
    case = {"value": P / dt, "unit": "cases/s", "cores": P, "kind": "port",
            "sample": f"{P} C2 cases (nw=1000, seeded JONSWAP) through oracle/raft_oracle.py loop=True (the "
                      f"reference's per-node/per-bin loop structure), one per single-threaded process on {P} "
                      f"cores ({cores_note}), {dt:.1f} s wall, {per_case:.1f} s/case/core; CPU {model}",
            "calibration": "port / reference time 0.84-1.11 (mean 0.99) on the four C2 golden cases, one core, the "
                           "reference re-timed case by case beside the port (tools/calibrate_cpu.py --interleave, "
                           "profiles/r04_v2/calibrate_cpu_interleaved.txt)"}
    ratio, cal = qtf_calibration()
    qtf = {"value": npairs / dq, "unit": "pairs/s", "cores": P, "kind": "port",
           "sample": f"{npairs} pairs (24-frequency subsets of the C3 400 grid) through oracle/qtf_oracle.py "
                     f"(vectorised over pairs) on {P} cores, {dq:.1f} s wall ({cores_note}); CPU {model}",
           "calibration": f"port / reference time {ratio:.3f} on the reference's 24-frequency C3 subset (300 pairs), "
                          f"one core, the reference timed beside the port ({cal}): the port is faster than the "
                          "reference's per-pair, per-node loops, so the reference-equivalent rate on these cores is "
                          "value x ratio",
           "reference_equivalent_value": npairs / dq * ratio}
    return case, qtf


QTF_CALIBRATION = os.path.join(ROOT, "profiles", "r06_v1", "qtf_cpu_calibration.json")


def qtf_calibration():
    """(port / reference time ratio of the QTF CPU port, its source): tools/calibrate_cpu.py --qtf,
    measured in the build container where the reference runs (it does not travel to the box)."""
    with open(QTF_CALIBRATION) as fh:
        d = json.load(fh)
    return float(d["mean_ratio"]), "tools/calibrate_cpu.py --qtf, " + os.path.relpath(QTF_CALIBRATION, ROOT)


CPU_BASELINE_CACHE = os.path.join("/tmp", "raft_bench_cpu_baseline.json")


def cpu_baseline_key():
    """What a cached baseline must match: the code that produced it (this file and the oracle
    sources, by content: the GPU box has no git history) and the host-core count it ran on."""
    import hashlib
    h = hashlib.sha256()
    for rel in ["bench.py", os.path.join("oracle", "raft_oracle.py"), os.path.join("oracle", "qtf_oracle.py")]:
        with open(os.path.join(ROOT, rel), "rb") as fh:
            h.update(fh.read())
    return f"{h.hexdigest()[:16]}-P{host_cores()[0]}"


def cpu_baselines_cached(harness=False, reuse=False):
    """The CPU baseline legs for this run, measured before the process touches the GPU.
    A plain single-process run (N = 1) always times them itself and leaves them in
    CPU_BASELINE_CACHE.  reuse=True (the ranks of a torchrun-launched N > 1 run) takes that
    file instead when it was written on this host in the last 24 h by the same code and core
    count (cpu_baseline_key) -- the relaunch() parent of `--gpus N` writes it just before it
    starts the ranks, and the driver's N = 1, 2, 4, 8 series runs N = 1 first -- and times them
    itself otherwise.  Every leg says whether it was reused ("cached") and where it came from.
    harness=True (--harness-check) writes a stub instead of timing the oracle."""
    import socket
    host, key = socket.gethostname(), cpu_baseline_key()
    if reuse:
        try:
            with open(CPU_BASELINE_CACHE) as fh:
                d = json.load(fh)
            if (d.get("host") == host and d.get("key") == key and time.time() - d.get("time", 0) < 86400
                    and d.get("stub", False) == harness):
                note = (f"reused: measured {time.time() - d['time']:.0f} s earlier on this host by the same code "
                        f"(key {key}), {CPU_BASELINE_CACHE}")
                return dict(d["case"], cached=True, provenance=note), dict(d["qtf"], cached=True, provenance=note)
        except (OSError, ValueError, KeyError):
            pass
    if harness:
        case = {"value": 0.0, "unit": "cases/s", "cores": 0, "kind": "stub", "sample": "harness check: no timing"}
        qtf = dict(case, unit="pairs/s")
    else:
        case, qtf = cpu_baselines()
    with open(CPU_BASELINE_CACHE, "w") as fh:
        json.dump({"host": host, "key": key, "time": time.time(), "stub": harness, "case": case, "qtf": qtf}, fh)
    return dict(case, cached=False), dict(qtf, cached=False)


def pack_outputs(res):
    """One contiguous f64 block [n, 6 + 6 nw + 1] of a batch's per-case outputs: std, PSD and
    the iteration count (exact in f64): what the response-spectrum gather moves."""
    import torch
    n = res["std"].shape[0]
    return torch.cat([res["std"].reshape(n, -1), res["psd"].reshape(n, -1),
                      res["iters"].to(torch.float64).reshape(n, 1)], 1)


def qtf_flops_per_pair(nsub, nkay, nwl):
    """SURVEY.md §8(d) fixed formula: F_pair = 1700 Nsub + 900 N_KAYint + 800 N_wl + 200."""
    return 1700 * nsub + 900 * nkay + 800 * nwl + 200


W400 = (0.04, 0.35, 0.000825)      # C3 second-order grid [Hz]: 400 frequencies, 80,200 pairs


def build_qtf(device):
    """C3: OC4semi-RAFT_QTF slender-body QTF on the 400-frequency grid, RAO Xi0 of the
    reference's first convergence (tests/golden/c3_qtf.npz).  Returns the model pieces; the
    QtfDevice (host tables incl. the hankel1 table + upload) is built by the caller, timed."""
    import raft
    import torch
    from raft.hydro_math import wave_numbers
    T = dict(np.load(os.path.join(ROOT, "tests", "golden", "c3_qtf.npz")))
    with open(os.path.join(ROOT, "tests", "golden", "designs", "OC4semi-RAFT_QTF.json")) as fh:
        design = json.load(fh)
    design["platform"]["outFolderQTF"] = None
    statics = {k: T[k] for k in ["M_struc", "B_struc", "C_struc", "C_hydro", "C_moor"]}
    m = raft.Model(design, statics=[statics], device=device)
    f = m.fowtList[0]
    f.setPosition(T["r6"])
    f.calcStatics()
    f.calcHydroConstants()
    w2 = np.arange(W400[0], W400[1] + 0.5 * W400[0], W400[2]) * 2 * np.pi
    k2 = wave_numbers(w2, f.depth)
    dd = f.device_design()
    X = torch.tensor(T["out_Xi0"], dtype=torch.complex128, device=dd.device)
    M66 = torch.tensor(f.M_struc, dtype=torch.float64, device=dd.device).contiguous()
    return T, f, dd, X, M66, w2, k2


QTF_NEW_REPS = 9


def bench_qtf(device, steps, warmup, world, rank, dist):
    """C3 throughput: one 400x400 QTF per step (upper triangle computed, Hermitian fill), 16 x 16
    pair tiles sharded over the ranks with one all-gather of packed pairs.  end_to_end_ms: a
    QTF of a new (design, grid, heading) in a warm process, including its tables (native host
    geometry, device Hankel table) and their upload, the median of QTF_NEW_REPS such QTFs;
    first_call_ms: the first QTF of the process, which also loads the QTF kernels."""
    import torch
    from raft.qtf import QtfDevice
    T, f, dd, X, M66, w2, k2 = build_qtf(device)
    group = dist.group.WORLD if world > 1 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    qd = QtfDevice(f, w2, k2, 0.0, device)
    q = qd.qtf(dd.w, X, M66, group=group)
    torch.cuda.synchronize()
    t_first = time.perf_counter() - t0     # first QTF of the process: includes loading its kernels
    del qd, q
    e2e, tab = [], []
    for _ in range(QTF_NEW_REPS):          # a new (design, grid, heading) in a warm process: median of 9
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        qd = QtfDevice(f, w2, k2, 0.0, device)
        tab.append(time.perf_counter() - t0)
        q = qd.qtf(dd.w, X, M66, group=group)
        torch.cuda.synchronize()
        e2e.append(time.perf_counter() - t0)
    t_e2e, t_tables = float(np.median(e2e)), float(np.median(tab))
    qm = qd.host["qmemb"]
    nkay = qd.nkr - int((qm[29] != 0).sum()) if qd.nmq else 0     # KAY rows minus one waterline row per member
    nwl = int((qm[0] != 0).sum()) if qd.nmq else 0
    n2 = len(w2)
    npair = n2 * (n2 + 1) // 2
    for _ in range(warmup):
        q = qd.qtf(dd.w, X, M66, group=group)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    # value: K QTFs one after another, no timing marks between them (as the C2 leg's value);
    # then the same K with HIP events around each one's kernels, for kernel_ms and the roofline
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        q = qd.qtf(dd.w, X, M66, group=group)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt_serial = time.perf_counter() - t0   # one GPU: a QTF at a time; N GPUs: each QTF tile-sharded
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):         # kernel time: start -> this rank's rows computed (before the exchange)
        ev[i][0].record(stream)
        q = qd.qtf(dd.w, X, M66, group=group, on_computed=lambda e=ev[i][1]: e.record(stream))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    ms_marked = (time.perf_counter() - t0) / steps * 1e3
    # The QTF stream pipelined over RAFT_BENCH_QTF_STREAMS HIP streams (default 3: with the
    # 4-wave GEMM, 3 streams 1.13e9 against 1.05e9 pairs/s for 2), each with its own tables and
    # workspace (QtfDevice): one QTF's short table and coefficient launches run beside the
    # others' GEMMs.  On N GPUs every rank runs its own stream of QTFs (weak scaling, no exchange:
    # QTFs of different headings / designs are independent), reported as `streams` beside the
    # tile-sharded QTF timed above (`value`).  The pipelined outputs equal a whole QTF bit for bit.
    if world > 1:
        q = qd.qtf(dd.w, X, M66)      # this GPU's whole QTF (the check below)
    nqs = int(os.environ.get("RAFT_BENCH_QTF_STREAMS", "3"))
    qds = [qd] + [QtfDevice(f, w2, k2, 0.0, device) for _ in range(nqs - 1)]
    streams = [stream] + [torch.cuda.Stream(device) for _ in range(nqs - 1)]
    outs = [torch.empty_like(q) for _ in range(nqs)]
    for i in range(2 * nqs):
        with torch.cuda.stream(streams[i % nqs]):
            qds[i % nqs].qtf(dd.w, X, M66, out=outs[i % nqs])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        with torch.cuda.stream(streams[i % nqs]):
            qds[i % nqs].qtf(dd.w, X, M66, out=outs[i % nqs])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    assert all(torch.equal(o, q) for o in outs), "pipelined QTF differs"
    # New RAOs on one design (the second passes of potSecOrder = 1 cases, raft/second_order.py):
    # each QTF is a full QTF of its own RAO (two RAOs alternate), the incident-wave parts -- Kim &
    # Yue tables and tile sums, node GEMM basis -- kept in the workspace from the first
    # (rh_qtf_slender_ext RH_QTF_INCIDENT_CACHED; the same bits as a full call: GPU test).  One QTF
    # at a time on one GPU, as `value`.
    Xb = (X * 0.9).contiguous()
    qc = QtfDevice(f, w2, k2, 0.0, device)
    qc.qtf(dd.w, X, M66, out=outs[0])
    for i in range(warmup):
        qc.qtf(dd.w, Xb if i % 2 else X, M66, out=outs[0], incident_cached=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        qc.qtf(dd.w, Xb if i % 2 else X, M66, out=outs[0], incident_cached=True)
    torch.cuda.synchronize()
    dt_cached = time.perf_counter() - t0
    t = torch.tensor([dt, t_e2e, t_tables, t_first, dt_serial, dt_cached], dtype=torch.float64, device=f"cuda:{device}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max, e2e_max, tab_max, first_max, ser_max, cached_max = (float(x) for x in t.cpu())
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    fpp = qtf_flops_per_pair(qd.nq, nkay, nwl)
    from raft.parallel import qtf_pairs_of
    mine = qtf_pairs_of(n2, rank, world)
    achieved = fpp * mine / (ms * 1e-3)
    # value: the C3 configuration itself -- one QTF at a time, tile-sharded over the N GPUs (strong
    # scaling; N = 1: the whole QTF on one GPU), as rounds 1-4 reported it.  streams: each GPU's
    # own pipelined stream of independent QTFs (weak scaling), beside it (round 5 had made that the
    # value; ADVICE r05: the metric must not change meaning).
    out = {"metric": "QTF pairs/sec", "value": npair * steps / ser_max, "unit": "pairs/s", "steps": steps,
           "ms_per_qtf": ser_max / steps * 1e3, "ms_per_qtf_with_event_marks": ms_marked, "scaling": "strong",
           "streams": {"value": world * npair * steps / dt_max, "unit": "pairs/s", "ms_per_qtf": dt_max / steps * 1e3,
                       "scaling": "weak",
                       "pipeline": f"each GPU's independent QTFs rotate over {nqs} HIP streams with their own tables "
                                   "and workspace (no exchange)",
                       "full_grid_equiv_per_s": world * n2 * n2 * steps / dt_max},
           "same_design_new_rao": {"value": npair * steps / cached_max, "unit": "pairs/s",
                                   "ms_per_qtf": cached_max / steps * 1e3, "scaling": "per GPU",
                                   "note": "each QTF of a new RAO (two alternate) on one design, grid and "
                                           "heading, its incident-wave parts (Kim & Yue, node GEMM basis) "
                                           "kept from the design's first QTF (RH_QTF_INCIDENT_CACHED)"},
           "end_to_end_ms": e2e_max * 1e3, "host_tables_ms": tab_max * 1e3,
           "first_call_ms": first_max * 1e3,
           "n_gpus": world, "n2": n2, "pairs_per_qtf": npair,
           "full_grid_equiv_per_s": n2 * n2 * steps / ser_max,
           "config": {"workload": "C3: OC4semi-RAFT_QTF slender-body QTF, 400x400 (w1,w2) grid, heading 0",
                      "submerged_nodes": qd.nq, "kay_intervals": nkay, "waterline_members": nwl,
                      "parallelism": f"tile-sharded x{world} + all-gather of packed pairs" if world > 1 else "one GPU"},
           "roofline": {"bound": "mfma", "achieved": achieved / 1e12, "peak": PEAK_FP64 / 1e12, "unit": "TFLOP/s",
                        "frac": achieved / PEAK_FP64,
                        "traffic": pmc_traffic("qtf", "k_qtf_tables", "k_qtf_lk", "k_qtf_gemm"),
                        **hw_util("qtf", ("k_qtf_tables", "k_qtf_lk", "k_qtf_gemm"), ms),
                        "kernel": "rh_qtf_slender%s: k_qtf_tables, k_qtf_lk, k_qtf_gemm (every launch of a "
                                  "QTF on this rank)" % ("_rows" if world > 1 else ""),
                        "kernel_ms": ms, "flops_per_pair": fpp, "pairs_this_rank": mine,
                        "note": "FP64: the pair sum as MFMA GEMMs (k_qtf_gemm) + VALU Kim & Yue epilogue (DESIGN.md "
                                "§4); peak = MI355X FP64 dense (matrix = vector rate); algorithmic FLOPs from SURVEY.md "
                                "§8(d) over this rank's pairs; traffic = HBM bytes of all three launches of a QTF (PMC)"}}
    return out


def build_c4(device, ncase=512, rank=0):
    """The C4 model (farm of 2 FOWTs, fixture mooring) and its prepared batch of `ncase` sea
    states (Model.prepareArrayBatch: case table + wave tables resident in HBM)."""
    import raft
    G = dict(np.load(os.path.join(ROOT, "tests", "golden", "c4_farm.npz")))
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_farm.json")) as fh:
        design = json.load(fh)
    design.pop("array_mooring", None)                 # the array stiffness comes from the fixture
    Ts = []
    i = 0
    while f"f{i}_w" in G:
        Ts.append({k[3:]: v for k, v in G.items() if k.startswith(f"f{i}_")})
        i += 1
    m = raft.Model(design, statics=[{k: T[k] for k in ["M_struc", "B_struc", "C_struc", "C_hydro", "C_moor"]}
                                    for T in Ts], device=device)
    m.K_array = G["K_array"]
    for f, T in zip(m.fowtList, Ts):
        f.setPosition(T["r6"])
        f.calcStatics()
        f.calcHydroConstants()
    cases = sea_states(ncase, 20241020 + rank)
    return m, m.prepareArrayBatch(cases)


def bench_c4(device, steps, world, rank, dist, ncase=512):
    """C4 (BASELINE.json configs[3]): tests/test_data/VolturnUS-S_farm.yaml, 2 coupled FOWTs,
    12-DOF system per bin, nw = 240; a step = `ncase` JONSWAP sea states per GPU through
    Model.analyzeArrayBatch: every (case, FOWT) drag fixed point in one launch, the wave
    excitation, the 12x12 system solves of every (case, bin) and the per-FOWT statistics; the
    case table is prepared once (Model.prepareArrayBatch), as C2's prepare_batch.
    Mooring: the reference-run fixture (FOWT C_moor + shared-line array stiffness), the
    configuration tests/golden/c4_farm.npz pins.  Weak scaling (cases per GPU fixed)."""
    import torch
    m, P = build_c4(device, ncase, rank)
    for _ in range(20):
        r = m.analyzeArrayBatch(prepared=P, host=False)
    torch.cuda.synchronize()
    # two events per step, around the fixed-point launch; the step's device time runs from one
    # step's first mark to the next one's (`end` closes the last step).  Every timing event is a
    # barrier packet: 4 per step cost 19 us of a 0.55 ms step (tools/ubench/event_cost.py)
    # value: the K steps with no timing marks (as the C2 and QTF legs); then the same K with the
    # marks, for the fixed point's kernel time and the device time per step
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(steps)]
    end = torch.cuda.Event(enable_timing=True)
    stream = torch.cuda.current_stream()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        r = m.analyzeArrayBatch(prepared=P, host=False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=f"cuda:{device}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    for i in range(steps):
        r = m.analyzeArrayBatch(prepared=P, host=False, marks=(ev[i][0], ev[i][1]))
    end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    kern_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    step_ms = ev[0][0].elapsed_time(end) / steps   # from the first step's launch mark: host-side prep excluded
    iters = r["iters"].cpu().numpy()
    dd = m.fowtList[0].device_design()
    circ = dd.node[N_CIRC()].cpu().numpy()
    nc, nr = int((circ != 0).sum()), int((circ == 0).sum())
    flops = float(sum(flops_per_case(int(k), dd.nw, nc, nr, dd.nn) for k in iters.ravel()))
    achieved = flops / (kern_ms * 1e-3)
    return {"metric": "coupled-array sea-state cases/sec (2 FOWTs, 12-DOF system)", "value": ncase * world * steps / dt,
            "unit": "cases/s", "scaling": "weak", "n_gpus": world, "steps": steps, "ms_per_step": dt / steps * 1e3,
            "device_ms_per_step": step_ms, "iterations_mean": float(iters.mean()),
            "config": {"workload": "C4: VolturnUS-S_farm, 2 FOWTs (x = 0 / 1600 m), nw=240, JONSWAP sea states",
                       "cases_per_step_per_gpu": ncase, "nw": dd.nw, "fowts": len(m.fowtList),
                       "parallelism": f"case-sharded x{world}"},
            "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_FP64 / 1e12, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_FP64, "traffic": pmc_traffic("c4", *solve_kernels(dd.nw)),
                         **hw_util("c4", solve_kernels(dd.nw), kern_ms),
                         "kernel": solve_kernel_name(dd.nw), "kernels_timed": list(solve_kernels(dd.nw)),
                         "chain_traffic": pmc_traffic("c4", *solve_kernels(dd.nw),
                                                      f"rh::k_array_resp<2, {str(dd.nw > 256).lower()}>"),
                         "kernel_ms": kern_ms, "flops_per_launch": flops,
                         "note": "the (case, FOWT) drag fixed point (kernels_timed); SURVEY.md §8(d) formula per "
                                 "(case, FOWT); traffic = HBM bytes of those launches, chain_traffic = of the whole "
                                 "step (fixed point, which also writes the array excitation F_wave, and the block "
                                 "solve with the motion statistics) from "
                                 + os.path.relpath(PMC_SUMMARY, ROOT)}}


C5_DESIGNS = 250


def c5_base():
    """The C5 baseline design (VolturnUS-S_example at nw=1000) and its mooring stiffness."""
    with open(os.path.join(ROOT, "tests", "golden", "designs", "VolturnUS-S_example.json")) as fh:
        base = json.load(fh)
    base["settings"]["min_freq"] = 0.0002
    return base, np.load(os.path.join(ROOT, "tests", "golden", "c2_nw1000.npz"))["C_moor"]


def c5_pool(world):
    """Host workers for the C5 design preparation, started before the GPU is initialised:
    min(16, this rank's share of the cores).  Each memoises the site's dispersion solution
    (the per-site cost; the single-process path has it warm from the C2 leg)."""
    from raft import Model
    from raft.batch import host_pool
    base, _ = c5_base()
    P = max(1, min(16, host_cores()[0] // max(1, world)))
    return host_pool(P, grids=[(Model.frequency_grid(base), float(base["site"]["water_depth"]))]), P


C5_PASSES = 3
# the first design block half the size of the others: the device starts sooner (the host
# prepares the later blocks while it solves); 0.2-0.8 ms better in four A/B pairs on two boxes
# (profiles/r06_v3/c5_block_path.txt, c5_first_ab.txt)
C5_FIRST = 0.5


def bench_c5(device, steps, world, rank, dist, pool=None, nproc=1):
    """C5 (BASELINE.json configs[4]): 250 parametersweep-style VolturnUS-S_example variants
    (raft/sweep.py) x 40 sea states (Hs 2..10 x Tp 6..20) = 10,000 cases at nw = 1000.
    The design-major case list is split in contiguous blocks over the ranks; a rank prepares
    only the designs its block touches, in C5_CHUNKS design blocks pipelined by
    raft/batch.py solve_sweep (native host preparation of block k+1 while block k solves),
    and the per-case outputs (std, PSD, iterations) are all-gathered over RCCL.  End-to-end
    time = everything from the design dicts to the gathered outputs (max over ranks), the median
    of C5_PASSES timed passes (each one whole job);
    solve-only = the blocks' launches alone, repeated `steps` times.  Strong scaling (fixed 10k)."""
    import torch
    from raft.batch import solve_sweep, sweep_cases, sweep_shard
    from raft.native_prep import SweepSpecs
    from raft.parallel import gather_cases
    from raft.sweep import sea_state_grid, sweep_multipliers
    base, C_moor = c5_base()
    mult = sweep_multipliers(C5_DESIGNS)
    grid = sea_state_grid()
    idx_all, cases_all = sweep_cases(C5_DESIGNS, grid)
    n = len(idx_all)
    lo, hi, dlo, dhi = sweep_shard(idx_all, rank, world)
    # inputs: the base design and this rank's multipliers.  Each block's spec records come from
    # them inside the timed pipeline (native_prep.sweep_specs: the base record with the swept
    # member fields rewritten), so no per-variant design dict is built or parsed.
    statics = {"C_moor": C_moor}
    designs = [base] * (dhi - dlo)               # site and frequency grid only
    threads = max(1, min(16, host_cores()[0] // max(1, world)))   # (the cgroup quota, not the affinity mask)

    parsed = {}

    def specs(a, b):   # the base record is parsed at the first block of a pass (SweepSpecs), inside the timing
        if a == 0 or "ss" not in parsed:
            parsed["ss"] = SweepSpecs(base, statics=statics)
        return parsed["ss"].records(mult[dlo + a:dlo + b])
    chunks = c5_chunks(world)
    local_idx = idx_all[lo:hi] - dlo
    want = ("psd", "std")
    state_idx = np.arange(lo, hi) % len(grid)          # design-major product
    # two untimed passes first (the host workers' first tasks, allocator growth), as the
    # warmup steps of the C2 leg
    for _ in range(2):
        w_out, w_keep = solve_sweep(designs, statics, local_idx, state_idx, grid, device=device, chunks=chunks,
                                    want=want, specs=specs, threads=threads, first=C5_FIRST)
        torch.cuda.synchronize()
        del w_out, w_keep
    e2e = []
    for rep in range(C5_PASSES):       # timed passes, each the whole job; the median is reported
        if rep:
            del res, keep, out
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res, keep = solve_sweep(designs, statics, local_idx, state_idx, grid, device=device, chunks=chunks,
                                want=want, specs=specs, threads=threads, first=C5_FIRST)
        out = gather_cases({"std": res["std"], "psd": res["psd"], "iters": res["iters"]}, n, dst=0)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e2e.append(time.perf_counter() - t0)
    host_s = sum(B.host_seconds for B, _, _, _ in keep)
    # solve only: the blocks' launches again, on their prepared tables
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(steps):
        ev[i][0].record(stream)
        for B, cs, prep, _ in keep:
            B.solve(None, cs, want=want, prepared=prep)
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t_solve = (time.perf_counter() - t1) / steps
    ts = torch.tensor(e2e + [t_solve, host_s], dtype=torch.float64, device=f"cuda:{device}")
    if world > 1:
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)      # per pass: the slowest rank
    ts = ts.cpu().numpy()
    passes = ts[:C5_PASSES]
    t_e2e, t_solve, t_host = float(np.median(passes)), float(ts[C5_PASSES]), float(ts[C5_PASSES + 1])
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    iters = out["iters"].cpu().numpy()
    return {"metric": "sweep cases/sec end-to-end (design prep + solve + gather)", "value": n / t_e2e,
            "unit": "cases/s", "scaling": "strong", "cases": n, "designs": C5_DESIGNS, "sea_states": len(grid),
            "end_to_end_s": t_e2e, "end_to_end_passes_s": [float(x) for x in passes], "host_prep_s": t_host,
            "blocks": chunks,
            "solve_only_cases_per_s": n / t_solve, "solve_ms": t_solve * 1e3, "kernel_ms_rank0": kern_ms,
            "iterations_mean": float(iters.mean()),
            "config": {"workload": "C5: 250 VolturnUS-S_example parametersweep variants (5 variables U(0.75,1.25)) "
                                   "x 40 sea states, nw=1000", "nw": keep[0][0].nw,
                       "parallelism": f"case-block-sharded x{world} + gather to rank 0 (std, PSD, iterations); "
                                      f"{chunks} design blocks per rank (the first half size), host preparation of block k+1 "
                                      "overlapped with the solve of block k",
                       "host_prep_threads_per_rank": threads,
                       "design_input": "base design + per-variant multipliers; spec records built in the timed "
                                       "pipeline (raft/native_prep.py SweepSpecs)"}}


def relaunch(nproc, argv):
    """`bench.py --gpus N` started as a plain process: run it again as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a CHILD process,
    before this process touches the GPU, and return its exit code."""
    import socket
    import subprocess
    if "--no-cpu-baseline" not in argv:
        cpu_baselines_cached(harness="--harness-check" in argv)   # this process never touches the GPU: fresh
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def harness_check(args, world, rank):
    """--harness-check: the multi-rank harness without a GPU (gloo, CPU): barrier, K timed
    stub steps, max-over-ranks time, one JSON line from rank 0.  tests/test_bench.py runs it."""
    import torch
    import torch.distributed as dist
    base = None
    if rank == 0 and not args.no_cpu_baseline:
        base = cpu_baselines_cached(harness=True, reuse=world > 1)
    if world > 1:
        dist.init_process_group("gloo")
    for _ in range(args.warmup):
        time.sleep(0.001)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    gathered = 0
    for _ in range(args.steps):
        time.sleep(0.001 * (1 + rank))
        if world > 1:   # the per-step output gather (a stub block of the real one's layout)
            res = {"std": torch.zeros(4, 6, dtype=torch.float64), "psd": torch.zeros(4, 6, 8, dtype=torch.float64),
                   "iters": torch.full((4,), 4 + rank, dtype=torch.int32)}
            blk = pack_outputs(res)
            out = [torch.empty_like(blk) for _ in range(world)] if rank == 0 else None
            dist.gather(blk, gather_list=out, dst=0)
            if rank == 0:
                gathered += int((torch.cat(out, 0)[:, -1] >= 4).sum())
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        line = {"metric": "harness check", "value": args.ncase * world * args.steps / float(t.item()),
                "unit": "cases/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": float(t.item()) / args.steps * 1e3, "ranks_seen": world}
        if world > 1:
            line["gather"] = {"cases_gathered_per_step": gathered // max(1, args.steps)}
        if base is not None:
            line["cpu_baseline"] = base[0]
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=200)   # ~0.2 s: the GPU comes out of the CPU-baseline idle at full clock
    ap.add_argument("--ncase", type=int, default=NCASE)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-qtf", action="store_true")
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--no-c4", action="store_true")
    ap.add_argument("--harness-check", action="store_true", help="multi-rank harness only (gloo, no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args.gpus, sys.argv[1:]))       # N ranks, one per GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; using {world} ranks", file=sys.stderr)
    if args.harness_check:
        return harness_check(args, world, rank)
    baselines = None
    if rank == 0 and not args.no_cpu_baseline:
        baselines = cpu_baselines_cached(reuse=world > 1)   # before this process initialises the GPU
    pool, nproc = None, 1     # C5 prepares designs on native host threads (no worker pool)
    import torch
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = local
    torch.cuda.set_device(device)

    from raft.solver import CaseSet, prepare_batch, solve_batch
    m, f, T = build_model(device)
    dd = f.device_design()
    cases = sea_states(args.ncase, 20241016 + rank)          # each rank: its own shard of sea states
    cs = CaseSet(np.zeros(len(cases), dtype=np.int32), [c["wave_heading"] for c in cases],
                 ["JONSWAP"] * len(cases), [c["wave_height"] for c in cases], [c["wave_period"] for c in cases],
                 [0.0] * len(cases))
    prep = prepare_batch([dd], cs)
    want = ("psd", "std", "zeta", "rao")
    stream = torch.cuda.current_stream()
    # Pipelined steps: consecutive steps alternate between two streams, each with its own wave
    # tables (a second DeviceDesign of the same FOWT) and its own outputs, so step i + 1's tables
    # and first workgroups start on the CUs that step i's last cases leave idle (its makespan
    # tail).  Every step still tabulates and solves its whole batch.
    from raft.prep import DeviceDesign
    nstream = int(os.environ.get("RAFT_BENCH_STREAMS", "2"))
    streams = [stream] + [torch.cuda.Stream(device) for _ in range(nstream - 1)]
    dds = [dd] + [DeviceDesign(f, device=device) for _ in range(nstream - 1)]
    preps = [prep]
    for k in range(1, nstream):
        with torch.cuda.stream(streams[k]):
            preps.append(prepare_batch([dds[k]], cs))
    torch.cuda.synchronize()

    def step(e=None, k=0):
        """One C2 step on stream k: the per-heading wave tables of the design (k_wave_tables,
        all headings of the batch in one launch) and the batched drag fixed point (k_solve_lds)."""
        s = streams[k]
        with torch.cuda.stream(s):
            if e is not None:
                e[0].record(s)
            dds[k].retabulate()
            if e is not None:
                e[1].record(s)
            return solve_batch([dds[k]], cs, m.nIter, m.XiStart, 0.01, want=want, prepared=preps[k])

    comm = torch.cuda.Stream(device) if world > 1 else None

    def gather_async(res, e_done):
        """Gather of this step's packed outputs to rank 0 on the comm stream, after the solve
        (event e_done), overlapping the next step's solve on the compute stream.  A gather, not
        an all-gather: only rank 0 consumes the response spectra, and on the fully connected
        xGMI node each rank's block then crosses one link once (DESIGN.md §6 byte budget)."""
        with torch.cuda.stream(comm):
            comm.wait_event(e_done)
            blk = pack_outputs(res)
            out = [torch.empty_like(blk) for _ in range(world)] if rank == 0 else None
            g0 = torch.cuda.Event(enable_timing=True)
            g0.record(comm)
            work = dist.gather(blk, gather_list=out, dst=0, async_op=True)
        for v in res.values():
            v.record_stream(comm)
        blk.record_stream(comm)
        return work, out, g0

    # The other legs run first: the CPU baseline leaves the GPU idle for 10-20 s, and a few
    # warmup steps alone start the C2 timing below its steady-state clock (round 3: 0.938 vs
    # 0.869 ms per step with 3 vs 200 warmup steps).  The C2 protocol itself is unchanged.
    legs = {}
    if not args.no_qtf:
        legs["qtf"] = bench_qtf(device, max(20, args.steps // 4), 10, world, rank, dist)
    if not args.no_c4:
        legs["c4"] = bench_c4(device, max(3, args.steps // 2), world, rank, dist)
    if not args.no_c5:
        legs["c5"] = bench_c5(device, max(3, args.steps // 4), world, rank, dist, pool, nproc)
    for i in range(args.warmup):
        res = step(None, i % nstream)
        if world > 1:
            e = torch.cuda.Event()
            e.record(streams[i % nstream])
            w, _, _ = gather_async(res, e)
            w.wait()
    torch.cuda.synchronize()

    def timed(gather, pipelined=False):
        # serial (one stream): two events per step, before the wave tables and before the solve;
        # the solve of step i ends where step i + 1 begins (ev[i + 1][0], or `end` after the last
        # step), nothing runs between them on the stream: the kernel times of the roofline.
        # (Each timing event is a barrier packet: a third one per step cost 4 us of the 0.87 ms
        # step, tools/ubench/event_cost.py.)  pipelined: steps alternate between the two streams,
        # no per-step events; the host clock between the synchronisations times the K steps.
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
        end = torch.cuda.Event(enable_timing=True)
        pend = []
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            k = i % nstream if pipelined else 0
            r = step(None if pipelined else ev[i], k)
            if gather:
                e_done = torch.cuda.Event()
                e_done.record(streams[k])
                pend.append(gather_async(r, e_done))
        end.record(stream)
        for work, _, _ in pend:
            work.wait()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=f"cuda:{device}")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        gms = None
        if pend:
            g1 = torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(comm):
                g1.record(comm)
            torch.cuda.synchronize()
            gms = pend[-1][2].elapsed_time(g1)   # the last step's gather (nothing overlaps it)
            if rank == 0:
                out = torch.cat(pend[-1][1], 0)
                assert out.shape[0] == world * args.ncase and torch.all(out[:, -1] >= 1)
        return float(t.item()), (ev, end), r, gms

    dt_serial, (ev, end), res, _ = timed(False)
    dt_ng, _, r_pipe, _ = timed(False, pipelined=True)
    # the pipelined steps solve the same batch: the same bits as the serial pass
    assert all(torch.equal(r_pipe[k], res[k]) for k in ("iters", "std", "psd")), "pipelined C2 step differs"
    dt_max, gather_ms = dt_ng, None
    if world > 1:
        dt_max, _, _, gather_ms = timed(True, pipelined=True)
    tab_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev]))
    nxt = [e[0] for e in ev[1:]] + [end]
    kern_ms = float(np.mean([e[1].elapsed_time(n) for e, n in zip(ev, nxt)]))

    iters = res["iters"].cpu().numpy()
    status = res["status"].cpu().numpy()
    circ = dd.node[N_CIRC()].cpu().numpy() if dd.nn else np.zeros(0)
    nc, nr = int((circ != 0).sum()), int((circ == 0).sum())
    flops = float(sum(flops_per_case(int(n), dd.nw, nc, nr, dd.nn) for n in iters))
    achieved = flops / (kern_ms * 1e-3)

    total_cases = args.ncase * world * args.steps
    line = {
        "metric": "sea-state cases/sec (converged RAO+PSD)",
        "value": total_cases / dt_max,
        "unit": "cases/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C2: VolturnUS-S_example nw=1000, 512 JONSWAP sea states per GPU per step "
                               "(step = per-heading wave tables + batched drag fixed point)",
                   "cases_per_step_per_gpu": args.ncase, "nw": dd.nw, "submerged_nodes": dd.nn,
                   "nodes_circ_rect": [nc, nr], "nIter": int(m.nIter), "headings": len(dd.headings),
                   "parallelism": f"case-sharded x{world}",
                   "pipeline": f"consecutive steps rotate over {nstream} HIP streams with their own wave "
                               "tables and outputs (value, ms_per_step); kernel_ms and the roofline from a "
                               "serial pass of the same K steps on one stream",
                   "ms_per_step_serial": dt_serial / args.steps * 1e3},
        "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_FP64 / 1e12, "unit": "TFLOP/s",
                     "frac": achieved / PEAK_FP64, "traffic": pmc_traffic("solve", *solve_kernels(dd.nw)),
                     **hw_util("solve", solve_kernels(dd.nw), kern_ms),
                     "l2": pmc_l2(solve_kernel_name(dd.nw), kern_ms),
                     "kernel": solve_kernel_name(dd.nw), "kernels_timed": list(solve_kernels(dd.nw)),
                     "kernel_ms": kern_ms,
                     "wave_tables_ms": tab_ms,
                     "flops_per_launch": flops,
                     "note": "FP64 VALU bound (no MFMA, DESIGN.md §4; peak = MI355X FP64 vector rate); algorithmic "
                             "FLOPs from SURVEY.md §8(d) over the solve call's launches (kernels_timed, HIP events on "
                             "their stream); traffic = HBM bytes of those launches from "
                             + os.path.relpath(PMC_SUMMARY, ROOT)},
        "iterations_mean": float(iters.mean()),
        "converged_frac": float((status == 1).mean()),
    }
    if world > 1:
        n_out = args.ncase * (6 + 6 * dd.nw + 1) * 8
        line["gather"] = {"included_in_value": True, "value_without_gather": total_cases / dt_ng,
                          "ms_per_step_without_gather": dt_ng / args.steps * 1e3,
                          "last_gather_ms": gather_ms, "bytes_per_rank_per_step": n_out,
                          "bytes_into_rank0_per_step": (world - 1) * n_out,
                          "note": "per step: gather (RCCL) of every rank's std, PSD and iteration counts to rank 0 on a "
                                  "second stream, overlapping the next step's solve (DESIGN.md §6 byte budget)"}
    line.update(legs)
    if pool is not None:
        pool.close()
        pool.join()
    if baselines is not None:
        line["cpu_baseline"] = dict(baselines[0])
        if "qtf" in line:
            line["qtf"]["cpu_baseline"] = baselines[1]
    if rank == 0:
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def N_CIRC():
    from raft import _native as N
    return N.NF["CIRC"]


if __name__ == "__main__":
    main()
