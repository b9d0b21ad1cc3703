"""CPU: the bench.py multi-rank harness.  `bench.py --gpus 2` started as a plain process
re-launches itself as two ranks (torch.distributed.run, 127.0.0.1) and rank 0 prints ONE JSON
line with n_gpus 2.  --harness-check replaces the GPU work by stub steps on gloo, so the
launch, barrier, max-over-ranks timing and printing are exercised without a GPU."""
import json
import os
import subprocess
import sys

from conftest import ROOT


def _run(*argv):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip().startswith("{")]
    return lines


def test_gpus2_launches_two_ranks_one_line():
    lines = _run("--gpus", "2", "--harness-check", "--steps", "3", "--warmup", "1")
    assert len(lines) == 1, lines
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["steps"] == 3
    # the per-step output gather and the CPU baseline (measured by the relaunch() parent before
    # any rank starts; a stub in harness mode) both reach rank 0's line
    assert d["gather"]["cases_gathered_per_step"] == 8
    assert d["cpu_baseline"]["kind"] == "stub"
    # rank 1 sleeps twice as long per step: the reported time is the max over ranks
    assert d["ms_per_step"] >= 2.0


def test_gpus1_single_rank():
    lines = _run("--gpus", "1", "--harness-check", "--steps", "2", "--warmup", "0")
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 1


def test_host_cores_respects_affinity():
    sys.path.insert(0, ROOT)
    import bench
    P, note = bench.host_cores()
    assert 1 <= P <= len(os.sched_getaffinity(0)) and "affinity" in note


def test_pmc_lookup_sections_and_exact_names(tmp_path, monkeypatch):
    """pmc_traffic reads the workload's section of a sectioned summary (tools/gpu.sh pmc),
    sums exactly the named kernels (k_qtf_kay is not k_qtf_kay_sum), and returns None when a
    named kernel is absent; a flat (older) summary serves every workload."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    rec = lambda r, w: {"hbm_read_bytes_corrected": r, "hbm_write_bytes": w}   # noqa: E731
    sec = {"solve": {"rh::k_a0_sums(rh::CaseArgs)": rec(1.0, 2.0),
                     "void rh::k_solve_lds<2, 512, false, 1>(rh::CaseArgs)": rec(10.0, 20.0)},
           "c4": {"rh::k_a0_sums(rh::CaseArgs)": rec(100.0, 0.0)},
           "qtf": {"rh::k_qtf_kay(rh_qtf_design, rh::QtfWork)": rec(5.0, 5.0),
                   "rh::k_qtf_kay_sum(rh_qtf_design, rh::QtfWork)": rec(7.0, 7.0)}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(sec))
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    assert bench.pmc_traffic("solve", "rh::k_a0_sums", *bench.solve_kernels(1000)) == 33.0
    assert bench.pmc_traffic("solve", *bench.solve_kernels(1000)) == 30.0
    assert bench.pmc_traffic("c4", "rh::k_a0_sums") == 100.0
    assert bench.pmc_traffic("qtf", "k_qtf_kay") == 10.0
    assert bench.pmc_traffic("c4", *bench.solve_kernels(240)) is None
    p.write_text(json.dumps(sec["solve"]))
    assert bench.pmc_traffic("qtf", "rh::k_a0_sums") == 3.0
    assert bench.solve_kernels(2000) == ("rh::k_solve_lds<2, 512, false, 2>",)


def test_pmc_hw_flops(tmp_path, monkeypatch):
    """pmc_hw_flops weighs the FP64 instruction counters (FMA 128 FLOPs per wave-instruction,
    MUL / ADD / transcendental 64, one MFMA_MOPS_F64 unit 512) and returns None when a counter
    is missing (a summary without the FP64 pass); hw_util turns them into a rate and a fraction."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    full = {"SQ_INSTS_VALU_FMA_F64": 10.0, "SQ_INSTS_VALU_MUL_F64": 2.0, "SQ_INSTS_VALU_ADD_F64": 3.0,
            "SQ_INSTS_VALU_TRANS_F64": 1.0, "SQ_INSTS_VALU_MFMA_MOPS_F64": 4.0}
    sec = {"solve": {"void rh::k_solve_lds<2, 512, false, 1>(rh::CaseArgs)": {"counters": full}},
           "qtf": {"rh::k_qtf_gemm(x)": {"counters": dict(full, SQ_INSTS_VALU_FMA_F64=0.0)},
                   "rh::k_qtf_lk(x)": {"counters": {"SQ_INSTS_VALU_FMA_F64": 1.0}}}}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(sec))
    monkeypatch.setattr(bench, "PMC_SUMMARY", str(p))
    f = 10 * 128 + (2 + 3 + 1) * 64 + 4 * 512
    assert bench.pmc_hw_flops("solve", *bench.solve_kernels(1000)) == f
    assert bench.pmc_hw_flops("qtf", "k_qtf_gemm") == f - 10 * 128
    assert bench.pmc_hw_flops("qtf", "k_qtf_gemm", "k_qtf_lk") is None
    u = bench.hw_util("solve", bench.solve_kernels(1000), 1.0)
    assert u["hw_flops"] == f and abs(u["hw_frac"] - f / 1e-3 / bench.PEAK_FP64) < 1e-15
    assert bench.hw_util("c4", bench.solve_kernels(240), 1.0)["hw_frac"] is None
