"""CPU: the ISA gate of tools/isa_check.py on the gfx950 device code of librafthip.

Compiles rh_abi.hip to assembly (hipcc cross-compiles without a GPU) and fails on
  * dynamic register indexing (s_set_gpr_idx / v_movrel) in any kernel -- the lowering that
    faulted k_qtf_hankel on the box in round 2;
  * scratch (spill) instructions inside a streaming loop of any kernel of the shipped library,
    counted twice: with a vector-memory load in flight (vmcnt modelled; a reload there drains the
    wave-table prefetch ring every node) and anywhere in the loop.  Only the general case solve
    k_solve_cases<NB> and the single-bin small-grid k_solve_lds<1, ...> are held to ratchets of
    their measured counts; the gate refuses a ratchet entry for any other kernel."""
import os
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_isa_gate():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_check.py")], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-2000:]
    assert all(f"k_solve_lds<{k}>" in p.stdout for k in ("2, 512, false, 1", "2, 128, true, 1", "2, 512, false, 2"))
    assert "k_a0_sums" not in p.stdout and "k_qtf_gemm32" not in p.stdout   # variant kernels stay out
    assert "FAIL" not in p.stdout
    assert all(k in p.stdout for k in ("k_qtf_lk", "k_qtf_gemm", "k_array_resp<2, false>", "k_array_resp<2, true>"))
    assert "k_qtf_lcoef" not in p.stdout and "k_qtf_kay(" not in p.stdout
    ratchets = [ln for ln in p.stdout.splitlines() if "ratchet" in ln]
    assert ratchets and all("k_solve_cases<" in ln or "k_solve_lds<1," in ln for ln in ratchets), ratchets
    # the benched kernels (C2, C4 fixed points, the QTF and array solves) have no scratch in any loop
    for k in ("k_solve_lds<2, 512, false, 1>", "k_solve_lds<2, 128, true, 1>", "k_qtf_gemm", "k_qtf_lk"):
        line = next(ln for ln in p.stdout.splitlines() if k in ln)
        assert "in_flight=  0 in_loops=  0" in line, line


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_variant_build_compiles():
    """The opt-in kernels moved out of the shipped library (tools/ubench/variants_src: the
    grouped and lane-pair solves, k_a0_sums, k_qtf_gemm32, the two-launch QTF) still compile
    with -DRH_VARIANTS, as tools/build_variants.sh builds them for on-box A/B timing, so that
    code cannot rot unnoticed."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_check
    path = isa_check.compile_asm(defines=("-DRH_VARIANTS",))
    try:
        with open(path) as fh:
            names = " ".join(isa_check.demangle(n) for n in isa_check.kernels(fh.read().split("\n")))
    finally:
        os.unlink(path)
    for k in ("k_solve_grp", "k_solve_pair", "k_a0_sums", "k_qtf_gemm32", "k_qtf_lcoef", "k_qtf_kay("):
        assert k in names, k
