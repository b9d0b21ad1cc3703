#!/bin/bash
# Round 5 PMC of the benched library (with the FP64 VALU and FP64-MFMA instruction counters:
# the hardware FLOPs beside the formula credit, bench.py pmc_hw_flops): one counter group per rocprofv3 run (never with tracing),
# over the C2 solve, the C3 QTF and the C4 step alone; then one summary with a section per
# workload ({"solve": ..., "qtf": ..., "c4": ...}, tools/pmc_summary.py), which bench.py's
# PMC_SUMMARY points at.  Each pass has its own time limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for wl in solve qtf c4; do
  case $wl in
    solve) cmd="$R/tools/ubench/time_solve.py pmc";;
    qtf) cmd="$R/tools/ubench/time_qtf.py pmc";;
    c4) cmd="$R/tools/ubench/time_c4.py 2";;
  esac
  i=0
  mkdir -p $OUT/pmc_$wl
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
             "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 100 rocprofv3 --pmc $grp -d $OUT/pmc_$wl/p$i -o run --output-format csv -- python3 $cmd > $OUT/pmc_$wl/p$i.log 2>&1
    rc=$?; echo "pmc $wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$wl/p$i.log; exit $rc; fi
  done
done
cd $R
python - <<'PY'
import json, subprocess, sys
out = {}
for wl in ("solve", "qtf", "c4"):
    r = subprocess.run([sys.executable, "tools/pmc_summary.py", f"gpurun_out/pmc_{wl}"], capture_output=True, text=True, check=True)
    out[wl] = json.loads(r.stdout)
json.dump(out, open("gpurun_out/pmc_summary.json", "w"), indent=1)
print("summary kernels:", {k: len(v) for k, v in out.items()})
PY
