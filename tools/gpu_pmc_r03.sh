#!/bin/bash
# PMC passes (one counter group per run, never with tracing) over the C2 solve, the C4 farm leg
# and the C3 QTF, then one merged per-kernel summary (tools/pmc_summary.py), plus the
# kernel-trace stats of the same three drivers.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for wl in ${WLS:-solve c4 qtf}; do
  case $wl in
    solve) cmd="$R/tools/ubench/time_solve.py pmc" ;;
    c4) cmd="$R/tools/ubench/time_c4.py 3" ;;
    qtf) cmd="$R/tools/ubench/time_qtf.py pmc" ;;
  esac
  i=0
  mkdir -p $OUT/pmc_$wl
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
             "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/pmc_$wl/p$i -o run --output-format csv -- python3 $cmd > $OUT/pmc_$wl/p$i.log 2>&1
    rc=$?; echo "pmc $wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$wl/p$i.log; exit $rc; fi
  done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_$wl -o run --output-format csv -- python3 $cmd > $OUT/kt_$wl.log 2>&1
  rc=$?; echo "trace $wl rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/kt_$wl.log; exit $rc; fi
done
cd $R
python - <<'PY'
import json, subprocess, sys
out = {}
import os
prev = os.environ.get("PMC_BASE")
if prev:
    out.update(json.load(open(prev)))
for wl in os.environ.get("WLS", "solve c4 qtf").split():
    r = subprocess.run([sys.executable, "tools/pmc_summary.py", f"gpurun_out/pmc_{wl}"], capture_output=True, text=True, check=True)
    out.update(json.loads(r.stdout))
json.dump(out, open("gpurun_out/pmc_summary.json", "w"), indent=1)
print("summary kernels:", len(out))
PY
