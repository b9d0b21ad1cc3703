#!/bin/bash
# PMC passes over tools/ubench/ab_solve.py (both solver modes in one process, so each kernel
# gets its own per-dispatch counters); one counter group per pass, never with tracing.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/ubench/ab_solve.py ${1:-2,0} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
cd $R && python tools/pmc_summary.py gpurun_out/pmc_ab solve > $OUT/summary.json && echo summary ok
