#!/bin/bash
# One full GPU measurement session (round artefacts):
#   1. GPU parity tests
#   2. rocprofv3 kernel-trace stats of the bench (no CPU baseline leg)
#   3. PMC passes over the C2 solve and the C3 QTF alone (one counter group per pass, never
#      combined with tracing; each pass a run of its own under a time limit)
#   4. the bench line itself (with the host-core CPU baseline)
# Every GPU step has its own time limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then tail -5 $OUT/bench_prof.log; exit $rc; fi
for wl in solve qtf; do
  i=0
  mkdir -p $OUT/pmc_$wl
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
             "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
             "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/pmc_$wl/p$i -o run --output-format csv -- python3 $R/tools/ubench/time_$wl.py pmc > $OUT/pmc_$wl/p$i.log 2>&1
    rc=$?; echo "pmc $wl pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$wl/p$i.log; exit $rc; fi
  done
done
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-300
exit $rc
