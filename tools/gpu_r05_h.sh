#!/bin/bash
# Round 5 (h): per-rank QTF timing with pair-balanced tile blocks, a kernel trace of the rank
# calls (which launch holds the per-rank time), then the round-5 PMC passes (FP64 counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05h
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 tools/ubench/time_qtf.py ranks 8 > $OUT/qtf_ranks.log 2>&1 || { tail -5 $OUT/qtf_ranks.log; exit 1; }
grep -v amdgpu.ids $OUT/qtf_ranks.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/qprof -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py ranks 8 > $OUT/qprof.log 2>&1
rc=$?; echo "qtf rocprof rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/qprof.log; exit $rc; fi
cd $R
bash tools/gpu_pmc_r05.sh > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/pmc.log
exit $rc
