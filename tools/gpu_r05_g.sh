#!/bin/bash
# Round 5 (g): GPU suite (member-major LDS rows in k_solve_lds, contiguous QTF tile blocks),
# per-rank QTF timing (rank r of 8 alone on one GPU), the bench legs and their kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05g
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 120 python3 tools/ubench/time_qtf.py ranks 8 > $OUT/qtf_ranks.log 2>&1 || { tail -5 $OUT/qtf_ranks.log; exit 1; }
grep -v amdgpu.ids $OUT/qtf_ranks.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400
if [ $rc -ne 0 ]; then tail -20 $OUT/bench.log; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*kernel_stats.csv" | head -2
exit $rc
