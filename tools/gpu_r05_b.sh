#!/bin/bash
# Round 5 (b): the GPU suite on the two-translation-unit library (max-ilp fast solve, pruned
# variants, NaN epilogue of failed cases), then the bench legs without the CPU baseline and a
# kernel trace of them.  Every GPU step has its own time limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05b
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-600
if [ $rc -ne 0 ]; then tail -20 $OUT/bench.log; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*kernel_stats.csv" | head -2
exit $rc
