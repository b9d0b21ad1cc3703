#!/bin/bash
# One GPU session: parity tests, kernel-trace profile of the bench, bench line.
# Every GPU step has its own time limit; a crash/timeout ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 $OUT/bench_prof.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log
exit $rc
