#!/bin/bash
# Quick GPU iteration: parity tests (all, not stopping at the first failure) + one bench
# line (no CPU baseline).  Every GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_quick.log
exit $rc
