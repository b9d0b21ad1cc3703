#!/bin/bash
# Round 5 (j): the C4 step with the array excitation written by the fixed point (F_wave, no
# k_array_exc launch) and the cheap tolCheck / epilogue adopted: full GPU suite, C2 / C4
# timings, the default bench line, and a kernel trace of the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05j
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/ubench/time_solve.py lib > $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
grep -v amdgpu.ids $OUT/timing.log
timeout -k 10 300 python3 bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
