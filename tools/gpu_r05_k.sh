#!/bin/bash
# Round 5 (k): F_wave stored by phase C of every iteration (no epilogue excitation sweep):
# array / parity subset, C2 and C4 timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05k
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python3 tools/ubench/time_solve.py lib >> $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/timing.log 2>&1 || { tail -5 $OUT/timing.log; exit 1; }
done
grep -v amdgpu.ids $OUT/timing.log
