#!/bin/bash
# Round 5 (i): A/B of the tolCheck without division / square root per entry (tol), the epilogue
# by multiplies (epi), both; then the parity subset with both.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05i
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
for lib in base tol epi both base tol epi both; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in base both; do
  echo "c4 $lib" >> $OUT/ab.log
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
grep -v amdgpu.ids $OUT/ab.log
RAFTHIP_LIB=$V/lib_both.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "fast_and_general or every_case or failed_cases or odd_grids or farm or margin or full_size" > $OUT/both_tests.log 2>&1
rc=$?; echo "both parity rc=$rc"; tail -3 $OUT/both_tests.log
exit $rc
