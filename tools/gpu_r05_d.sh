#!/bin/bash
# Round 5 (d): phase-C stagger and static priority A/B (C2 and C4 timings, RH_PROF phase splits),
# then the stagger library's parity subset.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05d
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
for lib in base stg prio stgprio base stg prio stgprio; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in base stg prio stgprio; do
  echo "c4 $lib" >> $OUT/ab.log
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in profbase profstg; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
grep -v amdgpu.ids $OUT/ab.log
RAFTHIP_LIB=$V/lib_stg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "fast_and_general or every_case or failed_cases or odd_grids or farm" > $OUT/stg_tests.log 2>&1
rc=$?; echo "stg parity rc=$rc"; tail -3 $OUT/stg_tests.log
exit $rc
