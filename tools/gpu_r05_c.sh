#!/bin/bash
# Round 5 (c): the GPU suite, then A/B of the phase-C joint sweep (variant libraries built without
# -DRH_VARIANTS: base / j2 / j3, and RH_PROF phase splits), and the joint sweep's parity.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05c
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/gpu_tests.log | head -20; exit $rc; fi
for lib in base j2 j3 base j2 j3; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in profbase profj2; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
grep -v amdgpu.ids $OUT/ab.log
RAFTHIP_LIB=$V/lib_j2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "fast_and_general or every_case or failed_cases or odd_grids" > $OUT/j2_tests.log 2>&1
rc=$?; echo "j2 parity rc=$rc"; tail -3 $OUT/j2_tests.log
exit $rc
