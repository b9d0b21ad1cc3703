#!/bin/bash
# Round 5 (f): the GPU suite (multi-sea-state batch fixed: its index tensors were freed before
# the call), then A/B of the member-major LDS layout of k_solve_lds (mm: factors [nm][18] and node
# coefficients [nn][5]; mm6: [nn][6]) against the committed kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05f
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -30; exit $rc; fi
for lib in base mm mm6 base mm mm6; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in base mm mm6; do
  echo "c4 $lib" >> $OUT/ab.log
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
for lib in profbase profmm; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
grep -v amdgpu.ids $OUT/ab.log
