#!/bin/bash
# Solve-kernel change: the C2/C4/C5 parity tests, then C2 timing of each library given.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_parity.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_parity.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/gpu_parity.log | head -20; exit $rc; fi
for rep in 1 2; do
  for lib in raft-teststuff_amd/librafthip.so "$@"; do
    RAFTHIP_LIB=$R/$lib timeout -k 10 120 python tools/ubench/time_solve.py $(basename $lib) >> $OUT/ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "time_solve $lib rc=$rc"; tail -5 $OUT/ab.log; exit $rc; fi
  done
done
grep -v amdgpu.ids $OUT/ab.log
