#!/bin/bash
# C4 A/B: the GPU suite with the candidate library (RAFTHIP_LIB=$1), then the C4 leg timed with
# each library given, alternating twice; RH_PROF libraries print their phase cycles.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
RAFTHIP_LIB=$R/$1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/c4ab_tests.log 2>&1
rc=$?; echo "pytest($1) rc=$rc"; tail -2 $OUT/c4ab_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/c4ab_tests.log | head -20; exit $rc; fi
shift
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib" >> $OUT/c4ab.log
    RAFTHIP_LIB=$R/$lib timeout -k 10 120 python tools/ubench/time_c4.py 10 >> $OUT/c4ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "time_c4 $lib rc=$rc"; tail -5 $OUT/c4ab.log; exit $rc; fi
  done
done
grep -v amdgpu.ids $OUT/c4ab.log
