#!/bin/bash
# Quick kernel iteration: all GPU parity tests, then the C2 solve timed with each library
# given as an argument (RAFTHIP_LIB), alternating twice.  Each GPU step has its own limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for lib in "$@"; do
    RAFTHIP_LIB=$R/$lib timeout -k 10 120 python tools/ubench/time_solve.py $(basename $lib) >> $OUT/ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "time_solve $lib rc=$rc"; tail -5 $OUT/ab.log; exit $rc; fi
  done
done
cat $OUT/ab.log
