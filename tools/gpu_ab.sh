#!/bin/bash
# Quick kernel A/B: targeted parity tests, then ab_solve.py timing of the solver modes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread -k "${1:-agree or full_size or batch}" > $OUT/gpu_ab_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/gpu_ab_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/ubench/ab_solve.py ${2:-2,0} > $OUT/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat $OUT/ab.log | tail -5
exit $rc
