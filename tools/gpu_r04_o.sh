#!/bin/bash
# Round 4 (o): the QTF resample's interval from the grid step (two loads instead of a bisection):
# QTF parity tests, then QTF timings.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_qtf.py tests/test_gpu_qtf12d.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04o_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04o_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/ubench/qtf_time.py o1 > $OUT/r04o_qtf.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py o2 >> $OUT/r04o_qtf.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/r04o_qtf.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof13 -o run --output-format csv -- python3 $R/tools/ubench/qtf_time.py prof > $OUT/qtf_prof13.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
