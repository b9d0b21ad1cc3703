#!/bin/bash
# Round 4 (i): k_qtf_lcoef + k_qtf_kay merged into one launch (k_qtf_lk, default) against two launches
# (rh_set_qtf_path 3): QTF parity tests (path 3 equals path 0 bit for bit), QTF timings 0 / 3 interleaved.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_qtf.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04i_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04i_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/ubench/qtf_time.py p0 --save $OUT/qtf_ref0.npy > $OUT/qtf_time_i.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py p3 --path 3 --check $OUT/qtf_ref0.npy >> $OUT/qtf_time_i.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py p0b >> $OUT/qtf_time_i.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py p3b --path 3 >> $OUT/qtf_time_i.log 2>&1 || exit $?
cat $OUT/qtf_time_i.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof12 -o run --output-format csv -- python3 $R/tools/ubench/qtf_time.py prof > $OUT/qtf_prof12.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
