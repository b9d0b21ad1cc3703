#!/bin/bash
# Round 4 (g): Kim & Yue member rows split over RH_KAY_SPLIT waves (default 2): QTF parity tests,
# then QTF timings of the default against the variants with 1 (round-4 form) and 4 waves per member.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_qtf.py tests/test_gpu_qtf12d.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04g_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04g_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
V=$R/raft-teststuff_amd/variants
RAFTHIP_LIB=$V/lib_kays1.so timeout -k 10 120 python tools/ubench/qtf_time.py s1 --save $OUT/qtf_s1.npy > $OUT/qtf_time_g.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py s2 --check $OUT/qtf_s1.npy >> $OUT/qtf_time_g.log 2>&1 || exit $?
RAFTHIP_LIB=$V/lib_kays4.so timeout -k 10 120 python tools/ubench/qtf_time.py s4 --check $OUT/qtf_s1.npy >> $OUT/qtf_time_g.log 2>&1 || exit $?
RAFTHIP_LIB=$V/lib_kays1.so timeout -k 10 120 python tools/ubench/qtf_time.py s1b >> $OUT/qtf_time_g.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py s2b >> $OUT/qtf_time_g.log 2>&1 || exit $?
cat $OUT/qtf_time_g.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof10 -o run --output-format csv -- python3 $R/tools/ubench/qtf_time.py prof > $OUT/qtf_prof10.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
