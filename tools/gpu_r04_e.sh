#!/bin/bash
# Round 4 (e): 32 x 32 QTF GEMM tiles for a whole QTF: QTF parity tests (incl. the row-sharded
# QTF equal to the whole one bit for bit), then QTF timings: default (32 x 32), 16 x 16 tiles
# (path 2) with one accumulation chain, and with the round-3 even/odd chains (variant library).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_qtf.py tests/test_gpu_qtf12d.py tests/test_gpu_rccl.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04e_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04e_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/ubench/qtf_time.py t32 --path 2 --save $OUT/qtf_ref32.npy > $OUT/qtf_time_e.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py t16 --check $OUT/qtf_ref32.npy >> $OUT/qtf_time_e.log 2>&1 || exit $?
RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_qsplit.so timeout -k 10 120 python tools/ubench/qtf_time.py t16split --check $OUT/qtf_ref32.npy >> $OUT/qtf_time_e.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py t32b --path 2 >> $OUT/qtf_time_e.log 2>&1 || exit $?
cat $OUT/qtf_time_e.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof8 -o run --output-format csv -- python3 $R/tools/ubench/qtf_time.py prof > $OUT/qtf_prof8.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
