#!/bin/bash
# Round 4: QTF launch restructure (Kim & Yue epilogue, tile sum in the GEMM epilogue) and the C4
# fused array response: parity tests, QTF timing of the default and a variant library, kernel
# trace of the bench legs.  Each GPU step has its own time limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 $OUT/r04_parity.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ubench/time_grid.py 1000 1000:noa0 1000 1000:noa0 200 200:noa0 2000 2000:noa0 2000:gen 1500 > $OUT/time_grid.log 2>&1 || exit $?
cat $OUT/time_grid.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_qtf.py tests/test_gpu_qtf12d.py tests/test_gpu_sweep.py tests/test_gpu_rccl.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/ubench/qtf_time.py default --save $OUT/qtf_ref.npy > $OUT/qtf_time.log 2>&1 || exit $?
RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_kay1.so timeout -k 10 120 python tools/ubench/qtf_time.py kay_wpe1 --check $OUT/qtf_ref.npy >> $OUT/qtf_time.log 2>&1 || exit $?
RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_qpf8.so timeout -k 10 120 python tools/ubench/qtf_time.py gemm_pf8 --check $OUT/qtf_ref.npy >> $OUT/qtf_time.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py default2 >> $OUT/qtf_time.log 2>&1 || exit $?
cat $OUT/qtf_time.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --steps 40 > $OUT/bench_prof4.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $OUT/bench_prof4.log | cut -c1-300
exit $rc
