#!/bin/bash
# Round 4 (n): k_qtf_lk's coefficient blocks frequency-block-major per XCD: QTF parity tests,
# QTF timings, and the HBM bytes of the QTF launches (FETCH_SIZE / WRITE_SIZE passes).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_qtf.py tests/test_gpu_rccl.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04n_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04n_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/ubench/qtf_time.py n1 > $OUT/r04n_qtf.log 2>&1 || exit $?
timeout -k 10 120 python tools/ubench/qtf_time.py n2 >> $OUT/r04n_qtf.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/r04n_qtf.log
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT/pmc_qtfn
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_qtfn/p1 -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py pmc > $OUT/pmc_qtfn/p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_qtfn/p2 -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py pmc > $OUT/pmc_qtfn/p2.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cd $R && python tools/pmc_summary.py gpurun_out/pmc_qtfn > $OUT/pmc_qtfn.json && echo summary ok
