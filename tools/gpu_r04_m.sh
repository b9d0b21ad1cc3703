#!/bin/bash
# Round 4 (m): C4 excitation launched in the fixed point's (design, heading) order with XCD
# slices: farm parity tests, the C4 leg, and the HBM read bytes of the C4 launches (one PMC pass).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04m_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04m_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python tools/ubench/time_c4.py 50 > $OUT/r04m_c4.log 2>&1 || exit $?
timeout -k 10 200 python tools/ubench/time_c4.py 50 >> $OUT/r04m_c4.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/r04m_c4.log
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT/pmc_c4m
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_c4m/p1 -o run --output-format csv -- python3 $R/tools/ubench/time_c4.py 2 > $OUT/pmc_c4m/p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_c4m/p2 -o run --output-format csv -- python3 $R/tools/ubench/time_c4.py 2 > $OUT/pmc_c4m/p2.log 2>&1
rc=$?; echo "pmc rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
cd $R && python tools/pmc_summary.py gpurun_out/pmc_c4m > $OUT/pmc_c4m.json && echo summary ok
