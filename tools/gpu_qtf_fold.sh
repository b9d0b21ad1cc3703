#!/bin/bash
# QTF path check: the GPU QTF tests (incl. sharded rows and .12d), then the C3 kernel trace and
# the C3 bench leg alone.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 120 --timeout-method thread $(grep -l "qtf\|QTF" tests/test_gpu*.py) > $OUT/qtf_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/qtf_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/qtf_tests.log | head -20; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kt_qtf2 -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py pmc > $OUT/kt_qtf2.log 2>&1
rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/kt_qtf2.log; exit $rc; fi
f=$(find $OUT/kt_qtf2 -name '*kernel_stats.csv' | head -1); grep qtf "$f" | cut -d, -f1-7 | sed 's/(rh_qtf_design[^"]*//'
cd $R
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 --no-c4 > $OUT/bench_c3.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 $OUT/bench_c3.log | cut -c1-600
exit $rc
