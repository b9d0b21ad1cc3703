#!/bin/bash
# Round-end GPU session: parity tests, smoke(), rocprof kernel stats of the bench (C2 + C3
# legs), the full bench line.  Every GPU step has its own time limit; a failure ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
if [ $rc -ne 0 ]; then tail -5 $OUT/bench_prof.log; exit $rc; fi
cd $R
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-400
exit $rc
