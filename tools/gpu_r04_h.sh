#!/bin/bash
# Round 4 (h): motion statistics fused into k_array_resp (one case per workgroup):
# sweep/farm and QTF parity tests, a short bench (C4 leg), the kernel trace of the C4 leg.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_qtf.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04h_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04h_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 40 --warmup 40 --no-cpu-baseline --no-c5 > $OUT/r04h_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/r04h_bench.log; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof11 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-c5 > $OUT/r04h_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
