#!/bin/bash
# Round 4 (b): the reworked k_a0_sums (8 waves, beta in LDS, whole row block in flight) and
# k_array_resp (member-factored excitation with a node prefetch ring): parity of the affected
# paths, A/B of the iteration-0 GEMM, and a kernel trace of the C2 / C4 bench legs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04b_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04b_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ubench/time_grid.py 1000 1000:noa0 1000 1000:noa0 200 200:noa0 > $OUT/time_grid_b.log 2>&1 || exit $?
cat $OUT/time_grid_b.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof5 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-qtf --steps 40 > $OUT/bench_prof5.log 2>&1
rc=$?; echo "rocprof rc=$rc"
exit $rc
