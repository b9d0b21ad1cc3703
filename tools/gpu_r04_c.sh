#!/bin/bash
# Round 4 (c): k_a0_sums with early loads and whole-row-block staging: parity of the C2/C4
# paths, A/B against per-case phase A, kernel trace, and two timing ablations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT/ablc; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04c_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04c_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ubench/time_grid.py 1000 1000:noa0 1000 1000:noa0 200 200:noa0 > $OUT/time_grid_c.log 2>&1 || exit $?
cat $OUT/time_grid_c.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof6 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-qtf --steps 40 > $OUT/bench_prof6.log 2>&1
rc=$?; echo "rocprof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in a0abl1 a0abl5; do
  RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_$lib.so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/ablc/$lib -o run --output-format csv -- python3 $R/tools/ubench/time_solve.py $lib > $OUT/ablc/$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cd $R
python3 - <<'PY'
import csv, glob
for d in sorted(glob.glob("gpurun_out/prof6/run_kernel_stats.csv") + glob.glob("gpurun_out/ablc/*/run_kernel_stats.csv")):
    for r in csv.DictReader(open(d)):
        print(f"{d.split('/')[-2]:10s} {r['Name'][:60]:60s} {float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']}")
PY
