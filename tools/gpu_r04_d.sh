#!/bin/bash
# Round 4 (d): the Xi-less C4 fixed point: parity of the affected paths, then the bench's C4 and
# C2 legs under a kernel trace, then a C4-only PMC pass pair (bytes of the whole chain).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/r04d_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/r04d_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof7 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c5 --no-qtf --steps 40 > $OUT/bench_prof7.log 2>&1
rc=$?; echo "rocprof rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
mkdir -p $OUT/pmc_c4d
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $grp -d $OUT/pmc_c4d/p$i -o run --output-format csv -- python3 $R/tools/ubench/time_c4.py 2 > $OUT/pmc_c4d/p$i.log 2>&1
  rc=$?; echo "pmc c4 pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
cd $R && python3 tools/pmc_summary.py gpurun_out/pmc_c4d > gpurun_out/pmc_c4d.json && echo pmc summary ok
