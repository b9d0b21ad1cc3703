#!/bin/bash
# Round 4 (q): the bench line under the driver's round-3 flags (--steps 20 --warmup 5) beside
# the default flags, same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20w5.log 2>&1
rc=$?; echo "bench s20w5 rc=$rc"; tail -1 $OUT/bench_s20w5.log | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1
rc=$?; echo "bench default rc=$rc"; tail -1 $OUT/bench_default.log | cut -c1-300; exit $rc
