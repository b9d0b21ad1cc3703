#!/bin/bash
# Round 4 (j): host cost of the C4 step (enqueue vs finish rate, cProfile of the enqueue loop).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python tools/ubench/c4_host.py > $OUT/c4_host.log 2>&1
rc=$?; echo "c4_host rc=$rc"; head -40 $OUT/c4_host.log; exit $rc
