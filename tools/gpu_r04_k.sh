#!/bin/bash
# Round 4 (k): wall-clock cost of the bench's per-step timing events (C2, C4).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 300 python tools/ubench/event_cost.py > $OUT/event_cost.log 2>&1
rc=$?; echo "event_cost rc=$rc"; cat $OUT/event_cost.log; exit $rc
