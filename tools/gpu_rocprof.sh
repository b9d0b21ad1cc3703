#!/bin/bash
# rocprofv3 kernel-trace stats of the bench's C2 + C3 legs only (the C5 leg launches the same
# solve kernel on 10k cases and would skew its average), then the plain bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c5 > $OUT/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 $OUT/bench_prof.log | cut -c1-200
exit $rc
