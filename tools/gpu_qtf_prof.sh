#!/bin/bash
# rocprofv3 kernel stats of the C3 QTF on the MFMA path (tools/ubench/qtf_kernels.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/qprof -o run --output-format csv -- python3 $R/tools/ubench/qtf_kernels.py 0 50 > $OUT/qtf_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; cat $OUT/qtf_prof.log | tail -3
f=$(find $OUT/qprof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20
exit $rc
