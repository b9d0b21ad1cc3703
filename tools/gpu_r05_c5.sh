#!/bin/bash
# C5 sweep: kernel trace and the HBM / L2 PMC passes of tools/ubench/c5_blocks.py (5 design blocks,
# three repetitions), to compare the per-case solve cost and traffic with C2's.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${C5OUT:-c5prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/tools/ubench/c5_blocks.py 5 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for grp in ${C5PMC:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"}; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $R/tools/ubench/c5_blocks.py 5 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
