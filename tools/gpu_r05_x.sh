#!/bin/bash
# Round 5 (x): per-rank QTF (rank r of 8, rh_qtf_slender_rows) and whole-QTF timings for the
# Kim & Yue row split (RH_KAY_SPLIT 1 / 2 / 4), with a kernel trace of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05x
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in base ks2; do
  echo "== $lib" >> $OUT/ranks.log
  RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_$lib.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_$lib -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py ranks 8 >> $OUT/ranks.log 2>&1 || { tail -5 $OUT/ranks.log; exit 1; }
done
grep -E "==|rank|whole" $OUT/ranks.log
