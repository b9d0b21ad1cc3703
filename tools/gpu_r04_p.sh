#!/bin/bash
# Round 4 (p): LLVM scheduler options for the whole library (variant builds of
# tools/build_variants.sh): C2-shaped solve (time_grid 1000), C4 leg, C3 QTF per library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
V=$R/raft-teststuff_amd/variants
: > $OUT/sched_ab2.log
for lib in s_base s_relax s_noclr s_base s_relax s_noclr; do
  echo "== $lib" >> $OUT/sched_ab2.log
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 200 python tools/ubench/time_grid.py 1000 >> $OUT/sched_ab2.log 2>&1 || exit $?
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 200 python tools/ubench/time_c4.py 20 >> $OUT/sched_ab2.log 2>&1 || exit $?
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python tools/ubench/qtf_time.py $lib >> $OUT/sched_ab2.log 2>&1 || exit $?
done
grep -v amdgpu.ids $OUT/sched_ab2.log
