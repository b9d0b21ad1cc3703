#!/bin/bash
# rocprofv3 kernel stats of the C3 QTF (MFMA path) for each library given (RAFTHIP_LIB).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  RAFTHIP_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/qv_$n -o run --output-format csv -- python3 $R/tools/ubench/qtf_kernels.py 0 30 > $OUT/qv_$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; if [ $rc -ne 0 ]; then tail -3 $OUT/qv_$n.log; exit $rc; fi
  f=$(find $OUT/qv_$n -name '*kernel_stats.csv' | head -1); grep qtf "$f" | cut -d, -f1-7 | sed 's/(rh_qtf_design[^"]*//'
done
