#!/bin/bash
# Stochastic PC sampling (rocprofv3, beta) of the C2 solve with the library given as $1.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RAFTHIP_LIB=$R/$1 timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval ${2:-1048576} -d $OUT/pcs -o run --output-format csv \
  -- python3 $R/tools/ubench/time_solve.py pcs > $OUT/pcs.log 2>&1
rc=$?; echo "pcsamp rc=$rc"; tail -3 $OUT/pcs.log; find $OUT/pcs -name "*.csv" | head; exit $rc
