#!/bin/bash
# Round 5, first session: C2 solve baseline timing, the RH_PROF phase split of the round-4
# kernel, and stochastic PC sampling of the benched library (the phase split the verdict asks for).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05a
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 tools/ubench/time_solve.py base > $OUT/time_base.log 2>&1 || { cat $OUT/time_base.log; exit 1; }
cat $OUT/time_base.log
RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_prof.so timeout -k 10 120 python3 tools/ubench/time_solve.py prof > $OUT/time_prof.log 2>&1 || { cat $OUT/time_prof.log; exit 1; }
cat $OUT/time_prof.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval 65536 -d $OUT/pcs -o run --output-format csv \
  -- python3 $R/tools/ubench/time_solve.py pcs > $OUT/pcs.log 2>&1
rc=$?; echo "pcsamp rc=$rc"; tail -3 $OUT/pcs.log; find $OUT/pcs -name "*.csv" | head
exit $rc
