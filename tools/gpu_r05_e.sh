#!/bin/bash
# Round 5 (e): the GPU suite with the batched multi-sea-state cases, the heterogeneous farm and
# the Bmat node stride (every GPU test, one process).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05e
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $OUT/gpu_tests.log | head -30; fi
exit $rc
