#!/bin/bash
# C2 bench step A/B: the GPU suite with the candidate library ($1), then the C2 leg of bench.py
# (wave tables + solve per step) with each library given, alternating twice, and one rocprof
# kernel trace per library.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
RAFTHIP_LIB=$R/$1 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/stepab_tests.log 2>&1
rc=$?; echo "pytest($1) rc=$rc"; tail -2 $OUT/stepab_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $OUT/stepab_tests.log | head -20; exit $rc; fi
shift
for rep in 1 2; do
  for lib in "$@"; do
    RAFTHIP_LIB=$R/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-qtf --no-c5 --no-c4 --steps 50 > $OUT/stepab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "bench $lib rc=$rc"; tail -5 $OUT/stepab.log; exit $rc; fi
    echo "$lib $(grep -o '"ms_per_step": [0-9.]*' $OUT/stepab.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $OUT/stepab.log | head -1)"
  done
done
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  RAFTHIP_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/st_$n -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-qtf --no-c5 --no-c4 --steps 10 > $OUT/st_$n.log 2>&1
  rc=$?; echo "trace $n rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
