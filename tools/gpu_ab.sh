#!/bin/bash
# On-box A/B helper: tools/gpu_ab.sh OUTDIR [tests] [time LIBS...] [pmc LIBS...]
#   tests      the parity / sweep GPU subset on the shipped library
#   time LIBS  C2 solve and C4 step timings, twice each, per library (name = variants/lib_NAME.so,
#              "lib" = the shipped build)
#   pmc LIBS   WRITE_SIZE and FETCH_SIZE passes of the C2 solve and the C4 step per library
# Every GPU step has its own time limit; the first failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
libpath() { if [ "$1" = lib ]; then echo $R/raft-teststuff_amd/librafthip.so; else echo $V/lib_$1.so; fi; }
mode=""; tl=(); pl=(); tests=0
for a in "$@"; do
  case $a in tests) tests=1;; time) mode=t;; pmc) mode=p;; *) if [ $mode = t ]; then tl+=($a); else pl+=($a); fi;; esac
done
if [ $tests = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for lib in "${tl[@]}"; do
    RAFTHIP_LIB=$(libpath $lib) timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
    echo "c4 $lib" >> $OUT/ab.log
    RAFTHIP_LIB=$(libpath $lib) timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  done
done
[ ${#tl[@]} -gt 0 ] && grep -v amdgpu.ids $OUT/ab.log
cd /tmp && export TMPDIR=/tmp
for lib in "${pl[@]}"; do
  for wl in solve c4; do
    case $wl in solve) cmd="$R/tools/ubench/time_solve.py pmc";; c4) cmd="$R/tools/ubench/time_c4.py 2";; esac
    mkdir -p $OUT/pmc_${lib}_$wl
    for grp in WRITE_SIZE FETCH_SIZE; do
      d=$OUT/pmc_${lib}_$wl/$grp
      RAFTHIP_LIB=$(libpath $lib) timeout -s KILL 100 rocprofv3 --pmc $grp -d $d -o run --output-format csv -- python3 $cmd > $d.log 2>&1
      rc=$?; echo "pmc $lib $wl $grp rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
    done
  done
done
exit 0
