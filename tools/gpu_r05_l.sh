#!/bin/bash
# Round 5 (l): where the fixed point's HBM writes come from.  x0 = per-entry stores of passing
# Xi entries (round-4/5 so far), x1 = per-wave (shipped now), x2 = last-iteration stores only
# (traffic floor, wrong Xi: A/B only).  Parity subset on the shipped build, timings, then
# WRITE_SIZE passes of the C2 solve and the C4 step per variant.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05l
mkdir -p $OUT
cd $R
V=$R/raft-teststuff_amd/variants
if [ "$1" != pmc ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for lib in x0 x1 x2 x0 x1 x2; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_solve.py $lib >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
  echo "c4 $lib" >> $OUT/ab.log
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 120 python3 tools/ubench/time_c4.py 50 >> $OUT/ab.log 2>&1 || { tail -5 $OUT/ab.log; exit 1; }
done
grep -v amdgpu.ids $OUT/ab.log
fi
cd /tmp && export TMPDIR=/tmp
for lib in x0 x1 x2; do
  for wl in solve c4; do
    case $wl in solve) cmd="$R/tools/ubench/time_solve.py pmc";; c4) cmd="$R/tools/ubench/time_c4.py 2";; esac
    for grp in WRITE_SIZE FETCH_SIZE; do
      d=$OUT/pmc_${lib}_$wl/$grp
      mkdir -p $OUT/pmc_${lib}_$wl
      RAFTHIP_LIB=$V/lib_$lib.so timeout -s KILL 100 rocprofv3 --pmc $grp -d $d -o run --output-format csv -- python3 $cmd > $d.log 2>&1
      rc=$?; echo "pmc $lib $wl $grp rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $d.log; exit $rc; fi
    done
  done
done
