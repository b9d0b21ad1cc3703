#!/bin/bash
# C2 solve A/B of the libraries given, then PC sampling of the first one (rocprofv3, beta).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT; cd $R
for rep in 1 2; do
  for lib in "$@"; do
    RAFTHIP_LIB=$R/$lib timeout -k 10 120 python tools/ubench/time_solve.py $(basename $lib) >> $OUT/ab.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "time_solve $lib rc=$rc"; tail -5 $OUT/ab.log; exit $rc; fi
  done
done
grep -v amdgpu.ids $OUT/ab.log
bash tools/gpu_pcsamp.sh $1 262144
