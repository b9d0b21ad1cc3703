#!/bin/bash
# Host cost of the C2 step for each library given (RAFTHIP_LIB).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for lib in "$@"; do
  echo "== $lib"
  RAFTHIP_LIB=$R/$lib timeout -k 10 200 python tools/ubench/host_step.py 2>&1 | grep -v amdgpu.ids
  rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
done
