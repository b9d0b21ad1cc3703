#!/bin/bash
# Time the default library and every tools/ubench/var_*.so on the C2 batch (one process each).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 120 python tools/ubench/time_solve.py full || exit $?
for so in tools/ubench/var_*.so; do
  n=$(basename $so .so)
  RAFTHIP_LIB=$R/$so timeout -k 10 120 python tools/ubench/time_solve.py ${n#var_} || exit $?
done
