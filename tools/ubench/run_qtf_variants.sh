#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 120 python tools/ubench/time_qtf.py full || exit $?
for so in tools/ubench/var_q*.so; do
  n=$(basename $so .so)
  RAFTHIP_LIB=$R/$so timeout -k 10 120 python tools/ubench/time_qtf.py ${n#var_} || exit $?
done
