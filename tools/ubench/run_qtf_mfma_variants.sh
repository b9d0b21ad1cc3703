#!/bin/bash
# total C3 QTF time of the MFMA path for the ablated libraries tools/ubench/var_[kg]*.so
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
shopt -s nullglob
timeout -k 10 120 python tools/ubench/qtf_kernels.py 0 50 || exit $?
for so in tools/ubench/var_k*.so tools/ubench/var_g*.so; do
  n=$(basename $so .so)
  printf "%s: " "${n#var_}"
  RAFTHIP_LIB=$R/$so timeout -k 10 120 python tools/ubench/qtf_kernels.py 0 50 || exit $?
done
