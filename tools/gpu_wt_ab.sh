cd /tmp && export TMPDIR=/tmp
for l in base lib; do
  if [ $l = lib ]; then L=$GRAFT_REPO_ROOT/raft-teststuff_amd/librafthip.so; else L=$GRAFT_REPO_ROOT/raft-teststuff_amd/variants/lib_base.so; fi
  RAFTHIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/wt_$l -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ubench/time_solve.py $l || exit 1
done
