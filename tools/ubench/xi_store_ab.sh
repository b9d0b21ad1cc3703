R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06xs; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in xs1 xs0 xs2; do
    RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_$v.so timeout -k 10 120 python3 tools/ubench/time_solve.py $v >> $O/xs.log 2>&1 || exit 1
  done
done
