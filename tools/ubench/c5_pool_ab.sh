# rh_prep_designs with and without its kept worker threads (round 6), alternating on one box:
# tools/ubench/c5_rank.py at N = 1 (16 host threads) and as rank 0 of 8 (2 threads).
#   lib_nopool: the library before the pool (threads spawned and joined per call), built by
#   VARIANT_BASE="" tools/build_variants.sh nopool "" from that source; main: the tree's library.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5pool}; mkdir -p $O; cd $R
for rep in 1 2 3; do
  for v in nopool main; do
    L=$R/raft-teststuff_amd/librafthip.so
    [ $v = nopool ] && L=$R/raft-teststuff_amd/variants/lib_nopool.so
    echo "== $v rep $rep N=1" >> $O/c5_pool.log
    RAFTHIP_LIB=$L timeout -k 10 120 python3 tools/ubench/c5_rank.py 1 >> $O/c5_pool.log 2>&1 || exit 1
    echo "== $v rep $rep rank 0 of 8" >> $O/c5_pool.log
    RAFTHIP_LIB=$L timeout -k 10 120 python3 tools/ubench/c5_rank.py 8 0 >> $O/c5_pool.log 2>&1 || exit 1
  done
done
