# k_qtf_lk A/B (round 6): the library before the per-call Kim & Yue split (head, built by
#   git stash; VARIANT_BASE="" tools/build_variants.sh head ""; git stash pop) against the tree's
# (main), alternating on one box: tools/ubench/time_qtf.py ranks N (rank r of N and the whole QTF).
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06ks2; mkdir -p $O; cd $R
for rep in 1 2 3; do
  for v in head main; do
    L=$R/raft-teststuff_amd/librafthip.so
    [ $v != main ] && L=$R/raft-teststuff_amd/variants/lib_$v.so
    for n in 8 2; do
      echo "== $v rep $rep ranks $n" >> $O/split.log
      RAFTHIP_LIB=$L timeout -k 10 120 python3 tools/ubench/time_qtf.py ranks $n >> $O/split.log 2>&1 || exit 1
    done
  done
done
