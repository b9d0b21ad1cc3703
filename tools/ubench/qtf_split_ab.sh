# k_qtf_lk's per-call choice (round 6): Kim & Yue tiles with one wave per member (kay1: never
# split), one wave per part of a member's rows (kay2: always), and the shipped rule (main:
# split up to ncu / 2 tiles per call), alternating on one box.  tools/ubench/time_qtf.py ranks
# N: rank r of N (rh_qtf_slender_rows) and the whole QTF, microseconds per call.
#   VARIANT_BASE="" tools/build_variants.sh kay1 "-DRH_KAY_SPLIT_MAX_TILES(n)=0" kay2 "-DRH_KAY_SPLIT_MAX_TILES(n)=100000"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-qtfsplit}; mkdir -p $O; cd $R
for rep in 1 2; do
  for v in kay1 kay2 main; do
    L=$R/raft-teststuff_amd/librafthip.so
    [ $v != main ] && L=$R/raft-teststuff_amd/variants/lib_$v.so
    for n in 8 4 2; do
      echo "== $v rep $rep ranks $n" >> $O/split.log
      RAFTHIP_LIB=$L timeout -k 10 120 python3 tools/ubench/time_qtf.py ranks $n >> $O/split.log 2>&1 || exit 1
    done
  done
done
