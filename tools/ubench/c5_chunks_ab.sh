# C5 per-rank design-block count A/B on one box (tools/ubench/c5_rank.py WORLD RANK THREADS CHUNKS),
# twice each, for the rank 0 share of N = 2, 4, 8 and the whole sweep at N = 1.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5chunks}; mkdir -p $O; cd $R
for rep in 1 2; do
  for wc in "1 4" "1 5" "1 6" "2 2" "2 3" "2 4" "4 1" "4 2" "4 3" "8 1" "8 2"; do
    set -- $wc
    timeout -k 10 120 python3 tools/ubench/c5_rank.py $1 0 0 $2 >> $O/c5_chunks.log 2>&1 || exit 1
  done
done
