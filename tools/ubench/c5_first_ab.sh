# C5 pipeline A/B on one box: first-block weights (C5_FIRST) of tools/ubench/c5_rank.py, twice each.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5ab}; mkdir -p $O; cd $R
for f in 1 0.5 1 0.5; do
  C5_FIRST=$f timeout -k 10 120 python3 tools/ubench/c5_rank.py 1 >> $O/c5_first.log 2>&1 || exit 1
done
C5_FIRST=1 timeout -k 10 120 python3 tools/ubench/c5_rank.py 8 >> $O/c5_first.log 2>&1
