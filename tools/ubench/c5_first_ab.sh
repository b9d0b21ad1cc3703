# C5 pipeline A/B on one box: first-block weights (C5_FIRST) of tools/ubench/c5_rank.py,
# alternating; usage: c5_first_ab.sh TAG [WEIGHTS...] (default 1 0.5)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-c5ab}; mkdir -p $O; cd $R
shift
W=${@:-1 0.5}
for rep in 1 2; do
  for f in $W; do
    C5_FIRST=$f timeout -k 10 120 python3 tools/ubench/c5_rank.py 1 >> $O/c5_first.log 2>&1 || exit 1
  done
done
