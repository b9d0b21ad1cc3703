cd $GRAFT_REPO_ROOT
for n in 480 496 504 510 512; do timeout -k 10 100 python tools/ubench/ab_solve.py 0 $n 2>&1 | grep mode || exit 1; done
