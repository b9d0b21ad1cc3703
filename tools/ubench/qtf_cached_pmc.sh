# HBM bytes of a QTF with the incident-wave parts kept (tools/ubench/time_qtf.py pmc_cached):
# two rocprofv3 --pmc passes, then tools/pmc_last.py over the last 20 dispatches per kernel.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-qtfpmc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/tools/ubench/time_qtf.py pmc_cached > $O/p$i.log 2>&1 || exit 1
done
cd $R && python3 tools/pmc_last.py $O 20 qtf > $O/qtf_cached_pmc.json
