#!/bin/bash
# Round 4: timing ablations of k_a0_sums (RH_A0_ABL) and k_array_resp (RH_ARR_ABL), variant
# libraries of tools/build_variants.sh; per-kernel times from rocprofv3 --kernel-trace --stats
# of the C2 solve (tools/ubench/time_solve.py) and the C4 step (tools/ubench/time_c4.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in a0abl0 a0abl1 a0abl2 a0abl4 a0abl7 arrabl1 arrabl2; do
  for wl in solve c4; do
    [ $wl = solve ] && arg=$lib || arg=3
    RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_$lib.so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $OUT/abl/$lib-$wl -o run --output-format csv -- python3 $R/tools/ubench/time_$wl.py $arg > $OUT/abl/$lib-$wl.log 2>&1
    rc=$?; echo "$lib $wl rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/abl/$lib-$wl.log; exit $rc; fi
  done
done
cd $R
python3 - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/abl/*/run_kernel_stats.csv")):
    tag = d.split("/")[2]
    for r in csv.DictReader(open(d)):
        if any(k in r["Name"] for k in ("k_a0_sums", "k_solve_lds", "k_array_resp")):
            print(f"{tag:18s} {r['Name'][:50]:50s} {float(r['AverageNs'])/1e3:9.1f} us  x{r['Calls']}")
PY
