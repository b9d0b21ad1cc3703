# k_array_resp A/B (round 6): the shipped kernel (A^-1 K12 slab in LDS, one workgroup per CU)
# against a version that formed the Schur complement in registers column by column (no slab),
# at one and two waves per SIMD (RH_ARR_WPE), built by
#   VARIANT_BASE="" tools/build_variants.sh arr_old "" arr_w1 "-DRH_ARR_WPE=1" arr_w2 "-DRH_ARR_WPE=2"
# (arr_w1 / arr_w2 from that version's source, not kept: DESIGN.md §5 Round 6,
# profiles/r06_v6/array_resp_ab.txt).  Per variant a kernel trace of the C4 bench leg; the
# k_array_resp<2, false> launch durations are summarised by tools/launch_durations.py.
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06arr; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
for rep in 1 2; do
  for v in arr_old arr_w1 arr_w2; do
    RAFTHIP_LIB=$R/raft-teststuff_amd/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$v.$rep -o run \
      --output-format csv -- python3 $R/tools/ubench/time_c4.py 30 > $O/$v.$rep.log 2>&1 || exit 1
    echo "== $v rep $rep: $(tail -1 $O/$v.$rep.log)"
    python3 $R/tools/launch_durations.py $O/$v.$rep/run_kernel_trace.csv "$v rep $rep" | grep -i "array\|solve_lds"
  done
done
