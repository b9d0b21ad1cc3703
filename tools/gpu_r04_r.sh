#!/bin/bash
# Round 4 (r): the max-ilp scheduler in the bench's steady state (variant builds via RAFTHIP_LIB,
# interleaved with the default scheduler's build).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
V=$R/raft-teststuff_amd/variants
: > $OUT/ilp_steady.log
for lib in base ilp base ilp; do
  RAFTHIP_LIB=$V/lib_$lib.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-c5 > $OUT/b_$lib.log 2>&1 || exit $?
  python - "$lib" $OUT/b_$lib.log >> $OUT/ilp_steady.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], "C2 kernel_ms %.4f step %.4f" % (d["roofline"]["kernel_ms"], d["ms_per_step"]),
      "QTF %.4f" % d["qtf"]["roofline"]["kernel_ms"], "C4 fixed point %.4f step %.4f" % (d["c4"]["roofline"]["kernel_ms"], d["c4"]["ms_per_step"]))
PY
done
cat $OUT/ilp_steady.log
