#!/bin/bash
# Build librafthip variants for on-box A/B timing (tools/ubench/time_solve.py via RAFTHIP_LIB),
# with the opt-in kernels of tools/ubench/variants_src (-DRH_VARIANTS) compiled in.  Each variant
# is the shipped build (__graft_entry__.compile_library: both translation units, their flags) plus
# the given defines.
# usage: tools/build_variants.sh name "-DFLAG=.. -DFLAG2=.." [name2 "flags2" ...]
# (VARIANT_BASE="" builds without -DRH_VARIANTS: the shipped kernels' register allocation, for A/B
# timing of a compile-time option of a shipped kernel)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/raft-teststuff_amd/variants
pids=()
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as G; G.compile_library('$R/raft-teststuff_amd/variants/lib_$name.so', '${VARIANT_BASE--DRH_VARIANTS} $flags'.split())" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la $R/raft-teststuff_amd/variants/
