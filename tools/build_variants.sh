#!/bin/bash
# Build librafthip variants for on-box A/B timing (tools/ubench/time_solve.py via RAFTHIP_LIB),
# with the opt-in kernels of tools/ubench/variants_src (-DRH_VARIANTS) compiled in.
# usage: tools/build_variants.sh name "-DFLAG=.. -DFLAG2=.." [name2 "flags2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/raft-teststuff_amd/variants
pids=()
while [ $# -gt 1 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -Wno-unused-result -DRH_VARIANTS $flags \
    -o $R/raft-teststuff_amd/variants/lib_$name.so $R/raft-teststuff_amd/csrc/rh_abi.hip &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
ls -la $R/raft-teststuff_amd/variants/
