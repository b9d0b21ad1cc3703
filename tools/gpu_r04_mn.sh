#!/bin/bash
# Round 4 (m + n): the C4 excitation in the fixed point's order with XCD slices, and k_qtf_lk's
# coefficient blocks frequency-block-major per XCD.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_r04_m.sh && bash $R/tools/gpu_r04_n.sh
