#!/bin/bash
# Round 4 end: the QTF resample check (tools/gpu_r04_o.sh), then the round-end session
# (tools/gpu_final.sh: GPU suite, smoke, kernel stats, bench line).
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/tools/gpu_r04_o.sh && bash $R/tools/gpu_final.sh
