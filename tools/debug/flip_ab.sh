#!/bin/bash
# A/B of the general-kernel regression: current library, the general kernel of round 1 in the
# current library (B), and the whole round-1 library.
cd ${GRAFT_REPO_ROOT:-.}
echo "== current"; timeout -k 10 120 python tools/debug/flip_cases.py || exit $?
echo "== B (round-1 general kernel)"; RAFTHIP_LIB=$PWD/raft-teststuff_amd/variants/librafthip_B.so timeout -k 10 120 python tools/debug/flip_cases.py || exit $?
echo "== round-1 library"; RAFTHIP_OLD_ABI=1 RAFTHIP_LIB=$PWD/raft-teststuff_amd/variants/librafthip_r1.so timeout -k 10 120 python tools/debug/flip_cases.py
