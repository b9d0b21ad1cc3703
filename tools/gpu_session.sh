R=$GRAFT_REPO_ROOT; cd $R
true
true
for l in raft-teststuff_amd/librafthip.so tools/ubench/var_cPrefA.so tools/ubench/var_prof.so tools/ubench/var_cPrefA_prof.so; do RAFTHIP_LIB=$R/$l timeout -k 10 100 python tools/ubench/time_solve.py $(basename $l) || exit 1; done
