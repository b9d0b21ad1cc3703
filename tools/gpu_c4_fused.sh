R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py -x -v -m gpu --timeout 200 --timeout-method thread > $OUT/c4_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/c4_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 40 --no-qtf --no-c5 --no-cpu-baseline > $OUT/c4_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; exit $rc
