#!/bin/bash
# One parameterised GPU session (replaces the per-experiment tools/gpu_r0*_?.sh scripts):
#   tools/gpu.sh TAG STEP [STEP ...]
# runs the steps in order on the box, each under its own time limit, writing under
# gpurun_out/TAG/; the first failing step ends the session (no GPU step after a fault).
# Steps:
#   tests[=PATTERN]   pytest -m gpu (optionally -k PATTERN), tests.log
#   smoke             __graft_entry__.smoke(), smoke.log
#   bench[=ARGS]      python bench.py ARGS (commas become spaces), bench.log
#   prof[=ARGS]       rocprofv3 --kernel-trace --stats over the C2 + C3 + C4 bench legs (bench ARGS,
#                     commas become spaces; default --steps 10 --warmup 2 --no-cpu-baseline --no-c5), prof/
#   pmc[=WORKLOADS]   one rocprofv3 --pmc pass per counter group (never with tracing) over the
#                     ubench drivers of solve,qtf,c4 (default: all three), pmc_<wl>/ and the
#                     per-workload summary pmc_summary.json (tools/pmc_summary.py)
#   ubench=SCRIPT[,ARGS]  python tools/ubench/SCRIPT ARGS, ubench_<SCRIPT>.log
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?usage: tools/gpu.sh TAG STEP...}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R

run() {   # run LIMIT LOG CMD...: one GPU step under its own time limit; stop the session on failure
  local lim=$1 log=$2
  shift 2
  timeout -k 10 $lim "$@" > $log 2>&1
  local rc=$?
  echo "[$(date +%T)] $(basename $log) rc=$rc"
  if [ $rc -ne 0 ]; then tail -25 $log; exit $rc; fi
}

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$step" != "$name" ] && arg=${step#*=}
  case $name in
    tests)
      if [ -n "$arg" ]; then
        run 900 $OUT/tests.log python -u -m pytest tests -x -v -m gpu -k "$arg" --timeout 300 --timeout-method thread
      else
        run 900 $OUT/tests.log python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
      fi
      tail -1 $OUT/tests.log;;
    smoke)
      run 300 $OUT/smoke.log python3 -c "import __graft_entry__ as G; G.smoke()"
      tail -1 $OUT/smoke.log;;
    bench)
      run 400 $OUT/bench.log python3 bench.py ${arg//,/ }
      tail -1 $OUT/bench.log | cut -c1-400;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      pargs=${arg:-"--steps,10,--warmup,2,--no-cpu-baseline,--no-c5"}
      run 300 $OUT/prof.log rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
        python3 $R/bench.py ${pargs//,/ }
      cd $R;;
    pmc)
      wls=${arg:-solve,qtf,c4}
      cd /tmp && export TMPDIR=/tmp
      for wl in ${wls//,/ }; do
        case $wl in
          solve) cmd="$R/tools/ubench/time_solve.py pmc";;
          qtf) cmd="$R/tools/ubench/time_qtf.py pmc";;
          c4) cmd="$R/tools/ubench/time_c4.py 2";;
          *) echo "unknown pmc workload $wl"; exit 2;;
        esac
        mkdir -p $OUT/pmc_$wl
        i=0
        for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
                   "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM" \
                   "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
                   "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE"; do
          i=$((i+1))
          timeout -s KILL 100 rocprofv3 --pmc $grp -d $OUT/pmc_$wl/p$i -o run --output-format csv -- python3 $cmd \
            > $OUT/pmc_$wl/p$i.log 2>&1
          rc=$?; echo "pmc $wl pass $i rc=$rc"
          if [ $rc -ne 0 ]; then tail -5 $OUT/pmc_$wl/p$i.log; exit $rc; fi
        done
      done
      cd $R
      python3 - "$OUT" "$wls" <<'PY'
import json, subprocess, sys
out_dir, wls = sys.argv[1], sys.argv[2].split(",")
out = {}
for wl in wls:
    r = subprocess.run([sys.executable, "tools/pmc_summary.py", f"{out_dir}/pmc_{wl}"], capture_output=True, text=True,
                       check=True)
    out[wl] = json.loads(r.stdout)
json.dump(out, open(f"{out_dir}/pmc_summary.json", "w"), indent=1)
print("pmc summary:", {k: len(v) for k, v in out.items()})
PY
      ;;
    ubench)
      script=${arg%%,*}
      rest=""
      [ "$arg" != "$script" ] && rest=${arg#*,}
      run 300 $OUT/ubench_${script%.py}.log python3 tools/ubench/$script ${rest//,/ }
      tail -3 $OUT/ubench_${script%.py}.log;;
    *)
      echo "unknown step $step"; exit 2;;
  esac
done
echo "session $TAG done"
