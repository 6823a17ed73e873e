#!/bin/bash
# Round-3 GPU session: parity tests, ping-pong staging A/B in the lab, a short bench.  Each GPU step has its
# own time limit; a fault / abort / timeout ends the script (test failures, rc 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -4 $OUT/$name.log
  case $rc in 0|1) return 0;; *) echo "fatal rc=$rc in $name"; exit $rc;; esac
}
for s in ${STEPS:-pytest pplab bench}; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    pytestk) run pytest_gpu_k 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${K_EXPR}" ;;
    pplab)  run pplab 240 lab/build/pp_lab 4096 4096 4096 9 pp1,pp2,pp2_nostore,pp1_nostore ;;
    pplab8) run pplab8 240 lab/build/pp_lab 8192 4096 4096 5 pp1,pp2 ;;
    ppclock) run ppclock 240 lab/build/pp_lab 4096 4096 4096 0 clock ;;
    w4)     run w4 300 lab/build/w4_lab 4096 4096 4096 7 ;;
    f4)     run f4 300 lab/build/w4_lab 4096 4096 4096 9 pp2,pp2_nostore,f4,f4_nostore,ppF,ppF_nostore ;;
    w4big)  run w4big 300 lab/build/w4_lab 8192 4096 4096 5 pp2,w4 ;;
    w4clock) run w4clock 300 lab/build/w4_lab 4096 4096 4096 0 clock ;;
    fused)  run fused 240 lab/build/fused_lab 7 ;;
    pmc)    CFG=${CFG:-c2} run pmc 900 bash scripts/pmc_bench.sh ;;
    bench)  run bench 600 python bench.py --steps 200 --warmup 50 --no-cpu-baseline --node-reps 0 --cold-steps 0 ;;
    benchfull) run benchfull 600 python bench.py ;;
    *) echo "unknown step $s";;
  esac
done
echo done
