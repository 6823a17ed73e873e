#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.  Each GPU step has its own
# time limit; a fault / abort / timeout ends the script (test FAILURES (rc 1) do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
fatal() { case $1 in 0|1) return 1;; *) echo "fatal rc=$1 in $2"; exit $1;; esac; }
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; date
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -5 $OUT/$name.log
  fatal $rc $name || true
  return $rc
}
STEPS="${STEPS:-pytest bench prof}"
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 1200 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 600 python bench.py ;;
    benchq) run benchq 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline ;;
    prof)   run prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-error-stats ;;
    timing) run timing 600 quantized-gemm-for-transformer-inference_amd/build/timing_quantize -m 4096 -n 4096 -k 4096 -r 3 ;;
    lab)    run lab 300 lab/build/gemm_lab 4096 4096 4096 5 ;;
    *) echo "unknown step $s";;
  esac
done
echo done
