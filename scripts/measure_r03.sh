#!/bin/bash
# Round-3 measurement session: the bench at every config and a rocprofv3 kernel trace of each (summaries
# under gpurun_out/m03/prof_<cfg>/).  Each GPU step has its own time limit; a fault / abort / timeout (rc > 1)
# ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/m03; mkdir -p $OUT
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -c 400 $OUT/$name.log; echo
  [ $rc -le 1 ] || exit $rc
}
CFGS="${CFGS:-c2 c3_up c3_down c4_shard c5_encoder c2_prepacked c2_outlier}"
for s in ${STEPS:-bench prof}; do
  case $s in
    timing)
      B=quantized-gemm-for-transformer-inference_amd/build
      step timing_2048x512x512 300 $B/timing_quantize -m 2048 -n 512 -k 512
      step timing_2048cube 300 $B/timing_quantize -m 2048 -n 2048 -k 2048 ;;
    bench)
      for c in $CFGS; do
        if [ $c = c2 ]; then step bench_c2 300 python3 bench.py
        else step bench_$c 300 python3 bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline --cold-steps 0; fi
      done ;;
    prof)
      for c in $CFGS; do
        step prof_$c 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0
      done ;;
    pmc)
      for c in $CFGS; do
        CFG=$c step pmc_$c 600 bash scripts/pmc_bench.sh
        case $c in c3_up) D="2048 16384 4096";; c3_down) D="2048 4096 16384";; c4_shard) D="8192 4096 4096";; *) D="4096 4096 4096";; esac
        python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$c $OUT/pmc_$c.json $D > /dev/null && echo "pmc $c summarized"
      done ;;
  esac
done
echo done
