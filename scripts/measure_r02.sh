#!/bin/bash
# Round-2 measurement session: reference-methodology harness lines, the bench at every config, the
# rocprofv3 kernel trace of the headline bench and its PMC passes.  Each GPU step has its own time
# limit; a fault / abort / timeout (rc > 1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/m02; mkdir -p $OUT
B=quantized-gemm-for-transformer-inference_amd/build
step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "rc=$rc"; tail -c 600 $OUT/$name.log; echo
  [ $rc -le 1 ] || exit $rc
}
STEPS="${STEPS:-timing bench configs prof pmc}"
for s in $STEPS; do
  case $s in
    timing)
      step timing_2048x512x512 300 $B/timing_quantize -m 2048 -n 512 -k 512
      step timing_2048cube 300 $B/timing_quantize -m 2048 -n 2048 -k 2048 ;;
    bench) step bench_c2 300 python3 bench.py ;;
    configs)
      for c in c3_up c3_down c4_shard c5_encoder; do
        step bench_$c 300 python3 bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline --cold-steps 0
      done ;;
    prof) step prof_c2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 ;;
    pmc) CFG=c2 step pmc_c2 900 bash scripts/pmc_bench.sh
         python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/c2 $OUT/pmc_c2.json > /dev/null && echo pmc summarized ;;
  esac
done
