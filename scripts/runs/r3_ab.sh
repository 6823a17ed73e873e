#!/bin/bash
# A/B of environment-selected variants on the C2 bench, interleaved: VARS="NAME=VAL ..." (one per variant,
# "-" = default), REPS rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/ab; mkdir -p $OUT
CFG=${CFG:-c2}
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARS}; do
    name=$(echo $v | tr '=' '_')
    if [ "$v" = "-" ]; then e=""; else e="$v"; fi
    env $e timeout -k 10 200 python3 bench.py --config $CFG --steps 200 --warmup 50 --no-cpu-baseline --cold-steps 0 --node-reps 0 --no-error-stats > $OUT/${name}_$r.log 2>&1
    rc=$?; [ $rc -le 1 ] || { echo "rc=$rc at $name"; exit $rc; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['gemm_kernel_ms'])" $OUT/${name}_$r.log $v $r
  done
done
