#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py configs: CONFIGS="c2 c2_outlier ..." RUN=<dir under gpurun_out>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6prof}
mkdir -p $OUT
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$c -o run --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-error-stats --node-reps 0 --cold-steps 0 > $OUT/$c.log 2>&1 || exit $?
done
echo done
