#!/bin/bash
# Round 3: gemm_i8_fm split-K (product) vs the ping-pong split-K kernel at FFN down, then the GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/split; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?
        echo "rc=$rc"; tail -c 700 $OUT/$name.log; echo; [ $rc -le 1 ] || exit $rc; }
run pytest_split 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "full_size or split or c3 or graph"
for i in 1 2; do
  run c3down_fm_$i 200 python bench.py --config c3_down --steps 100 --warmup 20 --no-cpu-baseline --cold-steps 0 --no-error-stats
  QGEMM_SPLIT_KERNEL=pp run c3down_pp_$i 200 python bench.py --config c3_down --steps 100 --warmup 20 --no-cpu-baseline --cold-steps 0 --no-error-stats
done
run pytest_all 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
