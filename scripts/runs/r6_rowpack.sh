#!/bin/bash
# round 6: 2-row pack blocks below 2 048 rows -- the lab sweep, the whole -m gpu suite, the C5 bench twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
out=gpurun_out/rowpack3; mkdir -p $out
for s in "512 1024" "512 4096" "2048 4096" "100 1000" "300 4096"; do
  timeout -k 10 60 lab/build/rowpack_lab $s 30 >> $out/lab.log 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c5_encoder --no-cpu-baseline >> $out/bench.log 2>&1 || exit 1
done
grep -E "median|DIFF" $out/lab.log | head -70
grep -o '"value": [0-9.]*' $out/bench.log
