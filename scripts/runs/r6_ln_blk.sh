#!/bin/bash
# round 6: add + layernorm with 16-element lane blocks (one hop per block) -- lab parity/timing against the
# interleaved layout in the same binary, the encoder parity tests, then the C5 bench twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/ln_blk; mkdir -p $out
for shape in "512 1024 50" "100 1000 20" "33 8 20" "64 260 20" "3 1028 20" "5 2052 20" "7 4096 20" "9 4092 20" "2 12 20"; do
  timeout -k 10 60 lab/build/ln_lab $shape >> $out/ln_lab.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > $out/pytest.log 2>&1 || exit 1
tail -2 $out/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c5_encoder --no-cpu-baseline >> $out/bench.log 2>&1 || exit 1
done
grep -E "kernel: median|mismatch|same|DIFF|wrong" $out/ln_lab.log | head -80
grep -o '"value": [0-9.]*' $out/bench.log
