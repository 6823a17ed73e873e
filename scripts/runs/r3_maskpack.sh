#!/bin/bash
# masked (outlier) single-pass pack at 4 vs 5 waves per SIMD: parity + c2_outlier A/B
set -o pipefail
out=gpurun_out/maskpack; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_outlier.py > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do
  for V in 5 4; do
    QGEMM_MASKPACK_WPE=$V timeout -k 10 120 python bench.py --config c2_outlier --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_${V}_$i.log 2>&1 || exit 1
    echo "wpe=$V $i $(grep -o '"value": [0-9.]*' $out/bench_${V}_$i.log | head -1)"
  done
done
