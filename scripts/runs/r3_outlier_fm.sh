#!/bin/bash
# outlier epilogue on gemm_i8_fm (f32-MFMA chain) vs the ping-pong kernel's VALU chain: parity + c2_outlier A/B
set -o pipefail
out=gpurun_out/outlier_fm; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_outlier.py > $out/pytest_fm.log 2>&1 || { tail -30 $out/pytest_fm.log; exit 1; }
tail -1 $out/pytest_fm.log
QGEMM_OUTLIER_KERNEL=pp timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_outlier.py -k "negative_zero or benched" > $out/pytest_pp.log 2>&1; tail -1 $out/pytest_pp.log
for i in 1 2; do
  for K in fm pp; do
    QGEMM_OUTLIER_KERNEL=$K timeout -k 10 120 python bench.py --config c2_outlier --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_${K}_$i.log 2>&1 || exit 1
    echo "$K $i $(grep -o '"value": [0-9.]*' $out/bench_${K}_$i.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.]*' $out/bench_${K}_$i.log | head -1)"
  done
done
