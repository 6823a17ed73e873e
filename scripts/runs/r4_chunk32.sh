#!/bin/bash
# outlier flags with 32-row chunks (512 blocks) vs 64 (256 blocks): c2_outlier A/B interleaved (library swapped
# between processes), then the outlier tests on the 32-row build
set -o pipefail
out=gpurun_out/r4c32; mkdir -p $out
so=quantized-gemm-for-transformer-inference_amd/build/libqgemm.so
cp $so /tmp/libqgemm_a.so || exit 1
for i in 1 2 3; do
  cp /tmp/libqgemm_a.so $so && timeout -k 10 200 python bench.py --config c2_outlier --no-cpu-baseline > $out/a$i.log 2>&1 || exit 1
  cp lab/build/libqgemm_c32.so $so && timeout -k 10 200 python bench.py --config c2_outlier --no-cpu-baseline > $out/b$i.log 2>&1 || exit 1
  echo "a$i $(grep -o '"value": [0-9.]*' $out/a$i.log | head -1)  b$i $(grep -o '"value": [0-9.]*' $out/b$i.log | head -1)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_outlier.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_b.log 2>&1 || { tail -20 $out/pytest_b.log; exit 1; }
tail -1 $out/pytest_b.log
cp /tmp/libqgemm_a.so $so
