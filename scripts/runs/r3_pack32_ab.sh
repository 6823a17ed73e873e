#!/bin/bash
# 32-column pack strip order: parity at the FFN-up shape, then c3_up bench A/B (xcd order vs grouped order)
set -o pipefail
out=gpurun_out/pack32_ab; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "full_size or wide or single_pass" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do
  for O in xcd grouped; do
    QGEMM_PACK32_ORDER=$O timeout -k 10 120 python bench.py --config c3_up --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_${O}_$i.log 2>&1 || exit 1
    echo "$O $i $(grep -o '"value": [0-9.]*' $out/bench_${O}_$i.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.]*' $out/bench_${O}_$i.log | head -1)"
  done
done
