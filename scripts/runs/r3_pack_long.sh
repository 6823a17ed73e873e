#!/bin/bash
# single-read W pack for 4096 < K <= 16384: parity, then c3_down bench A/B (two-pass vs single read)
set -o pipefail
out=gpurun_out/pack_long; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "long_k or full_size or split_k or ragged" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for i in 1 2; do
  for L in 0 1; do
    QGEMM_PACK_LONG=$L timeout -k 10 120 python bench.py --config c3_down --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_${L}_$i.log 2>&1 || exit 1
    echo "long=$L $i $(grep -o '"value": [0-9.]*' $out/bench_${L}_$i.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.]*' $out/bench_${L}_$i.log | head -1)"
  done
done
