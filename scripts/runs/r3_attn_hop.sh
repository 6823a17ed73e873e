#!/bin/bash
# attention lane-hop sums: lab old/new interleaved, encoder parity tests, C5 bench
set -o pipefail
out=gpurun_out/attn_hop; mkdir -p $out
for i in 1 2; do
  timeout -k 10 60 lab/build/attn_lab_old > $out/attn_old_$i.log 2>&1 || exit 1
  timeout -k 10 60 lab/build/attn_lab > $out/attn_new_$i.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > $out/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python bench.py --config c5_encoder --steps 200 --warmup 20 >> $out/bench.log 2>&1 || exit 1
done
