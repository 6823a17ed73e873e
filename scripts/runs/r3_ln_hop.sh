#!/bin/bash
# layernorm lane-hop chain: lab correctness/timing over shapes, encoder parity tests, C5 bench
set -o pipefail
out=gpurun_out/ln_hop; mkdir -p $out
for shape in "512 1024 50" "100 1000 20" "33 8 20" "64 260 20" "3 1028 20" "5 2052 20" "7 4096 20"; do
  timeout -k 10 60 lab/build/ln_lab $shape >> $out/ln_lab.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_encoder.py > $out/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 120 python bench.py --config c5_encoder --steps 200 --warmup 20 >> $out/bench.log 2>&1 || exit 1
done
