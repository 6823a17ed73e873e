#!/bin/bash
# K > 4096: X rows packed last (after W's two column passes) vs fused into W's column-max launch
set -u
export TMPDIR=/tmp
out=gpurun_out/xlast; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "long_k or c3_down" > $out/pytest.log 2>&1; echo "pytest rc=$?"; tail -1 $out/pytest.log
QGEMM_XLAST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "long_k or c3_down" > $out/pytest_x.log 2>&1; echo "pytest xlast rc=$?"; tail -1 $out/pytest_x.log
for i in 1 2; do
  for X in 0 1; do
    QGEMM_XLAST=$X timeout -k 10 120 python bench.py --config c3_down --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_${X}_$i.log 2>&1 || exit 1
    echo "xlast=$X $i $(grep -o '"value": [0-9.]*' $out/bench_${X}_$i.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.]*' $out/bench_${X}_$i.log | head -1)"
  done
done
QGEMM_XLAST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --config c3_down --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/prof.log 2>&1
echo "prof rc=$?"
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cut -c1-140 "$f"
