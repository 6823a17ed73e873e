#!/bin/bash
# outlier flags -> pack fold: the outlier GPU tests, then the c2_outlier bench line + kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4fold; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_outlier.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --config c2_outlier --no-cpu-baseline > $out/bench_c2_outlier.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2_outlier.log | head -1
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c2_outlier -o run --output-format csv -- python bench.py --config c2_outlier --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace.log 2>&1 || exit 1
echo done
