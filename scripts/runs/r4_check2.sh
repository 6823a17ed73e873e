#!/bin/bash
# round 4 check 2 (ticket-first split-K in the product): full -m gpu suite, c3_down bench + kernel trace, PMC passes
# over c3_down and c2 (traffic, hit rate, MFMA busy)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4check2; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --config c3_down --no-cpu-baseline > $out/bench_c3_down.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c3_down -o run --output-format csv -- python bench.py --config c3_down --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_c3_down.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*\|"gemm_kernel_ms": [0-9.]*' $out/bench_c3_down.log
for cfg in c3_down c2; do
  CFG=$cfg timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_$cfg.log 2>&1 || { tail $out/pmc_$cfg.log; exit 1; }
  if [ $cfg = c3_down ]; then dims="2048 4096 16384"; else dims="4096 4096 4096"; fi
  python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$cfg $out/pmc_$cfg.json $dims > $out/pmc_$cfg.sum 2>&1 || exit 1
done
echo done
