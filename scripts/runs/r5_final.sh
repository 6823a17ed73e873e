#!/bin/bash
# round 5 final measurements: GPU suite, smoke, the default bench line (C2, CPU baseline included), every config's
# bench line + kernel trace, the default bench under rocprofv3 --stats, PMC passes for c2 and c3_up
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5final; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_c2.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_c2.log 2>&1 || exit 1
for c in c3_up c3_down c4_shard c5_encoder c2_prepacked c2_outlier; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $out/bench_$c.log 2>&1 || exit 1
  grep -o '"value": [0-9.]*' $out/bench_$c.log | head -1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$c -o run --output-format csv -- python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_$c.log 2>&1 || exit 1
done
for cfg in c2 c3_up; do
  CFG=$cfg timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_$cfg.log 2>&1 || { tail $out/pmc_$cfg.log; exit 1; }
  if [ $cfg = c3_up ]; then dims="2048 16384 4096"; else dims="4096 4096 4096"; fi
  python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$cfg $out/pmc_$cfg.json $dims > $out/pmc_$cfg.sum 2>&1 || exit 1
done
echo done
