#!/bin/bash
# round 5 measurements of the committed tree: GPU suite, smoke, the default bench line (C2, CPU baseline included),
# the default bench under rocprofv3 --stats, every config's bench line + kernel trace, the mask-pack lab, PMC passes
# for c2 and c2_outlier
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5final; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_c2.log 2>&1 || { tail $out/bench_c2.log; exit 1; }
grep -o '"value": [0-9.]*' $out/bench_c2.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c2 -o run --output-format csv -- python bench.py --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_c2.log 2>&1 || exit 1
for c in c2_outlier c3_up c3_down c4_shard c5_encoder c2_prepacked; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $out/bench_$c.log 2>&1 || { tail $out/bench_$c.log; exit 1; }
  grep -o '"value": [0-9.]*' $out/bench_$c.log | head -1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$c -o run --output-format csv -- python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_$c.log 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/bench_c2_again.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2_again.log | head -1
timeout -k 10 200 lab/build/maskpack_lab 4096 4096 4096 7 > $out/maskpack.log 2>&1 || { tail $out/maskpack.log; exit 1; }
cat $out/maskpack.log
for cfg in c2 c2_outlier; do
  CFG=$cfg timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_$cfg.log 2>&1 || { tail $out/pmc_$cfg.log; exit 1; }
  python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$cfg $out/pmc_$cfg.json 4096 4096 4096 > $out/pmc_$cfg.sum 2>&1 || exit 1
done
echo done
