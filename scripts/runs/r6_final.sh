#!/bin/bash
# round 6 measurements of the committed tree: GPU suite, smoke, the default bench line (C2, CPU baseline included),
# the default bench under rocprofv3 --stats, every config's bench line + kernel trace, PMC passes
# for c2, c2_outlier and c3_up (RUN = output dir under gpurun_out)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${RUN:-r6final}; mkdir -p $out
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
for cfg in c2 c2_outlier c3_up; do
  CFG=$cfg timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_$cfg.log 2>&1 || { tail $out/pmc_$cfg.log; exit 1; }
  python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$cfg $out/pmc_$cfg.json $(case $cfg in c3_up) echo 2048 16384 4096;; *) echo 4096 4096 4096;; esac) > $out/pmc_$cfg.sum 2>&1 || exit 1
done
echo done
