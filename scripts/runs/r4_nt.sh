#!/bin/bash
# non-temporal pass-2 loads (FFN-down): GPU suite, c3_down bench line + kernel trace, PMC of the FFN-down call
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4nt; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --config c3_down --no-cpu-baseline > $out/bench_c3_down.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c3_down.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c3_down -o run --output-format csv -- python bench.py --config c3_down --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_c3_down.log 2>&1 || exit 1
CFG=c3_down timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_c3_down.log 2>&1 || { tail $out/pmc_c3_down.log; exit 1; }
python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/c3_down $out/pmc_c3_down.json 2048 4096 16384 > $out/pmc_c3_down.sum 2>&1 || exit 1
echo done
