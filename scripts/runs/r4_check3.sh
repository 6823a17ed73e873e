#!/bin/bash
# round 4 check 3 (FFN-down pack: W-only pass 1, pass 2 with X rows at its end): full -m gpu suite, c3_down bench + trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4check3; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python bench.py --config c3_down --no-cpu-baseline > $out/bench_c3_down.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_c3_down -o run --output-format csv -- python bench.py --config c3_down --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_c3_down.log 2>&1 || exit 1
grep -ho '"value": [0-9.]*\|"gemm_kernel_ms": [0-9.]*' $out/bench_c3_down.log
python3 -c "
import csv
for r in csv.DictReader(open('$out/trace_c3_down/run_kernel_stats.csv')):
    print('%-90s %8.1f' % (r['Name'][:90], float(r['AverageNs'])/1000))
"
