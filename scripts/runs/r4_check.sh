#!/bin/bash
# round 4 check: full -m gpu suite, smoke, bench lines (C2 default, C3 down/up) with kernel traces, LDS PMC of the
# FFN-up pack after the read-back fix
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4check; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $out/bench_c2.log 2>&1 || exit 1
for c in c3_down c3_up; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $out/bench_$c.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$c -o run --output-format csv -- python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_$c.log 2>&1 || exit 1
done
grep -ho '"value": [0-9.]*\|"gemm_kernel_ms": [0-9.]*' $out/bench_*.log
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d $out/ldsattr -o run --output-format csv -- lab/build/ldsattr_lab > $out/ldsattr.log 2>&1 || exit 1
echo done
