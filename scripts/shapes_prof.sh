#!/bin/bash
# Per-config bench lines + rocprofv3 kernel traces for the BASELINE shapes (c2, c3_up, c3_down,
# c4_shard), and the lab's in-kernel clock at the multi-tile GEMM shapes.  Each GPU step has its own
# time limit; any failure ends the script.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/shapes
mkdir -p $OUT
CFGS="${CFGS:-c2 c3_up c3_down c4_shard}"
for c in $CFGS; do
  echo "== $c"
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline --no-error-stats > $OUT/bench_$c.log 2>&1
  tail -1 $OUT/bench_$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['unit'],d['ms_per_step'],d.get('gemm_kernel_ms'),d['roofline']['frac'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-error-stats > $OUT/prof_$c.log 2>&1
done
if [ -n "${LAB:-}" ]; then
  for s in $LAB; do
    IFS=x read m n k <<< "$s"
    echo "== lab clock $m $n $k"
    timeout -k 10 200 lab/build/gemm_lab $m $n $k 0 clock > $OUT/labclock_$s.log 2>&1
    cat $OUT/labclock_$s.log
  done
fi
echo done
