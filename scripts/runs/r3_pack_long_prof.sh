#!/bin/bash
# kernel trace of c3_down with the single-read W pack
set -u
export TMPDIR=/tmp
out=gpurun_out/pack_long_prof; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --config c3_down --steps 30 --warmup 5 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/prof.log 2>&1
echo "rc=$?"
f=$(find $out/prof -name "*kernel_stats.csv" | head -1); cat "$f" | cut -c1-160
