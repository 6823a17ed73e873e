#!/bin/bash
# kernel trace of the whole-node C4 problem on one GPU (bench.py's c4_node object: 65536 x 4096 x 4096)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4node; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 10 > $out/trace.log 2>&1 || exit 1
echo done
