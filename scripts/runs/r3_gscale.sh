#!/bin/bash
# epilogue scales from global memory (no barrier) vs the LDS copy + barrier, 256-tile GEMM (lab)
set -o pipefail
out=gpurun_out/gscale; mkdir -p $out
for shape in "4096 4096 4096" "8192 4096 4096" "4096 4096 4096"; do
  echo "# $shape" >> $out/gscale.log
  timeout -k 10 120 lab/build/w4_lab $shape 9 stride >> $out/gscale.log 2>&1 || exit 1
done
grep -E "^#|check|f4nt  |gscale" $out/gscale.log
