#!/bin/bash
# output row stride probe of the 256-tile GEMM (lab/w4_lab.hip stride mode)
set -o pipefail
out=gpurun_out/stride; mkdir -p $out
for shape in "2048 16384 4096" "8192 4096 4096" "4096 4096 4096"; do
  echo "# $shape" >> $out/stride.log
  timeout -k 10 120 lab/build/w4_lab $shape 7 stride >> $out/stride.log 2>&1 || exit 1
done
cat $out/stride.log
