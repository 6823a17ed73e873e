#!/bin/bash
# 8-column single-pass pack: role orders (lab/pack32_lab.hip) at the C2 and C4-shard shapes
set -o pipefail
out=gpurun_out/pack8; mkdir -p $out
for shape in "4096 4096 4096" "8192 4096 4096" "4096 4096 4096"; do
  echo "# $shape" >> $out/pack8.log
  timeout -k 10 120 lab/build/pack32_lab $shape 10 >> $out/pack8.log 2>&1 || exit 1
done
grep -E "^#|order|strip" $out/pack8.log
