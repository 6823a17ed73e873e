#!/bin/bash
# direct-load small-tile GEMM (gemm_i8_sd) vs the LDS-DMA small kernels at the encoder / small shapes
set -o pipefail
out=gpurun_out/sd_lab; mkdir -p $out
for shape in "512 3072 1024" "512 1024 1024" "512 4096 1024" "512 1024 4096" "256 1024 1024" "64 4096 4096" "128 2048 2048"; do
  echo "# $shape" >> $out/sd_lab.log
  timeout -k 10 120 lab/build/gemm_lab $shape 5 small >> $out/sd_lab.log 2>&1 || exit 1
done
