#!/bin/bash
# 32-column single-pass pack: block -> strip orders (lab/pack32_lab.hip) at the FFN-up shape
set -o pipefail
out=gpurun_out/pack32; mkdir -p $out
timeout -k 10 120 lab/build/pack32_lab 2048 16384 4096 10 > $out/pack32.log 2>&1 || exit 1
timeout -k 10 120 lab/build/pack32_lab 2048 16384 4096 10 >> $out/pack32.log 2>&1 || exit 1
cat $out/pack32.log
