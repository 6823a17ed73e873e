#!/bin/bash
# round-5: per-block stamps of the product GEMM (w4_lab spread mode: f4 = gemm_i8_fm's loop + epilogue) at 4096^3
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5spread; mkdir -p $out
timeout -k 10 200 lab/build/w4_lab 4096 4096 4096 5 spread > $out/spread.log 2>&1 || { tail $out/spread.log; exit 1; }
python3 scripts/spread_analysis.py $out/spread.log | tee $out/spread_summary.txt
echo done
