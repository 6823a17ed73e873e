#!/bin/bash
# round-5: masked-pack cost attribution (lab/maskpack_lab.hip built with lab/maskpack_knobs_experiment.patch at
# QG_MASK_LAB_FLAGS = 0 / 1 no xo stores / 2 no wo stores / 3 neither / 4 no X-row mask loop / 8 no W-strip mask
# loop / 12 neither loop) and the GEMM's per-block stamps (w4_lab spread)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5mask2; mkdir -p $out
for f in 0 1 2 3 4 8 12; do
  echo "== QG_MASK_LAB_FLAGS=$f" >> $out/maskpack.log
  timeout -k 10 200 lab/build/maskpack_lab_f$f 4096 4096 4096 7 >> $out/maskpack.log 2>&1 || { tail $out/maskpack.log; exit 1; }
done
cat $out/maskpack.log
timeout -k 10 200 lab/build/w4_lab 4096 4096 4096 5 spread > $out/spread.log 2>&1 || { tail $out/spread.log; exit 1; }
python3 scripts/spread_analysis.py $out/spread.log | tee $out/spread_summary.txt
echo done
