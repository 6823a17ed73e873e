#!/bin/bash
# Lab: the encoder forward under each forced fp32-MFMA configuration (QGEMM_F32_CFG), kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/f32probe; mkdir -p $OUT
for c in ${CFGS:-0 2 3 4 5 8 9 10 11 12}; do
  export QGEMM_F32_CFG=$c
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c$c -o run --output-format csv -- python3 scripts/encoder_probe.py > $OUT/c$c.log 2>&1
  rc=$?; echo "cfg $c rc=$rc $(grep forwards $OUT/c$c.log)"
  [ $rc -eq 0 ] || exit $rc
done
