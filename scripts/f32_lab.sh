#!/bin/bash
# Lab: encoder forward with the fp32 MFMA kernel's stores (1) / MFMAs (2) disabled (QGEMM_F32_LAB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/f32lab; mkdir -p $OUT
for l in 0 1 2 3; do
  export QGEMM_F32_LAB=$l
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/l$l -o run --output-format csv -- python3 scripts/encoder_probe.py > $OUT/l$l.log 2>&1
  rc=$?; echo "lab $l rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
