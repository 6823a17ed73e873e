#!/bin/bash
# PMC passes over GEMM lab variants (counters in separate passes, kernel-trace only; no sys/runtime trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc; mkdir -p $OUT
LAB=lab/build/gemm_lab
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for V in ${VARIANTS:-v3p_nostore v5_s3}; do
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $P --output-format csv -d $OUT/$V -o pass$i -- $LAB 4096 4096 4096 2 $V > $OUT/$V.pass$i.log 2>&1
    rc=$?; echo "$V pass$i rc=$rc"
    case $rc in 0) ;; *) echo "stop"; exit $rc;; esac
  done
done
echo done
