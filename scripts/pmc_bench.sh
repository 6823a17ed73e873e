#!/bin/bash
# PMC passes over bench.py (counters in separate passes; kernel dispatch counters only -- no
# sys/runtime/hip trace domains with --pmc).  Output: gpurun_out/pmc_bench/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_bench; mkdir -p $OUT
CFG=${CFG:-c2}
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT/$CFG -o pass$i -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-error-stats --gemm-timing none --node-reps 0 --cold-steps 0 --prewarm-ms 0 --config $CFG > $OUT/$CFG.pass$i.log 2>&1
  rc=$?; echo "pass$i ($P) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo done
