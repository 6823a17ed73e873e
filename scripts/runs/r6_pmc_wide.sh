#!/bin/bash
# write-path counters of the FFN-up GEMM (64-KiB output rows) against its C4-shard twin, one box:
# write requests, average write latency (WRREQ_LEVEL / WRREQ), DRAM-credit and EA stalls; separate --pmc passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r6pmcw; mkdir -p $OUT
for CFG in c3_up c4_shard; do
  i=0
  for P in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum" \
           "TCC_EA0_WRREQ_64B_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_EA0_WRREQ" "WRITE_SIZE" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/$CFG -o pass$i -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-error-stats --gemm-timing none --node-reps 0 --cold-steps 0 --prewarm-ms 0 --config $CFG > $OUT/$CFG.pass$i.log 2>&1
    rc=$?; echo "$CFG pass$i ($P) rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
echo done
