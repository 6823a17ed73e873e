#!/bin/bash
# L1 (TCP) hit behaviour of the 256-tile GEMM: f4 (product structure) vs f4sync, K 4096 and 8192
set -u
export TMPDIR=/tmp
out=gpurun_out/l1pmc; mkdir -p $out
timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1; echo "list rc=$?"
for K in 4096 8192; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $out/k$K -o tcp -- lab/build/w4_lab 4096 4096 $K 2 f4,f4sync > $out/k$K.log 2>&1
  rc=$?; echo "K=$K rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
