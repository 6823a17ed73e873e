#!/bin/bash
# round 5: gemm_i8_fm with transposed accumulators and register stores -- GPU suite, lab A/B against the lab copies of
# the LDS-image epilogue's successors, bench lines of every 256-tile config
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5ds; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 150 lab/build/ds_lab 4096 4096 4096 9 fm,dsPn,dsp > $out/lab_c2.log 2>&1 || { tail $out/lab_c2.log; exit 1; }
timeout -k 10 150 lab/build/ds_lab 2048 16384 4096 7 fm,fmrot,dsp > $out/lab_c3up.log 2>&1 || { tail $out/lab_c3up.log; exit 1; }
grep -v check $out/lab_c2.log $out/lab_c3up.log
for c in c2 c3_up c3_down c4_shard c2_outlier c2_prepacked; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $out/bench_$c.log 2>&1 || { tail $out/bench_$c.log; exit 1; }
  echo "$c $(grep -o '"value": [0-9.]*' $out/bench_$c.log | head -1) $(grep -o '"gemm_kernel_ms": [0-9.e-]*' $out/bench_$c.log | head -1)"
done
echo done
