#!/bin/bash
# same-box comparison against hipBLASLt (torch._int_mm) with the round-3 kernels, two shapes
set -o pipefail
out=gpurun_out/vendor; mkdir -p $out
timeout -k 10 300 python scripts/vendor_compare.py > $out/vendor_4096.log 2>&1 || exit 1
timeout -k 10 300 python scripts/vendor_compare.py 8192 4096 4096 > $out/vendor_8192.log 2>&1 || exit 1
cat $out/vendor_4096.log $out/vendor_8192.log
