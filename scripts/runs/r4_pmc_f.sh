#!/bin/bash
# PMC passes of the f2 / f3 configs (weight-cache drop-in, LLM.int8() decomposition) for their roofline traffic
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r4pmcf; mkdir -p $out
for cfg in c2_prepacked c2_outlier; do
  CFG=$cfg timeout -k 10 400 bash scripts/pmc_bench.sh > $out/pmc_$cfg.log 2>&1 || { tail $out/pmc_$cfg.log; exit 1; }
  python3 scripts/summarize_pmc.py gpurun_out/pmc_bench/$cfg $out/pmc_$cfg.json 4096 4096 4096 > $out/pmc_$cfg.sum 2>&1 || exit 1
done
echo done
