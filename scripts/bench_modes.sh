#!/bin/bash
# Compare GEMM-timing modes of bench.py in one session (each its own time limit; stop on fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in none record ext none record; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --gemm-timing $m > gpurun_out/bench_$m.log 2>&1
  rc=$?; echo "mode=$m rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.loads(open('gpurun_out/bench_$m.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['gemm_kernel_ms'])"
done
