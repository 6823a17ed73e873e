#!/bin/bash
# Headline artifacts for profiles/: the default bench line (c2), the rocprofv3 kernel trace of the
# same command, then the PMC passes (scripts/pmc_bench.sh).  Each GPU step has its own time limit;
# any failure ends the script.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c2; mkdir -p $OUT
if [ -z "${PMC_ONLY:-}" ]; then
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['gemm_kernel_ms'],d['roofline']['frac'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py > $OUT/prof.log 2>&1
grep '^{"metric"' $OUT/prof.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('profiled run', d['value'],d['gemm_kernel_ms'])"
fi
bash scripts/pmc_bench.sh
echo done
