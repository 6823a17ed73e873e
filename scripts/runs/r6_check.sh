#!/bin/bash
# round 6 GPU check: the whole -m gpu suite, then bench at C2, FFN up and c2_outlier (RUN = output dir name)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6c2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --no-cpu-baseline --node-reps 0 > $OUT/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c3_up --no-cpu-baseline > $OUT/bench_c3_up.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2_outlier --no-cpu-baseline > $OUT/bench_c2_outlier.log 2>&1 || exit $?
tail -c 600 $OUT/bench_c2.log; echo; tail -c 400 $OUT/bench_c3_up.log; echo; tail -c 400 $OUT/bench_c2_outlier.log
