#!/bin/bash
# GPU check (whole -m gpu suite) then kernel traces of CONFIGS; RUN = output dir under gpurun_out
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/${RUN:-r6cp}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:-} > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
for c in ${CONFIGS:-c2}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --node-reps 0 > $OUT/bench_$c.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-error-stats --node-reps 0 --cold-steps 0 > $OUT/prof_$c.log 2>&1 || exit $?
done
echo done
