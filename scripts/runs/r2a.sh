set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r2a.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_r2a.log; echo "rc=$rc"
[ $rc -le 1 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/bench_r2a.log 2>&1; rc=$?; tail -c 3000 gpurun_out/bench_r2a.log; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== chain"; timeout -k 10 120 lab/build/chain2_lab 30 > gpurun_out/chain_r2a.log 2>&1; rc=$?; tail -3 gpurun_out/chain_r2a.log; echo "rc=$rc"
