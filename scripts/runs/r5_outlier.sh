#!/bin/bash
# round-5: the fused flags+index launch (outlier tests, c2_outlier vs c2 on one box, kernel trace) and the mask-pack lab
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5outlier; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 200 lab/build/maskpack_lab 4096 4096 4096 9 > $out/maskpack.log 2>&1 || { tail $out/maskpack.log; exit 1; }
cat $out/maskpack.log
for i in 1 2; do
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline --node-reps 0 --cold-steps 0 --no-error-stats > $out/bench_c2_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2_$i.log | head -1
timeout -k 10 300 python bench.py --config c2_outlier --no-cpu-baseline --cold-steps 0 --no-error-stats > $out/bench_c2_outlier_$i.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $out/bench_c2_outlier_$i.log | head -1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c2_outlier --no-cpu-baseline --cold-steps 0 --no-error-stats --steps 50 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$out/prof.log; exit 1; }
python3 $GRAFT_REPO_ROOT/scripts/rocpd_top.py $GRAFT_REPO_ROOT/$out/prof/run_results.db | tee $GRAFT_REPO_ROOT/$out/kernel_stats.txt
echo done
