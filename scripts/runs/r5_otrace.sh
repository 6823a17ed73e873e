#!/bin/bash
# round 5: kernel traces of c2 and c2_outlier on one box (GEMM durations side by side), then the lab's outlier-epilogue
# variants (fm / fo0 / fo8)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5otrace; mkdir -p $out
for c in c2 c2_outlier; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_$c -o run --output-format csv -- python bench.py --config $c --steps 60 --warmup 10 --no-cpu-baseline --no-error-stats --cold-steps 0 --node-reps 0 > $out/trace_$c.log 2>&1 || exit 1
done
timeout -k 10 150 lab/build/ds_lab 4096 4096 4096 9 fm,fo0,fo8 > $out/lab.log 2>&1 || exit 1
grep -v check $out/lab.log
for c in c2 c2_outlier; do
  f=$(find $out/trace_$c -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$c" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    n = n[:n.index('(')] if '(' in n else n
    print(f"{sys.argv[2]:11s} {int(r['Calls']):6d} {float(r['AverageNs'])/1000:8.2f} us  {n[-70:]}")
PY
done
echo done
