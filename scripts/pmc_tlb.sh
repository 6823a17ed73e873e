#!/bin/bash
# UTCL1 (per-CU address translation) counters of the two pack strip widths at a narrow and a wide W:
# does the wide-W slowdown come with translation misses?  One --pmc pass per shape.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=lab/build/pack2_lab
for s in "512 8192 4096" "512 16384 4096"; do
  tag=$(echo $s | tr ' ' x)
  timeout -s KILL 90 rocprofv3 --pmc ${PMC:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum} -d gpurun_out/pmc_tlb_$tag -o run --output-format csv -- $B $s 3 > gpurun_out/pmc_tlb_$tag.log 2>&1
  python3 - "$tag" <<'PY'
import csv, glob, sys, collections
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/pmc_tlb_{tag}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(tag, k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
done
