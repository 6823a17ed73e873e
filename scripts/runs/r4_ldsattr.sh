#!/bin/bash
# round 4: Infinity-Cache reuse of a streamed read (lab/reuse_lab.hip), and LDS bank-conflict attribution of the
# FFN-up single pass by role (lab/ldsattr_lab.hip, one --pmc pass)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 lab/build/reuse_lab > gpurun_out/r4_reuse_lab.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/ldsattr -o run --output-format csv -- lab/build/ldsattr_lab > gpurun_out/r4_ldsattr.log 2>&1 || exit $?
python3 - <<'PY' >> gpurun_out/r4_ldsattr.log
import csv, glob, collections
f = glob.glob("gpurun_out/ldsattr/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "pack_single_pass32" not in r["Kernel_Name"]: continue
    acc[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for g, d in sorted(acc.items(), reverse=True):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print("grid", g, {c: round(v) for c, v in m.items()},
          "conflict/active = %.4f" % (m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_LDS_IDX_ACTIVE"])))
PY
