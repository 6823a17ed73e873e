#!/bin/bash
# round 4: LDS bank-conflict attribution of the FFN-up W-strip role by read-back mode (lab/ldsattr_lab.hip)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES -d gpurun_out/ldsattr2 -o run --output-format csv -- lab/build/ldsattr_lab > gpurun_out/r4_ldsattr2.log 2>&1 || exit $?
python3 - <<'PY' >> gpurun_out/r4_ldsattr2.log
import csv, glob, collections
f = glob.glob("gpurun_out/ldsattr2/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "strip32" not in r["Kernel_Name"] and "pack_single_pass32" not in r["Kernel_Name"]: continue
    acc[(r["Kernel_Name"][:48], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for g, d in sorted(acc.items(), key=lambda x: -x[0][1]):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(g, {c: round(v) for c, v in m.items()}, "conflict/active = %.4f" % (m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_LDS_IDX_ACTIVE"])),
          "conflict per wave = %.1f" % (m["SQ_LDS_BANK_CONFLICT"] / max(1.0, m["SQ_WAVES"])))
PY
