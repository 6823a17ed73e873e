#!/usr/bin/env python3
"""Median per-dispatch value of every counter in rocprofv3 --pmc passes, per kernel (short name), per config dir.
usage: pmc_table.py <dir> [<dir> ...]   (each dir holds pass*_counter_collection.csv)"""
import csv
import glob
import statistics
import sys
from collections import defaultdict


def short(name):
    for key in ("gemm_i8_fm", "gemm_i8_small", "pack_single_pass32", "pack_single_pass8", "pack_single_pass",
                "outlier", "colmax", "pack_cols", "pack_rows"):
        if key in name:
            return key
    return name[:30]


for d in sys.argv[1:]:
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(f"{d}/pass*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            vals[k]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for k in sorted(vals):
        if not (k.startswith("gemm") or k.startswith("pack")):
            continue
        print(f"{d} {k}:")
        for c, v in sorted(vals[k].items()):
            print(f"    {c:40s} {statistics.median(v):16.1f}  (n={len(v)})")
