#!/usr/bin/env python3
"""Median duration per kernel in each third (or N parts) of a rocprofv3 kernel-trace CSV: the phases of a
probe that times a few configurations in sequence.  Usage: trace_phases.py run_kernel_trace.csv [parts]"""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    parts = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    out = collections.defaultdict(list)
    for i, r in enumerate(rows):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out[(i * parts) // len(rows), r["Kernel_Name"][:90]].append(d)
    for (ph, name), v in sorted(out.items()):
        if len(v) >= 10:
            print(f"{ph} {statistics.median(v):8.2f} us n={len(v):4d} {name}")


if __name__ == "__main__":
    main()
