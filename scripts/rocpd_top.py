#!/usr/bin/env python3
"""Per-kernel summary (calls, average and total duration) from a rocprofv3 rocpd database (`run_results.db`,
the default output format): the same columns as `--stats`'s kernel_stats.csv.  Usage: rocpd_top.py <db> [csv]"""
import sqlite3
import sys


def main(path, csv_out=None):
    cur = sqlite3.connect(path).cursor()
    rows = cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    lines = ["Name,Calls,TotalDurationNs,AverageNs,Percentage"]
    for name, calls, tot, avg, pct in rows:
        short = name if len(name) < 160 else name[:157] + "..."
        lines.append(f'"{short}",{calls},{float(tot) * 1e3:.0f},{float(avg) * 1e3:.1f},{float(pct):.2f}')
    text = "\n".join(lines)
    print(text)
    if csv_out:
        open(csv_out, "w").write(text + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
