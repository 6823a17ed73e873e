#!/usr/bin/env python3
"""Per-dispatch timeline from a rocprofv3 SQLite output (kernels view): the last `n` dispatches with their
start offset, duration and the gap after the previous dispatch's end.  Usage: rocpd_timeline.py DB [n]"""
import re
import sqlite3
import sys

db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))[-n:]
t0, prev = rows[0][1], None
tot_k = tot_g = 0.0
for name, s, e in rows:
    short = re.sub(r"\(.*", "", name).replace("qgemm::", "").replace("(anonymous namespace)::", "")[:70]
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    tot_k += (e - s) / 1e3
    tot_g += gap
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} gap {gap:6.2f}  {short}")
    prev = e
print(f"kernels {tot_k:.1f} us, gaps {tot_g:.1f} us, span {(rows[-1][2] - rows[0][1]) / 1e3:.1f} us")
