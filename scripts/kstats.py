"""Print a rocprofv3 kernel_stats.csv compactly: calls, average us, share, short name."""
import csv
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        rows = list(csv.DictReader(f))
    for r in rows:
        name = r["Name"].replace("qgemm::", "").replace("(anonymous namespace)::", "")
        name = name[:70]
        print(f'{int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:9.2f} us {float(r["Percentage"]):6.2f}%  {name}')
