"""Print the top kernels of a rocprofv3 kernel_stats.csv (usage: kstats.py FILE [N])."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 24]:
    print(f"{r['Name'][:72]:72s} calls={r['Calls']:>5} avg_us={float(r['AverageNs']) / 1e3:9.1f}")
