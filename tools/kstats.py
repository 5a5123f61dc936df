"""Summarise a rocprofv3 kernel_stats.csv per training step: tools/kstats.py <csv> <steps> [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {int(r['Calls']) / steps:7.1f}/step "
          f"{float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:110]}")
print(f"total {tot / 1e6 / steps:.2f} ms/step")
