"""Print calls / average / total per kernel from a rocprofv3 kernel_stats.csv (optional name filter)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if pat in r["Name"]:
        print(f"  {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} us  {float(r['TotalDurationNs']) / 1e6:9.2f} ms  "
              f"{r['Name'][:80]}")
