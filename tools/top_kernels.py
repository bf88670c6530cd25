"""Top kernels of a rocprofv3 kernel_stats.csv by total time: name, calls, average microseconds."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 8]:
    print(r["Name"][:100], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
