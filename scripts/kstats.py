"""Print the top kernels of a rocprofv3 kernel_stats.csv (share of GPU time, calls, average)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms")
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% calls={r['Calls']:>7} "
          f"avg={float(r['AverageNs']) / 1000:8.1f}us {r['Name'][:100]}")
