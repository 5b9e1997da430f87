"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, average us, share of time.

    python tools/kstats.py run_kernel_stats.csv [N]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[1])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    name = r["Name"].replace("mocr::(anonymous namespace)::", "").replace("void ", "")
    print(f'{name[:78]:78s} n={r["Calls"]:>6s} avg={float(r["AverageNs"]) / 1e3:8.2f}us '
          f'{100 * float(r["TotalDurationNs"]) / tot:5.1f}%')
