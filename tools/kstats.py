"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, average us, share of time.

    python tools/kstats.py run_kernel_stats.csv [N] [--no-load]

--no-load leaves out the load-time kernels (decoder weight folding, fragment packing), so
the shares are of the run's encode + decode work.
"""
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
rows = list(csv.DictReader(open(args[0])))
if "--no-load" in sys.argv:
    rows = [r for r in rows if "fold_mm_kernel" not in r["Name"] and "frag_pack_kernel" not in r["Name"]]
n = int(args[1]) if len(args) > 1 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(args[0] + (" (load-time kernels left out)" if "--no-load" in sys.argv else ""))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    name = r["Name"].replace("mocr::(anonymous namespace)::", "").replace("void ", "")
    print(f'{name[:78]:78s} n={r["Calls"]:>6s} avg={float(r["AverageNs"]) / 1e3:8.2f}us '
          f'{100 * float(r["TotalDurationNs"]) / tot:5.1f}%')
