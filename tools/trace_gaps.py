"""Per decode-kernel average duration and the average gap from the previous kernel's
end in the same queue, from a rocprofv3 run_kernel_trace.csv (last 2/3 of the trace)."""
import collections
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "mocr" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 3:]
dur = collections.defaultdict(list)
gap = collections.defaultdict(list)
last = {}
for r in rows:
    k = r["Kernel_Name"].replace("void ", "").replace("mocr::(anonymous namespace)::", "").split("(")[0]
    a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r["Queue_Id"]
    dur[k].append(b - a)
    if q in last:
        gap[k].append(a - last[q])
    last[q] = b
tot = 0
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    d = sum(dur[k]) / len(dur[k]) / 1e3
    g = sum(gap[k]) / max(1, len(gap[k])) / 1e3
    print(f"{k:45s} n={len(dur[k]):6d} dur {d:6.2f} us  gap-before {g:6.2f} us")
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e6
print("span ms", round(span, 2), "kernels", len(rows))
