"""GPU occupancy of a rocprofv3 kernel trace: over the window from the first to the last
dispatch whose name contains WINDOW (default: every dispatch), the fraction of time at
least one kernel runs (union of [start, end)), the mean number running, and per queue
(HIP stream) its busy fraction and the gaps between its consecutive kernels.

    python tools/trace_busy.py run_kernel_trace.csv [WINDOW]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, window=""):
    rows = [r for r in csv.DictReader(open(path)) if r["Kind"] == "KERNEL_DISPATCH"]
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows)
    hit = [k for k in ks if window in k[3]]
    t0, t1 = hit[0][0], max(k[1] for k in hit)
    ks = [k for k in ks if k[1] > t0 and k[0] < t1]
    ev = sorted([(max(s, t0), 1) for s, e, q, n in ks] + [(min(e, t1), -1) for s, e, q, n in ks])
    busy = run = 0
    last, cur = t0, 0
    for t, d in ev:
        if cur > 0:
            busy += t - last
        run += cur * (t - last)
        cur += d
        last = t
    span = t1 - t0
    print(f"window {span / 1e6:.2f} ms, {len(ks)} dispatches: GPU busy {busy / span:.3f}, mean kernels running {run / span:.2f}")
    per = defaultdict(list)
    for s, e, q, n in ks:
        per[q].append((s, e))
    for q, iv in sorted(per.items()):
        b = sum(e - s for s, e in iv)
        gaps = [iv[i + 1][0] - iv[i][1] for i in range(len(iv) - 1)]
        gaps_pos = [g for g in gaps if g > 0]
        med = statistics.median(gaps_pos) / 1e3 if gaps_pos else 0.0
        big = sum(g for g in gaps if g > 50_000) / 1e6
        print(f"  queue {q}: {len(iv)} kernels, busy {b / span:.3f}, median gap {med:.2f} us, "
              f"gaps > 50 us total {big:.2f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:3])
