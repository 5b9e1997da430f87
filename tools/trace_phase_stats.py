#!/usr/bin/env python3
"""Per-kernel duration statistics of the bench's isolated phase, from a rocprofv3
kernel trace of `bench.py` (run_kernel_trace.csv).

bench.py measures the roofline kernels with HIP events while ONE replica runs alone,
after the loaded (all-replica) timed region.  rocprofv3 --stats averages every dispatch
of the run, the loaded ones included, so it reads higher under contention.  This script
takes the dispatches of the last `--iso-batches` batches of one kernel (the isolated
phase; bench.py runs 3) and prints their statistics beside the whole-run ones, so the
HIP-event average can be checked against the profiler's clock for the same dispatches.
Only the kernel's full-batch dispatches (its largest grid) are counted.

usage: tools/trace_phase_stats.py TRACE.csv KERNEL_SUBSTRING PER_BATCH [--iso-batches 3] [--json OUT]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("kernel")
    ap.add_argument("per_batch", type=int, help="launches of the kernel per batch (s3.fc1: 6)")
    ap.add_argument("--iso-batches", type=int, default=3)
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            if a.kernel in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])))
    # the bench's B = 1 latency engine runs after the isolated phase and may use the same
    # kernel on a smaller grid: keep the full-batch dispatches (the largest grid)
    if rows:
        big = max(r[3] for r in rows)
        rows = [r[:3] for r in rows if r[3] == big]
    rows.sort()
    if not rows:
        raise SystemExit(f"no dispatch of {a.kernel!r}")
    names = {n for _, _, n in rows}
    if len(names) > 1:
        raise SystemExit(f"{a.kernel!r} matches several kernels: {sorted(names)}")
    dur = [(e - s) / 1e3 for s, e, _ in rows]
    n_iso = a.per_batch * a.iso_batches
    iso = dur[-n_iso:]
    out = {
        "kernel": rows[0][2],
        "all": {"dispatches": len(dur), "avg_us": statistics.mean(dur), "min_us": min(dur), "max_us": max(dur)},
        "isolated": {"dispatches": len(iso), "avg_us": statistics.mean(iso), "median_us": statistics.median(iso),
                     "min_us": min(iso), "max_us": max(iso)},
    }
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
