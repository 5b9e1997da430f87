"""Overlap of encoder and decoder kernels in a rocprofv3 kernel trace of bench.py
(run_kernel_trace.csv): over the pipelined (multi-replica) window, the fraction of wall
time in which encoder kernels, decode kernels, both, or neither are running, and each
class's summed kernel time.  Usage: python tools/trace_overlap.py run_kernel_trace.csv"""
import csv
import sys

DEC = ("foldgemm", "foldwide", "dec_", "rowgemm", "beam_")


def main(path):
    rows = [r for r in csv.DictReader(open(path)) if "mocr" in r["Kernel_Name"] and "fold_mm" not in r["Kernel_Name"]]
    ev = []
    tot = {"enc": 0, "dec": 0}
    res = {"enc": {}, "dec": {}}
    for r in rows:
        c = "dec" if any(k in r["Kernel_Name"] for k in DEC) else "enc"
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        ev += [(a, c, 1), (b, c, -1)]
        tot[c] += b - a
        res[c].setdefault((r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size_X"]), set()).add(
            r["Kernel_Name"].split("(")[0][-60:])
    ev.sort()
    # the pipelined window: middle 60 % of the trace span
    t0, t1 = ev[0][0], ev[-1][0]
    w0, w1 = t0 + 0.2 * (t1 - t0), t0 + 0.8 * (t1 - t0)
    act = {"enc": 0, "dec": 0}
    span = {"enc": 0, "dec": 0, "both": 0, "none": 0}
    prev = ev[0][0]
    for t, c, d in ev:
        lo, hi = max(prev, w0), min(t, w1)
        if hi > lo:
            k = "both" if act["enc"] and act["dec"] else "enc" if act["enc"] else "dec" if act["dec"] else "none"
            span[k] += hi - lo
        act[c] += d
        prev = t
    W = w1 - w0
    print({k: round(v / W, 3) for k, v in span.items()}, "window ms", round(W / 1e6, 2))
    print("summed kernel ms", {k: round(v / 1e6, 1) for k, v in tot.items()})
    for c in res:
        print(c)
        for k, v in sorted(res[c].items()):
            print("  vgpr/agpr/lds/wg", k, sorted(v)[:3])


if __name__ == "__main__":
    main(sys.argv[1])
