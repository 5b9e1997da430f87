"""Per-kernel summary (calls, total/avg us, grid) from a rocprofv3 sqlite results db."""
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"mocr::\(anonymous namespace\)::", "", name)
    return name[:90]


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rows = c.execute("select * from kernels").fetchall()
    i_name = cols.index("kernel_name") if "kernel_name" in cols else cols.index("name")
    i_s, i_e = cols.index("start"), cols.index("end")
    i_g = cols.index("grid_size_x") if "grid_size_x" in cols else None
    agg = {}
    t0, t1 = min(r[i_s] for r in rows), max(r[i_e] for r in rows)
    for r in rows:
        d = agg.setdefault(short(r[i_name]), [0, 0.0, r[i_g] if i_g is not None else None])
        d[0] += 1
        d[1] += (r[i_e] - r[i_s]) / 1e3
    return agg, (t1 - t0) / 1e3


if __name__ == "__main__":
    agg, span = stats(sys.argv[1])
    tot = sum(v[1] for v in agg.values())
    print(f"span {span/1e3:.1f} ms, kernel-time sum {tot/1e3:.1f} ms")
    for k, (n, t, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
        print(f"{t/1e3:9.2f} ms {n:7d} x {t/n:8.2f} us  grid {g}  {k}")
