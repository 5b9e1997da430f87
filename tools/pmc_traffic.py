"""Per-kernel-class HBM traffic from two rocprofv3 PMC passes of tools/profile_encoder.py.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d F -o run -- python tools/profile_encoder.py
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d W -o run -- python tools/profile_encoder.py
    python tools/pmc_traffic.py F/run_counter_collection.csv W/run_counter_collection.csv OUT.json

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B request for
wide (16 B/lane) streaming reads on gfx950, so it is doubled; WRITE_SIZE is taken as is
(exact for 16 B/lane stores, uncalibrated for the 2-4 B/lane epilogue stores here).
Both counters are in KiB.  Dispatches are mapped to the engine's kernel classes
(engine.hip encode()) by their order in one encode.
"""
import csv
import os
import json
import sys


def classes_in_order(mlp_fused=()):
    """Encoder dispatch classes in launch order; stages in `mlp_fused` run norm2 + MLP as one
    kernel (mlp.hip) instead of layernorm, fc1, fc2."""
    names = ["split(weights)", "split(kv-weights)", "stem"]
    depth = (2, 2, 6, 2)
    for s in range(4):
        for _ in range(depth[s]):
            names += [f"s{s+1}.ln_partition", f"s{s+1}.qkv", f"s{s+1}.wattn", f"s{s+1}.proj"]
            names += [f"s{s+1}.mlp"] if s + 1 in mlp_fused else [f"s{s+1}.layernorm", f"s{s+1}.fc1", f"s{s+1}.fc2"]
        if s < 3:
            names += [f"merge{s+1}.ln", f"merge{s+1}"]
    names += ["split(memory)", "memproj", "crosskv"]
    return names


def main(fetch_csv, write_csv, out):
    # encoder dispatches only (the load-time decoder weight folding is not an encoder kernel)
    keep = lambda r: "mocr" in r["Kernel_Name"] and "fold_mm" not in r["Kernel_Name"]
    f = [r for r in csv.DictReader(open(fetch_csv)) if keep(r)]
    w = [r for r in csv.DictReader(open(write_csv)) if keep(r)]
    fused = sorted({1 if "mlp_fused_kernel<96" in r["Kernel_Name"] else 2 for r in f if "mlp_fused" in r["Kernel_Name"]})
    names = classes_in_order(fused)
    fp32 = len(f) == len(names) - 3  # fp32 mode has no bf16 split kernels
    if fp32:
        names = [n for n in names if not n.startswith("split")]
    assert len(f) == len(w) == len(names), (len(f), len(w), len(names))
    agg = {}
    for name, a, b in zip(names, f, w):
        assert a["Kernel_Name"] == b["Kernel_Name"]
        d = agg.setdefault(name, {"launches": 0, "fetch_bytes": 0.0, "write_bytes": 0.0, "kernel": a["Kernel_Name"]})
        d["launches"] += 1
        d["fetch_bytes"] += 2 * float(a["Counter_Value"]) * 1024
        d["write_bytes"] += float(b["Counter_Value"]) * 1024
    for d in agg.values():
        d["hbm_bytes_per_launch"] = (d["fetch_bytes"] + d["write_bytes"]) / d["launches"]
    json.dump({"source": [os.path.relpath(p, os.path.dirname(os.path.abspath(out))) for p in (fetch_csv, write_csv)], "fetch_correction": 2.0, "classes": agg}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:4])
