"""Per-kernel-class HBM traffic from two rocprofv3 PMC passes of tools/profile_encoder.py.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d F -o run -- python tools/profile_encoder.py
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d W -o run -- python tools/profile_encoder.py
    python tools/pmc_traffic.py F/run_counter_collection.csv W/run_counter_collection.csv OUT.json [STEPS [BATCH]]

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B request for
wide (16 B/lane) streaming reads on gfx950, so it is doubled; WRITE_SIZE is taken as is.
Round 6 calibrated both on the decode step's own access patterns (tools/fetch_calib.hip,
profiles/r06/fetch_calib.md): 16-, 8- and 4-B lane loads and the fold GEMMs' 64-B row
segments all reach L2's fabric side as 128-B requests (TCC_EA0_RDREQ_128B), which gfx950's
FETCH_SIZE formula tallies at 64 B (TCC_BUBBLE reads 0), so x2 holds for every read here;
WRITE_SIZE is exact for 16-, 4-B and the V4 epilogue's 128-B-row stores.
Both counters are in KiB.  Encoder dispatches are mapped to the engine's kernel classes
(engine.hip encode()) by their order in one encode; every dispatch after the encoder
(``profile_encoder.py --decode-steps N``: the embedding kernel, then N graph-captured
greedy steps) is summed into ``decode.step`` (bytes per step) and listed per kernel.
"""
import csv
import os
import json
import sys


def classes_in_order(mlp_fused=(), attn_fused=(), attn_noproj=(), lnqkv=(), lnmerge=(), tail=()):
    """Encoder dispatch classes in launch order; stages in `mlp_fused` run norm2 + MLP as one
    kernel (mlp.hip) instead of layernorm, fc1, fc2, stages in `attn_fused` run norm1 +
    qkv + W-MSA + proj as one kernel (wattn.hip), stages in `attn_noproj` norm1 + qkv +
    W-MSA as one kernel, then the proj GEMM; stages in `lnqkv` norm1 + qkv as one kernel
    (mlp.hip lngemm384_kernel), merges in `lnmerge` gather + norm + reduction as one, stages in
    `tail` (with `attn_noproj`) proj + residual + norm2 + MLP as one (mlp384_kernel PROJ)."""
    names = ["split(weights)", "split(kv-weights)", "stem"]
    depth = (2, 2, 6, 2)
    for s in range(4):
        for _ in range(depth[s]):
            if s + 1 in attn_fused:
                names += [f"s{s+1}.attn"]
            elif s + 1 in attn_noproj and s + 1 in tail:
                names += [f"s{s+1}.attn", f"s{s+1}.tail"]
                continue
            elif s + 1 in attn_noproj:
                names += [f"s{s+1}.attn", f"s{s+1}.proj"]
            elif s + 1 in lnqkv:
                names += [f"s{s+1}.lnqkv", f"s{s+1}.wattn", f"s{s+1}.proj"]
            else:
                names += [f"s{s+1}.ln1", f"s{s+1}.qkv", f"s{s+1}.wattn", f"s{s+1}.proj"]
            names += [f"s{s+1}.mlp"] if s + 1 in mlp_fused else [f"s{s+1}.ln2", f"s{s+1}.fc1", f"s{s+1}.fc2"]
        if s < 3:
            names += [f"merge{s+1}"] if s + 1 in lnmerge else [f"merge{s+1}.ln", f"merge{s+1}"]
    names += ["split(memory)", "memproj", "crosskv"]
    return names


def with_memkv24(names, kn):
    """bf16x3 engines append the fp24 split (one dispatch per layer) or the int16
    quantisation (one dispatch) of the cross K/V unless the crosskv epilogue quantises."""
    n = sum("split_kv_fp24" in k for k in kn)
    q = sum("quant_kv_i16" in k for k in kn)
    return names + ["memkv(fp24)"] * n + ["memkv(i16)"] * q


def main(fetch_csv, write_csv, out, decode_steps=0, batch=0):
    decode_steps = int(decode_steps)
    # engine dispatches only (the load-time decoder weight folding is not an encoder kernel)
    keep = lambda r: "mocr" in r["Kernel_Name"] and "fold_mm" not in r["Kernel_Name"] and "frag_pack" not in r["Kernel_Name"]
    f = [r for r in csv.DictReader(open(fetch_csv)) if keep(r)]
    w = [r for r in csv.DictReader(open(write_csv)) if keep(r)]
    assert len(f) == len(w)
    kn = [r["Kernel_Name"] for r in f]
    fused = sorted({1 if "mlp_fused_kernel<96" in k else 2 for k in kn if "mlp_fused" in k} |
                   ({3} if any("mlp384_kernel" in k for k in kn) else set()))
    afused = sorted({1 if "swin_attn_kernel<96" in k else 2 for k in kn if "swin_attn_kernel" in k})
    anoproj = [3] if any("swin_attn_noproj_kernel" in k for k in kn) else []
    n_lng = sum("lngemm384_kernel" in k for k in kn)  # 6 stage-3 blocks and / or merge 1
    lnqkv = [3] if n_lng >= 6 else []
    # merge 1 as one dispatch: lngemm384 (rounds 4-5, and maps whose W/2 % 16 != 0) or the
    # persistent merge1_kernel (merge.hip, round 6)
    lnmerge = [1] if n_lng in (1, 7) or any("merge1_kernel" in k for k in kn) else []
    tail = [3] if any("mlp384_kernel<" in k and ", true" in k for k in kn) else []
    names = with_memkv24(classes_in_order(fused, afused, anoproj, lnqkv, lnmerge, tail), kn)
    # load-time bf16 splits before the stem: weights, kv-weights, and (bf16x3) the folded
    # decoder weights; fp32 mode has none
    n_split = next(i for i, k in enumerate(kn) if "stem" in k)
    names = names[n_split - min(n_split, 2):] if n_split < 2 else names
    if n_split == 0:
        names = [n for n in names if not n.startswith("split(w") and not n.startswith("split(kv")]
    elif n_split > 2:
        names = names[:2] + [f"split(load {i})" for i in range(2, n_split)] + names[2:]
    n_enc = len(names)
    assert len(f) >= n_enc, (len(f), n_enc)
    if not decode_steps:
        assert len(f) == n_enc, (len(f), n_enc)
    agg = {}
    dec_kernels = {}
    for i, (a, b) in enumerate(zip(f, w)):
        assert a["Kernel_Name"] == b["Kernel_Name"]
        fb = 2 * float(a["Counter_Value"]) * 1024
        wb = float(b["Counter_Value"]) * 1024
        if i < n_enc:
            name = names[i]
        else:
            name = "decode.step"
            k = a["Kernel_Name"].replace("void ", "").replace("mocr::(anonymous namespace)::", "").split("(")[0]
            dk = dec_kernels.setdefault(k, {"launches": 0, "fetch_bytes": 0.0, "write_bytes": 0.0})
            dk["launches"] += 1
            dk["fetch_bytes"] += fb
            dk["write_bytes"] += wb
        d = agg.setdefault(name, {"launches": 0, "fetch_bytes": 0.0, "write_bytes": 0.0, "kernel": a["Kernel_Name"]})
        d["launches"] += 1
        d["fetch_bytes"] += fb
        d["write_bytes"] += wb
    for d in agg.values():
        d["hbm_bytes_per_launch"] = (d["fetch_bytes"] + d["write_bytes"]) / d["launches"]
    if decode_steps and "decode.step" in agg:
        d = agg["decode.step"]
        d["kernel"] = "greedy decode step (all dispatches after the encoder / steps)"
        d["dispatches"] = d["launches"]
        d["launches"] = decode_steps
        d["hbm_bytes_per_launch"] = (d["fetch_bytes"] + d["write_bytes"]) / decode_steps
        for dk in dec_kernels.values():
            dk["hbm_bytes_per_launch"] = (dk["fetch_bytes"] + dk["write_bytes"]) / dk["launches"]
    json.dump({"batch": int(batch), "source": [os.path.relpath(p, os.path.dirname(os.path.abspath(out))) for p in (fetch_csv, write_csv)],
               "fetch_correction": 2.0, "decode_steps": decode_steps, "classes": agg, "decode_kernels": dec_kernels},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
