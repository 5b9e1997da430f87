"""tools/pmc_traffic.py maps an encode's dispatches to the engine's kernel classes by launch
order (CPU; synthetic counter CSVs in the rocprofv3 layout)."""
import csv
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_tool():
    spec = importlib.util.spec_from_file_location("pmc_traffic", os.path.join(ROOT, "tools", "pmc_traffic.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def bench_dispatches():
    """The B = 256 bf16x3 encode of the bench, as the library launches it: fused stage-1/2
    attention and MLP, merge 1 on lngemm384, stage 3 on lngemm384 + window attention + proj
    + mlp384, stage 4 unfused, the crosskv GEMM quantising the int16 K/V (no split pass)."""
    k = ["mocr::split_bf16_kernel", "mocr::split_bf16_kernel", "mocr::stem16_kernel"]
    k += ["mocr::swin_attn_kernel<96, 3, 3>", "mocr::mlp_fused_kernel<96, 2, 64, 3>"] * 2
    k += ["mocr::lngemm384_kernel<3, 2>"]
    k += ["mocr::swin_attn_kernel<192, 3, 2>", "mocr::mlp_fused_kernel<192, 1, 32, 3>"] * 2
    k += ["mocr::ln_group_kernel<64, 12, 2>", "mocr::gemm_x3_stagq_kernel<0, 9, 3, 3, 3>"]
    k += ["mocr::lngemm384_kernel<3, 2>", "mocr::window_attention_mfma_kernel<3>",
          "mocr::gemm_x3_stagq_kernel<2, 9, 3, 3, 3>", "mocr::mlp384_kernel<3>"] * 6
    k += ["mocr::ln_group_kernel<64, 24, 2>", "mocr::gemm_x3_stagq_kernel<0, 9, 3, 3, 3>"]
    k += ["mocr::ln_group_kernel<64, 12, 0>", "mocr::gemm_x3_stagq_kernel<0, 9, 3, 3, 3>",
          "mocr::window_attention_mfma_kernel<3>", "mocr::gemm_x3_stagq_kernel<2, 9, 3, 3, 3>",
          "mocr::ln_group_kernel<64, 12, 0>", "mocr::gemm_x3_stagq_kernel<1, 9, 4, 3, 2>",
          "mocr::gemm_x3_stagq_kernel<2, 9, 3, 3, 3>"] * 2
    k += ["mocr::split_bf16_kernel", "mocr::gemm_bf16_ring_kernel<4, 4, 2, 2, 0, 3, 2, false>",
          "mocr::gemm_x3_stagq_kernel<6, 9, 4, 3, 2>"]
    return k


def write_csv(path, names, value):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Value"])
        w.writeheader()
        for n in names:
            w.writerow({"Kernel_Name": n, "Counter_Value": value})


def test_round3_encode_maps_to_its_classes(tmp_path):
    tool = load_tool()
    names = bench_dispatches()
    write_csv(tmp_path / "f.csv", names, 1.0)
    write_csv(tmp_path / "w.csv", names, 3.0)
    out = tmp_path / "out.json"
    tool.main(str(tmp_path / "f.csv"), str(tmp_path / "w.csv"), str(out))
    cls = json.load(open(out))["classes"]
    assert cls["s3.lnqkv"]["launches"] == 6 and "lngemm384" in cls["s3.lnqkv"]["kernel"]
    assert cls["merge1"]["launches"] == 1 and "lngemm384" in cls["merge1"]["kernel"]
    assert "merge1.ln" not in cls and "s3.ln1" not in cls and "s3.qkv" not in cls
    assert cls["s3.wattn"]["launches"] == 6 and "window_attention" in cls["s3.wattn"]["kernel"]
    assert cls["s3.mlp"]["launches"] == 6 and "mlp384" in cls["s3.mlp"]["kernel"]
    assert cls["merge2.ln"]["launches"] == 1 and cls["s4.fc1"]["launches"] == 2
    assert "stagq_kernel<6" in cls["crosskv"]["kernel"] and "memkv(i16)" not in cls
    # FETCH_SIZE is doubled (gfx950 correction), both counters are KiB
    assert cls["stem"]["hbm_bytes_per_launch"] == (2 * 1.0 + 3.0) * 1024


def test_unfused_ln_gemm_and_the_quantisation_pass(tmp_path):
    tool = load_tool()
    names = []
    for n in bench_dispatches():
        if "lngemm384" in n:  # MOCR_VARIANT_UNFUSED_LN_GEMM: LayerNorm, then the GEMM
            names += ["mocr::ln_group_kernel<32, 12, 0>", "mocr::gemm_x3_stagq_kernel<0, 9, 3, 3, 3>"]
        else:
            names.append(n)
    names.append("mocr::quant_kv_i16_kernel")  # M != 144: the separate int16 pass
    write_csv(tmp_path / "f.csv", names, 1.0)
    write_csv(tmp_path / "w.csv", names, 1.0)
    tool.main(str(tmp_path / "f.csv"), str(tmp_path / "w.csv"), str(tmp_path / "o.json"))
    cls = json.load(open(tmp_path / "o.json"))["classes"]
    assert cls["s3.ln1"]["launches"] == 6 and cls["s3.qkv"]["launches"] == 6
    assert cls["merge1.ln"]["launches"] == 1 and "s3.lnqkv" not in cls
    assert cls["memkv(i16)"]["launches"] == 1


def test_stage3_block_tail_maps_to_s3_tail(tmp_path):
    """Round 6: stage 3 on the fused attention (no proj) and the block-tail kernel
    (mlp384_kernel PROJ: proj + residual + norm2 + MLP), two dispatches per block."""
    tool = load_tool()
    k = bench_dispatches()
    a = k.index("mocr::lngemm384_kernel<3, 2>", k.index("mocr::ln_group_kernel<64, 12, 2>"))  # stage 3's first block
    b = k.index("mocr::ln_group_kernel<64, 24, 2>")  # merge 3
    names = k[:a] + ["mocr::swin_attn_noproj_kernel<384, 3, 3, 12, 2>", "mocr::mlp384_kernel<3, true, 4>"] * 6 + k[b:]
    write_csv(tmp_path / "f.csv", names, 1.0)
    write_csv(tmp_path / "w.csv", names, 1.0)
    tool.main(str(tmp_path / "f.csv"), str(tmp_path / "w.csv"), str(tmp_path / "o.json"))
    cls = json.load(open(tmp_path / "o.json"))["classes"]
    assert cls["s3.attn"]["launches"] == 6 and "noproj" in cls["s3.attn"]["kernel"]
    assert cls["s3.tail"]["launches"] == 6 and "mlp384_kernel<3, true" in cls["s3.tail"]["kernel"]
    assert "s3.proj" not in cls and "s3.mlp" not in cls and cls["merge1"]["launches"] == 1


def test_round6_encode_merge1_kernel(tmp_path):
    """Round 6 production at 640 images: merge 1 on the persistent merge1_kernel (merge.hip),
    stage 3 as fused attention + block tail, so no lngemm384 dispatch remains."""
    tool = load_tool()
    k = bench_dispatches()
    a = k.index("mocr::lngemm384_kernel<3, 2>", k.index("mocr::ln_group_kernel<64, 12, 2>"))
    b = k.index("mocr::ln_group_kernel<64, 24, 2>")
    names = k[:a] + ["mocr::swin_attn_noproj_kernel<384, 3, 3, 12, 2>", "mocr::mlp384_kernel<3, true, 4>"] * 6 + k[b:]
    names = [("mocr::merge1_kernel<3>" if "lngemm384" in n else n) for n in names]
    names = [("mocr::stem16w_kernel" if "stem" in n else n) for n in names]
    assert not any("lngemm384" in n for n in names)
    write_csv(tmp_path / "f.csv", names, 1.0)
    write_csv(tmp_path / "w.csv", names, 1.0)
    tool.main(str(tmp_path / "f.csv"), str(tmp_path / "w.csv"), str(tmp_path / "o.json"))
    cls = json.load(open(tmp_path / "o.json"))["classes"]
    assert cls["merge1"]["launches"] == 1 and "merge1_kernel" in cls["merge1"]["kernel"]
    assert "merge1.ln" not in cls and cls["s3.tail"]["launches"] == 6
    assert "ln_group_kernel<64, 12, 2>" in cls["merge2.ln"]["kernel"]
