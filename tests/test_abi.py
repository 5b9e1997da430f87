"""CPU: the C-ABI library loads and exports what include/mathocr.h declares; host-side
queries that do not touch the GPU."""
import ctypes
import os
import re

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(REPO, "include", "mathocr.h")).read()
    return sorted(set(re.findall(r"\b(mocr_[a-z_0-9]+)\s*\(", text)))


def test_header_symbols_exported(pkg):
    lib = pkg.load_library()
    names = declared_symbols()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(pkg.engine.exported_symbols()) == names
    header = open(os.path.join(os.path.dirname(__file__), "..", "include", "mathocr.h")).read()
    version = int(re.search(r"#define MOCR_ABI_VERSION (\d+)", header).group(1))
    assert lib.mocr_abi_version() == version == pkg.engine.ABI_VERSION
    # the ctypes mirror of mocr_config has the header's fields, in order
    body = re.search(r"typedef struct mocr_config \{(.*?)\} mocr_config;", header, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = [f.strip() for decl in re.findall(r"int32_t([^;]*);", body) for f in decl.split(",")]
    assert fields == [n for n, _ in pkg.engine.MocrConfig._fields_]


def test_weight_count_matches_spec(pkg):
    lib = pkg.load_library()
    for vocab in (5075, 1000):
        cfg = pkg.engine.make_config(img_hw=(384, 384), vocab=vocab)
        n = lib.mocr_weight_count(ctypes.byref(cfg))
        expect = sum(int(torch.tensor(s).prod()) for _, s, _, _ in pkg.synth.param_specs(vocab))
        assert n == expect
    cfg = pkg.engine.make_config(img_hw=(384, 384))
    assert lib.mocr_weight_count(ctypes.byref(cfg)) == 36_679_757  # 37.45M minus unused swin.norm/head


def test_memory_tokens(pkg):
    lib = pkg.load_library()
    for hw, m in (((384, 384), 144), ((96, 320), 30), ((224, 224), 49)):
        cfg = pkg.engine.make_config(img_hw=hw)
        assert lib.mocr_memory_tokens(ctypes.byref(cfg)) == m


def test_bad_config_rejected(pkg):
    lib = pkg.load_library()
    cfg = pkg.engine.make_config(img_hw=(384, 384))
    cfg.d_model = 512
    assert lib.mocr_weight_count(ctypes.byref(cfg)) == 0
    assert b"d_model" in lib.mocr_last_error(None)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure path")
def test_engine_fails_loudly_without_gpu(pkg):
    with pytest.raises(pkg.MocrError):
        pkg.Engine(img_hw=(96, 320), max_batch=1)


def test_production_build_tag(pkg):
    """the library bakes its build tag beside the source hash; the
    in-tree library is a production build (no compile-time definitions)."""
    lib = pkg.load_library()
    assert lib.mocr_build_tag().decode() == "production"


def test_non_production_build_is_refused(pkg, tmp_path, monkeypatch):
    """A library built with compile-time definitions (Makefile MOCR_DEFS) or by a tools/
    A/B script cannot load as the production library; the bench's --lib loads it as an A/B
    build and reports the tag."""
    import subprocess
    src = tmp_path / "fake.c"
    src.write_text('const char* mocr_source_hash(void) { return "x"; }\n'
                   'const char* mocr_build_tag(void) { return "defs:-DMOCR_FOLD_TS"; }\n')
    so = tmp_path / "libfake.so"
    subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)], check=True)
    monkeypatch.setattr(pkg.engine, "_lib", None)
    with pytest.raises(RuntimeError, match="not a production build"):
        pkg.engine.load_library(str(so))
    # as an A/B build it passes the tag check and stops at the source hash
    with pytest.raises(RuntimeError, match="other sources"):
        pkg.engine.load_library(str(so), ab_build=True)
    monkeypatch.setattr(pkg.engine, "_lib", None)
