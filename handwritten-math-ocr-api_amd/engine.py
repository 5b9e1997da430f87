"""ctypes binding of libmathocr.so (include/mathocr.h) and the ``Engine`` class.

``Engine`` is what the reference's ``model`` object becomes: the callers that took a
``FormulaRecognitionModel`` (``src/inference.py:7``, ``app/src/im2latex.py:15``) take an
``Engine`` instead (see ``inference.py`` / ``im2latex.py`` in this package).  There is no
PyTorch op dispatch and no CPU fallback on this path: if the HIP library is missing or
no GPU is visible, construction raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import synth

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmathocr.so")

PRECISION = {"fp32": 0, "bf16": 1, "bf16x3": 2}
STOP = {"batch": 0, "none": 1}
ARCH = {"swin": 0, "res18trans": 1}
ABI_VERSION = 6
# kernel-path variants (include/mathocr.h MOCR_VARIANT_*): 0 = production
VARIANT = {"unfused_attn": 1, "unfused_mlp": 2, "dec_unfolded": 4, "s4_fused_attn": 8, "window_rows": 16, "dec_narrow": 32,
           "logits_f32": 64, "s3_large_batch": 128, "kv_f32": 256,
           "cross_kv_f24": 512, "unfused_ln_gemm": 1024, "self_kv_f24": 2048, "beam_unfolded": 4096,
           "unfused_s3_tail": 8192}


class MocrConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "img_h", "img_w", "vocab", "d_model", "n_heads", "d_ff", "n_layers", "max_pos",
        "sos_id", "eos_id", "pad_id", "max_batch", "precision", "max_beam", "arch", "variant")]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 48), ("launches", ctypes.c_int64), ("total_ms", ctypes.c_double),
                ("flops", ctypes.c_double), ("bytes", ctypes.c_double)]


_lib = None


def load_library(path: str = LIB_PATH, ab_build: bool = False):
    """Load libmathocr.so once.  Raises if it has not been built (no silent fallback), if
    it was built from other sources, or if it is not a production build (its baked
    ``mocr_build_tag`` is not "production": compile-time definitions or a tools/ A/B build)
    unless ``ab_build`` (the probes' and bench's ``--lib``, which report the tag)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    lib.mocr_source_hash.restype = ctypes.c_char_p
    lib.mocr_source_hash.argtypes = []
    lib.mocr_build_tag.restype = ctypes.c_char_p
    lib.mocr_build_tag.argtypes = []
    tag = lib.mocr_build_tag().decode()
    if tag != "production" and not ab_build:
        raise RuntimeError(f"{path} is not a production build (build tag {tag!r}): rebuild it with "
                           f"`python -c 'import __graft_entry__ as g; g.build()'`, or load it as an A/B build")
    want = source_hash()
    if want is not None and lib.mocr_source_hash().decode() != want:
        raise RuntimeError(f"{path} was built from other sources (hash {lib.mocr_source_hash().decode()}, "
                           f"sources {want}): rebuild it with `python -c 'import __graft_entry__ as g; g.build()'`")
    P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    i32p = ctypes.POINTER(ctypes.c_int32)
    f32p = ctypes.POINTER(ctypes.c_float)
    cfgp = ctypes.POINTER(MocrConfig)
    sigs = {
        "mocr_abi_version": (I, []),
        "mocr_device_count": (I, []),
        "mocr_weight_count": (SZ, [cfgp]),
        "mocr_memory_tokens": (I, [cfgp]),
        "mocr_create": (I, [cfgp, I, ctypes.POINTER(P)]),
        "mocr_destroy": (I, [P]),
        "mocr_last_error": (ctypes.c_char_p, [P]),
        "mocr_load_weights": (I, [P, f32p, SZ]),
        "mocr_set_images": (I, [P, f32p, I]),
        "mocr_set_images_device": (I, [P, P, I]),
        "mocr_encode": (I, [P, I]),
        "mocr_get_memory": (I, [P, f32p]),
        "mocr_decode": (I, [P, I, I, i32p, i32p, i32p, f32p, f32p]),
        "mocr_decode_device": (I, [P, I, I, P, i32p]),
        "mocr_decode_beam": (I, [P, I, I, I, i32p, f32p, i32p, i32p]),
        "mocr_set_encoder_pos": (I, [P, f32p, I]),
        "mocr_debug_encode_until": (I, [P, I, I, f32p, SZ]),
        "mocr_set_timing": (I, [P, I]),
        "mocr_get_timing": (I, [P, ctypes.POINTER(KernelStat), I]),
        "mocr_set_cu_mask": (I, [P, ctypes.POINTER(ctypes.c_uint32), I]),
        "mocr_set_stream_priority": (I, [P, I]),
        "mocr_group_unique_id": (I, [ctypes.c_char_p]),
        "mocr_group_create": (I, [ctypes.c_char_p, I, I, I, ctypes.POINTER(P)]),
        "mocr_group_destroy": (I, [P]),
        "mocr_group_last_error": (ctypes.c_char_p, []),
        "mocr_group_gather_ids": (I, [P, P, I, I, P, P]),
        "mocr_group_size": (I, [P, ctypes.POINTER(ctypes.c_int)]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mocr_abi_version() != ABI_VERSION:
        raise RuntimeError("libmathocr.so ABI version mismatch")
    _lib = lib
    return lib


def source_hash():
    """sha256 (16 hex digits) of the sources the Makefile bakes into libmathocr.so
    (csrc/*.hip and csrc/*.h sorted, then include/mathocr.h), or None without sources."""
    import glob
    import hashlib
    files = sorted(glob.glob(os.path.join(_HERE, "csrc", "*.hip")) + glob.glob(os.path.join(_HERE, "csrc", "*.h")),
                   key=os.path.basename)
    hdr = os.path.join(os.path.dirname(_HERE), "include", "mathocr.h")
    if not files or not os.path.exists(hdr):
        return None
    h = hashlib.sha256()
    for f in files + [hdr]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def exported_symbols():
    return ["mocr_abi_version", "mocr_source_hash", "mocr_build_tag", "mocr_device_count", "mocr_weight_count", "mocr_memory_tokens", "mocr_create", "mocr_destroy",
            "mocr_last_error", "mocr_load_weights", "mocr_set_images", "mocr_set_images_device", "mocr_encode",
            "mocr_get_memory", "mocr_decode", "mocr_decode_device", "mocr_decode_beam", "mocr_debug_encode_until",
            "mocr_set_timing", "mocr_get_timing", "mocr_set_encoder_pos", "mocr_set_cu_mask", "mocr_set_stream_priority", "mocr_group_unique_id", "mocr_group_create",
            "mocr_group_destroy", "mocr_group_last_error", "mocr_group_gather_ids", "mocr_group_size"]


def make_config(img_hw=(96, 320), vocab=synth.VOCAB, max_batch=64, precision="fp32", n_layers=synth.N_LAYERS,
                max_pos=synth.MAX_POS, sos=synth.SOS_ID, eos=synth.EOS_ID, pad=synth.PAD_ID, max_beam=0,
                arch="swin", variant=()) -> MocrConfig:
    flags = 0
    for v in variant:
        flags |= VARIANT[v]
    return MocrConfig(img_h=img_hw[0], img_w=img_hw[1], vocab=vocab, d_model=synth.D_MODEL, n_heads=synth.N_HEADS,
                      d_ff=synth.D_FF, n_layers=n_layers, max_pos=max_pos, sos_id=sos, eos_id=eos, pad_id=pad,
                      max_batch=max_batch, precision=PRECISION[precision], max_beam=max_beam, arch=ARCH[arch], variant=flags)


def _f32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


@dataclass
class BeamResult:
    ids: np.ndarray        # [B, n_steps+1] int32 best hypothesis, column 0 = sos, pad after it ends
    scores: np.ndarray     # [B, K] summed log-probs, rank order
    beams: np.ndarray      # [B, K, n_steps+1] every hypothesis, rank order
    n_steps: int


@dataclass
class DecodeResult:
    ids: np.ndarray                 # [B, n_steps+1] int32, column 0 = sos
    n_steps: int
    logp: Optional[np.ndarray]      # [B, n_steps] log(softmax+1e-10) of the chosen token
    logits: Optional[np.ndarray]    # [B, n_steps, V]


class MocrError(RuntimeError):
    pass


def check_ids_tensor(ids_dev, batch: int, max_steps: int, device: int):
    """Validate the device tensor ``mocr_decode_device`` writes ``batch x (max_steps + 1)``
    int32 through (``Engine.decode_into``): a raw pointer crosses the C-ABI, so a wrong
    shape, dtype, layout or device would be an out-of-bounds device write, not an error.
    Raises ValueError unless ``ids_dev`` is a contiguous int32 CUDA tensor of shape
    ``[batch, max_steps + 1]`` on HIP device ``device``."""
    import torch
    if batch <= 0:
        raise ValueError("decode_into: no images set (encode a batch first)")
    if not 1 <= max_steps:
        raise ValueError("decode_into: max_steps must be >= 1")
    if not getattr(ids_dev, "is_cuda", False):
        raise ValueError("decode_into: ids must be a CUDA (HIP device) tensor")
    if ids_dev.dtype != torch.int32:
        raise ValueError(f"decode_into: ids must be int32, got {ids_dev.dtype}")
    want = (batch, max_steps + 1)
    if tuple(ids_dev.shape) != want:
        raise ValueError(f"decode_into: ids must be {list(want)} (encoded batch x (max_steps + 1)), "
                         f"got {list(ids_dev.shape)}")
    if not ids_dev.is_contiguous():
        raise ValueError("decode_into: ids must be contiguous")
    if ids_dev.device.index != device:
        raise ValueError(f"decode_into: ids are on cuda:{ids_dev.device.index}, the engine on device {device}")


class Engine:
    """One engine per GPU (hip device ordinal ``device``)."""

    def __init__(self, img_hw=(96, 320), vocab=synth.VOCAB, max_batch=64, precision="fp32", device=0,
                 n_layers=synth.N_LAYERS, max_pos=synth.MAX_POS, sos=synth.SOS_ID, eos=synth.EOS_ID,
                 pad=synth.PAD_ID, max_beam=0, arch="swin", variant=()):
        """``variant``: names from ``VARIANT`` selecting the unfused kernel sequences
        (parity tests); empty in production."""
        self.lib = load_library()
        self.cfg = make_config(img_hw, vocab, max_batch, precision, n_layers, max_pos, sos, eos, pad, max_beam, arch,
                               tuple(variant))
        self.max_beam = max_beam
        self.arch = arch
        self.img_hw = tuple(img_hw)
        self.vocab = vocab
        self.max_batch = max_batch
        self.max_pos = max_pos
        self.n_layers = n_layers
        self.sos, self.eos, self.pad = sos, eos, pad
        self.precision = precision
        self.device = device
        h = ctypes.c_void_p()
        rc = self.lib.mocr_create(ctypes.byref(self.cfg), device, ctypes.byref(h))
        if rc != 0:
            raise MocrError(f"mocr_create failed ({rc}): {self.lib.mocr_last_error(None).decode()}")
        self._h = h
        self.memory_tokens = self.lib.mocr_memory_tokens(ctypes.byref(self.cfg))
        self.batch = 0

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc, what):
        if rc != 0:
            raise MocrError(f"{what} failed ({rc}): {self.lib.mocr_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mocr_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def weight_count(self) -> int:
        return int(self.lib.mocr_weight_count(ctypes.byref(self.cfg)))

    # ------------------------------------------------------------------ weights
    def load_weights(self, weights):
        """``weights``: a flat float32 blob, or a state dict (numpy/torch values) with the
        reference key names (see ``weights.pack_state_dict``)."""
        from .weights import pack_state_dict
        blob = weights if isinstance(weights, np.ndarray) and weights.ndim == 1 else pack_state_dict(
            weights, vocab=self.vocab, max_pos=self.max_pos, n_layers=self.n_layers, arch=self.arch)
        blob = np.ascontiguousarray(blob, dtype=np.float32)
        self._check(self.lib.mocr_load_weights(self._h, _f32p(blob), blob.size), "mocr_load_weights")

    # ------------------------------------------------------------------ encoder
    def set_images(self, images):
        """images: [B,1,H,W] float32 numpy array, or a contiguous float32 torch tensor
        (CPU, or CUDA on this engine's device — then no host round trip)."""
        if hasattr(images, "data_ptr") and getattr(images, "is_cuda", False):
            B = int(images.shape[0])
            self._shape_check(tuple(images.shape))
            if not images.is_contiguous() or str(images.dtype) != "torch.float32":
                raise ValueError("device images must be contiguous float32")
            self._check(self.lib.mocr_set_images_device(self._h, ctypes.c_void_p(images.data_ptr()), B),
                        "mocr_set_images_device")
        else:
            if hasattr(images, "numpy"):
                images = images.detach().cpu().numpy()
            a = np.ascontiguousarray(images, dtype=np.float32)
            self._shape_check(a.shape)
            B = a.shape[0]
            self._check(self.lib.mocr_set_images(self._h, _f32p(a), B), "mocr_set_images")
        self.batch = B

    def set_encoder_pos(self, table):
        """ResNet18-trans: the positional table [M, 256] the encoder adds after the
        projection (drawn fresh per forward by the reference, src/model_res18trans.py:57-59;
        ``synth.make_pos_table(seed, M)`` is torch's draw after ``torch.manual_seed(seed)``)."""
        t = np.ascontiguousarray(table, dtype=np.float32)
        if t.shape != (self.memory_tokens, synth.D_MODEL):
            raise ValueError(f"positional table must be [{self.memory_tokens}, {synth.D_MODEL}], got {list(t.shape)}")
        self._check(self.lib.mocr_set_encoder_pos(self._h, _f32p(t), t.shape[0]), "mocr_set_encoder_pos")

    def _shape_check(self, shape):
        if len(shape) != 4 or shape[1] != 1 or tuple(shape[2:]) != self.img_hw:
            raise ValueError(f"images must be [B,1,{self.img_hw[0]},{self.img_hw[1]}], got {list(shape)}")
        if not 1 <= shape[0] <= self.max_batch:
            raise ValueError(f"batch {shape[0]} outside [1, {self.max_batch}]")

    def encode(self, images=None):
        if images is not None:
            self.set_images(images)
        self._check(self.lib.mocr_encode(self._h, self.batch), "mocr_encode")

    def memory(self) -> np.ndarray:
        out = np.empty((self.batch, self.memory_tokens, synth.D_MODEL), dtype=np.float32)
        self._check(self.lib.mocr_get_memory(self._h, _f32p(out)), "mocr_get_memory")
        return out

    def encode_until(self, k: int, shape) -> np.ndarray:
        """Encoder output after torchvision ``features[k]`` (NHWC ``shape``), for parity debugging."""
        out = np.empty(shape, dtype=np.float32)
        self._check(self.lib.mocr_debug_encode_until(self._h, self.batch, k, _f32p(out), out.size),
                    "mocr_debug_encode_until")
        return out

    # ------------------------------------------------------------------ decoder
    def decode(self, max_steps=150, stop="batch", forced=None, want_logp=False, want_logits=False) -> DecodeResult:
        B = self.batch
        ids = np.empty((B, max_steps + 1), dtype=np.int32)
        n = ctypes.c_int32(0)
        logp = np.empty((B, max_steps), dtype=np.float32) if want_logp else None
        logits = np.empty((B, max_steps, self.vocab), dtype=np.float32) if want_logits else None
        fp = None
        if forced is not None:
            f = np.ascontiguousarray(forced, dtype=np.int32)
            if f.shape != (B, max_steps + 1):
                raise ValueError(f"forced ids must be [B, max_steps+1] = {[B, max_steps + 1]}")
            fp = _i32p(f)
        rc = self.lib.mocr_decode(self._h, max_steps, STOP[stop], fp, _i32p(ids), ctypes.byref(n),
                                  _f32p(logp) if logp is not None else None,
                                  _f32p(logits) if logits is not None else None)
        self._check(rc, "mocr_decode")
        k = n.value
        return DecodeResult(ids[:, :k + 1], k, logp[:, :k] if logp is not None else None,
                            logits[:, :k] if logits is not None else None)

    def beam_search(self, beam=4, max_steps=256, stop="batch") -> BeamResult:
        """Beam search of the encoded batch (``mocr_decode_beam``; semantics:
        oracle/model_ref.py ``beam_search``)."""
        B = self.batch
        W = max_steps + 1
        beams = np.empty((B, beam, W), np.int32)
        scores = np.empty((B, beam), np.float32)
        n = ctypes.c_int32()
        self._check(self.lib.mocr_decode_beam(self._h, beam, max_steps, STOP[stop], None, _f32p(scores),
                                              _i32p(beams), ctypes.byref(n)), "mocr_decode_beam")
        k = n.value
        return BeamResult(ids=beams[:, 0, :k + 1].copy(), scores=scores, beams=beams[:, :, :k + 1].copy(), n_steps=k)

    def decode_into(self, ids_dev, max_steps=150, stop="batch") -> int:
        """Decode and write ids [B, max_steps+1] int32 into a device tensor (e.g. a torch
        CUDA tensor that is then all-gathered).  Returns the number of steps run.
        The C side writes batch x (max_steps + 1) int32 through the raw pointer, so the
        tensor is checked first (``check_ids_tensor``)."""
        check_ids_tensor(ids_dev, self.batch, max_steps, self.device)
        n = ctypes.c_int32(0)
        self._check(self.lib.mocr_decode_device(self._h, max_steps, STOP[stop], ctypes.c_void_p(ids_dev.data_ptr()),
                                                ctypes.byref(n)), "mocr_decode_device")
        return n.value

    def greedy(self, images, max_steps=150, stop="batch") -> DecodeResult:
        self.encode(images)
        return self.decode(max_steps, stop)

    def set_cu_mask(self, cus=None):
        """Run this engine's stream on the CUs in ``cus`` (iterable of CU indices; None:
        all CUs)."""
        if cus is None:
            self._check(self.lib.mocr_set_cu_mask(self._h, None, 0), "mocr_set_cu_mask")
            return
        cus = list(cus)
        words = (max(cus) // 32 + 1) if cus else 1
        arr = (ctypes.c_uint32 * words)()
        for c in cus:
            arr[c // 32] |= 1 << (c % 32)
        self._check(self.lib.mocr_set_cu_mask(self._h, arr, words), "mocr_set_cu_mask")

    def set_stream_priority(self, priority: int):
        """Recreate the engine's stream at the device's highest (> 0), lowest (< 0) or the
        normal (0) HIP stream priority."""
        self._check(self.lib.mocr_set_stream_priority(self._h, int(priority)), "mocr_set_stream_priority")

    # ------------------------------------------------------------------ timing
    def set_timing(self, enabled: bool):
        self._check(self.lib.mocr_set_timing(self._h, int(bool(enabled))), "mocr_set_timing")

    def timing(self):
        n = self.lib.mocr_get_timing(self._h, None, 0)
        if n < 0:
            self._check(n, "mocr_get_timing")
        buf = (KernelStat * max(n, 1))()
        self.lib.mocr_get_timing(self._h, buf, n)
        return {buf[i].name.decode(): dict(launches=buf[i].launches, total_ms=buf[i].total_ms, flops=buf[i].flops,
                                           bytes=buf[i].bytes) for i in range(n)}
