"""FastAPI surface of the reference (``app/src/main.py``) on top of the MI355X engine.

Routes and payloads follow the reference:

- ``POST /predict`` (:439-509): multipart image -> ``PredictionResponse``;
- ``POST /predict/batch`` (:511-595): 1..10 base64 images -> ``BatchPredictionResponse``;
- ``GET /status`` (:597), ``/health`` (:613), ``/model/info`` (:651), ``/metrics`` (:675).

Differences, all on the compute side:

- ``/predict/batch`` decodes every valid image of the request as ONE batch on the GPU. The reference loops image by image. Per-image results are unchanged; see ``im2latex.predict_batch``. If the batched call fails, each image is retried alone, so only the images that fail on their own are reported ``success: false`` (the reference's per-image error isolation, :562-570).
- ``/predict`` requests that arrive together are decoded together: a micro-batcher (``app/batcher.py``) opens a 2 ms window at the first request and sends every request inside it, up to the engine's ``max_batch``, to the engine as one call. Each request gets the result its image gets alone (the reference calls the model once per request, :486).
- Engine calls run in a worker thread. The reference calls the model synchronously on the event loop (:486). ctypes releases the GIL, and a lock serialises calls on the one engine.
- ``/metrics`` adds the engine's images/s and a histogram of engine-call latencies to the reference's keys.

Rate limiting, API keys, CORS and cloud logging are product policy, not the hot path, and
are not rebuilt: ``/health`` reports ``rate_limiter_initialized: false``
and does not count it, ``/metrics`` reports the rate limiter as not available, as the
reference does when its limiter is missing.
"""
from __future__ import annotations

import asyncio
import base64
import io
import os
import threading
import time
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional

import numpy as np
from fastapi import FastAPI, HTTPException, Request
from pydantic import BaseModel, Field, field_validator
from starlette.concurrency import run_in_threadpool

from .. import im2latex
from ..config import config
from ..preprocess import preprocess_image
from .batcher import MicroBatcher

API_TITLE = "Handwritten Math Formula Recognition API"
API_VERSION = "1.0.0"


# ---------------------------------------------------------------- schemas (app/src/models.py)
class PredictionResponse(BaseModel):
    formula: str
    confidence: Optional[float] = Field(None, ge=0.0, le=1.0)
    processing_time: float = Field(..., ge=0.0)
    timestamp: str


class BatchPredictionRequest(BaseModel):
    images: List[str] = Field(..., min_length=1, max_length=config.max_batch_images)

    @field_validator("images")
    @classmethod
    def _max_images(cls, v):
        if len(v) > config.max_batch_images:
            raise ValueError(f"Maximum {config.max_batch_images} images allowed per batch")
        return v


class BatchPredictionResponse(BaseModel):
    results: List[Dict[str, Any]]
    total_images: int
    successful_predictions: int
    processing_time: float
    timestamp: str


class StatusResponse(BaseModel):
    status: str
    api_version: str
    model_loaded: bool
    vocab_loaded: bool
    device: str
    model_load_time: Optional[float] = None
    total_predictions: int
    uptime: float


class HealthResponse(BaseModel):
    healthy: bool
    checks: Dict[str, Any]
    timestamp: str


def _now():
    return time.strftime("%Y-%m-%d %H:%M:%S")


def _multipart_file(body: bytes, content_type: str):
    """(filename, bytes) of the ``file`` field of a multipart/form-data body.

    python-multipart (what FastAPI's ``UploadFile`` needs) is not installed in this
    image, so the one file field the reference's /predict takes is parsed here.
    """
    import email.parser
    import email.policy
    if "multipart/form-data" not in content_type:
        raise HTTPException(status_code=400, detail="Expected multipart/form-data with a 'file' field")
    msg = email.parser.BytesParser(policy=email.policy.HTTP).parsebytes(
        b"Content-Type: " + content_type.encode() + b"\r\n\r\n" + body)
    for part in msg.iter_parts():
        if part.get_param("name", header="content-disposition") == "file":
            return part.get_filename(), part.get_payload(decode=True) or b""
    raise HTTPException(status_code=400, detail="Missing 'file' field")


def _decode_image(data: bytes):
    from PIL import Image
    try:
        return Image.open(io.BytesIO(data))
    except Exception as e:  # noqa: BLE001
        raise HTTPException(status_code=400, detail="Invalid image data") from e


# engine-call latency histogram bucket bounds (ms), Prometheus-style cumulative counts
LATENCY_BUCKETS_MS = (5, 10, 25, 50, 100, 250, 500, 1000, 2500)


class State:
    """Model state of one server process (the reference keeps module globals)."""

    def __init__(self, engine=None, vocab=None, idx2char=None, predictor: Optional[Callable] = None,
                 device: str = "cuda:0", model_dir: Optional[str] = None, checkpoint: str = "model.pth",
                 batch_window_ms: Optional[float] = None, max_batch: Optional[int] = None):
        """``batch_window_ms`` / ``max_batch``: the /predict micro-batcher's window (default
        ``MOCR_BATCH_WINDOW_MS`` or 2 ms) and largest batch (default the engine's
        ``max_batch``, or ``config.max_batch_images`` with an injected predictor)."""
        self.engine = engine
        self.vocab = vocab
        self.idx2char = idx2char
        self.predictor = predictor or (lambda imgs: im2latex.predict_batch(self.engine, imgs, self.vocab,
                                                                            self.idx2char))
        self.device = device
        self.model_dir = model_dir
        self.checkpoint = checkpoint
        self.lock = threading.Lock()
        self.start = time.time()
        self.load_time: Optional[float] = None
        self.predictions = 0
        self.images_done = 0
        self.gpu_seconds = 0.0
        self.latency_counts = [0] * (len(LATENCY_BUCKETS_MS) + 1)
        if batch_window_ms is None:
            batch_window_ms = float(os.environ.get("MOCR_BATCH_WINDOW_MS", "2"))
        if max_batch is None:
            max_batch = engine.max_batch if engine is not None else config.max_batch_images
        self.batch_window_ms = batch_window_ms
        self.max_batch = max_batch
        self._batcher: Optional[MicroBatcher] = None
        self._batcher_lock = threading.Lock()

    @property
    def batcher(self) -> MicroBatcher:
        """The /predict micro-batcher, started on first use."""
        with self._batcher_lock:
            if self._batcher is None:
                self._batcher = MicroBatcher(self.run, self.max_batch, self.batch_window_ms * 1e-3)
            return self._batcher

    def close(self):
        if self._batcher is not None:
            self._batcher.close()

    @property
    def loaded(self):
        return self.engine is not None or self.predictor is not None and self.vocab is not None

    def run(self, images: np.ndarray):
        with self.lock:
            t0 = time.time()
            out = self.predictor(images)
            dt = time.time() - t0
            self.gpu_seconds += dt
            self.images_done += images.shape[0]
            ms = dt * 1e3
            self.latency_counts[next((i for i, b in enumerate(LATENCY_BUCKETS_MS) if ms <= b),
                                     len(LATENCY_BUCKETS_MS))] += 1
            return out

    def device_available(self) -> bool:
        if self.engine is None:
            return self.predictor is not None  # injected predictor (tests): no device to check
        try:
            return self.engine.lib.mocr_device_count() > self.engine.device
        except Exception:  # noqa: BLE001
            return False


def load_state(model_dir: str, device: str = "cuda:0", precision: str = "bf16x3") -> State:
    """``initialize_model`` (:178-210): vocab.json + a state-dict checkpoint in model_dir."""
    from ..utils import load_vocab
    t0 = time.time()
    vocab, idx2char = load_vocab(os.path.join(model_dir, "vocab.json"))
    ckpt = next((os.path.join(model_dir, n) for n in ("model_state.pth", "best_model.pth", "model.pth")
                 if os.path.exists(os.path.join(model_dir, n))), None)
    if ckpt is None:
        raise FileNotFoundError(f"no checkpoint in {model_dir}")
    eng = im2latex.load_model(ckpt, vocab, device, precision=precision)
    st = State(eng, vocab, idx2char, device=device, model_dir=model_dir, checkpoint=os.path.basename(ckpt))
    st.load_time = time.time() - t0
    return st


def create_app(state: Optional[State] = None, model_dir: Optional[str] = None) -> FastAPI:
    app = FastAPI(title=API_TITLE, version=API_VERSION)
    holder = {"state": state}
    app_start = time.time()

    def get_state() -> State:
        if holder["state"] is None:
            if model_dir is None:
                raise HTTPException(status_code=500, detail="Model is not loaded")
            try:
                holder["state"] = load_state(model_dir)
            except Exception as e:  # noqa: BLE001
                raise HTTPException(status_code=500, detail=f"Model initialization failed: {e}") from e
        return holder["state"]

    @app.get("/")
    async def root():
        st = holder["state"]
        return {"title": API_TITLE, "version": API_VERSION, "model_loaded": bool(st and st.loaded)}

    @app.post("/predict", response_model=PredictionResponse)
    async def predict_formula(request: Request):
        t0 = time.time()
        st = get_state()
        filename, data = _multipart_file(await request.body(), request.headers.get("content-type", ""))
        if filename and Path(filename).suffix.lower() not in config.allowed_extensions:
            raise HTTPException(status_code=400,
                                detail=f"Invalid file format. Allowed: {', '.join(config.allowed_extensions)}")
        if not data:
            raise HTTPException(status_code=400, detail="Empty file uploaded")
        if len(data) > config.max_file_size:
            raise HTTPException(status_code=413, detail=f"File too large. Maximum size: {config.max_file_size} bytes")
        image = preprocess_image(_decode_image(data))
        try:
            # joins the requests arriving within the batching window: one engine call for all
            formula, confidence = await asyncio.wrap_future(st.batcher.submit(image))
        except Exception as e:  # noqa: BLE001
            raise HTTPException(status_code=500, detail=f"Prediction failed: {e}") from e
        st.predictions += 1
        return PredictionResponse(formula=formula, confidence=confidence, processing_time=time.time() - t0,
                                  timestamp=_now())

    @app.post("/predict/batch", response_model=BatchPredictionResponse)
    async def predict_batch(req: BatchPredictionRequest):
        t0 = time.time()
        st = get_state()
        results: List[Dict[str, Any]] = [None] * len(req.images)  # type: ignore[list-item]
        ok_idx, tensors = [], []
        for i, b64 in enumerate(req.images):
            try:
                data = base64.b64decode(b64)
                tensors.append(preprocess_image(_decode_image(data)))
                ok_idx.append(i)
            except Exception as e:  # noqa: BLE001 - per-image failure, as the reference
                detail = e.detail if isinstance(e, HTTPException) else str(e)
                results[i] = {"index": i, "formula": "", "confidence": None, "success": False, "error": detail}
        if tensors:
            try:
                preds = await run_in_threadpool(st.run, np.concatenate(tensors, 0))
            except Exception:  # noqa: BLE001 - isolate the failing images (reference :562-570)
                preds = []
                for t in tensors:
                    try:
                        preds.append((await run_in_threadpool(st.run, t))[0])
                    except Exception as e:  # noqa: BLE001
                        preds.append(e)
            for i, pr in zip(ok_idx, preds):
                if isinstance(pr, Exception):
                    results[i] = {"index": i, "formula": "", "confidence": None, "success": False, "error": str(pr)}
                else:
                    formula, confidence = pr
                    results[i] = {"index": i, "formula": formula, "confidence": confidence, "success": True}
        st.predictions += len(req.images)
        ok = sum(1 for r in results if r["success"])
        return BatchPredictionResponse(results=results, total_images=len(req.images), successful_predictions=ok,
                                       processing_time=time.time() - t0, timestamp=_now())

    @app.get("/status", response_model=StatusResponse)
    async def status():
        st = holder["state"]
        return StatusResponse(status="healthy" if st and st.loaded else "unhealthy", api_version=API_VERSION,
                              model_loaded=bool(st and st.loaded),
                              vocab_loaded=bool(st and st.vocab is not None and st.idx2char is not None),
                              device=st.device if st else "none", model_load_time=st.load_time if st else None,
                              total_predictions=st.predictions if st else 0,
                              uptime=time.time() - (st.start if st else time.time()))

    @app.get("/health", response_model=HealthResponse)
    async def health():
        """Reference keys (:613-649); the rate limiter is not rebuilt."""
        st = holder["state"]
        mdir = (st.model_dir if st else None) or model_dir
        files = {}
        if mdir:
            ckpt = st.checkpoint if st else "model.pth"
            files = {ckpt: os.path.exists(os.path.join(mdir, ckpt)),
                     "vocab.json": os.path.exists(os.path.join(mdir, "vocab.json"))}
        checks = {"model_loaded": bool(st and st.loaded),
                  "vocab_loaded": bool(st and st.vocab is not None and st.idx2char is not None),
                  "device_available": bool(st and st.device_available()),
                  "rate_limiter_initialized": False,
                  "model_files_exist": files,
                  "environment": os.environ.get("ENVIRONMENT", "production")}
        healthy = (checks["model_loaded"] and checks["vocab_loaded"] and checks["device_available"]
                   and all(files.values()))
        return HealthResponse(healthy=healthy, checks=checks, timestamp=_now())

    @app.get("/model/info")
    async def model_info():
        """Reference keys (:651-673); 503 until the model is loaded."""
        st = holder["state"]
        if st is None or not st.loaded:
            raise HTTPException(status_code=503, detail="Model not loaded")
        eng = st.engine
        return {"model_config": {"img_height": config.img_h, "img_width": config.img_w, "d_model": config.d_model,
                                 "num_heads": config.nhead, "num_decoder_layers": config.num_decoder_layers,
                                 "dim_feedforward": config.dim_feedforward, "dropout": config.dropout,
                                 "max_seq_len": config.max_seq_len},
                "vocab_info": {"vocab_size": len(st.vocab) if st.vocab else 0,
                               "special_tokens": config.special_tokens},
                "device": st.device,
                # the engine's weights: the parameters the forward pass uses (the reference
                # also counts the registered but unused swin.norm / swin.head)
                "model_parameters": eng.weight_count() if eng is not None else 0,
                "engine": {"precision": eng.precision, "max_batch": eng.max_batch,
                           "arch": eng.arch} if eng is not None else None}

    @app.get("/metrics")
    async def metrics():
        """Reference keys (:675-702) plus the engine's throughput and call latencies."""
        import psutil
        st = holder["state"]
        uptime = time.time() - (st.start if st else app_start)
        total = st.predictions if st else 0
        out = {"predictions": {"total": total, "rate_per_second": total / uptime if uptime > 0 else 0},
               "system": {"cpu_percent": psutil.cpu_percent(), "memory_percent": psutil.virtual_memory().percent,
                          "disk_percent": psutil.disk_usage("/").percent},
               "rate_limiter": {"error": "Rate limiter not available"},
               "uptime_seconds": uptime}
        if st is not None:
            cum, buckets = 0, {}
            for b, n in zip(list(LATENCY_BUCKETS_MS) + ["+Inf"], st.latency_counts):
                cum += n
                buckets[f"le_{b}"] = cum
            b = st._batcher
            out["engine"] = {"images_processed": st.images_done, "engine_seconds": st.gpu_seconds,
                             "images_per_engine_second": st.images_done / st.gpu_seconds if st.gpu_seconds else None,
                             "call_latency_ms_histogram": buckets,
                             "predict_microbatch": {"window_ms": st.batch_window_ms, "max_batch": st.max_batch,
                                                    "engine_calls": b.calls if b else 0,
                                                    "mean_batch": (sum(b.batch_sizes) / len(b.batch_sizes))
                                                    if b and b.batch_sizes else None}}
        return out

    return app


app = create_app(model_dir=os.environ.get("MOCR_MODEL_DIR"))
