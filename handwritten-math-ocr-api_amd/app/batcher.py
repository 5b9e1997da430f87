"""Micro-batching of concurrent single-image ``/predict`` requests (the serving
surface "truly batched").

The reference serves ``POST /predict`` one image per model call, synchronously on the event
loop (``app/src/main.py:439-509``, ``im2latex.predict`` at :486).  On the GPU a decode
step over 8 rows costs about what one over 1 row costs (the step is a chain of dependent
launches), so requests that arrive together are decoded together: the
first request opens a window of ``window_s`` (2 ms by default), every request that arrives
inside it joins, up to ``max_batch``, and the batch goes to the engine as ONE call
(``im2latex.predict_batch``).  Each request gets its own row's result, which equals the
single-image result: Swin rows are independent and the decode's k order does not depend on
the batch (``tests/test_gpu_parity.py::test_serving_predict_matches_reference``), and a
row's tokens up to its EOS do not depend on when the batch-global stop ends the loop.

If a batched call raises, each image of it is retried alone, so only the requests whose
image fails on its own see the error (the per-image isolation of the reference's batch
route, :562-570).
"""
from __future__ import annotations

import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, List, Optional

import numpy as np


class _Item:
    __slots__ = ("image", "future")

    def __init__(self, image: np.ndarray):
        self.image = image
        self.future: Future = Future()


class MicroBatcher:
    """Collects single-image requests into engine calls on one worker thread.

    ``run(images[N, 1, H, W]) -> list of N results`` is the engine call (``State.run``);
    ``submit(image[1, 1, H, W])`` returns a ``concurrent.futures.Future`` of that image's
    result.  ``calls`` counts engine calls and ``batch_sizes`` records each call's size
    (``/metrics``)."""

    def __init__(self, run: Callable[[np.ndarray], List], max_batch: int, window_s: float = 0.002):
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self.run = run
        self.max_batch = int(max_batch)
        self.window_s = float(window_s)
        self.calls = 0
        self.batch_sizes: List[int] = []
        self._q: "queue.Queue[Optional[_Item]]" = queue.Queue()
        self._closed = False
        self._thread = threading.Thread(target=self._loop, name="mocr-microbatch", daemon=True)
        self._thread.start()

    def submit(self, image: np.ndarray) -> Future:
        image = np.ascontiguousarray(image, dtype=np.float32)
        if image.ndim != 4 or image.shape[0] != 1:
            raise ValueError(f"one image [1, C, H, W] per request, got {list(image.shape)}")
        if self._closed:
            raise RuntimeError("micro-batcher is closed")
        it = _Item(image)
        self._q.put(it)
        return it.future

    def close(self, timeout: float = 5.0):
        if not self._closed:
            self._closed = True
            self._q.put(None)
            self._thread.join(timeout)

    # ---------------------------------------------------------------- worker
    def _loop(self):
        stop = False
        while not stop:
            first = self._q.get()
            if first is None:
                break
            items = [first]
            deadline = time.monotonic() + self.window_s
            while len(items) < self.max_batch:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    nxt = self._q.get(timeout=left)
                except queue.Empty:
                    break
                if nxt is None:
                    stop = True
                    break
                items.append(nxt)
            # one engine call per image shape (every /predict image is preprocessed to the
            # model's shape, so normally one)
            by_shape = {}
            for it in items:
                by_shape.setdefault(it.image.shape, []).append(it)
            for group in by_shape.values():
                self._dispatch(group)
        # drain: requests queued behind the close sentinel fail instead of hanging
        while True:
            try:
                it = self._q.get_nowait()
            except queue.Empty:
                break
            if it is not None:
                it.future.set_exception(RuntimeError("micro-batcher is closed"))

    def _call(self, images: np.ndarray):
        self.calls += 1
        self.batch_sizes.append(images.shape[0])
        out = self.run(images)
        if len(out) != images.shape[0]:
            raise RuntimeError(f"engine returned {len(out)} results for {images.shape[0]} images")
        return out

    def _dispatch(self, items: List[_Item]):
        try:
            outs = self._call(np.concatenate([it.image for it in items], 0))
        except Exception as e:  # noqa: BLE001
            if len(items) == 1:
                items[0].future.set_exception(e)
                return
            for it in items:  # isolate the failing images
                try:
                    it.future.set_result(self._call(it.image)[0])
                except Exception as e1:  # noqa: BLE001
                    it.future.set_exception(e1)
            return
        for it, o in zip(items, outs):
            it.future.set_result(o)
