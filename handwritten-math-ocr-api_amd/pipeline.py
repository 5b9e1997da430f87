"""Batch pipelining on one GPU: R engine replicas, one host thread each.

A greedy decode step is a chain of small, latency-bound kernels, while the encoder is a
throughput-bound stream of large GEMMs.  Calls are independent, so R engines on the same
device, each driven by its own thread (ctypes releases the GIL; each engine has its own
HIP stream), overlap one call's decode with another call's encoder.  The GPU time of the
two halves still adds up rather than hiding one behind the other (docs/DESIGN_history_r01-r05.md §5.6;
tools/pipeline_probe.py measures encode-only, decode-only and both).

``imap`` preserves submission order, so callers can run an order-sensitive step
(e.g. the RCCL gather of token streams in ``bench.py``) on the results, identically on
every rank.
"""
from __future__ import annotations

import queue
import threading

from .engine import Engine


class ReplicaPool:
    def __init__(self, n_replicas: int = 3, engines=None, **engine_kwargs):
        if engines is not None:
            self.engines = list(engines)
        else:
            if n_replicas < 1:
                raise ValueError("n_replicas must be >= 1")
            self.engines = [Engine(**engine_kwargs) for _ in range(n_replicas)]

    def __len__(self):
        return len(self.engines)

    def load_weights(self, weights):
        from .weights import pack_state_dict
        e0 = self.engines[0]
        blob = weights if hasattr(weights, "ndim") and weights.ndim == 1 else pack_state_dict(
            weights, vocab=e0.vocab, max_pos=e0.max_pos, n_layers=e0.n_layers, arch=e0.arch)
        for e in self.engines:
            e.load_weights(blob)

    def imap(self, fn, items):
        """Yield fn(engine, item) for each item, in order; items run concurrently on the
        replicas (item i on a free replica).  Exceptions are re-raised in order."""
        items = list(items)
        work = queue.Queue()
        for i, it in enumerate(items):
            work.put((i, it))
        done = {}
        cv = threading.Condition()

        def worker(eng):
            while True:
                try:
                    i, it = work.get_nowait()
                except queue.Empty:
                    return
                try:
                    r = (True, fn(eng, it))
                except BaseException as ex:  # noqa: BLE001 - forwarded to the caller
                    r = (False, ex)
                with cv:
                    done[i] = r
                    cv.notify_all()

        threads = [threading.Thread(target=worker, args=(e,), daemon=True) for e in self.engines]
        for t in threads:
            t.start()
        try:
            for i in range(len(items)):
                with cv:
                    while i not in done:
                        cv.wait()
                    ok, val = done.pop(i)
                if not ok:
                    raise val
                yield val
        finally:
            for t in threads:
                t.join()

    def close(self):
        for e in self.engines:
            e.close()
