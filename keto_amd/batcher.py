"""Request batcher in front of the check engine.

The reference answers every ``Check`` RPC / REST call on its own goroutine
(``internal/check/handler.go:144-275``, gRPC ``Check`` at :248), one ``CheckIsMember`` each.  The
GPU engine wants batches, so concurrent callers submit here and a dispatcher thread gathers
whatever is pending into one ``kg_check_batch`` call: a batch closes when it reaches
``max_batch`` queries or when its oldest query has waited ``max_wait_us``.  Each caller gets the
answer of a loop of ``CheckIsMember``: allowed, or the per-query error.

While one batch runs on the GPU the next one fills, so under load the batch size grows to match
the arrival rate and the GPU stays busy; at low load a query waits at most ``max_wait_us`` plus
one batch.  ``latency_percentile`` reports the batch latency (submission of the oldest query to
its answer) that BASELINE.json's p99 metric names.
"""
from __future__ import annotations

import collections
import ctypes as C
import threading
import time
from concurrent.futures import Future
from typing import List, Optional, Tuple

import numpy as np

from . import _lib
from .engine import CheckError, Engine, queries_array
from .ketoapi import RelationTuple


class BatcherClosed(RuntimeError):
    pass


class CheckBatcher:
    STATS_WINDOW = 1 << 16  # latency / size samples kept (the most recent batches)

    def __init__(self, engine: Engine, max_batch: int = 1 << 16, max_wait_us: int = 200):
        if max_batch < 1 or max_wait_us < 0:
            raise ValueError("max_batch >= 1 and max_wait_us >= 0 required")
        self.engine = engine
        self.max_batch = max_batch
        self.max_wait = max_wait_us * 1e-6
        self._cv = threading.Condition()
        self._pending: List[Tuple[np.ndarray, Future, float]] = []
        self._closed = False
        self.batch_sizes: "collections.deque[int]" = collections.deque(maxlen=self.STATS_WINDOW)
        self.batch_latency_s: "collections.deque[float]" = collections.deque(maxlen=self.STATS_WINDOW)
        self.cancelled = 0
        self._thread = threading.Thread(target=self._run, name="kg-check-batcher", daemon=True)
        self._thread.start()

    # ---- submission
    def submit_ids(self, q7) -> Future:
        """One kg_query row (ns, obj, rel, sns, sobj, srel, max_depth) -> Future[(result u8, err u32)]."""
        row = np.ascontiguousarray(q7, np.uint32).reshape(7)
        f: Future = Future()
        with self._cv:
            if self._closed:
                raise BatcherClosed("batcher is closed")
            self._pending.append((row, f, time.perf_counter()))
            if len(self._pending) == 1 or len(self._pending) >= self.max_batch:
                self._cv.notify()
        return f

    def submit(self, t: RelationTuple, rest_depth: int) -> Future:
        it = getattr(self.engine, "interner", None) or self.engine.snapshot.interner  # a live engine: no rebuild
        return self.submit_ids(queries_array(np.asarray(it.tuple_ids(t), np.uint32), rest_depth)[0])

    def check_is_member(self, t: RelationTuple, rest_depth: int, timeout: Optional[float] = None) -> bool:
        """CheckIsMember through the batcher (internal/check/engine.go:54-60)."""
        res, err = self.submit(t, rest_depth).result(timeout)
        if res == _lib.KG_ERROR:
            raise CheckError(err)
        return res == _lib.KG_IS_MEMBER

    # ---- dispatcher
    def _take(self) -> List[Tuple[np.ndarray, Future, float]]:
        """The next batch of live (not cancelled) queries; [] once closed and drained."""
        while True:
            with self._cv:
                while not self._pending and not self._closed:
                    self._cv.wait()
                if not self._pending:
                    return []
                deadline = self._pending[0][2] + self.max_wait
                while len(self._pending) < self.max_batch and not self._closed:
                    left = deadline - time.perf_counter()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                batch, self._pending = self._pending[:self.max_batch], self._pending[self.max_batch:]
            # a caller may have cancelled its future (directly, or through asyncio.wrap_future when its
            # RPC was cancelled): drop it here, so result delivery never meets a cancelled future
            live = [b for b in batch if b[1].set_running_or_notify_cancel()]
            self.cancelled += len(batch) - len(live)
            if live:
                return live

    @staticmethod
    def _deliver(f: Future, result=None, exc: Optional[BaseException] = None) -> None:
        try:  # one broken future must never end the dispatcher (every later submit would hang)
            if exc is not None:
                f.set_exception(exc)
            else:
                f.set_result(result)
        except Exception:  # noqa: BLE001 -- InvalidStateError and the like
            pass

    def _run(self) -> None:
        while True:
            batch = self._take()
            if not batch:
                return
            q = np.stack([b[0] for b in batch])
            try:
                out, err = self.engine.batch_check_ids(q)
            except BaseException as e:  # the whole batch failed (library status): every caller sees it
                for _, f, _t in batch:
                    self._deliver(f, exc=e)
                continue
            done = time.perf_counter()
            self.batch_sizes.append(len(batch))
            self.batch_latency_s.append(done - batch[0][2])
            for i, (_, f, _t) in enumerate(batch):
                self._deliver(f, (int(out[i]), int(err[i])))

    # ---- lifecycle / stats
    def close(self) -> None:
        """Stop accepting queries; pending ones are still answered."""
        with self._cv:
            self._closed = True
            self._cv.notify_all()
        self._thread.join()

    def __enter__(self) -> "CheckBatcher":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def latency_percentile(self, p: float = 99.0) -> float:
        """Batch latency percentile in ms (oldest submission -> answers delivered)."""
        if not self.batch_latency_s:
            return 0.0
        return float(np.percentile(np.asarray(self.batch_latency_s), p) * 1e3)


class NativeBatcher:
    """The library's request batcher (kg_batcher_*, keto_amd/csrc/kg_batcher.cpp): one BLOCKING call
    per request, the shape a Go handler goroutine binds through cgo.  Calls from
    many Python threads run concurrently in the library (ctypes releases the GIL for the wait)."""

    def __init__(self, snapshot, max_read_depth: int = 5, max_batch: int = 1 << 16, max_wait_us: int = 200,
                 dispatchers: int = 4):
        self.snapshot = snapshot
        self.L = _lib.load()
        self._h = C.c_void_p()
        _lib.check(self.L.kg_batcher_create(snapshot.handle, max_read_depth, max_batch, max_wait_us, dispatchers,
                                            C.byref(self._h)), "kg_batcher_create")

    @property
    def handle(self):
        return self._h

    def check_ids(self, q) -> Tuple[np.ndarray, np.ndarray]:
        """(n, 7) kg_query rows of ONE caller -> (result u8, err u32); blocks until answered."""
        q = np.ascontiguousarray(q, np.uint32).reshape(-1, 7)
        out = np.zeros(q.shape[0], np.uint8)
        err = np.zeros(q.shape[0], np.uint32)
        _lib.check(self.L.kg_batcher_check(self._h, q.ctypes.data_as(C.c_void_p), q.shape[0],
                                           out.ctypes.data_as(C.c_void_p), err.ctypes.data_as(C.c_void_p)),
                   "kg_batcher_check")
        return out, err

    def check_is_member(self, t: RelationTuple, rest_depth: int) -> bool:
        """CheckIsMember through the native batcher (internal/check/engine.go:54-60)."""
        it = self.snapshot.interner
        out, err = self.check_ids(queries_array(np.asarray(it.tuple_ids(t), np.uint32), rest_depth))
        if out[0] == _lib.KG_ERROR:
            raise CheckError(int(err[0]))
        return bool(out[0] == _lib.KG_IS_MEMBER)

    def stats(self) -> dict:
        st = _lib.kg_batcher_stats_t()
        _lib.check(self.L.kg_batcher_stats(self._h, C.byref(st)), "kg_batcher_stats")
        return {n: getattr(st, n) for n, _ in st._fields_}

    def reset_stats(self) -> None:
        self.L.kg_batcher_reset_stats(self._h)

    def close(self) -> None:
        if self._h:
            self.L.kg_batcher_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self) -> "NativeBatcher":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
