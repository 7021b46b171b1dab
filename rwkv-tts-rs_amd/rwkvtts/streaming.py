"""StreamingInference on the MI355X engine (host mirror of src/streaming_inference.rs:14-416).

The reference's type surface is kept -- InferenceRequest{id, tokens, context_length, priority,
cache_result}, InferenceResult{request_id, logits, inference_time, from_cache, completed_at},
BatchConfig, StreamingStats, start/stop/submit_request/get_stats/reset_stats/adjust_batch_size
-- but the body is real: the reference's `process_batch` fills logits with random numbers
(:329-360); here a scheduler thread collects up to max_batch_size requests in priority order
(highest first, FIFO within a priority, :289-320) and runs them as ONE ragged `infer` over
fresh state slots, returning each request's last-token logits. Results with cache_result are
memoised by token sequence (the reference keeps a result cache keyed the same way).
"""
import dataclasses
import threading
import time
from collections import deque
from concurrent.futures import Future
from typing import Dict, List, Optional, Sequence

import numpy as np

from .runtime import RnnInput, RnnInputBatch, SharedRwkvRuntime


@dataclasses.dataclass
class InferenceRequest:  # :14-55
    id: str
    tokens: List[int]
    context_length: int = 0
    priority: int = 5
    created_at: float = dataclasses.field(default_factory=time.monotonic)
    cache_result: bool = True

    def with_priority(self, priority: int) -> "InferenceRequest":
        self.priority = priority
        return self

    def with_cache(self, cache_result: bool) -> "InferenceRequest":
        self.cache_result = cache_result
        return self


@dataclasses.dataclass
class InferenceResult:  # :57-69
    request_id: str
    logits: np.ndarray
    inference_time: float
    from_cache: bool
    completed_at: float


@dataclasses.dataclass
class BatchConfig:  # :72-97
    max_batch_size: int = 8
    batch_timeout: float = 0.050
    dynamic_batching: bool = True
    min_batch_size: int = 2
    prefetch_window: int = 4


@dataclasses.dataclass
class StreamingStats:  # :99-135
    total_requests: int = 0
    total_batches: int = 0
    cache_hits: int = 0
    avg_batch_size: float = 0.0
    avg_inference_time_ms: float = 0.0
    avg_wait_time_ms: float = 0.0
    prefetch_hits: int = 0
    pipeline_efficiency: float = 0.0

    def cache_hit_rate(self) -> float:
        return 0.0 if self.total_requests == 0 else self.cache_hits / self.total_requests

    def reset(self):
        for f in dataclasses.fields(self):
            setattr(self, f.name, f.default)


class StreamingInference:  # :141-416
    def __init__(self, runtime: SharedRwkvRuntime, config: Optional[BatchConfig] = None):
        self.runtime = runtime
        self.config = config or BatchConfig()
        self._queues: Dict[int, deque] = {}
        self._lock = threading.Lock()
        self._wake = threading.Condition(self._lock)
        self._cache: Dict[tuple, np.ndarray] = {}
        self._stats = StreamingStats()
        self._thread: Optional[threading.Thread] = None
        self._running = False

    # ---- lifecycle (:178-227)
    def start(self):
        if self._running:
            return
        self._running = True
        self._thread = threading.Thread(target=self._scheduler, name="rwkvtts-streaming", daemon=True)
        self._thread.start()

    def stop(self):
        with self._lock:
            self._running = False
            self._wake.notify_all()
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    # ---- submission (:229-270)
    def submit_request(self, request: InferenceRequest, timeout: float = 30.0) -> InferenceResult:
        if not self._running:
            raise RuntimeError("StreamingInference is not running")
        if not request.tokens:
            raise ValueError("request has no tokens")
        key = tuple(request.tokens)
        with self._lock:
            self._stats.total_requests += 1
            if request.cache_result and key in self._cache:
                self._stats.cache_hits += 1
                now = time.monotonic()
                return InferenceResult(request.id, self._cache[key].copy(), 0.0, True, now)
            fut: Future = Future()
            self._queues.setdefault(request.priority, deque()).append((request, fut))
            self._wake.notify()
        return fut.result(timeout=timeout)

    def _collect(self) -> List[tuple]:  # :289-320: highest priority first, FIFO inside
        batch = []
        for prio in sorted(self._queues, reverse=True):
            q = self._queues[prio]
            while q and len(batch) < min(self.config.max_batch_size, self.runtime.max_slots):
                batch.append(q.popleft())
        return batch

    def _scheduler(self):
        while True:
            with self._lock:
                while self._running and not any(self._queues.values()):
                    self._wake.wait(self.config.batch_timeout)
                if not self._running:
                    pending = [x for q in self._queues.values() for x in q]
                    self._queues.clear()
                    for _, fut in pending:
                        fut.set_exception(RuntimeError("StreamingInference stopped"))
                    return
                batch = self._collect()
            if batch:
                self._process(batch)

    def _process(self, batch: Sequence[tuple]):
        t0 = time.monotonic()
        slots = list(range(len(batch)))
        inp = RnnInput([RnnInputBatch(list(r.tokens)) for r, _ in batch], self.runtime.token_chunk_size)
        outs = [None] * len(batch)
        try:
            # the whole batch (slot resets + every infer call) holds the runtime's lock, so another
            # thread's generate_batch / infer on the same engine cannot touch these slots meanwhile
            with self.runtime._lock:
                for s in slots:
                    self.runtime.reset_slot(s)
                while any(o is None for o in outs):  # feed until every request produced its logits
                    idx = [i for i, o in enumerate(outs) if o is None]
                    sub = RnnInput([inp.batches[i] for i in idx], inp.token_chunk_size)
                    rem, got = self.runtime.infer(sub, slots=[slots[i] for i in idx])
                    for j, i in enumerate(idx):
                        inp.batches[i] = rem.batches[j]
                        if got[j].size:
                            outs[i] = got[j]
        except Exception as ex:  # noqa: BLE001 -- every waiter gets the failure
            for _, fut in batch:
                fut.set_exception(ex)
            return
        dt = time.monotonic() - t0
        now = time.monotonic()
        with self._lock:
            st = self._stats
            st.total_batches += 1
            st.avg_batch_size += (len(batch) - st.avg_batch_size) / st.total_batches
            st.avg_inference_time_ms += (1000.0 * dt - st.avg_inference_time_ms) / st.total_batches
            waits = [1000.0 * (t0 - r.created_at) for r, _ in batch]
            st.avg_wait_time_ms += (float(np.mean(waits)) - st.avg_wait_time_ms) / st.total_batches
            for (r, _), lg in zip(batch, outs):
                if r.cache_result:
                    self._cache[tuple(r.tokens)] = lg
        for (r, fut), lg in zip(batch, outs):
            fut.set_result(InferenceResult(r.id, lg, dt, False, now))

    # ---- stats / config (:380-416)
    def get_stats(self) -> StreamingStats:
        with self._lock:
            return dataclasses.replace(self._stats)

    def reset_stats(self):
        with self._lock:
            self._stats.reset()

    def adjust_batch_size(self, target_latency_ms: float):
        """:390-406: over 1.2x the target latency shrink the batch (floor min_batch_size),
        under 0.8x grow it (cap 16)."""
        if not self.config.dynamic_batching:
            return
        cur = self.get_stats().avg_inference_time_ms
        if cur > target_latency_ms * 1.2:
            self.config.max_batch_size = max(self.config.max_batch_size - 1, self.config.min_batch_size)
        elif cur < target_latency_ms * 0.8:
            self.config.max_batch_size = min(self.config.max_batch_size + 1, 16)

    def get_config(self) -> BatchConfig:
        return self.config

    def update_config(self, config: BatchConfig):
        self.config = config
