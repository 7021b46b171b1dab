"""Host-side mirror of the reference's runtime / sampler / batch-manager interfaces, over the
C-ABI (include/rwkvtts.h). Names and argument meaning follow the Rust originals:

* `SharedRwkvRuntime`      -- src/shared_runtime.rs:44-284 (model load, state slots, infer)
* `RnnInput`, `RnnInputBatch`, `RnnOption` -- web-rwkv runtime::infer types as used at
  src/normal_mode_inference.rs:62-80 (a call consumes <= token_chunk_size tokens and returns
  the remaining input; an output's logits are empty while its input is still pending)
* `StdRng`                 -- rand 0.8 StdRng::seed_from_u64 (stateless key + draw index)
* `sample_logits_with_top_p_k` -- src/rwkv_sampler.rs:55-211, run on the GPU
* `SamplerArgs`, `TtsBatchRequest`, `DynamicBatchConfig` -- src/rwkv_sampler.rs:222-290,
  src/batch_types.rs:67-97
* `DynamicBatchManager`    -- src/dynamic_batch_manager.rs:22-164: generate_tts /
  generate_tts_batch over the native request manager (include/rwkvtts.h rwkvtts_manager_*):
  thread-safe submit, the reference's collect window, one engine per GPU, continuous batching.
"""
import ctypes
import dataclasses
import threading
from typing import List, Optional, Sequence

import numpy as np

from . import _ffi
from ._ffi import check, lib


class StdRng:
    """rand 0.8.5 StdRng (ChaCha12) as (32-byte key, next-draw index)."""

    def __init__(self, rng_struct):
        self._s = rng_struct

    @classmethod
    def seed_from_u64(cls, seed: int) -> "StdRng":
        s = _ffi.Rng()
        lib().rwkvtts_rng_seed_from_u64(ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), ctypes.byref(s))
        return cls(s)

    @property
    def key(self):
        return list(self._s.key)

    @property
    def draw_index(self):
        return int(self._s.draw_index)


class RnnOption:
    Last = _ffi.OPT_LAST
    Full = _ffi.OPT_FULL


@dataclasses.dataclass
class RnnInputBatch:
    tokens: List[int]
    option: int = RnnOption.Last

    def push(self, tok: int):
        self.tokens.append(int(tok))


@dataclasses.dataclass
class RnnInput:
    batches: List[RnnInputBatch]
    token_chunk_size: int = 512


def _locked(fn):
    def wrapper(self, *a, **k):
        with self._lock:
            return fn(self, *a, **k)
    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    return wrapper


def request_struct(r: "TtsBatchRequest"):
    """TtsBatchRequest -> (_ffi.Request, keepalive arrays)."""
    keep = []

    def arr(x):
        if x is None:
            return None
        a = np.ascontiguousarray(np.asarray(x, dtype=np.int32))
        keep.append(a)
        return a
    P = ctypes.POINTER(ctypes.c_int32)
    q = _ffi.Request()
    tt, pt, rg, rs = arr(r.text_tokens), arr(r.property_tokens), arr(r.ref_global_tokens), arr(r.ref_semantic_tokens)
    q.text_tokens = tt.ctypes.data_as(P) if tt is not None and len(tt) else None
    q.n_text = 0 if tt is None else len(tt)
    q.property_tokens = pt.ctypes.data_as(P) if pt is not None and len(pt) else None
    q.n_property = 0 if pt is None else len(pt)
    # Some(empty) stays distinguishable from None: a non-null pointer with count 0
    q.ref_global = (rg.ctypes.data_as(P) if len(rg) else ctypes.cast(ctypes.pointer(_EMPTY), P)) if rg is not None else None
    q.n_ref_global = 0 if rg is None else len(rg)
    q.ref_semantic = (rs.ctypes.data_as(P) if len(rs) else ctypes.cast(ctypes.pointer(_EMPTY), P)) if rs is not None else None
    q.n_ref_semantic = 0 if rs is None else len(rs)
    q.has_seed = 0 if r.args.seed is None else 1
    q.seed = 0 if r.args.seed is None else int(r.args.seed) & 0xFFFFFFFFFFFFFFFF
    q.max_tokens = int(r.args.max_tokens)
    q.fixed_semantic = r.fixed_semantic
    q.greedy = 1 if r.greedy else 0
    lr = r.args.layered_randomness
    q.layered_set = 1
    q.use_independent_seeds = 1 if lr.use_independent_seeds else 0
    q.global_seed_offset = int(lr.global_seed_offset) & 0xFFFFFFFFFFFFFFFF
    q.semantic_seed_offset = int(lr.semantic_seed_offset) & 0xFFFFFFFFFFFFFFFF
    return q, keep


_EMPTY = ctypes.c_int32(0)


def _unpack_results(res, sem_bufs):
    """(global, semantic) per request; a failed request gives ([], []) like
    dynamic_batch_manager.rs:466-469. Also returns the per-request status codes."""
    out, status = [], []
    for i in range(len(res)):
        status.append(int(res[i].status))
        if res[i].status != 0:
            out.append(([], []))
            continue
        out.append((list(res[i].global_tokens[:res[i].n_global]), sem_bufs[i][:res[i].n_semantic].tolist()))
    return out, status


def parse_quant_type(s) -> int:
    """bin/server.rs:1029-1056 (parse_quant_type): none / int8 / nf4 / sf4, case-insensitive;
    anything else is an error. SF4 parses but the engine rejects it (table not available)."""
    if isinstance(s, int):
        return s
    t = {"none": _ffi.QUANT_NONE, "int8": _ffi.QUANT_INT8, "nf4": _ffi.QUANT_NF4, "sf4": _ffi.QUANT_SF4}.get(str(s).lower())
    if t is None:
        raise ValueError(f"unsupported quant type: {s}. supported: none, int8, nf4, sf4")
    return t


def quant_config(quant_layers: int, quant_type) -> tuple:
    """bin/server.rs:1059-1071 (create_quant_config): layers [0, quant_layers) quantised, or none."""
    t = parse_quant_type(quant_type)
    if quant_layers <= 0 or t == _ffi.QUANT_NONE:
        return 0, _ffi.QUANT_NONE
    return int(quant_layers), t


class SharedRwkvRuntime:
    """One engine per GPU: weights resident in HBM, `max_concurrent_batches` state slots.
    quant_layers / quant_type: the server's --quant-layers / --quant-type (web-rwkv Quant).
    forms: rwkvtts_engine_desc.forms (_ffi.FORM_*; 0 = the shipping decode forms)."""

    def __init__(self, weights: np.ndarray, device: int = 0, max_slots: int = 10,
                 token_chunk_size: int = 512, use_graphs: bool = True, weights_on_device: bool = False,
                 device_ptr: Optional[int] = None, wkv_variant: int = 0, quant_layers: int = 0,
                 quant_type="none", forms: int = 0):
        # the C ABI serialises calls per engine; this lock also keeps Python-side buffers of one
        # call from interleaving with another thread's
        self._lock = threading.RLock()
        ql, qt = quant_config(quant_layers, quant_type)
        desc = _ffi.EngineDesc(device, max_slots, token_chunk_size, 1 if use_graphs else 0, wkv_variant, ql, qt, forms)
        h = ctypes.c_void_p()
        if device_ptr is not None:
            check(lib().rwkvtts_engine_create(ctypes.byref(desc), ctypes.c_void_p(device_ptr),
                                              int(weights), 1, ctypes.byref(h)), "engine_create")
        else:
            w = np.ascontiguousarray(weights)
            check(lib().rwkvtts_engine_create(ctypes.byref(desc), w.ctypes.data_as(ctypes.c_void_p),
                                              w.nbytes, 0, ctypes.byref(h)), "engine_create")
        self._h = h
        self.max_slots = max_slots
        self.token_chunk_size = token_chunk_size
        d = _ffi.Dims()
        check(lib().rwkvtts_engine_dims(self._h, ctypes.byref(d)), "engine_dims")
        self.dims = {f: getattr(d, f) for f, _ in _ffi.Dims._fields_}

    def close(self):
        if self._h:
            lib().rwkvtts_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- state (State::init / load / back) ----
    @_locked
    def state_floats(self) -> int:
        return int(lib().rwkvtts_state_floats(self._h))

    @_locked
    def reset_slot(self, slot: int):
        check(lib().rwkvtts_slot_reset(self._h, slot), "slot_reset")

    @_locked
    def read_slot(self, slot: int) -> np.ndarray:
        out = np.empty(self.state_floats(), dtype=np.float32)
        check(lib().rwkvtts_slot_read(self._h, slot, out.ctypes.data_as(ctypes.c_void_p)), "slot_read")
        return out

    @_locked
    def write_slot(self, slot: int, state: np.ndarray):
        s = np.ascontiguousarray(state, dtype=np.float32)
        check(lib().rwkvtts_slot_write(self._h, slot, s.ctypes.data_as(ctypes.c_void_p)), "slot_write")

    # ---- Runtime<Rnn>::infer ----
    @_locked
    def infer(self, inp: RnnInput, head_rows: Optional[int] = None, slots: Optional[Sequence[int]] = None):
        """Returns (remaining RnnInput, outputs) where outputs[i] is an np.ndarray of logits
        (empty while batch i still has pending input). Batch index == state slot unless
        `slots` maps them."""
        head_rows = head_rows or self.dims["n_vocab"]
        n = len(inp.batches)
        arr = (_ffi.Input * n)()
        keep = []
        for i, b in enumerate(inp.batches):
            t = np.ascontiguousarray(np.asarray(b.tokens, dtype=np.uint32))
            keep.append(t)
            arr[i].slot = slots[i] if slots is not None else i
            arr[i].tokens = t.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
            arr[i].n_tokens = len(t)
            arr[i].option = b.option
        consumed = np.zeros(n, dtype=np.int32)
        has = np.zeros(n, dtype=np.int32)
        max_rows = sum(len(t) if b.option == RnnOption.Full else 1 for t, b in zip(keep, inp.batches))
        logits = np.zeros((max(max_rows, 1), head_rows), dtype=np.float32)
        check(lib().rwkvtts_infer(self._h, arr, n, head_rows, logits.ctypes.data_as(ctypes.c_void_p),
                                  consumed.ctypes.data_as(ctypes.c_void_p), has.ctypes.data_as(ctypes.c_void_p)),
              "infer")
        outputs, row = [], 0
        remaining = RnnInput([RnnInputBatch(list(b.tokens[c:]), b.option) for b, c in zip(inp.batches, consumed)],
                             inp.token_chunk_size)
        for i, b in enumerate(inp.batches):
            if b.option == RnnOption.Full:
                k = int(consumed[i])
                outputs.append(logits[row:row + k].copy())
                row += k
            elif has[i]:
                outputs.append(logits[row].copy())
                row += 1
            else:
                outputs.append(np.zeros(0, dtype=np.float32))
        return remaining, outputs

    # ---- device sampler ----
    @_locked
    def sample(self, logits: np.ndarray, temperature=1.0, top_p=0.85, top_k=0, forbid_token=None,
               rngs: Optional[Sequence[Optional[StdRng]]] = None) -> np.ndarray:
        lg = np.ascontiguousarray(np.atleast_2d(logits), dtype=np.float32)
        n_rows, n = lg.shape
        args = _ffi.SampleArgs(temperature, top_p, top_k, -1 if forbid_token is None else forbid_token)
        out = np.zeros(n_rows, dtype=np.int32)
        if rngs is None or all(r is None for r in rngs):
            ptrs = None
        else:
            ptrs = (ctypes.POINTER(_ffi.Rng) * n_rows)(*[ctypes.pointer(r._s) for r in rngs])
        check(lib().rwkvtts_sample(self._h, lg.ctypes.data_as(ctypes.c_void_p), n_rows, n, ctypes.byref(args),
                                   ptrs, out.ctypes.data_as(ctypes.c_void_p)), "sample")
        return out

    # ---- scheduler ----
    @_locked
    def generate_batch(self, requests: Sequence["TtsBatchRequest"]):
        """generate_tts_batch on this engine; failed requests give ([], []) (status in
        self.last_status)."""
        n = len(requests)
        reqs = (_ffi.Request * n)()
        res = (_ffi.Result * n)()
        keep, sem_bufs = [], []
        for i, r in enumerate(requests):
            q, k = request_struct(r)
            keep.append(k)
            reqs[i] = q
            sb = np.zeros(_ffi.SEMANTIC_LIMIT, dtype=np.int32)
            sem_bufs.append(sb)
            res[i].semantic_tokens = sb.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        check(lib().rwkvtts_generate_batch(self._h, reqs, n, res), "generate_batch")
        out, self.last_status = _unpack_results(res, sem_bufs)
        return out

    @_locked
    def stats(self):
        s = _ffi.Stats()
        check(lib().rwkvtts_get_stats(self._h, ctypes.byref(s)), "get_stats")
        return {f: getattr(s, f) for f, _ in _ffi.Stats._fields_}

    @_locked
    def set_profiling(self, on):
        """False / True (1): HIP events on eager launches; 2: in-graph sampled timing of the
        graph-replayed decode steps (rwkvtts.h rwkvtts_set_profiling)."""
        mode = on if isinstance(on, int) and not isinstance(on, bool) else (1 if on else 0)
        check(lib().rwkvtts_set_profiling(self._h, mode), "set_profiling")

    @_locked
    def profile(self):
        out = {}
        n = self.stats()["profile_kernel_count"]
        for i in range(n):
            name = ctypes.create_string_buffer(64)
            la = ctypes.c_int64()
            ms = ctypes.c_double()
            check(lib().rwkvtts_profile_entry(self._h, i, name, 64, ctypes.byref(la), ctypes.byref(ms)), "profile_entry")
            out[name.value.decode()] = (int(la.value), float(ms.value))
        return out


def sample_logits_with_top_p_k(runtime: SharedRwkvRuntime, logits, temperature: float, top_p: float,
                               top_k: int, forbid_token: Optional[int], rng: Optional[StdRng]) -> int:
    """src/rwkv_sampler.rs:55-62 signature (plus the runtime that owns the GPU)."""
    return int(runtime.sample(np.asarray(logits, dtype=np.float32)[None, :], temperature, top_p, top_k,
                              forbid_token, [rng] if rng is not None else None)[0])


@dataclasses.dataclass
class LayeredRandomnessConfig:  # src/rwkv_sampler.rs:251-275
    global_randomness: float = 0.1
    semantic_randomness: float = 0.4
    use_independent_seeds: bool = True
    global_seed_offset: int = 1000
    semantic_seed_offset: int = 2000


@dataclasses.dataclass
class SamplerArgs:  # src/rwkv_sampler.rs:234-290
    temperature: float = 1.0
    top_p: float = 0.85
    top_k: int = 0
    max_tokens: int = 2048
    seed: Optional[int] = None
    voice_fidelity: float = 0.8
    layered_randomness: LayeredRandomnessConfig = dataclasses.field(default_factory=LayeredRandomnessConfig)
    token_chunk_size: int = 512


@dataclasses.dataclass
class TtsBatchRequest:  # src/rwkv_sampler.rs:222-231 (text already tokenised)
    text_tokens: List[int]
    property_tokens: List[int] = dataclasses.field(default_factory=list)
    ref_global_tokens: Optional[List[int]] = None
    ref_semantic_tokens: Optional[List[int]] = None
    args: SamplerArgs = dataclasses.field(default_factory=SamplerArgs)
    voice_id: Optional[str] = None
    fixed_semantic: int = 0   # benchmark mode: EOS masked, exactly this many tokens
    greedy: bool = False      # config-1 plumbing check (top_k = 1)


@dataclasses.dataclass
class DynamicBatchConfig:  # src/batch_types.rs:67-97
    min_batch_size: int = 1
    max_batch_size: int = 10
    collect_timeout_ms: int = 50
    inference_timeout_ms: int = 60000
    max_concurrent_batches: int = 4
    semaphore_permits: int = 3
    token_chunk_size: int = 256


class DynamicBatchManager:
    """src/dynamic_batch_manager.rs:22-164 over the native manager (rwkvtts_manager_*): any
    thread may call generate_tts; the collector batches concurrent calls with the reference's
    collect window and routes each request to the least-loaded engine (one per device, one owner
    thread each), whose continuous batching decodes all its requests together. Per-request
    outputs equal the serial single-engine run."""

    def __init__(self, weights: np.ndarray, config: Optional[DynamicBatchConfig] = None,
                 devices: Sequence[int] = (0,), max_slots: int = 32, token_chunk_size: int = 512,
                 use_graphs: bool = True, wkv_variant: int = 0, tokenizer=None, quant_layers: int = 0,
                 quant_type="none", forms: int = 0):
        self.config = config or DynamicBatchConfig()
        devices = list(devices)
        if not 1 <= len(devices) <= _ffi.MAX_ENGINES:
            raise ValueError("1..16 engines")
        d = _ffi.ManagerDesc()
        d.n_engines = len(devices)
        for i, dev in enumerate(devices):
            d.devices[i] = dev
        ql, qt = quant_config(quant_layers, quant_type)
        d.engine = _ffi.EngineDesc(0, max_slots, token_chunk_size, 1 if use_graphs else 0, wkv_variant, ql, qt, forms)
        d.max_batch_size = self.config.max_batch_size
        d.collect_timeout_ms = self.config.collect_timeout_ms
        w = np.ascontiguousarray(weights)
        h = ctypes.c_void_p()
        check(lib().rwkvtts_manager_create(ctypes.byref(d), w.ctypes.data_as(ctypes.c_void_p), w.nbytes,
                                           ctypes.byref(h)), "manager_create")
        self._h = h
        self.devices = devices
        self.tokenizer = tokenizer
        # per calling thread: concurrent generate_tts callers (the server's worker threads) never
        # see each other's status codes
        self._tls = threading.local()
        # close() must not race a call that has not yet entered the native manager (rwkvtts.h:
        # destroy may not overlap the START of another call): calls are counted here, close()
        # refuses new ones and waits until every call still in flight is a waiter the native
        # manager has registered (those return inside destroy, before the handle is freed)
        self._gate = threading.Condition()
        self._inflight = 0
        self._closing = False

    def _enter(self):
        with self._gate:
            if self._closing or not getattr(self, "_h", None):
                raise _ffi.RwkvTtsError(_ffi.ECLOSED, "manager is closed")
            self._inflight += 1

    def _leave(self):
        with self._gate:
            self._inflight -= 1
            self._gate.notify_all()

    @property
    def last_status(self):
        """Status codes of this thread's last wait / generate_tts_batch call."""
        return getattr(self._tls, "last_status", [])

    def close(self):
        gate = getattr(self, "_gate", None)
        if gate is None:
            return
        with gate:
            if self._closing or not getattr(self, "_h", None):
                return
            self._closing = True
            # destroy only once every call in flight is a waiter blocked inside the native wait
            # (destroy returns those before it frees the handle); if the stats poll fails, once no
            # call is in flight at all. An interrupt here (KeyboardInterrupt in the wait) propagates
            # with _closing kept and the handle NOT destroyed: a leak, never a destroy that overlaps
            # the start of another call (rwkvtts.h rwkvtts_manager_destroy)
            while True:
                s = _ffi.ManagerStats()
                if lib().rwkvtts_manager_get_stats(self._h, ctypes.byref(s)) == _ffi.OK:
                    if self._inflight <= s.waiters:
                        break
                elif self._inflight == 0:
                    break
                gate.wait(0.005)
        try:
            lib().rwkvtts_manager_destroy(self._h)
        finally:
            with gate:
                self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _tokens(self, text):
        if isinstance(text, str):
            if self.tokenizer is None:
                raise ValueError("text given as a string but the manager has no tokenizer")
            return self.tokenizer.encode(text)  # dynamic_batch_manager.rs:512-515
        return list(text)

    def submit(self, request: "TtsBatchRequest") -> int:
        q, keep = request_struct(request)
        t = ctypes.c_uint64()
        self._enter()
        try:
            check(lib().rwkvtts_manager_submit(self._h, ctypes.byref(q), ctypes.byref(t)), "manager_submit")
        finally:
            self._leave()
        return int(t.value)

    def wait(self, ticket: int, timeout_ms: int = -1):
        """(global, semantic) or None if not ready within timeout_ms; ([], []) for a failed request."""
        out, status = self.wait_status(ticket, timeout_ms)
        self._tls.last_status = [] if status is None else [status]
        return out

    def wait_status(self, ticket: int, timeout_ms: int = -1):
        """((global, semantic), status code); (None, None) if not ready within timeout_ms."""
        r = _ffi.Result()
        sb = np.zeros(_ffi.SEMANTIC_LIMIT, dtype=np.int32)
        r.semantic_tokens = sb.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        self._enter()
        try:
            rc = lib().rwkvtts_manager_wait(self._h, ctypes.c_uint64(ticket), timeout_ms, ctypes.byref(r))
        finally:
            self._leave()
        if rc == _ffi.EBUSY:
            return None, None
        check(rc, "manager_wait")
        res = (_ffi.Result * 1)(r)
        out, status = _unpack_results(res, [sb])
        return out[0], status[0]

    def generate_tts(self, text, property_tokens, ref_global_tokens=None, ref_semantic_tokens=None,
                     voice_id=None, args: Optional[SamplerArgs] = None):
        req = TtsBatchRequest(self._tokens(text), list(property_tokens), ref_global_tokens, ref_semantic_tokens,
                              args or SamplerArgs(), voice_id)
        return self.wait(self.submit(req))

    def generate_tts_batch(self, requests: Sequence[TtsBatchRequest]):
        tickets = [self.submit(r) for r in requests]
        out, status = [], []
        for t in tickets:
            o, st = self.wait_status(t)
            out.append(o)
            status.append(st)
        self._tls.last_status = status
        return out

    def stats(self):
        s = _ffi.ManagerStats()
        self._enter()
        try:
            check(lib().rwkvtts_manager_get_stats(self._h, ctypes.byref(s)), "manager_get_stats")
        finally:
            self._leave()
        n = len(self.devices)
        return {"submitted": s.submitted, "completed": s.completed, "batches": s.batches,
                "served": list(s.served[:n]), "max_active": list(s.max_active[:n]), "steps": list(s.steps[:n]),
                "bcast_ranks": s.bcast_ranks, "bcast_rccl": s.bcast_rccl, "bcast_ms": s.bcast_ms,
                "waiters": s.waiters, "persistent": list(s.persistent[:n])}
