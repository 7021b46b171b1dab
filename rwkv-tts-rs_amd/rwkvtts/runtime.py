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
  generate_tts_batch; requests run concurrently in GPU slots (one slot per request).
"""
import ctypes
import dataclasses
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


class SharedRwkvRuntime:
    """One engine per GPU: weights resident in HBM, `max_concurrent_batches` state slots."""

    def __init__(self, weights: np.ndarray, device: int = 0, max_slots: int = 10,
                 token_chunk_size: int = 512, use_graphs: bool = True, weights_on_device: bool = False,
                 device_ptr: Optional[int] = None):
        desc = _ffi.EngineDesc(device, max_slots, token_chunk_size, 1 if use_graphs else 0)
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
    def state_floats(self) -> int:
        return int(lib().rwkvtts_state_floats(self._h))

    def reset_slot(self, slot: int):
        check(lib().rwkvtts_slot_reset(self._h, slot), "slot_reset")

    def read_slot(self, slot: int) -> np.ndarray:
        out = np.empty(self.state_floats(), dtype=np.float32)
        check(lib().rwkvtts_slot_read(self._h, slot, out.ctypes.data_as(ctypes.c_void_p)), "slot_read")
        return out

    def write_slot(self, slot: int, state: np.ndarray):
        s = np.ascontiguousarray(state, dtype=np.float32)
        check(lib().rwkvtts_slot_write(self._h, slot, s.ctypes.data_as(ctypes.c_void_p)), "slot_write")

    # ---- Runtime<Rnn>::infer ----
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
    def generate_batch(self, requests: Sequence["TtsBatchRequest"]):
        n = len(requests)
        reqs = (_ffi.Request * n)()
        res = (_ffi.Result * n)()
        keep, sem_bufs = [], []
        for i, r in enumerate(requests):
            def arr(x):
                if x is None:
                    return None
                a = np.ascontiguousarray(np.asarray(x, dtype=np.int32))
                keep.append(a)
                return a
            tt, pt, rg, rs = arr(r.text_tokens), arr(r.property_tokens), arr(r.ref_global_tokens), arr(r.ref_semantic_tokens)
            P = ctypes.POINTER(ctypes.c_int32)
            reqs[i].text_tokens = tt.ctypes.data_as(P) if tt is not None and len(tt) else None
            reqs[i].n_text = 0 if tt is None else len(tt)
            reqs[i].property_tokens = pt.ctypes.data_as(P) if pt is not None and len(pt) else None
            reqs[i].n_property = 0 if pt is None else len(pt)
            reqs[i].ref_global = rg.ctypes.data_as(P) if rg is not None else None
            reqs[i].n_ref_global = 0 if rg is None else len(rg)
            reqs[i].ref_semantic = rs.ctypes.data_as(P) if rs is not None else None
            reqs[i].n_ref_semantic = 0 if rs is None else len(rs)
            reqs[i].has_seed = 0 if r.args.seed is None else 1
            reqs[i].seed = 0 if r.args.seed is None else r.args.seed
            reqs[i].max_tokens = r.args.max_tokens
            reqs[i].fixed_semantic = r.fixed_semantic
            reqs[i].greedy = 1 if r.greedy else 0
            sb = np.zeros(_ffi.SEMANTIC_LIMIT, dtype=np.int32)
            sem_bufs.append(sb)
            res[i].semantic_tokens = sb.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        check(lib().rwkvtts_generate_batch(self._h, reqs, n, res), "generate_batch")
        out = []
        for i in range(n):
            g = list(res[i].global_tokens[:res[i].n_global])
            s = sem_bufs[i][:res[i].n_semantic].tolist()
            out.append((g, s))
        return out

    def stats(self):
        s = _ffi.Stats()
        check(lib().rwkvtts_get_stats(self._h, ctypes.byref(s)), "get_stats")
        return {f: getattr(s, f) for f, _ in _ffi.Stats._fields_}

    def set_profiling(self, on: bool):
        check(lib().rwkvtts_set_profiling(self._h, 1 if on else 0), "set_profiling")

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
    """generate_tts / generate_tts_batch over one GPU engine. Unlike the reference (which runs a
    collected batch sequentially on state slot 0), requests decode concurrently, one slot each;
    per-request outputs equal the serial run."""

    def __init__(self, runtime: SharedRwkvRuntime, config: Optional[DynamicBatchConfig] = None):
        self.runtime = runtime
        self.config = config or DynamicBatchConfig()

    def generate_tts(self, text_tokens, property_tokens, ref_global_tokens=None, ref_semantic_tokens=None,
                     voice_id=None, args: Optional[SamplerArgs] = None):
        req = TtsBatchRequest(list(text_tokens), list(property_tokens), ref_global_tokens, ref_semantic_tokens,
                              args or SamplerArgs(), voice_id)
        return self.runtime.generate_batch([req])[0]

    def generate_tts_batch(self, requests: Sequence[TtsBatchRequest]):
        return self.runtime.generate_batch(list(requests))
