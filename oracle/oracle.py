"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see oracle.h for what each function restates and
how it is pinned). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product library never calls it.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


class OracleRng(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint32 * 8), ("index", ctypes.c_uint64)]


class OracleResult(ctypes.Structure):
    _fields_ = [("n_global", ctypes.c_int32), ("n_semantic", ctypes.c_int32),
                ("global_tokens", ctypes.c_int32 * 32), ("semantic_tokens", ctypes.c_int32 * 2048),
                ("n_forward", ctypes.c_int32)]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def use_native():
    """Switch to the -march=native build (built on first use on this host; bench cpu_baseline)."""
    global LIB, _lib
    subprocess.check_call(["make", "-s", "-C", _HERE, "native"])
    LIB = os.path.join(_HERE, "liboracle_native.so")
    _lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        L.oracle_chacha_block.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        L.oracle_chacha_block_raw.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.oracle_rng_seed_from_u64.argtypes = [ctypes.c_uint64, ctypes.POINTER(OracleRng)]
        L.oracle_rng_next_u32.argtypes = [ctypes.POINTER(OracleRng)]
        L.oracle_rng_next_u32.restype = ctypes.c_uint32
        L.oracle_rng_gen_f32.argtypes = [ctypes.POINTER(OracleRng)]
        L.oracle_rng_gen_f32.restype = ctypes.c_float
        L.oracle_sample_dbg.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_float, ctypes.c_int,
                                        ctypes.c_int, ctypes.POINTER(OracleRng), ctypes.POINTER(ctypes.c_float),
                                        ctypes.POINTER(ctypes.c_float)]
        L.oracle_sample_dbg.restype = ctypes.c_int
        L.oracle_expf.argtypes = [ctypes.c_float]
        L.oracle_expf.restype = ctypes.c_float
        L.oracle_model_load.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_model_load.restype = ctypes.c_void_p
        L.oracle_model_free.argtypes = [ctypes.c_void_p]
        L.oracle_model_quantize.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_model_quantize.restype = ctypes.c_int
        L.oracle_state_floats.argtypes = [ctypes.c_void_p]
        L.oracle_state_floats.restype = ctypes.c_int64
        L.oracle_forward_token.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_generate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(OracleResult)]
        L.oracle_generate.restype = ctypes.c_int
        L.oracle_mel.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.oracle_mel.restype = ctypes.c_int
        L.oracle_codec_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_codec_decode.restype = ctypes.c_int
        _lib = L
    return _lib


class Rng:
    def __init__(self, seed):
        self.s = OracleRng()
        lib().oracle_rng_seed_from_u64(ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF), ctypes.byref(self.s))

    def next_u32(self):
        return lib().oracle_rng_next_u32(ctypes.byref(self.s))

    def gen_f32(self):
        return lib().oracle_rng_gen_f32(ctypes.byref(self.s))

    @property
    def key(self):
        return list(self.s.key)


def chacha_block(key, counter, stream=0, rounds=12):
    k = (ctypes.c_uint32 * 8)(*key)
    out = (ctypes.c_uint32 * 16)()
    lib().oracle_chacha_block(k, counter, stream, rounds, out)
    return list(out)


def chacha_block_raw(words16, rounds):
    inp = (ctypes.c_uint32 * 16)(*words16)
    out = (ctypes.c_uint32 * 16)()
    lib().oracle_chacha_block_raw(inp, rounds, out)
    return list(out)


def sample(logits, temperature=1.0, top_p=0.85, top_k=0, forbid=None, rng=None, debug=False):
    """src/rwkv_sampler.rs:55-211. rng: oracle.Rng (advanced in place) or None (StdRng(42))."""
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    s, r = ctypes.c_float(), ctypes.c_float()
    idx = lib().oracle_sample_dbg(lg.ctypes.data_as(ctypes.c_void_p), len(lg), temperature, top_p, top_k,
                                  -1 if forbid is None else forbid, ctypes.byref(rng.s) if rng else None,
                                  ctypes.byref(s), ctypes.byref(r))
    return (idx, s.value, r.value) if debug else idx


def expf(x):
    return lib().oracle_expf(float(x))


class Model:
    """RWKV-7 x070 f32 forward (web-rwkv Bundle<f32> arithmetic restated)."""

    def __init__(self, blob: np.ndarray, threads: int = 0, quant_layers: int = 0, quant_type: int = 0):
        b = np.ascontiguousarray(blob)
        self._blob = b
        self.h = lib().oracle_model_load(b.ctypes.data_as(ctypes.c_void_p), b.nbytes)
        if not self.h:
            raise ValueError("bad weight blob")
        if threads:
            lib().oracle_set_threads(threads)
        if quant_layers and quant_type:  # web-rwkv Quant restated (rwkv7.c): 1 Int8, 2 NF4
            if lib().oracle_model_quantize(self.h, int(quant_layers), int(quant_type)) != 0:
                raise ValueError("bad quantisation config")

    def __del__(self):
        try:
            lib().oracle_model_free(self.h)
        except Exception:
            pass

    def new_state(self):
        return np.zeros(lib().oracle_state_floats(self.h), dtype=np.float32)

    def forward(self, state, token, head_rows=0):
        out = np.zeros(max(head_rows, 1), dtype=np.float32)
        lib().oracle_forward_token(self.h, state.ctypes.data_as(ctypes.c_void_p), int(token),
                                   out.ctypes.data_as(ctypes.c_void_p) if head_rows else None, head_rows)
        return out if head_rows else None

    def generate(self, request_struct):
        """request_struct: rwkvtts._ffi.Request (the same struct the product ABI takes)."""
        res = OracleResult()
        lib().oracle_generate(self.h, ctypes.byref(request_struct), ctypes.byref(res))
        return (list(res.global_tokens[:res.n_global]), list(res.semantic_tokens[:res.n_semantic]),
                res.n_forward)


def codec_decode(dims_struct, weights: np.ndarray, semantic, global_tokens, threads: int = 0) -> np.ndarray:
    """f32 CPU restatement of the BiCodec decoder (codec.c) -> PCM [T * 320]."""
    if threads:
        lib().oracle_set_threads(threads)
    s = np.ascontiguousarray(semantic, dtype=np.int64)
    g = np.ascontiguousarray(global_tokens, dtype=np.int64)
    w = np.ascontiguousarray(weights, dtype=np.float32)
    pcm = np.empty(s.size * 320, dtype=np.float32)
    rc = lib().oracle_codec_decode(ctypes.byref(dims_struct), w.ctypes.data, s.ctypes.data, int(s.size),
                                   g.ctypes.data, pcm.ctypes.data)
    if rc != 0:
        raise ValueError(f"oracle_codec_decode failed ({rc})")
    return pcm


def mel(wav) -> np.ndarray:
    """f32 restatement of extract_mel_spectrogram_consistent -> [128][n_frames]."""
    w = np.ascontiguousarray(wav, dtype=np.float32)
    n_frames = max(1, (w.size + 1024 - 1024) // 320 + 1) if w.size > 0 else 1
    out = np.empty(128 * n_frames, dtype=np.float32)
    nf = ctypes.c_int(0)
    rc = lib().oracle_mel(w.ctypes.data if w.size else None, int(w.size), out.ctypes.data, ctypes.byref(nf))
    if rc != 0:
        raise ValueError(f"oracle_mel failed ({rc})")
    return out[: 128 * nf.value].reshape(128, nf.value)
