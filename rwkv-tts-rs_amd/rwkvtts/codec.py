"""BiCodec detokenizer on the MI355X (host mirror of the reference's vocoder calls).

Mirrors `LightweightTtsPipeline::decode_audio` / `decode_audio_batch` /
`detokenize_audio_with_session` (src/lightweight_tts_pipeline.rs:606-730): global tokens (32 FSQ
speaker codes, offset already removed) + semantic tokens -> 16 kHz f32 PCM, `T * 320` samples.
The batch call returns an empty array for an utterance that fails, as the reference's
spawn_blocking tasks do (:650-690); the single call raises.
"""
import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _ffi
from ._ffi import check, lib

# Assumed SparkTTS BiCodec decoder dims and a tiny variant for fast tests.
CODEC_DIMS_FULL = dict(codebook_size=8192, codebook_dim=8, latent_dim=1024, n_global=32, fsq_levels=4,
                       fsq_dims=6, spk_dim=1024, prenet_dim=384, prenet_inter=2048, prenet_layers=12,
                       dec_channels=1536, n_up=4, up_rates=(8, 5, 4, 2), up_kernels=(16, 11, 8, 4))
CODEC_DIMS_TINY = dict(codebook_size=8192, codebook_dim=8, latent_dim=128, n_global=32, fsq_levels=4,
                       fsq_dims=6, spk_dim=128, prenet_dim=64, prenet_inter=128, prenet_layers=2,
                       dec_channels=512, n_up=4, up_rates=(8, 5, 4, 2), up_kernels=(16, 11, 8, 4))


def make_codec_dims(d: dict) -> _ffi.CodecDims:
    c = _ffi.CodecDims()
    for k, v in d.items():
        if k in ("up_rates", "up_kernels"):
            arr = getattr(c, k)
            for i, x in enumerate(v):
                arr[i] = x
        else:
            setattr(c, k, v)
    return c


def codec_blob_floats(d: dict) -> int:
    return int(lib().rwkvtts_codec_blob_bytes(ctypes.byref(make_codec_dims(d)))) // 4


def synth_codec_blob(d: dict, seed: int = 20251205) -> np.ndarray:
    """Deterministic synthetic decoder weights (f32 blob; MFMA operands bf16-exact)."""
    out = np.empty(codec_blob_floats(d), dtype=np.float32)
    check(lib().rwkvtts_codec_synth_weights(ctypes.byref(make_codec_dims(d)), ctypes.c_uint64(seed),
                                            out.ctypes.data_as(ctypes.c_void_p)), "codec_synth_weights")
    return out


def synth_codec_blob_f32(d: dict, seed: int = 20251205, rel: float = 2.0 ** -12) -> np.ndarray:
    """synth_codec_blob with every weight perturbed by a relative 2^-12 (seeded): f32 values that
    bf16 cannot hold, as a real fp32 checkpoint's (the reference runs BiCodec in fp32 on ORT).
    The 64-float header (the dims) is left alone."""
    w = synth_codec_blob(d, seed)
    u = np.random.default_rng(seed ^ 0x5EED).uniform(-1.0, 1.0, w.size - 64)
    w[64:] = (w[64:].astype(np.float64) * (1.0 + rel * u)).astype(np.float32)
    return w


class BiCodecDetokenizer:
    """One decoder per GPU (replaces the 4-session ORT pool of src/onnx_session_pool.rs:204-279)."""

    def __init__(self, weights: np.ndarray, dims: Optional[dict] = None, device: int = 0,
                 weight_path: int = 0):
        """weight_path: _ffi.CODEC_WEIGHTS_AUTO (hi + lo weight planes iff some conv weight is not
        bf16-exact), CODEC_WEIGHTS_BF16 or CODEC_WEIGHTS_HILO (rwkvtts_codec_create_ex)."""
        self.dims = dict(dims or CODEC_DIMS_FULL)
        self._cd = make_codec_dims(self.dims)
        w = np.ascontiguousarray(weights, dtype=np.float32)
        h = ctypes.c_void_p()
        check(lib().rwkvtts_codec_create_ex(device, ctypes.byref(self._cd), w.ctypes.data_as(ctypes.c_void_p),
                                            int(weight_path), ctypes.byref(h)), "codec_create")
        self._h = h

    def set_forms(self, forms: int):
        """Verification forms of later decode calls (_ffi.CODEC_FORM_*; 0 = shipping, PCM bitwise equal)."""
        check(lib().rwkvtts_codec_set_forms(self._h, int(forms)), "codec_set_forms")

    def close(self):
        if self._h:
            lib().rwkvtts_codec_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode_audio(self, global_tokens: Sequence[int], semantic_tokens: Sequence[int]) -> np.ndarray:
        g = np.ascontiguousarray(global_tokens, dtype=np.int64)
        s = np.ascontiguousarray(semantic_tokens, dtype=np.int64)
        if g.size != self.dims["n_global"] or s.size == 0:
            raise ValueError(f"decode_audio: need {self.dims['n_global']} global and >0 semantic tokens")
        pcm = np.empty(s.size * _ffi.HOP, dtype=np.float32)
        check(lib().rwkvtts_codec_decode(self._h, s.ctypes.data_as(ctypes.c_void_p), int(s.size),
                                         g.ctypes.data_as(ctypes.c_void_p), pcm.ctypes.data_as(ctypes.c_void_p)),
              "codec_decode")
        return pcm

    def decode_audio_batch(self, batch: Sequence[tuple]) -> List[np.ndarray]:
        """[(global_tokens, semantic_tokens)] -> [pcm]; invalid items give empty arrays."""
        ok, gs, ss = [], [], []
        for g, s in batch:
            g = np.ascontiguousarray(g, dtype=np.int64)
            s = np.ascontiguousarray(s, dtype=np.int64)
            valid = g.size == self.dims["n_global"] and s.size > 0
            ok.append(valid)
            if valid:
                gs.append(g)
                ss.append(s)
        outs = [np.empty(s.size * _ffi.HOP, dtype=np.float32) for s in ss]
        if ss:
            n = len(ss)
            P = ctypes.c_void_p * n
            sem = P(*[s.ctypes.data for s in ss])
            glob = P(*[g.ctypes.data for g in gs])
            pcm = P(*[o.ctypes.data for o in outs])
            T = (ctypes.c_int * n)(*[s.size for s in ss])
            rc = lib().rwkvtts_codec_decode_batch(self._h, sem, T, glob, n, pcm)
            if rc != 0:
                outs = [np.empty(0, dtype=np.float32) for _ in ss]
        it = iter(outs)
        return [next(it) if v else np.empty(0, dtype=np.float32) for v in ok]

    # ---- profiling (per-stage HIP-event timing) ----
    def set_profiling(self, on: bool):
        check(lib().rwkvtts_codec_set_profiling(self._h, 1 if on else 0), "codec_set_profiling")

    def profile(self):
        out = {}
        for i in range(lib().rwkvtts_codec_profile_count(self._h)):
            name = ctypes.create_string_buffer(64)
            n = ctypes.c_int64()
            ms = ctypes.c_double()
            check(lib().rwkvtts_codec_profile_entry(self._h, i, name, 64, ctypes.byref(n), ctypes.byref(ms)),
                  "codec_profile_entry")
            out[name.value.decode()] = (n.value, ms.value)
        return out
