"""Reference-audio mel spectrogram on the MI355X vs the oracle restatement of
src/tts_pipeline_fixes.rs:12-159. The window, twiddles and filterbank come from the same glibc
calls and every device sum runs in the reference's order without contraction, so the result is
expected bit-exact (asserted)."""
import ctypes

import numpy as np
import pytest

from rwkvtts import _ffi

pytestmark = pytest.mark.gpu


def gpu_mel(wav):
    w = np.ascontiguousarray(wav, dtype=np.float32)
    nf_max = w.size // 320 + 2
    out = np.empty(128 * nf_max, dtype=np.float32)
    nf = ctypes.c_int(0)
    _ffi.check(_ffi.lib().rwkvtts_mel(0, w.ctypes.data_as(ctypes.c_void_p) if w.size else None, int(w.size),
                                      out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nf)), "mel")
    return out[: 128 * nf.value].reshape(128, nf.value)


@pytest.mark.parametrize("n", [0, 1, 319, 320, 1023, 1024, 4000, 16000 * 3 + 17])
def test_mel_bit_exact(oracle_mod, n):
    rs = np.random.default_rng(n)
    t = np.arange(n) / 16000.0
    wav = (0.3 * np.sin(2 * np.pi * 220 * t) + 0.05 * rs.standard_normal(n)).astype(np.float32)
    g, r = gpu_mel(wav), oracle_mod.mel(wav)
    assert g.shape == r.shape == (128, max(1, n // 320 + 1) if n else 1)
    assert np.array_equal(g, r), np.abs(g - r).max()


def test_mel_silence_and_impulse(oracle_mod):
    wav = np.zeros(3200, np.float32)
    assert not gpu_mel(wav).any()
    wav[1600] = 1.0
    assert np.array_equal(gpu_mel(wav), oracle_mod.mel(wav))
