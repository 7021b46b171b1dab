"""Zero-shot reference-audio features on the MI355X.

Mirrors `TtsPipelineFixes::extract_mel_spectrogram_consistent` (src/tts_pipeline_fixes.rs:12-159):
16 kHz f32 waveform -> mel magnitude spectrogram [128, n_frames] (n_fft 1024, hop 320, Hann,
Slaney-normalised filterbank 10 Hz - 8 kHz, no log), bit-identical to the reference's f32 math.
"""
import ctypes

import numpy as np

from . import _ffi
from ._ffi import check, lib

N_MELS, N_FFT, HOP = 128, 1024, 320


def n_frames(n_samples: int) -> int:
    padded = n_samples + N_FFT
    return 1 if padded <= N_FFT else (padded - N_FFT) // HOP + 1


def extract_mel_spectrogram_consistent(wav, device: int = 0) -> np.ndarray:
    w = np.ascontiguousarray(wav, dtype=np.float32).reshape(-1)
    nf = n_frames(w.size)
    out = np.empty(N_MELS * nf, dtype=np.float32)
    got = ctypes.c_int(0)
    check(lib().rwkvtts_mel(device, w.ctypes.data_as(ctypes.c_void_p) if w.size else None, int(w.size),
                            out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(got)), "mel")
    assert got.value == nf
    return out.reshape(N_MELS, nf)
