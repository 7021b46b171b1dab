"""Zero-shot reference-audio front end (host mirror of src/ref_audio_utilities.rs:115-222,532-631
and the clip / silence helpers it uses), feeding the HIP mel kernel (features.py).

* `load_audio(path, target_sr, volume_normalize)` (:115-222): WAV via the hound rules of
  `load_audio_with_hound` (:225-283: 16 / 24 / 32-bit int as s / 2^(bits-1), 32-bit float as is;
  1..8 channels, first channel kept; >= 0.1 s), resampled to target_sr, optionally
  volume-normalised (coeff 0.2), then leading / trailing silence (|x| <= 0.01) trimmed.
  MP3 (symphonia) is not supported: no decoder is available offline.
* `audio_volume_normalize` (:583-624), `detect_silence` / `trim_silence_only` (:1301-1356),
  `zero_mean_unit_variance_normalize` (:636-683), `get_ref_clip`
  (lightweight_tts_pipeline.rs:1130-1155): f32 restatements in the reference's order.
* `resample_audio_high_quality` (:532-576): rubato 0.15 `SincFixedIn` with the reference's
  parameters (sinc_len 256, f_cutoff 0.95, oversampling 256, linear interpolation between sinc
  tables, Blackman-Harris^2 window, one whole-signal chunk). rubato is not vendored and nothing
  in the reference pins its output: **parity unpinned**; restated from the library's published
  algorithm (the output keeps rubato's sinc_len / 2 input-sample delay and its
  ceil(n * ratio) output length).
"""
import struct
from typing import Tuple

import numpy as np

F32 = np.float32


# ---- WAV (hound) -------------------------------------------------------------------------
def read_wav(path: str) -> Tuple[np.ndarray, int, int]:
    """-> (interleaved f32 samples, sample_rate, channels) under load_audio_with_hound's rules."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    pos, fmt, pcm = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
            if fmt[0] == 0xFFFE and len(body) >= 26:  # WAVE_FORMAT_EXTENSIBLE: sub-format code
                fmt = (struct.unpack("<H", body[24:26])[0],) + fmt[1:]
        elif cid == b"data":
            pcm = body
        pos += 8 + size + (size & 1)
    if fmt is None or pcm is None:
        raise ValueError("WAV lacks fmt or data chunk")
    tag, ch, sr, _, _, bits = fmt
    if bits not in (16, 24, 32):
        raise ValueError(f"unsupported bit depth: {bits} (16/24/32)")
    if ch == 0 or ch > 8:
        raise ValueError(f"unsupported channel count: {ch} (1-8)")
    if sr == 0 or sr > 192000:
        raise ValueError(f"unsupported sample rate: {sr} Hz")
    if bits == 16:
        x = np.frombuffer(pcm[:len(pcm) // 2 * 2], dtype="<i2").astype(F32) / F32(32768.0)
    elif bits == 24:
        b = np.frombuffer(pcm[:len(pcm) // 3 * 3], dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(F32) / F32(8388608.0)
    elif tag == 3:
        x = np.frombuffer(pcm[:len(pcm) // 4 * 4], dtype="<f4").astype(F32)
    else:
        x = np.frombuffer(pcm[:len(pcm) // 4 * 4], dtype="<i4").astype(F32) / F32(2147483648.0)
    return x, sr, ch


# ---- rubato SincFixedIn ---------------------------------------------------------------------
def _blackman_harris2(n: int) -> np.ndarray:
    """rubato WindowFunction::BlackmanHarris2: the Blackman-Harris window squared."""
    k = np.arange(n, dtype=np.float64)
    w = (0.35875 - 0.48829 * np.cos(2 * np.pi * k / n) + 0.14128 * np.cos(4 * np.pi * k / n)
         - 0.01168 * np.cos(6 * np.pi * k / n))
    return (w * w).astype(F32)


def _make_sincs(npoints: int, factor: int, f_cutoff: float) -> np.ndarray:
    """rubato make_sincs: `factor` tables of `npoints` taps, normalised to unit DC gain."""
    tot = npoints * factor
    win = _blackman_harris2(tot)
    x = (np.arange(tot, dtype=np.float64) - tot // 2) * f_cutoff / factor
    y = (win.astype(np.float64) * np.sinc(x)).astype(F32)
    s = F32(np.sum(y, dtype=F32) / F32(factor))
    sincs = np.empty((factor, npoints), dtype=F32)
    for n in range(factor):
        sincs[factor - n - 1] = y[n::factor] / s
    return sincs


def resample_audio_high_quality(audio, original_sr: int, target_sr: int, sinc_len: int = 256,
                                f_cutoff: float = 0.95, oversampling: int = 256) -> np.ndarray:
    x = np.asarray(audio, dtype=F32)
    if original_sr == target_sr:
        return x.copy()
    ratio = target_sr / original_sr
    cutoff = f_cutoff if ratio >= 1.0 else f_cutoff * ratio
    sincs = _make_sincs(sinc_len, oversampling, cutoff)
    n_out = int(np.ceil(x.size * ratio))
    # input buffer as rubato holds it: sinc_len zeros of history, then the chunk
    buf = np.concatenate([np.zeros(sinc_len, F32), x, np.zeros(sinc_len, F32)])
    t_ratio = 1.0 / ratio
    idx = np.arange(n_out, dtype=np.float64) * t_ratio - sinc_len / 2.0  # rubato's start delay
    start = np.floor(idx).astype(np.int64)
    frac = idx - start
    pos = frac * oversampling
    p0 = np.floor(pos).astype(np.int64)
    w1 = (pos - p0).astype(F32)
    base = start + sinc_len  # into buf
    out = np.empty(n_out, dtype=F32)
    taps = np.arange(sinc_len)
    for i0 in range(0, n_out, 4096):  # linear interpolation between adjacent sinc tables
        sl = slice(i0, min(i0 + 4096, n_out))
        seg = buf[(base[sl, None] + taps[None, :] - sinc_len // 2 + 1).clip(0, buf.size - 1)]
        a = np.einsum("ij,ij->i", seg, sincs[p0[sl] % oversampling])
        b = np.einsum("ij,ij->i", seg, sincs[(p0[sl] + 1) % oversampling])
        out[sl] = a + (b - a) * w1[sl]
    return out


# ---- normalisation / trimming ------------------------------------------------------------
def audio_volume_normalize(audio, coeff: float = 0.2) -> np.ndarray:
    x = np.asarray(audio, dtype=F32).copy()
    temp = np.sort(np.abs(x))
    if temp.size and temp[-1] < F32(0.1):
        sf = max(temp[-1], F32(1e-3))
        x = x / F32(sf) * F32(0.1)
    temp = temp[temp > F32(0.01)]
    n = temp.size
    if n <= 10:
        return x
    a, b = int(F32(0.9) * F32(n)), int(F32(0.99) * F32(n))
    vol = F32(0.0)
    for v in temp[a:b]:  # sequential f32 sum (Iterator::sum)
        vol = F32(vol + v)
    vol = F32(vol / F32(b - a))
    scale = F32(min(max(F32(coeff) / vol, F32(0.1)), F32(10.0)))
    x = x * scale
    mx = F32(np.max(np.abs(x))) if x.size else F32(0)
    if mx > 1.0:
        x = x / mx
    return x


def detect_silence(audio, threshold: float) -> Tuple[int, int]:
    a = np.abs(np.asarray(audio, dtype=F32))
    n = a.size
    if n == 0:
        return 0, 0
    loud = np.nonzero(a > F32(threshold))[0]
    if loud.size == 0:
        return n // 2, n - n // 2
    start, end = int(loud[0]), int(n - 1 - loud[-1])
    if start + end >= n:
        return n // 2, n - n // 2
    return start, end


def trim_silence_only(audio, silence_threshold: float = 0.01) -> np.ndarray:
    x = np.asarray(audio, dtype=F32)
    s, e = detect_silence(x, silence_threshold)
    a, b = min(s, x.size), max(x.size - e, 0)
    if a >= b:
        return np.zeros(x.size, dtype=F32)
    return x[a:b].copy()


def zero_mean_unit_variance_normalize(values) -> np.ndarray:
    x = np.asarray(values, dtype=F32).copy()
    if x.size == 0:
        return x
    if x.size == 1:
        x[0] = 0.0
        return x
    s = F32(0.0)
    for v in x:
        s = F32(s + v)
    mean = F32(s / F32(x.size))
    if np.all(np.abs(x - mean) < F32(1e-10)):
        return np.zeros_like(x)
    acc = F32(0.0)
    for v in x:
        d = F32(v - mean)
        acc = F32(acc + F32(d * d))
    std = F32(np.sqrt(F32(F32(acc / F32(x.size)) + F32(1e-7))))
    return ((x - mean) / std).astype(F32)


def get_ref_clip(wav, sample_rate: int = 16000, ref_segment_duration: float = 6.0, hop: int = 320) -> np.ndarray:
    x = np.asarray(wav, dtype=F32)
    seg = int(F32(ref_segment_duration) * F32(sample_rate)) // hop * hop
    if seg > x.size:
        reps = seg // x.size + 1
        return np.tile(x, reps)[:seg].copy()
    return x[:seg].copy()


def load_audio(path: str, target_sr: int = 16000, volume_normalize: bool = True) -> np.ndarray:
    import os
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    size = os.path.getsize(path)
    if size == 0 or size > 100 * 1024 * 1024:
        raise ValueError("audio file empty or larger than 100 MB")
    if path.lower().endswith(".mp3"):
        raise NotImplementedError("MP3 decoding (symphonia) is not available")
    x, sr, ch = read_wav(path)
    if x.size == 0 or x.size < ch:
        raise ValueError("no audio samples")
    if x.size < int(F32(sr) * F32(0.1)):
        raise ValueError("audio shorter than 0.1 s")
    if ch > 1:
        x = x[::ch].copy()
    if sr != target_sr:
        x = resample_audio_high_quality(x, sr, target_sr)
    if volume_normalize:
        x = audio_volume_normalize(x, 0.2)
    return trim_silence_only(x, 0.01)
