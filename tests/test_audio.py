"""Zero-shot reference-audio front end (rwkvtts.audio; src/ref_audio_utilities.rs:115-683,
lightweight_tts_pipeline.rs:1130-1155). WAV decoding, normalisation, trimming and clipping are
restatements checked against hand-computed cases; the rubato resampler is parity unpinned
(crate not vendored) and is checked for its defining properties: sinc_len / 2 input-sample
delay, ceil(n * ratio) output length, pass-band fidelity. CPU only."""
import struct
import wave

import numpy as np
import pytest

from rwkvtts import audio as A


def _wav(path, data: bytes, sr, ch, bits, tag=1):
    fmt = struct.pack("<HHIIHH", tag, ch, sr, sr * ch * bits // 8, ch * bits // 8, bits)
    body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(data)) + data
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def test_read_wav_formats(tmp_path):
    p = tmp_path / "a16.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(2)
        w.setsampwidth(2)
        w.setframerate(16000)
        w.writeframes(struct.pack("<4h", 16384, -1, -32768, 7))
    x, sr, ch = A.read_wav(str(p))
    assert sr == 16000 and ch == 2 and x.tolist() == [0.5, -1 / 32768, -1.0, 7 / 32768]
    v24 = [(1 << 22), -(1 << 23), 5]
    raw = b"".join(int(v & 0xFFFFFF).to_bytes(3, "little") for v in v24)
    _wav(tmp_path / "a24.wav", raw, 24000, 1, 24)
    x, sr, ch = A.read_wav(str(tmp_path / "a24.wav"))
    assert x.tolist() == [0.5, -1.0, np.float32(5 / 8388608)]
    _wav(tmp_path / "f32.wav", struct.pack("<3f", 0.25, -2.0, 1e-3), 44100, 1, 32, tag=3)
    assert A.read_wav(str(tmp_path / "f32.wav"))[0].tolist() == [0.25, -2.0, np.float32(1e-3)]
    _wav(tmp_path / "i32.wav", struct.pack("<2i", 1 << 30, -(1 << 31)), 8000, 1, 32)
    assert A.read_wav(str(tmp_path / "i32.wav"))[0].tolist() == [0.5, -1.0]
    _wav(tmp_path / "u8.wav", b"\x80\x80", 8000, 1, 8)
    with pytest.raises(ValueError):
        A.read_wav(str(tmp_path / "u8.wav"))


def test_volume_normalize():
    # quiet signal: scaled to peak 0.1 first; the 90-99 % quantile mean is then taken over the
    # sorted magnitudes of the ORIGINAL samples (the reference does not re-sort, :589-607)
    rs = np.random.default_rng(0)
    x = (rs.standard_normal(4000) * 0.01).astype(np.float32)
    y = A.audio_volume_normalize(x, 0.2)
    t = np.sort(np.abs(x))
    t = t[t > 0.01]
    a, b = int(np.float32(0.9) * len(t)), int(np.float32(0.99) * len(t))
    vol = np.float32(0)
    for v in t[a:b]:
        vol = np.float32(vol + v)
    scale = np.float32(min(max(np.float32(0.2) / np.float32(vol / np.float32(b - a)), 0.1), 10.0))
    exp = (x / np.float32(max(np.abs(x).max(), 1e-3)) * np.float32(0.1)) * scale
    if np.abs(exp).max() > 1:
        exp = exp / np.abs(exp).max()
    assert np.array_equal(y, exp.astype(np.float32))
    few = np.array([0.5, 0.02, 0.0], np.float32)  # <= 10 values above 0.01: unchanged
    assert np.array_equal(A.audio_volume_normalize(few), few)


def test_trim_clip_and_zmuv():
    x = np.array([0, 0.005, 0.2, -0.3, 0.01, 0], np.float32)
    assert A.trim_silence_only(x, 0.01).tolist() == [np.float32(0.2), np.float32(-0.3)]
    assert A.trim_silence_only(np.zeros(5, np.float32)).tolist() == [0.0] * 5
    c = A.get_ref_clip(np.arange(1000, dtype=np.float32))
    assert c.size == 96000 and c[1000] == 0 and c[1999] == 999
    assert A.get_ref_clip(np.ones(200000, np.float32)).size == 96000
    z = A.zero_mean_unit_variance_normalize([1.0, 2.0, 3.0])
    assert np.allclose(z, (np.array([1, 2, 3]) - 2) / np.sqrt(2 / 3 + 1e-7), atol=1e-6)
    assert A.zero_mean_unit_variance_normalize([4.0]).tolist() == [0.0]


@pytest.mark.parametrize("sr0,sr1,f", [(24000, 16000, 440.0), (8000, 16000, 300.0), (44100, 16000, 1000.0)])
def test_resampler_properties(sr0, sr1, f):
    n = sr0
    x = np.sin(2 * np.pi * f * np.arange(n) / sr0).astype(np.float32)
    y = A.resample_audio_high_quality(x, sr0, sr1)
    assert y.size == int(np.ceil(n * sr1 / sr0))
    t = np.arange(y.size) * sr0 / sr1 - 128  # sinc_len / 2 input samples of delay
    e = np.sin(2 * np.pi * f * t / sr0)
    m = slice(int(400 * sr1 / sr0) + 300, y.size - 300)
    assert np.abs(y[m] - e[m]).max() < 2e-3
    assert np.array_equal(A.resample_audio_high_quality(x, sr0, sr0), x)


def test_load_audio_pipeline(tmp_path):
    sr = 24000
    t = np.arange(sr) / sr
    x = np.concatenate([np.zeros(2400), 0.05 * np.sin(2 * np.pi * 220 * t), np.zeros(2400)])
    p = tmp_path / "ref.wav"
    with wave.open(str(p), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(sr)
        w.writeframes((x * 32767).astype("<i2").tobytes())
    y = A.load_audio(str(p), 16000, True)
    assert 15000 < y.size < 17000           # silence trimmed, 1 s of tone at 16 kHz
    assert abs(y[0]) > 0.01 and abs(y[-1]) > 0.01
    assert 0.2 < np.abs(y).max() <= 1.0     # volume-normalised
