"""BiCodec decoder on the MI355X (HIP MFMA conv stack) vs the oracle f32 restatement.

Parity vs ORT is unpinned (the ONNX graph is absent); these tests pin the GPU
path to the oracle on synthetic weights. Tolerance: the MFMA matrices are bf16-exact in both
paths; the GPU splits activations into bf16 hi + lo planes (|rel err| <= 2^-17 per product)
and accumulates in a different order, through ~50 layers, then tanh. PCM lies in (-1, 1).
"""
import json
import os

import numpy as np
import pytest

from rwkvtts import codec

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PCM_ATOL = 5e-4      # max |gpu - oracle| per sample
PCM_RTOL_L2 = 1e-4   # ||gpu - oracle||_2 / ||oracle||_2


def _check(gpu, ref):
    assert gpu.shape == ref.shape
    err = np.abs(gpu - ref)
    rel = np.linalg.norm(gpu - ref) / max(np.linalg.norm(ref), 1e-12)
    assert err.max() <= PCM_ATOL and rel <= PCM_RTOL_L2, (err.max(), rel)


@pytest.fixture(scope="module")
def tiny():
    d = codec.CODEC_DIMS_TINY
    w = codec.synth_codec_blob(d, seed=11)
    c = codec.BiCodecDetokenizer(w, d)
    yield d, w, c
    c.close()


@pytest.mark.parametrize("T", [1, 2, 5, 37, 130])
def test_tiny_vs_oracle(tiny, oracle_mod, T):
    d, w, c = tiny
    rs = np.random.default_rng(T)
    sem, g = rs.integers(0, 8192, T), rs.integers(0, 4096, 32)
    _check(c.decode_audio(g, sem), oracle_mod.codec_decode(codec.make_codec_dims(d), w, sem, g, threads=16))


def test_tiny_batch_equals_single(tiny):
    """decode_audio_batch over ragged utterances == one decode per utterance, bitwise."""
    d, w, c = tiny
    rs = np.random.default_rng(5)
    items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T)) for T in (3, 64, 17, 129, 1)]
    batch = c.decode_audio_batch(items)
    for (g, s), pcm in zip(items, batch):
        assert np.array_equal(pcm, c.decode_audio(g, s))


def test_batch_invalid_item_is_empty(tiny):
    d, w, c = tiny
    rs = np.random.default_rng(6)
    good = (rs.integers(0, 4096, 32), rs.integers(0, 8192, 4))
    out = c.decode_audio_batch([good, (np.zeros(5, np.int64), [1, 2]), good])
    assert out[1].size == 0 and np.array_equal(out[0], out[2]) and out[0].size == 4 * 320
    with pytest.raises(RuntimeError):
        c.decode_audio(np.zeros(32, np.int64), [8192])


def test_full_dims_raf_tokens_vs_oracle(oracle_mod):
    """Full SparkTTS dims on the real BiCodecTokenize outputs of the reference's RAF fixture."""
    d = codec.CODEC_DIMS_FULL
    w = codec.synth_codec_blob(d)
    c = codec.BiCodecDetokenizer(w, d)
    r = json.load(open(os.path.join(HERE, "golden", "raf_voice_05d8f5ed.json")))
    g, sem = r["global_tokens"], r["semantic_tokens"][:24]
    try:
        _check(c.decode_audio(g, sem), oracle_mod.codec_decode(codec.make_codec_dims(d), w, sem, g, threads=16))
    finally:
        c.close()


def test_full_dims_batch_of_32_vs_oracle(oracle_mod):
    """The bench's launch shape: 32 utterances in ONE batched decode at the full dims (ragged
    lengths of a few frames each), every utterance against the oracle."""
    d = codec.CODEC_DIMS_FULL
    w = codec.synth_codec_blob(d)
    c = codec.BiCodecDetokenizer(w, d)
    rs = np.random.default_rng(32)
    items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, 2 + (i % 5))) for i in range(32)]
    try:
        outs = c.decode_audio_batch(items)
        cd = codec.make_codec_dims(d)
        for (g, s), pcm in zip(items, outs):
            _check(pcm, oracle_mod.codec_decode(cd, w, s, g, threads=16))
    finally:
        c.close()
