"""BiCodec decoder: weight layout, synthetic weights and the oracle restatement (CPU only)."""
import json
import os

import numpy as np
import pytest

from rwkvtts import codec
from rwkvtts import _ffi

HERE = os.path.dirname(os.path.abspath(__file__))


def test_blob_layout_and_synth_determinism():
    d = codec.CODEC_DIMS_TINY
    n = codec.codec_blob_floats(d)
    assert n * 4 == _ffi.lib().rwkvtts_codec_blob_bytes(codec.make_codec_dims(d))
    a = codec.synth_codec_blob(d, seed=7)
    b = codec.synth_codec_blob(d, seed=7)
    c = codec.synth_codec_blob(d, seed=8)
    assert a.size == n and np.array_equal(a, b) and not np.array_equal(a, c)
    assert np.isfinite(a).all()
    # header carries the dims struct
    hdr = a[:22].view(np.int32)
    assert hdr[0] == d["codebook_size"] and hdr[2] == d["latent_dim"] and hdr[10] == d["dec_channels"]


def test_full_blob_size():
    # SURVEY §8a-7 dims: ~90M parameters (prenet 12 ConvNeXt blocks + 4 up blocks)
    n = codec.codec_blob_floats(codec.CODEC_DIMS_FULL)
    assert 80e6 < n < 100e6


def test_oracle_shape_range_and_determinism(oracle_mod):
    d = codec.CODEC_DIMS_TINY
    w = codec.synth_codec_blob(d)
    rs = np.random.default_rng(1)
    sem, g = rs.integers(0, 8192, 9), rs.integers(0, 4096, 32)
    cd = codec.make_codec_dims(d)
    p1 = oracle_mod.codec_decode(cd, w, sem, g, threads=4)
    p2 = oracle_mod.codec_decode(cd, w, sem, g, threads=2)
    assert p1.shape == (9 * 320,)
    assert np.array_equal(p1, p2)  # thread count does not change the f32 result
    assert np.abs(p1).max() < 1.0 and p1.std() > 0.05  # tanh output, not saturated
    # the speaker tokens condition the whole utterance
    g2 = g.copy()
    g2[0] = (g2[0] + 1) % 4096
    assert not np.allclose(p1, oracle_mod.codec_decode(cd, w, sem, g2))


def test_oracle_causality_window(oracle_mod):
    """Changing the last semantic code only changes samples within the receptive field of the
    final frames (the decoder is a finite stack of convolutions)."""
    d = codec.CODEC_DIMS_TINY
    w = codec.synth_codec_blob(d)
    rs = np.random.default_rng(2)
    sem, g = rs.integers(0, 8192, 40), rs.integers(0, 4096, 32)
    cd = codec.make_codec_dims(d)
    a = oracle_mod.codec_decode(cd, w, sem, g)
    sem2 = sem.copy()
    sem2[-1] = (sem2[-1] + 1) % 8192
    b = oracle_mod.codec_decode(cd, w, sem2, g)
    diff = np.nonzero(a != b)[0]
    assert diff.size > 0
    # prenet: embed k7 + 2 dwconv k7 -> 9 frames; conv_in k7 -> 3; convT + residual units
    # (dilations 1, 3, 9 at 8/40/160/320 samples per frame) -> ~7.3 more: ~19.3 frames in all
    assert diff.min() >= (40 - 1 - 20) * 320


def test_oracle_rejects_bad_codes(oracle_mod):
    d = codec.CODEC_DIMS_TINY
    w = codec.synth_codec_blob(d)
    cd = codec.make_codec_dims(d)
    with pytest.raises(ValueError):
        oracle_mod.codec_decode(cd, w, [8192], np.zeros(32, np.int64))
    with pytest.raises(ValueError):
        oracle_mod.codec_decode(cd, w, [0], np.full(32, 4096, np.int64))


def test_raf_fixture_tokens_in_codec_range():
    for f in ("raf_voice_05d8f5ed.json", "raf_voice_d897f5e1.json"):
        r = json.load(open(os.path.join(HERE, "golden", f)))
        assert len(r["global_tokens"]) == 32
        assert all(0 <= t < 4096 for t in r["global_tokens"])
        assert all(0 <= t < 8192 for t in r["semantic_tokens"])
