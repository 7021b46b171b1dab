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

import rwkvtts
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


def test_full_dims_bench_shape_512_frames_vs_oracle(oracle_mod):
    """The bench's vocoder launch at its full shape: 32 utterances x 512 frames
    (163,840 samples each) in ONE batched decode at the full dims -- long-T tiling, halo windows
    across many time tiles and the blockIdx.z batching at T = 512 -- with the first and last
    utterance compared against the oracle over all 163,840 samples (~10 s of oracle time each at
    16 threads)."""
    d = codec.CODEC_DIMS_FULL
    w = codec.synth_codec_blob(d)
    c = codec.BiCodecDetokenizer(w, d)
    rs = np.random.default_rng(512)
    items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, 512)) for _ in range(32)]
    try:
        outs = c.decode_audio_batch(items)
        assert all(o.size == 512 * 320 for o in outs)
        cd = codec.make_codec_dims(d)
        for i in (0, 31):
            g, s = items[i]
            _check(outs[i], oracle_mod.codec_decode(cd, w, s, g, threads=16))
        # and the same utterance decoded alone is bitwise the batched one
        assert np.array_equal(outs[31], c.decode_audio(*items[31]))
    finally:
        c.close()


def _decoder(w, d, wlo=None):
    """A decoder with the conv weight path forced (rwkvtts_codec_create_ex) or automatic."""
    F = rwkvtts._ffi
    path = F.CODEC_WEIGHTS_AUTO if wlo is None else (F.CODEC_WEIGHTS_HILO if wlo else F.CODEC_WEIGHTS_BF16)
    return codec.BiCodecDetokenizer(w, d, weight_path=path)


def test_weight_lo_path_bit_identical_on_bf16_weights():
    """The three-product (weight hi + lo) kernels on bf16-exact weights add exact zeros: PCM is
    bitwise the two-product path's, at every stage's tile choice (tiny and full dims)."""
    rs = np.random.default_rng(77)
    for d, T in ((codec.CODEC_DIMS_TINY, 37), (codec.CODEC_DIMS_FULL, 6)):
        w = codec.synth_codec_blob(d, seed=3)
        items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T - i)) for i in range(3)]
        a, b = _decoder(w, d, False), _decoder(w, d, True)
        try:
            for x, y in zip(a.decode_audio_batch(items), b.decode_audio_batch(items)):
                assert np.array_equal(x, y)
        finally:
            a.close()
            b.close()


def test_full_dims_f32_weights_vs_oracle(oracle_mod):
    """f32 weights that bf16 cannot hold (a real fp32 checkpoint's; synth + 2^-12 relative
    perturbation): the decoder picks the weight hi + lo path automatically and matches the f32
    oracle at the same PCM tolerance as bf16-exact weights. The forced bf16-weight path's error
    on the same input is reported (test output) as the bound the hi + lo split removes; the
    full-batch vocoder time of both paths is reported too."""
    import time
    d = codec.CODEC_DIMS_FULL
    w = codec.synth_codec_blob_f32(d, seed=21)
    r = json.load(open(os.path.join(HERE, "golden", "raf_voice_05d8f5ed.json")))
    g, sem = r["global_tokens"], r["semantic_tokens"][:24]
    ref = oracle_mod.codec_decode(codec.make_codec_dims(d), w, sem, g, threads=16)
    c, cb = _decoder(w, d), _decoder(w, d, False)
    try:
        got = c.decode_audio(g, sem)
        _check(got, ref)
        lo = cb.decode_audio(g, sem)
        e_lo = (float(np.abs(lo - ref).max()), float(np.linalg.norm(lo - ref) / np.linalg.norm(ref)))
        e_hi = (float(np.abs(got - ref).max()), float(np.linalg.norm(got - ref) / np.linalg.norm(ref)))
        # the bench's launch shape: 32 x 512 frames
        rs = np.random.default_rng(1)
        items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, 512)) for _ in range(32)]
        ms = []
        for dec in (c, cb):
            dec.decode_audio_batch(items)
            t0 = time.perf_counter()
            dec.decode_audio_batch(items)
            ms.append(1e3 * (time.perf_counter() - t0))
        print(f"f32 weights: hi+lo path max|err| {e_hi[0]:.2e} rel-L2 {e_hi[1]:.2e}; bf16-weight path "
              f"max|err| {e_lo[0]:.2e} rel-L2 {e_lo[1]:.2e}; 32 x 512 frames: {ms[0]:.1f} ms hi+lo, {ms[1]:.1f} ms bf16")
        d_rep = os.environ.get("RWKVTTS_REPORT_DIR")
        if d_rep:
            os.makedirs(d_rep, exist_ok=True)
            json.dump({"hi_lo": {"max_abs": e_hi[0], "rel_l2": e_hi[1], "batch_ms": ms[0]},
                       "bf16_weights": {"max_abs": e_lo[0], "rel_l2": e_lo[1], "batch_ms": ms[1]}},
                      open(os.path.join(d_rep, "codec_f32_weights.json"), "w"), indent=1)
    finally:
        c.close()
        cb.close()


def test_fused_residual_unit_bit_identical():
    """The 96-channel residual units as one launch (conv7 -> Snake -> conv1 -> + residual, the
    intermediate planes kept in LDS) give bitwise the two-launch result: same products, same
    per-element accumulation order (RWKVTTS_CODEC_FORM_SEPARATE_RESUNIT switches the fusion off)."""
    rs = np.random.default_rng(96)
    for d, T in ((codec.CODEC_DIMS_TINY, 41), (codec.CODEC_DIMS_FULL, 7)):
        w = codec.synth_codec_blob(d, seed=9)
        items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T - 2 * i)) for i in range(3)]
        c = codec.BiCodecDetokenizer(w, d)
        try:
            fused = c.decode_audio_batch(items)
            c.set_forms(rwkvtts._ffi.CODEC_FORM_SEPARATE_RESUNIT)
            plain = c.decode_audio_batch(items)
            c.set_forms(0)
            for x, y in zip(fused, plain):
                assert np.array_equal(x, y)
        finally:
            c.close()


def test_channel_blocked_planes_bit_identical():
    """The WaveGenerator's activation planes channel-blocked ([C / 32][rows][32], the default) or
    channel-last (RWKVTTS_CODEC_FORM_CHANNEL_LAST): only addresses change, so PCM is bitwise
    equal -- with and without the fused residual units, the weight-lo kernels, ragged lengths."""
    rs = np.random.default_rng(32)
    for d, T, wlo in ((codec.CODEC_DIMS_TINY, 41, None), (codec.CODEC_DIMS_FULL, 9, None),
                      (codec.CODEC_DIMS_FULL, 5, True)):
        w = codec.synth_codec_blob(d, seed=12)
        items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T - 2 * i)) for i in range(3)]
        c = _decoder(w, d, wlo)
        try:
            outs = []
            F = rwkvtts._ffi
            for forms in (0, F.CODEC_FORM_CHANNEL_LAST, F.CODEC_FORM_SEPARATE_RESUNIT,
                          F.CODEC_FORM_CHANNEL_LAST | F.CODEC_FORM_SEPARATE_RESUNIT):
                c.set_forms(forms)
                outs.append(c.decode_audio_batch(items))
            for o in outs[1:]:
                for x, y in zip(outs[0], o):
                    assert np.array_equal(x, y)
        finally:
            c.close()
