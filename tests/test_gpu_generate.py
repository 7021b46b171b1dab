"""End-to-end phase controller + scheduler on the GPU vs the oracle's serial reference loop
(src/normal_mode_inference.rs, src/zero_shot_inference.rs)."""
import json
import os

import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import make_request, synth_text, to_struct

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", params=["bf16", "f16"])
def setup(request):
    # f16 = fp16 matrices (config 5 / the reference's web-rwkv numerics): f16 MFMA + f16 planes
    dt = rwkvtts._ffi.DTYPE_F16 if request.param == "f16" else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(W.DIMS_TINY, seed=99, dtype=dt)
    import oracle
    om = oracle.Model(blob)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=8, token_chunk_size=128, use_graphs=True)
    yield om, rt
    rt.close()


def _oracle(om, req):
    q, keep = to_struct(req)
    g, s, _ = om.generate(q)
    return g, s


def test_normal_mode_matches_oracle(setup):
    om, rt = setup
    reqs = [make_request(synth_text(100 + i), seed=50 + i, max_tokens=48) for i in range(3)]
    got = rt.generate_batch(reqs)
    for r, (g, s) in zip(reqs, got):
        og, os_ = _oracle(om, r)
        assert g == og
        assert s == os_
        assert len(g) == 32 and all(0 <= x < 4096 for x in g)


def test_fixed_length_and_greedy(setup):
    om, rt = setup
    reqs = [make_request(synth_text(7), seed=1, fixed=40), make_request(synth_text(8), seed=2, fixed=25, greedy=True)]
    got = rt.generate_batch(reqs)
    for r, (g, s) in zip(reqs, got):
        og, os_ = _oracle(om, r)
        assert (g, s) == (og, os_)
        assert len(s) == r.fixed_semantic
        assert rwkvtts.EOS_TOKEN not in s


def test_batched_equals_serial(setup):
    """8 concurrent slots give exactly the per-request results of 1-at-a-time runs."""
    om, rt = setup
    reqs = [make_request(synth_text(200 + i), seed=300 + i, max_tokens=30 + 3 * i) for i in range(8)]
    together = rt.generate_batch(reqs)
    for i, r in enumerate(reqs):
        assert rt.generate_batch([r])[0] == together[i]


def test_zero_shot_with_raf_globals(setup):
    """Zero-shot prompt uses the 32 global tokens of the reference's own RAF fixture."""
    om, rt = setup
    raf = json.load(open(os.path.join(GOLDEN, "raf_voice_05d8f5ed.json")))
    req = make_request(synth_text(5, n=10), props=[], seed=77, ref_global=raf["global_tokens"],
                       ref_semantic=raf["semantic_tokens"][:50])
    (g, s), = rt.generate_batch([req])
    og, os_ = _oracle(om, req)
    assert g == og == raf["global_tokens"]
    assert s == os_
    assert len(s) >= 18  # hard minimum ceil(10 * 1.8)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
def test_mid_model_generation_matches_oracle(dt):
    """Two layers at the full 0.4B widths: the 0.4B-specialised decode kernels (LoRA ranks
    64/64/32/128, 4 split-K slabs, C = 1024) stay token-exact against the oracle."""
    dtype = rwkvtts._ffi.DTYPE_F16 if dt == "f16" else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(W.DIMS_MID, seed=5, dtype=dtype)
    import oracle
    om = oracle.Model(blob)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=128, use_graphs=True)
    try:
        reqs = [make_request(synth_text(400 + i), seed=600 + i, fixed=24) for i in range(3)]
        got = rt.generate_batch(reqs)
        for r, (g, s) in zip(reqs, got):
            assert (g, s) == _oracle(om, r)
    finally:
        rt.close()
