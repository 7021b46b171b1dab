"""Decode steps run the token embedding inside layer 0's LayerNorm launch (lm_kernels.hip
k_ln1024 EMB form, engine.hip launch_forward); prefill steps and engines created with
forms = RWKVTTS_FORM_SEPARATE_EMBED run k_embed as its own launch. Both must give the same bits: the same
token streams and bitwise-identical recurrent state after generation."""
import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import make_request, synth_text

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dt", ["bf16", "f16"])
def test_fused_embedding_is_bitwise_identical(dt):
    dtype = rwkvtts._ffi.DTYPE_F16 if dt == "f16" else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(W.DIMS_MID, seed=5, dtype=dtype)  # n_embd 1024: the fused form applies
    reqs = [make_request(synth_text(300 + i), seed=70 + i, max_tokens=40) for i in range(3)]
    out, states = [], []
    for off in (False, True):
        rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=128, use_graphs=True,
                                       forms=rwkvtts._ffi.FORM_SEPARATE_EMBED if off else 0)
        try:
            out.append(rt.generate_batch(reqs))
            states.append([rt.read_slot(s) for s in range(len(reqs))])
        finally:
            rt.close()
    assert out[0] == out[1]
    assert sum(len(s) for _, s in out[0]) > 0
    for a, b in zip(states[0], states[1]):
        assert np.array_equal(a, b)
