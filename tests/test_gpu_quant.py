"""Quantised layers (web-rwkv Quant::Int8 / NF4 via the server's --quant-layers / --quant-type,
bin/server.rs:1029-1071) on the GPU vs the oracle's independent restatement (oracle/rwkv7.c
oracle_model_quantize): both quantise the same 16-bit matrices with the same block rules, the
GPU dequantises in registers and feeds w = hi + lo to three MFMAs per product. Parity vs web-rwkv
itself is unpinned (the crate is not vendored)."""
import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import PROPS, make_request, synth_text, to_struct

pytestmark = pytest.mark.gpu

LOGIT_ATOL = 2e-3  # as tests/test_gpu_forward.py: hi/lo planes for activations and weights

CASES = [  # (dims, dtype, quant type, quantised layers)
    ("tiny", "bf16", "int8", 2),
    ("tiny", "f16", "nf4", 1),
    ("small", "bf16", "nf4", 4),
    ("small", "f16", "int8", 3),
    ("mid", "bf16", "int8", 2),
    ("mid", "f16", "nf4", 2),
]


@pytest.mark.parametrize("case", CASES, ids=["-".join(map(str, c)) for c in CASES])
def test_quantised_logits_and_tokens(case):
    name, dt, qt, ql = case
    dims = {"tiny": W.DIMS_TINY, "small": W.DIMS_SMALL, "mid": W.DIMS_MID}[name]
    dtype = rwkvtts._ffi.DTYPE_F16 if dt == "f16" else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(dims, seed=321, dtype=dtype)
    import oracle
    qcode = rwkvtts.runtime.parse_quant_type(qt)
    om = oracle.Model(blob, quant_layers=ql, quant_type=qcode)
    om_full = oracle.Model(blob)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=64, use_graphs=True,
                                   quant_layers=ql, quant_type=qt)
    try:
        toks = PROPS + [rwkvtts.TAG_2] + synth_text(11) + [rwkvtts.TAG_0]
        st, st_full = om.new_state(), om_full.new_state()
        ref = np.stack([om.forward(st, t, 8193) for t in toks])
        full = np.stack([om_full.forward(st_full, t, 8193) for t in toks])
        rt.reset_slot(0)
        _, out = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(toks), rwkvtts.RnnOption.Full)], 64),
                          head_rows=8193)
        err = np.abs(out[0] - ref).max()
        assert err < LOGIT_ATOL, err
        # the device runs the quantised model, not the 16-bit one
        assert err < np.abs(out[0] - full).max()
        reqs = [make_request(synth_text(500 + i), seed=700 + i, fixed=20) for i in range(3)]
        got = rt.generate_batch(reqs)
        for r, (g, s) in zip(reqs, got):
            q, keep = to_struct(r)
            og, os_, _ = om.generate(q)
            assert (g, s) == (og, os_)
    finally:
        rt.close()


def test_sf4_rejected():
    blob = W.synth_blob(W.DIMS_TINY, seed=1)
    with pytest.raises(rwkvtts._ffi.RwkvTtsError) as e:
        rwkvtts.SharedRwkvRuntime(blob, max_slots=2, quant_layers=1, quant_type="sf4")
    assert e.value.code == rwkvtts._ffi.EUNSUPPORTED
