"""RWKV-7 forward on the GPU (Runtime<Rnn>::infer semantics) vs the oracle f32 restatement."""
import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import PROPS, synth_text

pytestmark = pytest.mark.gpu

# bf16 weights are exact in both paths; the GPU feeds MFMA with activations split into two bf16
# planes (|error| <= 2^-17 relative) and accumulates in f32 in a different order. Observed max
# |logit diff| is ~1e-4 on logits of std ~1.6; the bound below leaves headroom.
LOGIT_ATOL = 2e-3


@pytest.fixture(scope="module", params=["tiny", "small", "mid", "tiny_f16", "small_f16", "mid_f16"])
def models(request):
    dims = {"tiny": W.DIMS_TINY, "small": W.DIMS_SMALL, "mid": W.DIMS_MID}[request.param.split("_")[0]]
    dt = rwkvtts._ffi.DTYPE_F16 if request.param.endswith("f16") else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(dims, seed=123, dtype=dt)
    import oracle
    om = oracle.Model(blob)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=8, token_chunk_size=64, use_graphs=False)
    yield dims, om, rt
    rt.close()


def infer_all(rt, inp, head_rows, slots=None):
    """Feed RnnInput until every batch produced its output (the loops at
    src/normal_mode_inference.rs:74-80): a call consumes <= token_chunk_size tokens in total."""
    outs = [None] * len(inp.batches)
    while any(o is None for o in outs):
        idx = [i for i, o in enumerate(outs) if o is None]
        sub = rwkvtts.RnnInput([inp.batches[i] for i in idx], inp.token_chunk_size)
        rem, out = rt.infer(sub, head_rows=head_rows, slots=[slots[i] if slots else i for i in idx])
        for j, i in enumerate(idx):
            inp.batches[i] = rem.batches[j]
            if out[j].size:
                outs[i] = out[j]
    return outs


def _prompt(seed):
    return PROPS + [rwkvtts.TAG_2] + synth_text(seed) + [rwkvtts.TAG_0]


def test_prefill_and_decode_logits(models):
    dims, om, rt = models
    toks = _prompt(1)
    st = om.new_state()
    ref = [om.forward(st, t, 8193) for t in toks]
    rt.reset_slot(0)
    rem, out = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(toks), rwkvtts.RnnOption.Full)], 64),
                        head_rows=8193)
    got = out[0]
    assert got.shape == (len(toks), 8193)
    err = np.abs(got - np.stack(ref)).max()
    assert err < LOGIT_ATOL, err
    # state after prefill matches
    s_gpu = rt.read_slot(0)
    assert np.abs(s_gpu - st).max() < 1e-3
    # decode 8 more tokens one by one (Last option), teacher-forced
    for t in [8196 + 5, 8196 + 77, 8194, 12, 4000, 8191, 3, 8192]:
        r = om.forward(st, t, 8193)
        _, o = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch([t])], 64), head_rows=8193)
        assert np.abs(o[0] - r).max() < LOGIT_ATOL


def test_chunked_prefill_is_bitwise_identical(models):
    dims, om, rt = models
    toks = _prompt(2)
    rt.reset_slot(1)
    _, full = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(toks))], 64), head_rows=4096, slots=[1])
    rt.reset_slot(2)
    inp = rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(toks))], 7)
    # engine chunk is fixed at creation; emulate RnnInput chunking by feeding 7-token pieces
    out = None
    for i in range(0, len(toks), 7):
        _, o = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch(toks[i:i + 7])], 64), head_rows=4096, slots=[2])
        out = o[0]
    assert np.array_equal(out, full[0])
    assert np.array_equal(rt.read_slot(1), rt.read_slot(2))


def test_batch_invariance(models):
    """A slot's logits do not depend on which other slots share the step."""
    dims, om, rt = models
    prompts = [_prompt(10 + i) for i in range(4)]
    for s in range(4):
        rt.reset_slot(s)
    together = infer_all(rt, rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(p)) for p in prompts], 512),
                         head_rows=8193, slots=[0, 1, 2, 3])
    for s in range(4):
        rt.reset_slot(4)
        alone = infer_all(rt, rwkvtts.RnnInput([rwkvtts.RnnInputBatch(list(prompts[s]))], 512), head_rows=8193,
                          slots=[4])
        assert np.array_equal(alone[0], together[s]), s


def test_state_roundtrip(models):
    dims, om, rt = models
    rt.reset_slot(0)
    rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch(_prompt(3))], 64), head_rows=16)
    s = rt.read_slot(0)
    rt.write_slot(5, s)
    assert np.array_equal(rt.read_slot(5), s)
    _, a = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch([100])], 64), head_rows=4096, slots=[0])
    _, b = rt.infer(rwkvtts.RnnInput([rwkvtts.RnnInputBatch([100])], 64), head_rows=4096, slots=[5])
    assert np.array_equal(a[0], b[0])
