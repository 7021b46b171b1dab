"""The decode step's two halves as persistent launches (csrc/lm_kernels.hip k_ffn_persist: LayerNorm
2 + mix, key GEMM, relu^2, value GEMM; k_att_persist: LayerNorm 1 + six mixes (layer 0 with the
embedding folded in), rkv + LoRA-down, WKV, Wo -- with in-launch write-through hand-offs) against
the launches they replace: the same bodies and reduction orders, so token streams must be
identical bit for bit -- at the bench shape (32 slots, 0.4B bf16, graph replay), with fewer rows
than slots (R < 32: padded LayerNorm blocks), eager launches, the fp16 model, two engines on one
GPU, and against the oracle. The forms are selected per engine by rwkvtts_engine_desc.forms
(RWKVTTS_FORM_*: each bit switches one fused form back to the launches it replaces)."""
import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import make_request, synth_text, to_struct

pytestmark = pytest.mark.gpu


# "both": both halves persistent (two launches per layer, the production decode path, forms 0). The
# one-launch per layer / per step variants and the rkv -> WKV granule hand-off were measured slower
# (rounds 4 and 5) and removed from the library in round 6 (tools/experiments/r06_shelved_forms.patch).
_F = rwkvtts._ffi
_SEP = _F.FORM_SEPARATE_ATT | _F.FORM_SEPARATE_FFN
MODES = {"off": _SEP,
         "ffn": _F.FORM_SEPARATE_ATT,
         "att": _F.FORM_SEPARATE_FFN,
         "both": 0,
         # one-row steps without the row-fused LayerNorm form (its LayerNorm rows as at R > 1)
         "both_rows": _F.FORM_LN_ROWS,
         # the row-fused form with the key -> value / WKV -> Wo hand-offs through partial slabs +
         # counters instead of data-tagged granules
         "both_slabs": _F.FORM_SLAB_HANDOFF,
         # separate launches with ln_out as its own launch (not folded into the one-row head GEMM)
         "off_lnout": _SEP | _F.FORM_SEPARATE_LNOUT,
         # the shipping forms with the exact sampler walk (no certificate): the same tokens
         "both_exact": _F.FORM_EXACT_SAMPLER}


def _runtime(blob, mode, **kw):
    if mode is True:
        mode = "both"
    elif mode is False:
        mode = "off"
    return rwkvtts.SharedRwkvRuntime(blob, forms=MODES[mode], **kw)


def _both(blob, reqs, modes=("off", "ffn", "att", "both"), **kw):
    """Token streams of every mode; the recurrent state after generation must be bitwise the
    first mode's as well (a 1-ulp difference that does not flip a token is still a difference)."""
    outs, profs, ref_states = [], [], None
    for persist in modes:
        rt = _runtime(blob, persist, **kw)
        try:
            outs.append(rt.generate_batch(reqs))
            states = [rt.read_slot(s) for s in range(min(len(reqs), 8))]
            if ref_states is None:
                ref_states = states
            else:
                for i, (x, y) in enumerate(zip(states, ref_states)):
                    assert np.array_equal(x, y), (persist, i, int(np.sum(x != y)))
            if not kw.get("use_graphs", True):
                rt.set_profiling(True)
                rt.generate_batch(reqs[:1])
                profs.append(rt.profile())
                rt.set_profiling(False)
        finally:
            rt.close()
    return outs, profs


@pytest.fixture(scope="module")
def blob04():
    return W.synth_blob(W.DIMS_04B, seed=20251205)


def test_persist_bench_shape_bitwise(blob04):
    reqs = [make_request(synth_text(100 + i), seed=i, fixed=40) for i in range(32)]
    outs, _ = _both(blob04, reqs, max_slots=32, token_chunk_size=2048, use_graphs=True)
    assert all(o == outs[0] for o in outs[1:])


def test_persist_fewer_rows_and_eager(blob04):
    import oracle
    reqs = [make_request(synth_text(200 + i), seed=50 + i, fixed=12 + i) for i in range(5)]
    outs, profs = _both(blob04, reqs, max_slots=8, token_chunk_size=512, use_graphs=False)
    assert all(o == outs[0] for o in outs[1:])
    b = outs[3]
    # the persistent launches ran (and the separate ones did not) in the decode steps
    assert "ffn_persist" in profs[1] and "ffn_persist" not in profs[0], profs[1].keys()
    assert "att_persist" in profs[2] and "wkv" in profs[0], profs[2].keys()
    assert "att_persist" in profs[3] and "ffn_persist" in profs[3], profs[3].keys()
    om = oracle.Model(blob04)
    q, keep = to_struct(reqs[2])
    g, s, _ = om.generate(q)
    assert b[2] == (g, s)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_persist_one_row_fused_layernorm_bitwise(dtype):
    """One decode row (a lone request): the persistent halves run their row-fused form (no LayerNorm
    workgroups: every rkv / key workgroup computes the row's LayerNorm itself, a trailing workgroup
    stores the residual and the token-shift row; the FFN key -> value hand-off as data-tagged
    granules; ln_out folded into the head GEMM). Bitwise the separate launches' (ln_out as its own
    launch, and folded), the LayerNorm-row form's, the slab hand-off's and the exact sampler's
    tokens and recurrent state, graph replay and eager."""
    dt = rwkvtts._ffi.DTYPE_F16 if dtype == "f16" else rwkvtts._ffi.DTYPE_BF16
    blob = W.synth_blob(W.DIMS_04B, seed=11, dtype=dt)
    reqs = [make_request(synth_text(500), seed=5, fixed=40)]
    for graphs in (True, False):
        outs, _ = _both(blob, reqs, modes=("off_lnout", "off", "both", "both_rows", "both_slabs", "both_exact"),
                        max_slots=4, token_chunk_size=512, use_graphs=graphs)
        assert all(o == outs[0] for o in outs[1:]), graphs


def test_persist_f16_bitwise():
    blob = W.synth_blob(W.DIMS_04B, seed=7, dtype=rwkvtts._ffi.DTYPE_F16)
    reqs = [make_request(synth_text(300 + i), seed=70 + i, fixed=16) for i in range(8)]
    outs, _ = _both(blob, reqs, max_slots=8, token_chunk_size=512, use_graphs=True)
    assert all(o == outs[0] for o in outs[1:])


def test_persist_under_the_manager_two_engines_one_device(blob04):
    """Two engines on one device decoding at the same time. Only the first engine created on the
    device holds the persistent slot (claim_persistent: two persistent launches in flight on one GPU
    can deadlock); the second runs the separate launches beside it, so one persistent launch and
    separate launches are in flight together -- asserted through the manager's per-engine flag."""
    m = rwkvtts.DynamicBatchManager(blob04, rwkvtts.DynamicBatchConfig(max_batch_size=64, collect_timeout_ms=5),
                                    devices=[0, 0], max_slots=32, token_chunk_size=512, forms=MODES["both"])
    try:
        reqs = [make_request(synth_text(400 + i), seed=90 + i, fixed=20) for i in range(48)]
        got = m.generate_tts_batch(reqs)
        st = m.stats()
        assert all(n > 0 for n in st["served"]), st
        assert sorted(st["persistent"]) == [0, 1], st  # exactly one engine per device is persistent
    finally:
        m.close()
    rt = _runtime(blob04, False, max_slots=32, token_chunk_size=512, use_graphs=True)
    try:
        ref = rt.generate_batch(reqs[:32]) + rt.generate_batch(reqs[32:])
    finally:
        rt.close()
    assert got == ref
