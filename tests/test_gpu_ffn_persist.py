"""The decode step's FFN half as ONE persistent launch (csrc/lm_kernels.hip k_ffn_persist:
LayerNorm 2 + mix, key GEMM, relu^2, value GEMM with in-launch write-through hand-offs) against
the three-launch path it replaces: the same bodies and reduction orders, so token streams must be
identical bit for bit -- at the bench shape (32 slots, 0.4B bf16, graph replay), with fewer rows
than slots (R < 32: padded LayerNorm blocks), eager launches, the fp16 model, and against the
oracle. RWKVTTS_FFN_PERSIST is read when an engine is created."""
import os

import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import make_request, synth_text, to_struct

pytestmark = pytest.mark.gpu


def _runtime(blob, persist, **kw):
    old = os.environ.get("RWKVTTS_FFN_PERSIST")
    os.environ["RWKVTTS_FFN_PERSIST"] = "1" if persist else "0"
    try:
        return rwkvtts.SharedRwkvRuntime(blob, **kw)
    finally:
        if old is None:
            os.environ.pop("RWKVTTS_FFN_PERSIST", None)
        else:
            os.environ["RWKVTTS_FFN_PERSIST"] = old


def _both(blob, reqs, **kw):
    outs, profs = [], []
    for persist in (False, True):
        rt = _runtime(blob, persist, **kw)
        try:
            outs.append(rt.generate_batch(reqs))
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
    (a, b), _ = _both(blob04, reqs, max_slots=32, token_chunk_size=2048, use_graphs=True)
    assert a == b


def test_persist_fewer_rows_and_eager(blob04):
    import oracle
    reqs = [make_request(synth_text(200 + i), seed=50 + i, fixed=12 + i) for i in range(5)]
    (a, b), profs = _both(blob04, reqs, max_slots=8, token_chunk_size=512, use_graphs=False)
    assert a == b
    # the persistent launch ran (and the three launches did not) in the decode steps
    assert "ffn_persist" in profs[1] and "ffn_persist" not in profs[0], profs[1].keys()
    om = oracle.Model(blob04)
    q, keep = to_struct(reqs[2])
    g, s, _ = om.generate(q)
    assert b[2] == (g, s)


def test_persist_f16_bitwise():
    blob = W.synth_blob(W.DIMS_04B, seed=7, dtype=rwkvtts._ffi.DTYPE_F16)
    reqs = [make_request(synth_text(300 + i), seed=70 + i, fixed=16) for i in range(8)]
    (a, b), _ = _both(blob, reqs, max_slots=8, token_chunk_size=512, use_graphs=True)
    assert a == b


def test_persist_under_the_manager_two_engines_one_device(blob04):
    """Two engines on one device decoding at the same time: two persistent launches in flight on
    the GPU together (dependencies only point to lower block indices: no deadlock)."""
    old = os.environ.get("RWKVTTS_FFN_PERSIST")
    os.environ["RWKVTTS_FFN_PERSIST"] = "1"
    try:
        m = rwkvtts.DynamicBatchManager(blob04, rwkvtts.DynamicBatchConfig(max_batch_size=64, collect_timeout_ms=5),
                                        devices=[0, 0], max_slots=32, token_chunk_size=512)
    finally:
        if old is None:
            os.environ.pop("RWKVTTS_FFN_PERSIST", None)
        else:
            os.environ["RWKVTTS_FFN_PERSIST"] = old
    try:
        reqs = [make_request(synth_text(400 + i), seed=90 + i, fixed=20) for i in range(48)]
        got = m.generate_tts_batch(reqs)
        st = m.stats()
        assert all(n > 0 for n in st["served"]), st
    finally:
        m.close()
    rt = _runtime(blob04, False, max_slots=32, token_chunk_size=512, use_graphs=True)
    try:
        ref = rt.generate_batch(reqs[:32]) + rt.generate_batch(reqs[32:])
    finally:
        rt.close()
    assert got == ref
