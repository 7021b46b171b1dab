"""StreamingInference mirror (src/streaming_inference.rs): CPU-side scheduling logic, and on the
GPU real logits equal to a direct infer of the same tokens on a fresh slot."""
import threading

import numpy as np
import pytest

from rwkvtts import streaming as S


class FakeRuntime:
    """Engine stand-in for the CPU tests: logits = one-hot-ish function of the token list."""
    max_slots = 4
    token_chunk_size = 64

    def __init__(self):
        self.calls = []
        self._lock = threading.RLock()

    def reset_slot(self, s):
        pass

    def infer(self, inp, slots=None, head_rows=None):
        from rwkvtts.runtime import RnnInput, RnnInputBatch
        self.calls.append([list(b.tokens) for b in inp.batches])
        outs = [np.array([float(sum(b.tokens)), float(len(b.tokens))], np.float32) for b in inp.batches]
        return RnnInput([RnnInputBatch([]) for _ in inp.batches], inp.token_chunk_size), outs


def test_priority_order_cache_and_stats():
    rt = FakeRuntime()
    si = S.StreamingInference(rt, S.BatchConfig(max_batch_size=2, batch_timeout=0.01))
    with pytest.raises(RuntimeError):
        si.submit_request(S.InferenceRequest("x", [1]))
    # queue three requests before the scheduler runs: the high-priority one goes first
    reqs = [S.InferenceRequest("a", [1, 2], priority=1), S.InferenceRequest("b", [3], priority=9),
            S.InferenceRequest("c", [4, 5, 6], priority=5)]
    for r in reqs:
        si._queues.setdefault(r.priority, __import__("collections").deque())
    si.start()
    res = {}
    ths = [threading.Thread(target=lambda r=r: res.__setitem__(r.id, si.submit_request(r))) for r in reqs]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert [res[k].logits[0] for k in "abc"] == [3.0, 3.0, 15.0]
    again = si.submit_request(S.InferenceRequest("a2", [1, 2]))
    assert again.from_cache and again.logits[0] == 3.0
    st = si.get_stats()
    assert st.total_requests == 4 and st.cache_hits == 1 and st.total_batches >= 2
    assert all(len(c) <= 2 for c in rt.calls)
    si.adjust_batch_size(target_latency_ms=1e9)  # far under target: grow
    assert si.get_config().max_batch_size == 3
    si.stop()


@pytest.mark.gpu
def test_streaming_matches_direct_infer():
    import rwkvtts
    from rwkvtts import weights as W
    import oracle
    blob = W.synth_blob(W.DIMS_TINY, seed=5)
    om = oracle.Model(blob)
    rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=16, use_graphs=False)
    si = S.StreamingInference(rt, S.BatchConfig(max_batch_size=4))
    si.start()
    toks = [[77823, 77838, 8195] + list(range(20000 + i, 20000 + i + 5 + 7 * i)) + [8193] for i in range(6)]
    got = [None] * 6
    ths = [threading.Thread(target=lambda i=i: got.__setitem__(i, si.submit_request(S.InferenceRequest(str(i), toks[i]))))
           for i in range(6)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    si.stop()
    for i in range(6):
        rt.reset_slot(0)
        inp = rwkvtts.RnnInput([rwkvtts.RnnInputBatch(toks[i])], 16)
        out = None
        while out is None or out.size == 0:
            inp, o = rt.infer(inp, slots=[0])
            out = o[0]
        assert np.array_equal(got[i].logits, out)
        # and against the oracle's f32 restatement (tolerance of test_gpu_forward.py)
        st = om.new_state()
        V = out.size
        ref = [om.forward(st, t, V) for t in toks[i]][-1]
        assert np.abs(got[i].logits - ref).max() < 2e-3
    rt.close()
