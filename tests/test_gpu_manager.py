"""The native request manager (rwkvtts_manager_*, dynamic_batch_manager.rs:33-405) at the
benchmarked shape and under failure:

* config 4's per-GPU path: DIMS_04B weights, 32 slots per engine, two engines, 48 requests from
  concurrent submitter threads, the weight blob uploaded once and (RWKVTTS_MANAGER_FORCE_RCCL)
  ncclBroadcast to the engines' devices -- on a one-GPU box both engines share device 0, so the
  broadcast is a one-rank RCCL call and the second engine copies device-to-device; sampled
  requests token-exact against the oracle; live statistics while the manager runs;
* config 4's whole workload on the one GPU: 8 engines x 32 slots (the 8-GPU node's engine count,
  all on device 0), 256 requests from 8 submitter threads, every engine serving, sampled
  requests token-exact against the oracle; one distinct device -> RCCL is not loaded;
* RCCL disabled (RWKVTTS_MANAGER_NO_RCCL): the manager still creates and serves;
* an injected admission failure (RWKVTTS_TEST_FAIL_ADMIT): every ticket still resolves;
* a second waiter on one ticket is refused; destroy with a waiter blocked returns its result;
* two engines on one device capturing their first decode graphs at the same moment.
"""
import os
import threading
import time

import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W
from helpers import make_request, synth_text, to_struct

pytestmark = pytest.mark.gpu


def _oracle(om, req):
    q, keep = to_struct(req)
    g, s, _ = om.generate(q)
    return g, s


def _run_concurrent(fns, timeout):
    out = [None] * len(fns)
    err = []

    def call(i):
        try:
            out[i] = fns[i]()
        except Exception as e:  # noqa: BLE001
            err.append((i, repr(e)))
    ths = [threading.Thread(target=call, args=(i,), daemon=True) for i in range(len(fns))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
    assert not any(t.is_alive() for t in ths), "threads still running after the timeout"
    assert not err, err
    return out


class _env:
    def __init__(self, **kv):
        self.kv = kv

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update({k: str(v) for k, v in self.kv.items()})

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_manager_04b_32_slots_two_engines_rccl():
    blob = W.synth_blob(W.DIMS_04B, seed=20251205)
    import oracle
    with _env(RWKVTTS_MANAGER_FORCE_RCCL=1):
        m = rwkvtts.DynamicBatchManager(blob, rwkvtts.DynamicBatchConfig(max_batch_size=50, collect_timeout_ms=20),
                                        devices=[0, 0], max_slots=32, token_chunk_size=512)
    try:
        st0 = m.stats()
        assert st0["bcast_rccl"] == 1 and st0["bcast_ranks"] == 1, st0
        reqs = [make_request(synth_text(5000 + i), seed=3000 + i, fixed=6 + i % 5) for i in range(48)]
        got = [None] * 48
        live = []

        def submitter(k):
            def run():
                tickets = [(i, m.submit(reqs[i])) for i in range(k, 48, 6)]
                for i, t in tickets:
                    got[i] = m.wait(t, timeout_ms=240000)
                    live.append(m.stats())
            return run
        _run_concurrent([submitter(k) for k in range(6)], timeout=300)
        assert all(g is not None for g in got), ("requests not served", m.stats())
        st = m.stats()
        assert st["completed"] == 48 and all(n > 0 for n in st["served"]), st
        # statistics are live: read while the manager runs, not only after destroy
        assert any(max(s["max_active"]) > 1 and max(s["steps"]) > 0 for s in live), live[-1]
        assert max(st["max_active"]) <= 32
        om = oracle.Model(blob)
        for i in (0, 13, 29, 47):
            assert got[i] == _oracle(om, reqs[i]), i
        for i in range(48):
            assert len(got[i][0]) == 32 and len(got[i][1]) == 6 + i % 5
    finally:
        m.close()


def test_manager_config4_eight_engines_256_requests():
    """Config 4's request-level data parallelism (dynamic_batch_manager.rs:33-87,185-405) at its
    full shape, on the one GPU: 8 engines x 32 slots, 256 requests, 8 submitter threads."""
    blob = W.synth_blob(W.DIMS_04B, seed=20251205)
    import oracle
    n_eng, n_req, n_thr = 8, 256, 8
    m = rwkvtts.DynamicBatchManager(blob, rwkvtts.DynamicBatchConfig(max_batch_size=64, collect_timeout_ms=20),
                                    devices=[0] * n_eng, max_slots=32, token_chunk_size=512)
    try:
        st0 = m.stats()
        # one distinct device: nothing to broadcast, RCCL is not even loaded
        assert st0["bcast_ranks"] == 1 and st0["bcast_rccl"] == 0, st0
        reqs = [make_request(synth_text(9000 + i), seed=4000 + i, fixed=3 + i % 4) for i in range(n_req)]
        got = [None] * n_req

        def submitter(k):
            def run():
                tickets = [(i, m.submit(reqs[i])) for i in range(k, n_req, n_thr)]
                for i, t in tickets:
                    got[i] = m.wait(t, timeout_ms=240000)
            return run
        _run_concurrent([submitter(k) for k in range(n_thr)], timeout=280)
        missing = [i for i in range(n_req) if got[i] is None]
        assert not missing, ("tickets not resolved", missing[:8], m.stats())
        st = m.stats()
        assert st["completed"] == n_req and sum(st["served"]) == n_req, st
        assert all(n > 0 for n in st["served"]), ("an engine served nothing", st["served"])
        assert max(st["max_active"]) <= 32, st
        assert sum(st["persistent"]) == 1, st  # one persistent engine on the device, 7 separate-launch ones
        for i in range(n_req):
            assert len(got[i][0]) == 32 and len(got[i][1]) == 3 + i % 4, i
        om = oracle.Model(blob)
        for i in (0, 31, 64, 100, 127, 170, 222, 255):
            assert got[i] == _oracle(om, reqs[i]), i
    finally:
        m.close()


def test_manager_without_rccl():
    """RCCL disabled: a one-device manager never needs it; a multi-engine one still creates,
    serves and reports bcast_rccl = 0 (single-GPU deployments carry no RCCL)."""
    blob = W.synth_blob(W.DIMS_TINY, seed=99)
    import oracle
    with _env(RWKVTTS_MANAGER_NO_RCCL=1):
        m = rwkvtts.DynamicBatchManager(blob, devices=[0, 0], max_slots=2, token_chunk_size=64)
    try:
        st = m.stats()
        assert st["bcast_rccl"] == 0 and st["bcast_ranks"] == 1, st
        reqs = [make_request(synth_text(8100 + i), seed=50 + i, max_tokens=10) for i in range(4)]
        got = m.generate_tts_batch(reqs)
        om = oracle.Model(blob)
        assert got == [_oracle(om, r) for r in reqs]
    finally:
        m.close()
    import torch
    assert torch.cuda.current_device() == 0


def test_manager_admission_failure_resolves_every_ticket():
    blob = W.synth_blob(W.DIMS_TINY, seed=99)
    import oracle
    os.environ["RWKVTTS_TEST_FAIL_ADMIT"] = "3"  # each engine's 3rd admission fails
    try:
        m = rwkvtts.DynamicBatchManager(blob, rwkvtts.DynamicBatchConfig(max_batch_size=4, collect_timeout_ms=5),
                                        devices=[0, 0], max_slots=2, token_chunk_size=64)
        try:
            reqs = [make_request(synth_text(6000 + i), seed=80 + i, max_tokens=8) for i in range(10)]
            tickets = [m.submit(r) for r in reqs]
            res = [m.wait_status(t, timeout_ms=60000) for t in tickets]
        finally:
            m.close()
    finally:
        del os.environ["RWKVTTS_TEST_FAIL_ADMIT"]
    assert all(o is not None for o, _ in res), "a ticket never resolved"
    status = [s for _, s in res]
    assert rwkvtts._ffi.EHIP in status, status
    om = oracle.Model(blob)
    for (o, s), r in zip(res, reqs):
        assert s in (0, rwkvtts._ffi.EHIP)
        if s == 0:
            assert o == _oracle(om, r)
        else:
            assert o == ([], [])


def test_manager_ticket_waiters():
    blob = W.synth_blob(W.DIMS_TINY, seed=99)
    m = rwkvtts.DynamicBatchManager(blob, devices=[0], max_slots=2, token_chunk_size=64)
    closed = False
    try:
        t = m.submit(make_request(synth_text(1), seed=1, fixed=400))
        first = []
        th = threading.Thread(target=lambda: first.append(m.wait(t, timeout_ms=120000)), daemon=True)
        th.start()
        time.sleep(0.3)
        with pytest.raises(rwkvtts._ffi.RwkvTtsError):
            m.wait(t, timeout_ms=0)  # claimed by the first waiter (or already released): refused
        # destroy while a waiter blocks on a long request: shutdown drains the request and the
        # waiter returns its result before the manager's memory goes away
        t2 = m.submit(make_request(synth_text(2), seed=2, fixed=300))
        second = []
        th2 = threading.Thread(target=lambda: second.append(m.wait_status(t2, timeout_ms=120000)), daemon=True)
        th2.start()
        # every waiter that has not returned yet is blocked inside the native wait (not merely
        # started) before destroy
        t_end = time.time() + 30
        while time.time() < t_end:
            need = (0 if first else 1) + (0 if second else 1)
            if m.stats()["waiters"] >= need:
                break
            time.sleep(0.005)
        else:
            raise AssertionError("waiter threads never blocked in rwkvtts_manager_wait")
        m.close()
        closed = True
        th.join(60)
        th2.join(60)
        assert first and len(first[0][1]) == 400
        assert second and second[0][1] in (0, rwkvtts._ffi.ECLOSED)
    finally:
        if not closed:
            m.close()


def test_two_engines_first_capture_concurrently():
    """Regression for the round-2 manager hang: two engines on one device, owned by
    two threads, capture and instantiate their first decode graphs at the same moment."""
    blob = W.synth_blob(W.DIMS_TINY, seed=99)
    import oracle
    rts = [rwkvtts.SharedRwkvRuntime(blob, device=0, max_slots=4, token_chunk_size=64, use_graphs=True)
           for _ in range(2)]
    try:
        reqs = [make_request(synth_text(7000 + i), seed=90 + i, max_tokens=12) for i in range(2)]
        gate = threading.Barrier(2)

        def run(i):
            def f():
                gate.wait()
                return rts[i].generate_batch([reqs[i]])[0]
            return f
        got = _run_concurrent([run(0), run(1)], timeout=120)
        om = oracle.Model(blob)
        assert got == [_oracle(om, r) for r in reqs]
    finally:
        for rt in rts:
            rt.close()
