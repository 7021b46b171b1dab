"""Shared test helpers: request builders and the SURVEY §8d synthetic prompt."""
import ctypes

import numpy as np

import rwkvtts
from rwkvtts import _ffi

PROPS = [77823, 77838, 77869, 77845, 77830, 77826]  # SURVEY §8d (age 15, gender 46, emotion 22, pitch 7, speed 3)


def synth_text(seed, n=24):
    """24 text ids uniform in [12293, 77821]."""
    rs = np.random.RandomState(seed)
    return rs.randint(12293, 77822, size=n).astype(np.int32).tolist()


def make_request(text, props=PROPS, seed=7, max_tokens=2048, fixed=0, greedy=False,
                 ref_global=None, ref_semantic=None):
    return rwkvtts.TtsBatchRequest(text_tokens=list(text), property_tokens=list(props),
                                   ref_global_tokens=ref_global, ref_semantic_tokens=ref_semantic,
                                   args=rwkvtts.SamplerArgs(seed=seed, max_tokens=max_tokens),
                                   fixed_semantic=fixed, greedy=greedy)


def to_struct(r):
    """rwkvtts.TtsBatchRequest -> (_ffi.Request, keepalive) for the oracle."""
    keep = []

    def arr(x):
        if x is None:
            return None
        a = np.ascontiguousarray(np.asarray(x, dtype=np.int32))
        keep.append(a)
        return a
    P = ctypes.POINTER(ctypes.c_int32)
    q = _ffi.Request()
    tt, pt, rg, rs = arr(r.text_tokens), arr(r.property_tokens), arr(r.ref_global_tokens), arr(r.ref_semantic_tokens)
    q.text_tokens = tt.ctypes.data_as(P) if tt is not None and len(tt) else None
    q.n_text = 0 if tt is None else len(tt)
    q.property_tokens = pt.ctypes.data_as(P) if pt is not None and len(pt) else None
    q.n_property = 0 if pt is None else len(pt)
    q.ref_global = rg.ctypes.data_as(P) if rg is not None else None
    q.n_ref_global = 0 if rg is None else len(rg)
    q.ref_semantic = rs.ctypes.data_as(P) if rs is not None else None
    q.n_ref_semantic = 0 if rs is None else len(rs)
    q.has_seed = 0 if r.args.seed is None else 1
    q.seed = r.args.seed or 0
    q.max_tokens = r.args.max_tokens
    q.fixed_semantic = r.fixed_semantic
    q.greedy = 1 if r.greedy else 0
    return q, keep
