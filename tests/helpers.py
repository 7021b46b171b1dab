"""Shared test helpers: request builders and the SURVEY §8d synthetic prompt."""
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
    """rwkvtts.TtsBatchRequest -> (_ffi.Request, keepalive) for the oracle (the same struct the
    product ABI takes)."""
    from rwkvtts.runtime import request_struct
    return request_struct(r)
