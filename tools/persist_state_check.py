"""Bitwise state / token comparison of the persistent-launch modes (off, ffn, att, both), each run
twice (a race shows as run-to-run variation). Usage: persist_state_check.py [f16|bf16] [mid|04b]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402
from helpers import make_request, synth_text  # noqa: E402

dt = sys.argv[1] if len(sys.argv) > 1 else "f16"
dims = W.DIMS_MID if (len(sys.argv) < 3 or sys.argv[2] == "mid") else W.DIMS_04B
blob = W.synth_blob(dims, seed=5, dtype=rwkvtts._ffi.DTYPE_F16 if dt == "f16" else rwkvtts._ffi.DTYPE_BF16)
reqs = [make_request(synth_text(300 + i), seed=70 + i, max_tokens=40) for i in range(3)]
modes = {"off": ("0", "0"), "ffn": ("5", "0"), "att": ("0", "5"), "both": ("5", "5")}
res = {}
for name, (f, a) in modes.items():
    for rep in range(2):
        os.environ["RWKVTTS_FFN_PERSIST"], os.environ["RWKVTTS_ATT_PERSIST"] = f, a
        rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=128, use_graphs=True)
        out = rt.generate_batch(reqs)
        st = [rt.read_slot(s) for s in range(3)]
        rt.close()
        res[(name, rep)] = (out, st)
ref_out, ref_st = res[("off", 0)]
for k, (o, st) in res.items():
    diff = [int(np.sum(a != b)) for a, b in zip(st, ref_st)]
    mx = max(float(np.max(np.abs(a - b))) for a, b in zip(st, ref_st))
    print(k, "tokens_equal", o == ref_out, "state elements differing", diff, "max abs", mx, flush=True)
