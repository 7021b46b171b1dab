"""Persistent-launch per-block stamps (layer 5 of the last decode step): k_ffn_persist
(RWKVTTS_DEBUG_STAMPS ffn=path; roles LayerNorm rows, key, value) or k_att_persist (att=path; roles
LayerNorm rows, rkv, WKV, Wo): per role the min / median / max of each stamp in us from the
launch's first block start. Usage: ffn_stamps.py [S] [ffn|att] [B] (B requests, default 32;
S semantic; DB_FORMS: rwkvtts_engine_desc.forms, e.g. 4 = the LayerNorm-row form at B = 1)."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
which = sys.argv[2] if len(sys.argv) > 2 else "ffn"
path = os.path.join(tempfile.mkdtemp(), "stamps.bin")
os.environ["RWKVTTS_DEBUG_STAMPS"] = ("ffn=" if which == "ffn" else "att=") + path
B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 32
blob = W.synth_blob(W.DIMS_04B, seed=20251205)
forms = int(os.environ.get("DB_FORMS", "0"))
rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=max(B, 1), token_chunk_size=2048, use_graphs=True, forms=forms)
reqs = []
for i in range(B):
    rs = np.random.RandomState(1000 + i)
    reqs.append(rwkvtts.TtsBatchRequest(text_tokens=rs.randint(12293, 77822, size=24).tolist(),
                                        property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                        args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=S))
for rep in range(2):
    rt.generate_batch(reqs)
    st = rt.stats()
    print(f"rep {rep}: decode {st['decode_ms'] / max(st['steps'], 1) * 1000:.1f} us/step")
rt.close()
a = np.fromfile(path, dtype=np.uint64).reshape(-1, 4).astype(np.float64)
nw = 16 * B  # WKV workgroups: one per (row, head)
ae = 244 + nw + 128
roles = ({"ln": (0, 32), "key": (32, 288), "value": (288, 544)} if which == "ffn" else
         {"ln": (0, 32), "rkv": (32, 244), "wkv": (244, 244 + nw), "wo": (244 + nw, ae)})
if B == 1 and not (forms & rwkvtts._ffi.FORM_LN_ROWS):  # the row-fused form (layer 5: no LN blocks)
    roles = ({"key": (0, 256), "value": (256, 512), "shift": (512, 513)} if which == "ffn" else
             {"rkv": (0, 212), "wkv": (212, 228), "wo": (228, 356), "shift": (356, 357)})
nb = max(e for _, e in roles.values())
t0 = a[:nb, 0][a[:nb, 0] > 0].min()
names = ["start", "wait_done", "work_done", "end"]
for r, (b, e) in roles.items():
    x = (a[b:e] - t0) * 0.01  # 100 MHz ticks -> us
    line = []
    for k in range(4):
        v = x[:, k][a[b:e, k] > 0]
        if v.size:
            line.append(f"{names[k]} {v.min():6.2f}/{np.median(v):6.2f}/{v.max():6.2f}")
    print(f"{r:6s} " + "  ".join(line))
