"""k_wkv2 phase stamps (layer 5, last decode step; RWKVTTS_WKV_STAMPS debug hook).
Phases: 0 start -> 1 partials+hidden staged -> 2 LoRA-up + channel terms -> 3 state update +
moments -> 4 GroupNorm/store -> 5 state stored; 6 = end of row 1 (prefill rows only)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
path = "/tmp/wkv2_stamps.bin"
os.environ["RWKVTTS_WKV_STAMPS"] = path
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=32, token_chunk_size=512)
reqs = [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=16) for i in range(32)]
rt.generate_batch(reqs)
st = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)[: 32 * 16].astype(np.int64)
names = ["loads->hidden staged", "LoRA-up + channel", "state update+moments", "GN + store", "state store"]
for k in range(5):
    d = st[:, k + 1] - st[:, k]
    print(f"  {names[k]:24s} median {np.median(d):7.0f}  p90 {np.percentile(d, 90):7.0f}")
print(f"  total median {np.median(st[:,5]-st[:,0]):.0f}")
