"""Phase timing of the layer-5 WKV kernel in the last decode step (s_memtime stamps,
RWKVTTS_WKV_STAMPS debug hook): per-phase median cycles and the spread of WG start/end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
path = "/tmp/wkv_stamps.bin"
os.environ["RWKVTTS_WKV_STAMPS"] = path
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

d = W.DIMS_04B
rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(d), max_slots=32, token_chunk_size=512)
reqs = [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=16) for i in range(32)]
rt.generate_batch(reqs)
st = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)[: 32 * 16].astype(np.int64)
names = ["segs->partials+LoRA staged", "LoRA up", "wave0 prep", "state update", "groupnorm/store", "state store"]
for k in range(6):
    dd = st[:, k + 1] - st[:, k]
    print(f"  {names[k]:28s} median {np.median(dd):8.0f}  p90 {np.percentile(dd, 90):8.0f} cycles")
tot = st[:, 6] - st[:, 0]
print(f"  per-WG total median {np.median(tot):.0f} cycles; start spread {st[:,0].max()-st[:,0].min()} ; "
      f"first start -> last end {st[:,6].max()-st[:,0].min()} cycles")
