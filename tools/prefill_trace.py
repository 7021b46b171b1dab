"""Prefill-only workload for a kernel trace: 32 requests of the bench's prompt shape (6 property
+ TAG + 32 text + TAG tokens), fixed_semantic=1, run twice (the second run is the one to read).
PF_CHUNK sets the engine's token_chunk_size (default 512)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import numpy as np  # noqa: E402
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=32,
                               token_chunk_size=int(os.environ.get("PF_CHUNK", "512")), use_graphs=True)
rs = np.random.RandomState(0)
reqs = [rwkvtts.TtsBatchRequest(text_tokens=rs.randint(12293, 77822, size=32).tolist(),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=1) for i in range(32)]
for _ in range(2):
    rt.generate_batch(reqs)
    st = rt.stats()
    print("prefill_ms", round(st["prefill_ms"], 3), "prefill_steps", st["prefill_steps"])
