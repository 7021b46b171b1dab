"""Short LM workload for counter passes: 32 requests (0.4B synthetic), 16 semantic tokens each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=32, token_chunk_size=512,
                               use_graphs=os.environ.get("LM_GRAPHS", "1") == "1")
reqs = [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=16) for i in range(32)]
rt.generate_batch(reqs)
print("ok")
