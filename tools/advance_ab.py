"""Per-kernel HIP-event times of a 32-request 0.4B batch (eager launches, the bench's profiling
pass) -- for A/B runs of the sampler / controller under environment switches (e.g.
RWKVTTS_SAMPLER_EXACT=1). Usage: advance_ab.py [S]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import numpy as np  # noqa: E402
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B, seed=20251205), max_slots=32, token_chunk_size=2048,
                               use_graphs=True)
reqs = []
for i in range(32):
    rs = np.random.RandomState(i)
    reqs.append(rwkvtts.TtsBatchRequest(text_tokens=rs.randint(12293, 77822, size=24).tolist(),
                                        property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                        args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=S))
rt.generate_batch(reqs)  # warm-up (graphs, caches)
rt.set_profiling(True)
out = rt.generate_batch(reqs)
prof = rt.profile()
rt.set_profiling(False)
tok = sum(sum(s) for _, s in out) % 1000003
for k in ("sample_advance", "gemm_head", "wkv", "embed"):
    n, ms = prof.get(k, (0, 0.0))
    print(f"{os.environ.get('AB_TAG', '')} {k:16s} launches {n:6d} avg {1000.0 * ms / max(n, 1):8.2f} us  (tokens {tok})")
rt.close()
