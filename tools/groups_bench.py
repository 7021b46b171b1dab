"""Slot-group experiment: G engines on ONE device, each serving B/G of the requests from its own
host thread (its own stream and graph), against one engine serving all B. If the decode chain is
launch/latency-bound, one group's kernels run inside the other's kernel boundaries.
Usage: groups_bench.py [S] [G]. Prints wall time per request-token and the token checksum of the
union of results (must equal the single-engine run's)."""
import hashlib
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import numpy as np  # noqa: E402
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
G = int(sys.argv[2]) if len(sys.argv) > 2 else 2
B = int(os.environ.get("DB_B", "32"))
blob = W.synth_blob(W.DIMS_04B, seed=20251205)
reqs = []
for i in range(B):
    rs = np.random.RandomState(1000 + i)
    reqs.append(rwkvtts.TtsBatchRequest(text_tokens=rs.randint(12293, 77822, size=24).tolist(),
                                        property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                        args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=S))


def run(groups):
    rts = [rwkvtts.SharedRwkvRuntime(blob, max_slots=B // groups, token_chunk_size=512, use_graphs=True)
           for _ in range(groups)]
    parts = [reqs[g * (B // groups):(g + 1) * (B // groups)] for g in range(groups)]
    for rt, p in zip(rts, parts):  # warm-up (graph capture)
        rt.generate_batch(p[:1])
    for rep in range(2):
        outs = [None] * groups

        def work(g):
            outs[g] = rts[g].generate_batch(parts[g])

        th = [threading.Thread(target=work, args=(g,)) for g in range(groups)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        out = [r for o in outs for r in o]
        h = hashlib.sha1(repr(out).encode()).hexdigest()[:12]
        steps = [rt.stats()["steps"] for rt in rts]
        print(f"groups={groups} rep {rep}: wall {wall * 1000:.1f} ms, {wall / (S + 33) * 1e6:.1f} us per step-equivalent "
              f"(steps {steps}), {B * (S + 33) / wall:.0f} tokens/s, tokens {h}", flush=True)
    for rt in rts:
        rt.close()


run(1)
run(G)
