"""Debug: one request alone (one-row decode steps) with and without the granule hand-off, eager
and graph replay; prints statuses and whether the token streams agree."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "rwkv-tts-rs_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402
from helpers import make_request, synth_text  # noqa: E402

blob = W.synth_blob(W.DIMS_04B, seed=11)
reqs = [make_request(synth_text(500), seed=5, fixed=20)]
res = {}
for graphs in (True, False):
    for gran in ("0", "1"):
        os.environ["RWKVTTS_GRAN"] = gran
        rt = rwkvtts.SharedRwkvRuntime(blob, device=0, max_slots=4, token_chunk_size=512, use_graphs=graphs)
        try:
            out = rt.generate_batch(reqs)
            res[(graphs, gran)] = out
            print("graphs", graphs, "gran", gran, "status", rt.last_status, "glob", out[0][0][:6], "sem", out[0][1][:8], flush=True)
        finally:
            rt.close()
for graphs in (True, False):
    print("graphs", graphs, "equal:", res[(graphs, "0")] == res[(graphs, "1")])
