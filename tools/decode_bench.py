"""Decode-loop microbenchmark: 32 requests (0.4B synthetic bf16), fixed S semantic tokens, graph
replay. Prints decode ms/step from the engine's own HIP events and a token checksum (a kernel
change that keeps the arithmetic must keep the checksum). Usage: decode_bench.py [S] [reps].
Env: DB_B requests (default 32), DB_F16=1 fp16 weights, DB_ZS=1 zero-shot prompts (32 reference
global tokens + 128 reference semantic tokens per request), DB_QUANT=int8|nf4 (every layer quantised,
the server's --quant-layers 24 --quant-type ...), DB_FORMS=n (rwkvtts_engine_desc.forms: RWKVTTS_FORM_* bits)."""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
f16 = os.environ.get("DB_F16", "0") == "1"
B = int(os.environ.get("DB_B", "32"))
zs = os.environ.get("DB_ZS", "0") == "1"
blob = W.synth_blob(W.DIMS_04B, seed=20251205, **({"dtype": rwkvtts._ffi.DTYPE_F16} if f16 else {}))
qt = os.environ.get("DB_QUANT", "none")
rt = rwkvtts.SharedRwkvRuntime(blob, max_slots=max(B, 1), token_chunk_size=512, use_graphs=True,
                               quant_layers=W.DIMS_04B["n_layer"] if qt != "none" else 0, quant_type=qt,
                               forms=int(os.environ.get("DB_FORMS", "0")))
del blob
import numpy as np  # noqa: E402
reqs = []
for i in range(B):
    rs = np.random.RandomState(1000 + i)
    ref = {}
    if zs:
        ref = dict(ref_global_tokens=rs.randint(0, 4096, size=32).tolist(),
                   ref_semantic_tokens=rs.randint(0, 8192, size=128).tolist())
    reqs.append(rwkvtts.TtsBatchRequest(text_tokens=rs.randint(12293, 77822, size=24).tolist(),
                                        property_tokens=[] if zs else [77823, 77838, 77869, 77845, 77830, 77826],
                                        args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=S, **ref))
for r in range(reps):
    t0 = time.perf_counter()
    out = rt.generate_batch(reqs)
    wall = time.perf_counter() - t0
    st = rt.stats()
    h = hashlib.sha1(repr(out).encode()).hexdigest()[:12]
    us = st['decode_ms'] / max(st['steps'], 1) * 1000
    print(f"rep {r}: B={B} f16={int(f16)} zs={int(zs)} quant={qt} decode {us:.1f} us/step over {st['steps']} steps "
          f"({B * 320 / us * 1e6:.0f} samples/s decode-only), "
          f"prefill {st['prefill_ms']:.2f} ms, wall {wall * 1000:.1f} ms, tokens {h}", flush=True)
rt.close()
