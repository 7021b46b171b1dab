"""Phase timing of two layer-5 GEMMs (rkv+LoRA-down, ffn_value) in the last decode step:
s_memtime stamps (RWKVTTS_GEMM_STAMPS debug hook). Phases: start -> X staged (W loads issued
before) -> MFMA done (W arrived) -> stores issued."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
path = "/tmp/gemm_stamps.bin"
os.environ["RWKVTTS_GEMM_STAMPS"] = path
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=32, token_chunk_size=512)
reqs = [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=16) for i in range(32)]
rt.generate_batch(reqs)
st = np.fromfile(path, dtype=np.uint64).reshape(2, 4096, 4).astype(np.int64)
for name, nwg, s in (("rkv_lora", 53 * 4, st[0]), ("ffn_value", 16 * 16, st[1])):
    s = s[:nwg]
    d = np.diff(s, axis=1)
    print(f"{name}: per-WG median total {np.median(s[:,3]-s[:,0]):.0f} cyc; phases "
          f"{' / '.join(f'{np.median(d[:,i]):.0f}' for i in range(3))}; "
          f"p90 total {np.percentile(s[:,3]-s[:,0], 90):.0f}; start spread {s[:,0].max()-s[:,0].min()} "
          f"span {s[:,3].max()-s[:,0].min()}")
