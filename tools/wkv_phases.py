"""WKV (k_wkv6 by default; RWKVTTS_WKV_VARIANT-style env of the engine picks k_wkv4) phase breakdown: runs 32 requests through the engine with RWKVTTS_DEBUG_STAMPS wkv=path set
(layer 5 of the last decode step records per-workgroup stamps) and prints the launch-wide span,
the workgroup start ramp and mean / max core-clock cycles per phase."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
path = os.path.join(ROOT, "gpurun_out", "wkv_stamps.bin")
os.environ["RWKVTTS_DEBUG_STAMPS"] = "wkv=" + path
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_04B), max_slots=32, token_chunk_size=512, use_graphs=True)
reqs = [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                args=rwkvtts.SamplerArgs(seed=i), fixed_semantic=16) for i in range(32)]
rt.generate_batch(reqs)
rt.close()
st = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)[:512].astype(np.int64)
st = st[st[:, 0] > 0]
rs, re_ = st[:, 0], st[:, 7]
print(f"workgroups {len(st)}: span {(re_.max() - rs.min()) * 0.01:.2f} us; starts spread {(rs.max() - rs.min()) * 0.01:.2f} us; "
      f"ends spread {(re_.max() - re_.min()) * 0.01:.2f} us; per-WG realtime {((re_ - rs) * 0.01).mean():.2f} us mean, "
      f"{((re_ - rs) * 0.01).max():.2f} max")
names = ["loads+hidden+barrier", "lora+mix+barrier", "state update", "store+GN barrier", "tail"]
d = np.diff(st[:, 1:7], axis=1)
for k, nm in enumerate(names):
    print(f"  {nm:22s} mean {d[:, k].mean():8.0f} cyc  max {d[:, k].max():8.0f}")
print(f"  total core cycles mean {(st[:, 6] - st[:, 1]).mean():.0f} max {(st[:, 6] - st[:, 1]).max():.0f}")
