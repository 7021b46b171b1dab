"""Per-phase s_memrealtime stamps (10 ns ticks) of k_advance (the device sampler + phase controller) in the last
decode step of a 32-request 0.4B batch (RWKVTTS_DEBUG_STAMPS adv=path debug hook). Usage: advance_stamps.py [S]"""
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(tempfile.gettempdir(), "adv_stamps.bin")
os.environ["RWKVTTS_DEBUG_STAMPS"] = "adv=" + path
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
for rep in range(2):
    rt.generate_batch(reqs)
    allst = np.fromfile(path, dtype=np.uint64).reshape(256, 16).astype(np.int64)
    st = allst[:32]
    acc = allst[255]
    print(f"all steps so far: per-row kernel time mean {acc[0] / max(acc[1], 1) * 0.01:.2f} us over {acc[1]} rows, "
          f"max {acc[2] * 0.01:.2f} us; not certifiable {acc[3]}, rejected by the certificate {acc[4]}, "
          f"mean candidates {acc[5] / max(acc[1], 1):.0f}; rejections by reason: top-k boundary {acc[7]}, "
          f"top-p cut {acc[8]}, draw in band {acc[9]}, sum {acc[10]}")
    order = [k for k in range(16) if (st[:, k] != 0).all()]
    order.sort(key=lambda k: st[:, k].mean())
    print(f"rep {rep}: s_memrealtime stamps of thread 0 (10 ns ticks; mean over 32 rows of the last step), in time order")
    for a, b in zip(order, order[1:]):
        d = st[:, b] - st[:, a]
        print(f"  {a:2d} -> {b:2d}  mean {d.mean():8.0f}  min {d.min():8d}  max {d.max():8d}")
    print(f"  total {(st[:, order[-1]] - st[:, order[0]]).mean():.0f}; first row start -> last row end "
          f"{st[:, order[-1]].max() - st[:, order[0]].min()}")
rt.close()
