"""Vocoder micro-benchmark: BiCodec decode of B utterances x T frames (full dims), per-stage
HIP-event profile and achieved TFLOP/s (algorithmic, f32-equivalent)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from rwkvtts import codec  # noqa: E402
from bench import codec_flops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
d = codec.CODEC_DIMS_FULL
c = codec.BiCodecDetokenizer(codec.synth_codec_blob(d), d)
rs = np.random.default_rng(0)
items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T)) for _ in range(B)]
pcm = c.decode_audio_batch(items)
if os.environ.get("CODEC_DIGEST"):
    import hashlib
    h = hashlib.sha256()
    for x in pcm:
        h.update(np.ascontiguousarray(x, dtype=np.float32).tobytes())
    print("pcm digest", h.hexdigest()[:16])
t0 = time.perf_counter()
for _ in range(3):
    c.decode_audio_batch(items)
dt = (time.perf_counter() - t0) / 3
fl = codec_flops(d, B * T)
print(f"B={B} T={T}: {dt*1e3:.2f} ms/batch, {sum(fl.values())/dt/1e12:.1f} TFLOP/s end-to-end")
c.set_profiling(True)
c.decode_audio_batch(items)
tot = 0.0
for k, (n, ms) in c.profile().items():
    tot += ms
    extra = f" {fl[k]/(ms*1e-3)/1e12:7.1f} TFLOP/s" if k in fl and ms > 0 else ""
    print(f"  {k:20s} {n:4d} launches {ms:9.3f} ms{extra}")
print(f"  total (eager, events) {tot:.3f} ms")
