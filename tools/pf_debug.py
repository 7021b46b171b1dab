import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "rwkv-tts-rs_amd"))
import numpy as np, ctypes
from rwkvtts import codec, _ffi
d = codec.CODEC_DIMS_FULL
c = codec.BiCodecDetokenizer(codec.synth_codec_blob(d), d)
rs = np.random.default_rng(512)
for T in (24, 64, 128, 256, 512):
    items = [(rs.integers(0, 4096, 32), rs.integers(0, 8192, T)) for _ in range(4)]
    outs = c.decode_audio_batch(items)
    print(T, [o.size for o in outs][:2], _ffi.lib().rwkvtts_last_error().decode() if hasattr(_ffi.lib().rwkvtts_last_error, "restype") else "", flush=True)
