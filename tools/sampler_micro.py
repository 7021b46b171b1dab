"""Sampler micro-benchmark: k_sample_rows on 32 rows per config (run under rocprofv3
--kernel-trace; dispatch order == CONFIGS order x REPS)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rwkv-tts-rs_amd"))
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

CONFIGS = [  # name, n, T, top_p, top_k
    ("sem_k80_p95", 8193, 1.0, 0.95, 80),
    ("glob_k20_p95", 4096, 1.0, 0.95, 20),
    ("sem_k80_p1", 8193, 1.0, 1.0, 80),
    ("sem_k0_p1", 8193, 1.0, 1.0, 0),
    ("n1024_k80_p95", 1024, 1.0, 0.95, 80),
]
REPS = 5
rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_TINY), max_slots=2, token_chunk_size=64, use_graphs=False)
rs = np.random.RandomState(0)
for name, n, T, p, k in CONFIGS:
    x = (rs.randn(32, n) * 1.6).astype(np.float32)
    for _ in range(REPS):
        rt.sample(x, T, p, k, None, [rwkvtts.StdRng.seed_from_u64(i) for i in range(32)])
json.dump({"configs": CONFIGS, "reps": REPS}, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/null", "w"))
