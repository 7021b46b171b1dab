"""Experiment: 32 requests as L independent engine lanes (own HIP stream each) driven from L
host threads concurrently (ctypes releases the GIL), vs one engine with 32 slots."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rwkv-tts-rs_amd"))
import numpy as np  # noqa: E402
import rwkvtts  # noqa: E402
from rwkvtts import weights as W  # noqa: E402

blob = W.synth_blob(W.DIMS_04B)
SEM = int(os.environ.get("SEM", "128"))


def reqs(n, off):
    return [rwkvtts.TtsBatchRequest(text_tokens=list(range(20000 + i, 20024 + i)),
                                    property_tokens=[77823, 77838, 77869, 77845, 77830, 77826],
                                    args=rwkvtts.SamplerArgs(seed=off + i), fixed_semantic=SEM) for i in range(n)]


for L in (1, 2, 4):
    per = 32 // L
    rts = [rwkvtts.SharedRwkvRuntime(blob, max_slots=per, token_chunk_size=512) for _ in range(L)]
    outs = [None] * L

    def work(j):
        outs[j] = rts[j].generate_batch(reqs(per, j * per))
    for rep in range(2):
        ths = [threading.Thread(target=work, args=(j,)) for j in range(L)]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt = time.perf_counter() - t0
    n = sum(len(s) for o in outs for _, s in o)
    print(f"lanes={L}: {dt*1e3:.1f} ms for {n} semantic tokens -> {n*320/dt/1e6:.2f} M samples/s", flush=True)
    for r in rts:
        r.close()
