"""Per-phase breakdown of the device sampler (s_memrealtime stamps, 10 ns ticks, via rwkvtts_debug_sample)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rwkv-tts-rs_amd"))
import rwkvtts  # noqa: E402
from rwkvtts import _ffi, weights as W  # noqa: E402

rt = rwkvtts.SharedRwkvRuntime(W.synth_blob(W.DIMS_TINY), max_slots=2, token_chunk_size=64, use_graphs=False)
f = _ffi.lib().rwkvtts_debug_sample
f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_ffi.SampleArgs),
              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
names = ["load", "max+exp", "sum", "div", "topk", "compact", "topp", "temp", "multinomial"]
rs = np.random.RandomState(0)
for n, p, k in [(8193, 0.95, 80), (4096, 0.95, 20), (1024, 0.95, 80), (8193, 1.0, 0)]:
    rows = (rs.randn(32, n) * 1.6).astype(np.float32)
    out = np.zeros(32, np.int32)
    for rep in range(3):
        dbg = np.zeros(32 * 34, np.float32)
        args = _ffi.SampleArgs(1.0, p, k, -1)
        f(rt.handle, rows.ctypes.data_as(ctypes.c_void_p), 32, n, ctypes.byref(args), None,
          out.ctypes.data_as(ctypes.c_void_p), dbg.ctypes.data_as(ctypes.c_void_p))
    st = dbg[64:].view(np.uint64).reshape(32, 16)[:, :10].astype(np.int64)
    d = np.diff(st, axis=1).mean(axis=0)
    print(f"n={n} p={p} k={k}: total {st[:, 9].mean() - st[:, 0].mean():.0f} ticks ;",
          " ".join(f"{nm}={x:.0f}" for nm, x in zip(names, d)))
    s2 = dbg[64:].view(np.uint64).reshape(32, 16).astype(np.int64)
    print("   sum: scan", (s2[:, 10] - s2[:, 2]).mean(), "sim", (s2[:, 11] - s2[:, 10]).mean(), "compose",
          (s2[:, 12] - s2[:, 11]).mean(), "walk", (s2[:, 13] - s2[:, 12]).mean(), "walk-only", (s2[:, 14] - s2[:, 12]).mean(),
          "serial-add cycles", s2[:, 15].mean())
