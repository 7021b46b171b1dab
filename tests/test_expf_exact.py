"""The expf the GPU sampler runs (csrc/exact_math.h) is bit-identical to glibc expf, which is what
Rust's f32::exp calls on Linux (src/rwkv_sampler.rs:83-87). CPU check of the same source via the
library's host hook; the exhaustive sweep over every float in [-104, 0] (1.12e9 values) was run
once with tools/expf_sweep.c and is repeated on a strided subset here."""
import ctypes

import numpy as np

from rwkvtts import _ffi


def test_expf_matches_glibc_strided(oracle_mod):
    L = _ffi.lib()
    f = L.rwkvtts_debug_expf
    f.argtypes = [ctypes.c_float]
    f.restype = ctypes.c_float
    libm = ctypes.CDLL("libm.so.6")
    libm.expf.argtypes = [ctypes.c_float]
    libm.expf.restype = ctypes.c_float
    # every 4099th float bit pattern from -0 down to -104, plus edge values
    bits = np.arange(0x80000000, 0xC2D00000, 4099, dtype=np.uint64).astype(np.uint32)
    xs = bits.view(np.float32)
    xs = np.concatenate([xs, np.float32([-0.0, 0.0, -1e-45, -87.33655, -103.97207, -104.0, -np.inf])])
    bad = [x for x in xs.tolist() if np.float32(f(x)).view(np.uint32) != np.float32(libm.expf(x)).view(np.uint32)]
    assert not bad, bad[:5]
