"""The C-ABI library loads and exports every symbol include/rwkvtts.h declares (CPU-only)."""
import os
import re

import rwkvtts
from rwkvtts import _ffi
from conftest import ROOT


def declared_functions():
    src = open(os.path.join(ROOT, "include", "rwkvtts.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"static inline[^{]*\{.*?\n\}", "", src, flags=re.S)
    return set(re.findall(r"\b(rwkvtts_[a-z0-9_]+)\s*\(", src)) - {
        "rwkvtts_tensor_shape", "rwkvtts_tensor_offset", "rwkvtts_blob_bytes"}


def test_header_symbols_exported():
    L = _ffi.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in sorted(names):
        assert hasattr(L, n), f"{n} declared in include/rwkvtts.h but not exported"
    assert names == set(_ffi.EXPORTS), "python binding out of sync with the header"


def test_errors_are_status_codes():
    import ctypes
    import numpy as np
    desc = _ffi.EngineDesc(0, 1, 16, 0)
    h = ctypes.c_void_p()
    bad = np.zeros(256, dtype=np.uint8)
    rc = _ffi.lib().rwkvtts_engine_create(ctypes.byref(desc), bad.ctypes.data_as(ctypes.c_void_p), 256, 0,
                                          ctypes.byref(h))
    assert rc != 0 and not h.value
    assert b"magic" in _ffi.lib().rwkvtts_last_error() or len(_ffi.lib().rwkvtts_last_error()) > 0


def test_rng_seed_matches_oracle(oracle_mod):
    for seed in (0, 1, 42, 1042, 2042, 2**63 + 5):
        assert rwkvtts.StdRng.seed_from_u64(seed).key == oracle_mod.Rng(seed).key
