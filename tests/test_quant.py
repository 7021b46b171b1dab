"""CPU checks of the quantisation config (bin/server.rs:1029-1071 parse_quant_type /
create_quant_config) and of the oracle's Int8 / NF4 restatement (oracle/rwkv7.c)."""
import numpy as np
import pytest

from rwkvtts import _ffi, runtime
from rwkvtts import weights as W


def test_parse_quant_type():
    assert runtime.parse_quant_type("none") == _ffi.QUANT_NONE
    assert runtime.parse_quant_type("INT8") == _ffi.QUANT_INT8
    assert runtime.parse_quant_type("nf4") == _ffi.QUANT_NF4
    assert runtime.parse_quant_type("Sf4") == _ffi.QUANT_SF4
    with pytest.raises(ValueError):
        runtime.parse_quant_type("int4")


def test_quant_config():
    assert runtime.quant_config(0, "int8") == (0, _ffi.QUANT_NONE)    # quant_layers == 0 -> None
    assert runtime.quant_config(12, "none") == (0, _ffi.QUANT_NONE)
    assert runtime.quant_config(12, "nf4") == (12, _ffi.QUANT_NF4)


def _logits(om, toks):
    st = om.new_state()
    return np.stack([om.forward(st, t, 256) for t in toks])


def test_oracle_quantised_forward():
    import oracle
    blob = W.synth_blob(W.DIMS_TINY, seed=5)
    toks = [77823, 77838, 65530, 20000, 30000, 12345, 77828]
    full = _logits(oracle.Model(blob), toks)
    none = _logits(oracle.Model(blob, quant_layers=0, quant_type=1), toks)
    assert np.array_equal(full, none)
    q8 = _logits(oracle.Model(blob, quant_layers=2, quant_type=1), toks)
    q4 = _logits(oracle.Model(blob, quant_layers=2, quant_type=2), toks)
    q8_1 = _logits(oracle.Model(blob, quant_layers=1, quant_type=1), toks)
    e8, e4, e81 = (np.abs(x - full).max() for x in (q8, q4, q8_1))
    scale = np.abs(full).max()
    # int8 (256 levels per 128-block) is far closer to the 16-bit model than NF4 (16 levels per
    # 64-block); quantising fewer layers moves the logits less
    assert 0 < e8 < 0.05 * scale and e8 < e4 and e81 <= e8
    with pytest.raises(ValueError):
        oracle.Model(blob, quant_layers=2, quant_type=3)
