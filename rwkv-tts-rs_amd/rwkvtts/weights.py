"""Weight blobs for the engine (include/rwkvtts.h layout).

* `synth_blob` -- deterministic synthetic RWKV-7 weights produced by the library's
  C++ generator (`rwkvtts_synth_weights`);
* `synth_blob_numpy` -- an independent numpy implementation of the same counter-based scheme,
  used by the tests to cross-check the packed layout;
* `pack_checkpoint` -- packs an upstream RWKV-7 x070 state dict (tensor names of SURVEY A.3,
  as web-rwkv's Loader reads them: src/shared_runtime.rs:109-123) into the blob.
"""
import ctypes

import numpy as np

from . import _ffi

# RWKV-TTS 0.4B (assumed dims): L=24 C=1024 N=64 F=4096 V=77923, LoRA 64/64/32/128
DIMS_04B = dict(n_layer=24, n_embd=1024, head_size=64, n_ffn=4096, n_vocab=77923,
                d_decay=64, d_aaa=64, d_mv=32, d_gate=128)
# tiny model for fast oracle comparisons (keeps the real vocabulary so prompt ids are valid)
DIMS_TINY = dict(n_layer=2, n_embd=128, head_size=64, n_ffn=512, n_vocab=77923,
                 d_decay=16, d_aaa=16, d_mv=16, d_gate=32)
DIMS_SMALL = dict(n_layer=4, n_embd=256, head_size=64, n_ffn=1024, n_vocab=77923,
                  d_decay=32, d_aaa=32, d_mv=16, d_gate=64)

# two layers at the full 0.4B widths: exercises the 0.4B-specialised decode kernels against the
# oracle at a cost the CPU restatement finishes in seconds
DIMS_MID = dict(n_layer=2, n_embd=1024, head_size=64, n_ffn=4096, n_vocab=77923,
                d_decay=64, d_aaa=64, d_mv=32, d_gate=128)

G_EMB, G_LN0_W, G_LN0_B, G_LNOUT_W, G_LNOUT_B, G_HEAD, G_COUNT = range(7)
(L_LN1_W, L_LN1_B, L_LN2_W, L_LN2_B, L_XR, L_XW, L_XK, L_XV, L_XA, L_XG, L_W0, L_A0, L_V0, L_KK,
 L_KA, L_RK, L_LNX_W, L_LNX_B, L_FFN_XK, L_WR, L_WK, L_WV, L_WO, L_W1T, L_A1T, L_V1T, L_G1T,
 L_W2T, L_A2T, L_V2T, L_G2T, L_FFN_K, L_FFN_V, L_COUNT) = range(34)
L_FIRST_MAT = L_WR


def make_dims(d):
    return _ffi.Dims(**d) if isinstance(d, dict) else d


def tensor_shape(d, layer, t):
    """(rows, cols, is_matrix) -- mirrors rwkvtts_tensor_shape."""
    C, V, F = d["n_embd"], d["n_vocab"], d["n_ffn"]
    if layer < 0:
        if t in (G_EMB, G_HEAD):
            return V, C, True
        return 1, C, False
    mats = {L_WR: (C, C), L_WK: (C, C), L_WV: (C, C), L_WO: (C, C),
            L_W1T: (d["d_decay"], C), L_A1T: (d["d_aaa"], C), L_V1T: (d["d_mv"], C),
            L_G1T: (d["d_gate"], C), L_W2T: (C, d["d_decay"]), L_A2T: (C, d["d_aaa"]),
            L_V2T: (C, d["d_mv"]), L_G2T: (C, d["d_gate"]), L_FFN_K: (F, C), L_FFN_V: (C, F)}
    if t in mats:
        return mats[t][0], mats[t][1], True
    return 1, C, False


def layout(d):
    """[(layer, t, offset, rows, cols, is_mat)], total bytes -- mirrors rwkvtts_tensor_offset."""
    off = 256
    out = []
    for layer in range(-1, d["n_layer"]):
        for t in range(G_COUNT if layer < 0 else L_COUNT):
            r, c, m = tensor_shape(d, layer, t)
            out.append((layer, t, off, r, c, m))
            nb = r * c * (2 if m else 4)
            off += (nb + 255) & ~255
    return out, off


def blob_bytes(d):
    return layout(d)[1]


def synth_blob(d, seed=20251205, dtype=_ffi.DTYPE_BF16):
    """Synthetic weights from the library's generator (uint8 numpy array)."""
    nb = blob_bytes(d)
    buf = np.empty(nb, dtype=np.uint8)
    _ffi.check(_ffi.lib().rwkvtts_synth_weights(ctypes.byref(make_dims(d)), dtype, seed,
                                                buf.ctypes.data_as(ctypes.c_void_p)), "synth_weights")
    return buf


# ---------------- independent numpy generator (test cross-check) ----------------
M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _normal(h):
    s = ((h & np.uint64(0xFFFF)).astype(np.float64) + ((h >> np.uint64(16)) & np.uint64(0xFFFF)).astype(np.float64)
         + ((h >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.float64) + (h >> np.uint64(48)).astype(np.float64))
    return (s / 65536.0 - 2.0) * 1.7320508075688772


def _uniform(h):
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _value(layer, t, h):
    if layer < 0:
        if t == G_EMB:
            return _normal(h) * 0.5
        if t == G_HEAD:
            return _normal(h) * 0.05
        if t in (G_LN0_W, G_LNOUT_W):
            return 1.0 + 0.1 * _normal(h)
        return 0.02 * _normal(h)
    if t in (L_LN1_W, L_LN2_W):
        return 1.0 + 0.1 * _normal(h)
    if t in (L_LN1_B, L_LN2_B, L_LNX_B):
        return 0.02 * _normal(h)
    if t in (L_XR, L_XW, L_XK, L_XV, L_XA, L_XG, L_FFN_XK):
        return _uniform(h)
    if t == L_W0:
        return -4.0 + 6.0 * _uniform(h)
    if t in (L_A0, L_V0):
        return -1.0 + 2.0 * _uniform(h)
    if t in (L_KK, L_KA):
        return 0.5 + 0.5 * _uniform(h)
    if t == L_RK:
        return 0.1 * _normal(h)
    if t == L_LNX_W:
        return 0.5 + 0.5 * _uniform(h)
    return 0.02 * _normal(h)


def f32_to_bf16_bits(x):
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)
    return u.astype(np.uint16)


def bf16_bits_to_f32(b):
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << np.uint32(16)).view(np.float32)


def header(d, dtype):
    """256-byte rwkvtts_blob_header."""
    hdr = np.zeros(64, dtype=np.int32)
    hdr.view(np.uint32)[0] = 0x37545752
    hdr[1] = 1
    hdr[2] = dtype
    names = ["n_layer", "n_embd", "head_size", "n_ffn", "n_vocab", "d_decay", "d_aaa", "d_mv", "d_gate"]
    for i, n in enumerate(names):
        hdr[4 + i] = d[n]
    return hdr.view(np.uint8)


def synth_blob_numpy(d, seed=20251205):
    """bf16 blob, bit-identical to rwkvtts_synth_weights(dtype=BF16)."""
    ents, nb = layout(d)
    buf = np.zeros(nb, dtype=np.uint8)
    buf[:256] = header(d, _ffi.DTYPE_BF16)
    for layer, t, off, r, c, m in ents:
        tid = np.uint64((layer + 1) * 64 + t + 1)
        with np.errstate(over="ignore"):
            key = _splitmix64(np.uint64(seed) ^ (np.uint64(0xD1B54A32D192ED03) * tid))
        n = r * c
        zero_v = layer == 0 and t in (L_V0, L_V1T, L_V2T)
        idx = np.arange(n, dtype=np.uint64)
        vals = np.zeros(n) if zero_v else _value(layer, t, _splitmix64(key ^ idx))
        f = vals.astype(np.float32)
        if m:
            buf[off:off + 2 * n] = f32_to_bf16_bits(f).view(np.uint8)
        else:
            buf[off:off + 4 * n] = f.view(np.uint8)
    return buf


# ---------------- real checkpoints ----------------
def pack_checkpoint(sd, d, dtype=_ffi.DTYPE_BF16):
    """Pack an RWKV-7 x070 state dict (numpy arrays, upstream names -- SURVEY A.3) into a blob.
    LoRA matrices are transposed so every projection reads [out][in] rows."""
    ents, nb = layout(d)
    buf = np.zeros(nb, dtype=np.uint8)
    buf[:256] = header(d, dtype)
    gmap = {G_EMB: "emb.weight", G_LN0_W: "blocks.0.ln0.weight", G_LN0_B: "blocks.0.ln0.bias",
            G_LNOUT_W: "ln_out.weight", G_LNOUT_B: "ln_out.bias", G_HEAD: "head.weight"}
    lmap = {L_LN1_W: ("ln1.weight", None), L_LN1_B: ("ln1.bias", None), L_LN2_W: ("ln2.weight", None),
            L_LN2_B: ("ln2.bias", None), L_XR: ("att.x_r", None), L_XW: ("att.x_w", None),
            L_XK: ("att.x_k", None), L_XV: ("att.x_v", None), L_XA: ("att.x_a", None),
            L_XG: ("att.x_g", None), L_W0: ("att.w0", None), L_A0: ("att.a0", None),
            L_V0: ("att.v0", None), L_KK: ("att.k_k", None), L_KA: ("att.k_a", None),
            L_RK: ("att.r_k", None), L_LNX_W: ("att.ln_x.weight", None), L_LNX_B: ("att.ln_x.bias", None),
            L_FFN_XK: ("ffn.x_k", None), L_WR: ("att.receptance.weight", None),
            L_WK: ("att.key.weight", None), L_WV: ("att.value.weight", None),
            L_WO: ("att.output.weight", None), L_W1T: ("att.w1", "T"), L_A1T: ("att.a1", "T"),
            L_V1T: ("att.v1", "T"), L_G1T: ("att.g1", "T"), L_W2T: ("att.w2", "T"),
            L_A2T: ("att.a2", "T"), L_V2T: ("att.v2", "T"), L_G2T: ("att.g2", "T"),
            L_FFN_K: ("ffn.key.weight", None), L_FFN_V: ("ffn.value.weight", None)}
    for layer, t, off, r, c, m in ents:
        if layer < 0:
            name, tr = gmap[t], None
        else:
            nm, tr = lmap[t]
            name = f"blocks.{layer}.{nm}"
        if name not in sd:
            if layer == 0 and t in (L_V0, L_V1T, L_V2T):
                continue  # layer 0 has no value-residual LoRA
            raise KeyError(name)
        a = np.asarray(sd[name], dtype=np.float32)
        if tr == "T":
            a = a.T
        a = np.ascontiguousarray(a.reshape(r, c))
        if m:
            bits = f32_to_bf16_bits(a) if dtype == _ffi.DTYPE_BF16 else a.astype(np.float16).view(np.uint16)
            buf[off:off + 2 * r * c] = bits.reshape(-1).view(np.uint8)
        else:
            buf[off:off + 4 * r * c] = a.reshape(-1).view(np.uint8)
    return buf
