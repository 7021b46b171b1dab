"""Packed weight layout: C++ generator == independent numpy generator; header round-trip;
checkpoint packer transposes LoRA matrices (CPU-only)."""
import numpy as np

from rwkvtts import weights as W


def test_synth_c_equals_numpy():
    a = W.synth_blob(W.DIMS_TINY, seed=5)
    b = W.synth_blob_numpy(W.DIMS_TINY, seed=5)
    assert a.nbytes == b.nbytes == W.blob_bytes(W.DIMS_TINY)
    assert np.array_equal(a, b)


def test_pack_checkpoint_roundtrip():
    d = W.DIMS_TINY
    blob = W.synth_blob_numpy(d, seed=3)
    ents, _ = W.layout(d)
    names = {W.L_W1T: "att.w1", W.L_W2T: "att.w2", W.L_WR: "att.receptance.weight", W.L_FFN_K: "ffn.key.weight"}
    # rebuild a state dict from the blob, then pack it again
    gnames = {W.G_EMB: "emb.weight", W.G_LN0_W: "blocks.0.ln0.weight", W.G_LN0_B: "blocks.0.ln0.bias",
              W.G_LNOUT_W: "ln_out.weight", W.G_LNOUT_B: "ln_out.bias", W.G_HEAD: "head.weight"}
    lnames = {W.L_LN1_W: "ln1.weight", W.L_LN1_B: "ln1.bias", W.L_LN2_W: "ln2.weight", W.L_LN2_B: "ln2.bias",
              W.L_XR: "att.x_r", W.L_XW: "att.x_w", W.L_XK: "att.x_k", W.L_XV: "att.x_v", W.L_XA: "att.x_a",
              W.L_XG: "att.x_g", W.L_W0: "att.w0", W.L_A0: "att.a0", W.L_V0: "att.v0", W.L_KK: "att.k_k",
              W.L_KA: "att.k_a", W.L_RK: "att.r_k", W.L_LNX_W: "att.ln_x.weight", W.L_LNX_B: "att.ln_x.bias",
              W.L_FFN_XK: "ffn.x_k", W.L_WR: "att.receptance.weight", W.L_WK: "att.key.weight",
              W.L_WV: "att.value.weight", W.L_WO: "att.output.weight", W.L_W1T: "att.w1", W.L_A1T: "att.a1",
              W.L_V1T: "att.v1", W.L_G1T: "att.g1", W.L_W2T: "att.w2", W.L_A2T: "att.a2", W.L_V2T: "att.v2",
              W.L_G2T: "att.g2", W.L_FFN_K: "ffn.key.weight", W.L_FFN_V: "ffn.value.weight"}
    sd = {}
    for layer, t, off, r, c, m in ents:
        if m:
            a = W.bf16_bits_to_f32(blob[off:off + 2 * r * c].view(np.uint16)).reshape(r, c)
        else:
            a = blob[off:off + 4 * r * c].view(np.float32).reshape(r, c)
        if layer < 0:
            sd[gnames[t]] = a.copy()
        else:
            if layer == 0 and t in (W.L_V0, W.L_V1T, W.L_V2T):
                continue
            if t in (W.L_W1T, W.L_A1T, W.L_V1T, W.L_G1T, W.L_W2T, W.L_A2T, W.L_V2T, W.L_G2T):
                a = a.T  # checkpoint orientation ([C, D] / [D, C])
            sd[f"blocks.{layer}.{lnames[t]}"] = a.copy()
    assert sd["blocks.1.att.w1"].shape == (d["n_embd"], d["d_decay"])
    packed = W.pack_checkpoint(sd, d)
    assert np.array_equal(packed, blob)
