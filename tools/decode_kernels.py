"""The B=32 decode-step kernels of the 0.4B model as rocprofv3 sees them: bench profile name ->
(symbol prefixes, grid size). Shared by make_pmc_json.py and decode_kernel_summary.py."""

# (kernel symbol prefixes, grid size) of each decode-step launch at 32 rows (0.4B dims). Matched by
# prefix so template arguments appended later do not drop a kernel (round 3 lost both LayerNorm
# launches when k_ln1024 gained its EMB argument): the attention LayerNorm covers both the layer-0
# launch with the embedding folded in (EMB = true) and the other layers'.
DECODE = {
    "gemm_rkv_lora": (("k_gemm2<2, 8, 0, false, 1, 2, false>",), 54272),
    "gemm_ffn_key": (("k_gemm2<2, 8, 0, false, 1, 0, false>",), 65536),
    "gemm_wo": (("k_gemm2<2, 4, 0, false, 1, 0, false>",), 32768),
    "gemm_ffn_value": (("k_gemm2<2, 8, 1, false, 4, 0, false>",), 65536),
    "wkv": (("k_wkv6<false, false>", "k_wkv6<false>"), 131072),
    "ln_mix_att": (("k_ln1024<false, 1, 6, 16",), 8192),
    "ln_mix_ffn": (("k_ln1024<false, 1, 1, 8",), 8192),
    # the persistent decode launches: 32 LN + 212 rkv + 512 WKV + 128 Wo blocks and 32 LN + 256 key +
    # 256 value blocks of 256 threads
    "att_persist": (("k_att_persist<false,",), 884 * 256),
    "ffn_persist": (("k_ffn_persist<false",), 544 * 256),
}
# persistent attention launch grid (threads) -> rows of the decode step: 32 LN + 212 rkv + 16 R WKV +
# 128 Wo blocks (the tail form: 212 + 16 R + 128 + 32 LN2 blocks, the same count for layers > 0)
ATT_GRIDS = {(372 + 16 * r) * 256: r for r in range(1, 33)}


def match(acc, prefixes, grid):
    """All launches of symbols starting with one of `prefixes` at this grid size."""
    vals, syms = [], []
    for (name, g), v in acc.items():
        if g == grid and any(name.startswith(p) for p in prefixes):
            vals += v
            syms.append(name)
    return vals, sorted(set(syms))
