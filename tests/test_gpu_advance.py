"""The production decode-step sampler k_advance (csrc/sampler.hip: advance_prep -- candidates
collected from registers, the tight per-addition softmax-sum bound, ChaCha12 blocks cached in
the slot control block -- feeding the prepped sample_block and its certified fast path) on
adversarial synthetic logit rows, token-for-token against the oracle restatement of
src/rwkv_sampler.rs:55-211 and the phase rules of normal_mode_inference.rs:237-391 /
zero_shot_inference.rs:256-309 (the rows the end-to-end streams never produce).

Rows: near-uniform (the bench's random-weight logits), wide, peaked (top-p cut active),
k-th / (k+1)-th largest logits tied and 1 ulp apart, heavy exact ties, EOS-dominated rows (stop,
zero-shot re-draw with EOS masked, window rule), at top_k 20 and 80, with draw indices that cross
16-word ChaCha blocks over 20 consecutive launches (the cached block path). Every case runs with
the certified fast path allowed and with the exact walk forced; both must equal the oracle."""
import ctypes

import numpy as np
import pytest

import rwkvtts
from rwkvtts import _ffi
from rwkvtts import weights as W

pytestmark = pytest.mark.gpu
EOS = 8192
LD = EOS + 1
STEPS = 20


class Row(ctypes.Structure):  # engine.h DebugAdvanceRow
    _fields_ = [("mode", ctypes.c_int32), ("phase", ctypes.c_int32), ("top_k", ctypes.c_int32),
                ("fixed", ctypes.c_int32), ("n_sem", ctypes.c_int32), ("hard_min", ctypes.c_int32),
                ("win_bits", ctypes.c_int32), ("win_len", ctypes.c_int32), ("key", ctypes.c_uint32 * 8),
                ("draw", ctypes.c_uint64)]


assert ctypes.sizeof(Row) == 72


@pytest.fixture(scope="module")
def rt():
    blob = W.synth_blob(W.DIMS_TINY)
    r = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=64, use_graphs=False)
    yield r
    r.close()


def _gpu(rt, logits, rows, exact):
    f = _ffi.lib().rwkvtts_debug_advance  # argtypes from _ffi.EXPORTS
    n = len(rows)
    arr = (Row * n)(*rows)
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    assert lg.shape == (n, LD)
    tok, used, ph = (np.zeros((STEPS, n), np.int32) for _ in range(3))
    rc = f(rt.handle, lg.ctypes.data_as(ctypes.c_void_p), n, ctypes.cast(arr, ctypes.c_void_p), int(exact), STEPS,
           tok.ctypes.data_as(ctypes.c_void_p), used.ctypes.data_as(ctypes.c_void_p), ph.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, _ffi.lib().rwkvtts_last_error()
    return tok, used, ph


def _rng_at(oracle_mod, seed, draw):
    r = oracle_mod.Rng(seed)
    for _ in range(draw):
        r.gen_f32()
    return r


def _reference(oracle_mod, row_logits, c):
    """The oracle's tokens / draws / phases for STEPS launches of one row (same logits each time)."""
    toks, useds, phases = [], [], []
    phase, n_sem, bits, wl, draw, nglob = c["phase"], c["n_sem"], c["win_bits"], c["win_len"], c["draw"], 0
    rng = _rng_at(oracle_mod, c["seed"], draw)
    for _ in range(STEPS):
        if phase == 3:
            toks.append(-1); useds.append(0); phases.append(3)
            continue
        if phase == 0:
            t = oracle_mod.sample(row_logits[:4096], 1.0, 0.95, c["top_k"], None, rng)
            nglob += 1
            if nglob == 32:
                phase = 1
            toks.append(t); useds.append(1); phases.append(phase)
            continue
        lg = row_logits[:LD].copy()
        if c["fixed"] or (c["mode"] == 1 and n_sem < c["hard_min"]):
            lg[EOS] = -np.inf
        t = oracle_mod.sample(lg, 1.0, 0.95, c["top_k"], None, rng)
        used, stop = 1, False
        if t == EOS:
            if c["mode"] == 0:
                stop = True
            else:
                non_eos = bin(bits & ((1 << wl) - 1)).count("1")
                ratio = np.float32(non_eos) / np.float32(wl) if wl > 0 else np.float32(0)
                if wl >= 12 and ratio >= np.float32(0.7):
                    stop = True
                else:
                    lg[EOS] = -np.inf
                    t = oracle_mod.sample(lg, 1.0, 0.95, c["top_k"], None, rng)
                    used = 2
        if stop:
            phase = 3
            toks.append(-1); useds.append(used); phases.append(3)
            continue
        if c["mode"] == 1:
            bits = ((bits << 1) | (1 if t != EOS else 0)) & 0xFFF
            wl = min(12, wl + 1)
        n_sem += 1
        toks.append(t); useds.append(used); phases.append(phase)
    return toks, useds, phases


def _kth_tied(rs, k, ulps):
    """Near-uniform row whose k-th and (k+1)-th largest logits (over the first 4096 and over all
    8193) are equal (ulps = 0) or `ulps` ulps apart."""
    x = (rs.randn(LD) * 0.5).astype(np.float32)
    for n in (4096, LD):
        order = np.argsort(-x[:n], kind="stable")
        a, b = order[k - 1], order[k]
        v = x[a]
        x[b] = v if ulps == 0 else np.nextafter(v, np.float32(-np.inf), dtype=np.float32)
        for _ in range(ulps - 1):
            x[b] = np.nextafter(x[b], np.float32(-np.inf), dtype=np.float32)
    return x


def _row_kinds(rs, k):
    out = {}
    out["near_uniform"] = (rs.randn(LD) * 0.3).astype(np.float32)
    out["wide"] = (rs.randn(LD) * 4.0).astype(np.float32)
    p = rs.randn(LD).astype(np.float32)
    p[rs.randint(0, 4096, 3)] += np.float32([9.0, 7.5, 6.0])  # top-p cut inside the top-k
    out["peaked"] = p
    out["kth_tied"] = _kth_tied(rs, k, 0)
    out["kth_1ulp"] = _kth_tied(rs, k, 1)
    out["quantised_ties"] = (np.round(rs.randn(LD) * 4) / 4).astype(np.float32)
    e = (rs.randn(LD) * 0.5).astype(np.float32)
    e[EOS] = 6.0  # EOS carries most of the mass
    out["eos_heavy"] = e
    e2 = (rs.randn(LD) * 0.5).astype(np.float32)
    e2[EOS] = 3.5  # EOS drawn on some steps only
    out["eos_some"] = e2
    return out


def _cases(oracle_mod, top_k):
    rs = np.random.RandomState(1000 + top_k)
    logits, rows, meta = [], [], []
    draws = (0, 15, 16, 31, 1007)
    i = 0
    for kind, x in _row_kinds(rs, top_k).items():
        configs = [
            dict(mode=0, phase=0, fixed=0, n_sem=0, hard_min=0, win_bits=0, win_len=0),     # global phase
            dict(mode=0, phase=2, fixed=0, n_sem=0, hard_min=0, win_bits=0, win_len=0),     # semantic, EOS stops
            dict(mode=0, phase=2, fixed=1, n_sem=5, hard_min=0, win_bits=0, win_len=0),     # bench: EOS masked
            dict(mode=1, phase=2, fixed=0, n_sem=3, hard_min=10, win_bits=0, win_len=0),    # zero-shot below hard_min
            dict(mode=1, phase=2, fixed=0, n_sem=40, hard_min=10, win_bits=0xFFF, win_len=12),  # window may stop
            dict(mode=1, phase=2, fixed=0, n_sem=40, hard_min=10, win_bits=0x0FF, win_len=12),  # ratio 8/12 < 0.7: re-draw
            dict(mode=1, phase=2, fixed=0, n_sem=40, hard_min=10, win_bits=0x1F, win_len=5),    # short window: re-draw
        ]
        for c in configs:
            seed = 7919 * (i + 1) + top_k
            c = dict(c, top_k=top_k, seed=seed, draw=draws[i % len(draws)], kind=kind)
            key = oracle_mod.Rng(seed).key
            rows.append(Row(c["mode"], c["phase"], top_k, c["fixed"], c["n_sem"], c["hard_min"], c["win_bits"],
                            c["win_len"], (ctypes.c_uint32 * 8)(*key), c["draw"]))
            logits.append(x)
            meta.append(c)
            i += 1
    return np.stack(logits), rows, meta


@pytest.mark.parametrize("top_k", [20, 80])
@pytest.mark.parametrize("exact", [0, 1])
def test_advance_adversarial_rows_vs_oracle(rt, oracle_mod, top_k, exact):
    logits, rows, meta = _cases(oracle_mod, top_k)
    tok, used, ph = _gpu(rt, logits, rows, exact)
    bad = []
    for i, c in enumerate(meta):
        rt_, ru, rp = _reference(oracle_mod, logits[i], c)
        if list(tok[:, i]) != rt_ or list(used[:, i]) != ru or list(ph[:, i]) != rp:
            bad.append((c["kind"], {k: c[k] for k in ("mode", "phase", "fixed", "n_sem", "win_bits", "draw")},
                        list(tok[:, i]), rt_))
    assert not bad, bad[:3]
    # the cases reach every branch: stops, re-draws (2 draws in one step) and emitted tokens
    assert (ph == 3).any() and (used == 2).any() and (tok >= 0).sum() > len(meta) * STEPS // 2
