"""CPU restatement of the sampler's binade-run exact sum (csrc/sampler.hip, exact_seq_sum_runs):
the whole-range safety test, the segmented composition of parity maps across threads, the run table and the
walk, checked bit-exact against the sequential f32 sum (rwkv_sampler.rs:88) on softmax-like rows,
power-of-two rows (ties), sparse rows and short rows. This pins the ALGORITHM and its safety band;
the GPU kernel itself is checked against the oracle in tests/test_gpu_sampler.py."""
import struct

import numpy as np
import pytest

NO = 1 << 20
def f2b(x): return struct.unpack('<I', struct.pack('<f', x))[0]
def b2f(b): return struct.unpack('<f', struct.pack('<I', b))[0]
def d2b(x): return struct.unpack('<Q', struct.pack('<d', x))[0]
def comp(a, b):
    n0 = a[0] + (b[1] if a[0] & 1 else b[0]); n1 = a[1] + (b[1] if (1 + a[1]) & 1 else b[0])
    return (min(n0, 0x2000000), min(n1, 0x2000000))
def elem(b, E):
    ef = (b >> 23) & 0xFF; M = b & 0x7FFFFF
    if ef == 0: ex = -149
    else: M |= 0x800000; ex = ef - 150
    sh = (E - 23) - ex
    if M == 0 or sh > 25: return (0, 0)
    if sh <= 0: return (M << -sh, M << -sh)
    a = M >> sh; r = M & ((1 << sh) - 1); half = 1 << (sh - 1)
    if r > half: return (a + 1, a + 1)
    if r < half: return (a, a)
    return (a + (a & 1), a + ((a + 1) & 1))
def runs_sum(p, NT=512):
    """exact_seq_sum_runs: whole thread ranges inside one binade's safe band compose their maps,
    runs of such ranges with one binade are composed in order, everything else is added serially."""
    n = len(p); EMIN, NR = -100, 128
    rstart = [0] * NR; rend = [-1] * NR; rt = [(0, 0)] * NR
    lg = 0
    while (1 << lg) < n - 1: lg += 1
    DM = (1 << (52 - (23 - lg))) >> 32; DMAX = (1 << 20) - 2 * DM
    SUB = (n + NT - 1) // NT
    rng = [(min(n, t * SUB), min(n, min(n, t * SUB) + SUB)) for t in range(NT)]
    ds = [sum(float(p[i]) for i in range(b, e)) for b, e in rng]
    pre = np.concatenate([[0.0], np.cumsum(ds)])[:-1]
    tE, T = [], []
    for t, (b, e) in enumerate(rng):
        lw, hw = d2b(pre[t]) >> 32, d2b(pre[t] + ds[t]) >> 32
        E = (lw >> 20) - 1023
        safe = b < e and EMIN <= E <= EMIN + NR - 1 and (lw & 0xFFFFF) >= DM and \
            (hw >> 20) == (lw >> 20) and (hw & 0xFFFFF) < DMAX
        m = (0, 0)
        if safe:
            for i in range(b, e): m = comp(m, elem(f2b(float(p[i])), E))
        tE.append(E if safe else NO); T.append(m)
    carry, c = [], (0, 0)
    for t in range(NT):
        carry.append(c)
        contL = tE[t] != NO and t > 0 and tE[t - 1] == tE[t]
        c = comp(c, T[t]) if contL else T[t]
    for t, (b, e) in enumerate(rng):
        if tE[t] == NO: continue
        contL = t > 0 and tE[t - 1] == tE[t]
        contR = t + 1 < NT and tE[t + 1] == tE[t]
        if not contL: rstart[tE[t] - EMIN] = b
        if not contR:
            rend[tE[t] - EMIN] = e; rt[tE[t] - EMIN] = comp(carry[t], T[t]) if contL else T[t]
    s = np.float32(0); pos = 0; nser = 0; fails = 0; nruns = 0
    def ser(s, a, b):
        for i in range(a, b): s = np.float32(s + p[i])
        return s
    for k in range(NR):
        if rend[k] < 0: continue
        nruns += 1
        rs, re = rstart[k], rend[k]
        assert rs >= pos, (rs, pos)
        s = ser(s, pos, rs); nser += rs - pos
        sb = f2b(float(s)); ef = (sb >> 23) & 0xFF; mm = (sb & 0x7FFFFF) | 0x800000
        T_ = rt[k][1] if mm & 1 else rt[k][0]
        if ef != 0 and ef - 127 == k + EMIN and mm + T_ < 0x1000000:
            s = np.float32(b2f((sb & 0xFF800000) | ((mm + T_) & 0x7FFFFF)))
        else:
            fails += 1; s = ser(s, rs, re)
        pos = re
    s = ser(s, pos, n); nser += n - pos
    return s, nser, fails, nruns
def seq(p):
    s = np.float32(0)
    for x in p: s = np.float32(s + x)
    return s


@pytest.mark.parametrize("trial", range(8))
def test_runs_sum_bit_exact(trial):
    rs = np.random.RandomState(100 + trial)
    n = [8193, 4096, 1024, 100, 8193, 16384, 5, 8193][trial]
    if trial == 4:  # powers of two: ties at half an ulp everywhere
        p = (2.0 ** rs.randint(-30, 0, size=n)).astype(np.float32)
    elif trial == 7:  # sparse ones among zeros: prefixes exactly at powers of two
        p = np.zeros(n, np.float32)
        p[rs.randint(0, n, 50)] = 1.0
    else:
        lg = (rs.randn(n) * 1.6).astype(np.float32)
        p = np.exp(lg - lg.max()).astype(np.float32)
    got, nser, fails, nruns = runs_sum(p, NT=512)
    assert got == seq(p)
    assert fails == 0  # the safety band is never violated
    if trial in (0, 1, 5):
        assert nser < n // 10  # only the ranges holding a binade crossing are added one by one
