"""The certified sampler's tight bound on the sequential f32 softmax sum (csrc/sampler.hip,
advance_prep): S = e_0 + e_1 + ... formed left to right in f32 (rwkv_sampler.rs: probs.iter().sum())
satisfies |S - E| <= B = sum_{i>=1} 2^(floor(log2(P_i (1 + eps0))) - 24) with P_i the real prefix
sums, E their total and eps0 = n 2^-23 the crude bound. Checked here on the host (numpy f64 for the
real sums) over row shapes the sampler sees: near-uniform, peaked, wide dynamic range, ties and
values near binade boundaries."""
import numpy as np


def seq_sum_f32(e):
    s = np.float32(0.0)
    for v in e:
        s = np.float32(s + v)
    return float(s)


def tight_bound(e):
    n = len(e)
    eps0 = n * 2.0 ** -23 + 2.0 ** -36
    P = np.cumsum(e.astype(np.float64))
    up = P[1:] * (1.0 + eps0 + 2.0 ** -30)
    k = np.maximum(np.floor(np.log2(up)), -126)
    return float(np.sum(2.0 ** (k - 24))), float(P[-1]), eps0


def rows():
    rs = np.random.RandomState(7)
    for n in (64, 1000, 4096, 8193):
        for sd in (0.3, 1.6, 4.0, 12.0):
            lg = (rs.randn(n) * sd).astype(np.float32)
            yield np.exp((lg - lg.max()).astype(np.float64)).astype(np.float32)
    yield np.ones(8193, np.float32)                            # every addition at a binade edge
    yield np.full(8193, np.float32(1.0 - 2.0 ** -24))           # just below
    yield (1.0 + rs.randint(0, 3, 4096) * 2.0 ** -23).astype(np.float32)  # half-ulp ties
    e = np.zeros(8193, np.float32)
    e[rs.randint(0, 8193, 5)] = 1.0
    yield e                                                     # one-hot-ish (peaked)
    yield (2.0 ** rs.uniform(-140, 0, 8193)).astype(np.float32)  # subnormal prefixes


def test_tight_bound_holds_and_beats_crude():
    ratios = []
    for e in rows():
        S = seq_sum_f32(e)
        B, E, eps0 = tight_bound(e)
        assert abs(S - E) <= B, (len(e), S, E, B)
        ratios.append(B / (eps0 * E))
    # the point of the bound: typically several times tighter than n 2^-23 E
    assert np.median(ratios) < 0.35
