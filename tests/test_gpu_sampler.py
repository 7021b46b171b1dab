"""GPU sampler (csrc/sampler.hip) vs the oracle restatement of src/rwkv_sampler.rs:55-211:
bit-exact token indices on identical logits and RNG streams."""
import numpy as np
import pytest

import rwkvtts
from rwkvtts import weights as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    blob = W.synth_blob(W.DIMS_TINY)
    r = rwkvtts.SharedRwkvRuntime(blob, max_slots=4, token_chunk_size=64, use_graphs=False)
    yield r
    r.close()


def _rows(kind, n, count, seed):
    rs = np.random.RandomState(seed)
    if kind == "normal":
        return (rs.randn(count, n) * rs.uniform(0.3, 4.0, size=(count, 1))).astype(np.float32)
    if kind == "peaky":
        x = rs.randn(count, n).astype(np.float32)
        x[np.arange(count), rs.randint(0, n, count)] += 12.0
        return x
    if kind == "ties":  # heavy ties: quantised logits
        return (np.round(rs.randn(count, n) * 2) / 2).astype(np.float32)
    if kind == "masked":  # semantic-style: tail masked to -inf
        x = rs.randn(count, n).astype(np.float32)
        x[:, 8193:] = -np.inf
        return x
    raise ValueError(kind)


CASES = [  # (n, temperature, top_p, top_k)
    (4096, 1.0, 0.95, 20),    # global phase (normal_mode_inference.rs:237-287)
    (8193, 1.0, 0.95, 80),    # semantic phase (:333-360)
    (8193, 1.0, 0.95, 1),     # greedy plumbing
    (8193, 1.0, 0.5, 80),
    (4096, 1.0, 1.0, 20),     # top-p disabled
    (1000, 1.0, 0.85, 0),     # SamplerArgs::default (top_k 0, top_p 0.85)
    (3000, 1.0, 0.3, 0),
    (16384, 1.0, 1.0, 0),     # plain multinomial over a long row
    (77923 // 8, 1.0, 0.9, 64),
    # candidate fast path (top-k <= 256, T = 1) edges and its fallbacks
    (8193, 1.0, 0.0, 80),     # top_p <= 0: survivors are the ties of the maximum
    (8193, 1.0, -1.0, 7),
    (4096, 1.0, 0.02, 256),   # largest fast k
    (4096, 1.0, 0.95, 257),   # first k past the fast path
    (300, 1.0, 0.95, 299),    # k = n - 1
    (17, 1.0, 0.9, 3),        # fewer elements than candidate threads
]


@pytest.mark.parametrize("kind", ["normal", "peaky", "ties"])
@pytest.mark.parametrize("case", CASES)
def test_sampler_bit_exact(rt, oracle_mod, kind, case):
    n, T, p, k = case
    rows = _rows(kind, n, 24, seed=n * 7 + k)
    seeds = [1000 + i * 17 for i in range(len(rows))]
    dev = rt.sample(rows, T, p, k, None, [rwkvtts.StdRng.seed_from_u64(s) for s in seeds])
    ref = [oracle_mod.sample(rows[i], T, p, k, None, oracle_mod.Rng(seeds[i])) for i in range(len(rows))]
    assert dev.tolist() == ref


def test_sampler_masked_full_vocab_equivalence(rt, oracle_mod):
    # semantic sampling sees the full 77923-wide vector with j > 8192 at -inf; the device samples the
    # 8193-row prefix: identical results
    rows = _rows("masked", 77923, 6, seed=3)
    seeds = list(range(6))
    dev = rt.sample(np.ascontiguousarray(rows[:, :8193]), 1.0, 0.95, 80, None,
                    [rwkvtts.StdRng.seed_from_u64(s) for s in seeds])
    ref = [oracle_mod.sample(rows[i], 1.0, 0.95, 80, None, oracle_mod.Rng(seeds[i])) for i in range(6)]
    assert dev.tolist() == ref


@pytest.mark.parametrize("kind", ["normal", "ties"])
@pytest.mark.parametrize("case", [(77923, 1.0, 0.85, 0),     # SamplerArgs::default on the full vocabulary
                                  (77923, 1.0, 0.95, 80),
                                  (20000, 1.0, 0.3, 5000),   # top-k past the LDS candidate path
                                  (77923, 1.0, 1.0, 0)])
def test_sampler_full_vocab_rows(rt, oracle_mod, kind, case):
    """Rows longer than the LDS row (16384) run from a device scratch: bit-exact for every
    top-k / top-p combination, including top-p without top-k over ~10^4 positive candidates."""
    n, T, p, k = case
    rows = _rows(kind, n, 4, seed=n + k)
    seeds = [77 + i for i in range(len(rows))]
    dev = rt.sample(rows, T, p, k, None, [rwkvtts.StdRng.seed_from_u64(s) for s in seeds])
    ref = [oracle_mod.sample(rows[i], T, p, k, None, oracle_mod.Rng(seeds[i])) for i in range(len(rows))]
    assert dev.tolist() == ref


def test_sampler_rng_stream_advances(rt, oracle_mod):
    rows = _rows("normal", 4096, 1, seed=11)[0]
    dr = rwkvtts.StdRng.seed_from_u64(1042)
    orng = oracle_mod.Rng(1042)
    for step in range(40):  # crosses ChaCha block boundaries (16 draws / block)
        d = rwkvtts.sample_logits_with_top_p_k(rt, rows, 1.0, 0.95, 20, None, dr)
        o = oracle_mod.sample(rows, 1.0, 0.95, 20, None, orng)
        assert d == o, step
    assert dr.draw_index == 40


def test_sampler_no_rng_and_forbid(rt, oracle_mod):
    rows = _rows("normal", 2048, 8, seed=5)
    for forbid in (None, 0, 17):
        dev = rt.sample(rows, 1.0, 0.9, 40, forbid, None)
        ref = [oracle_mod.sample(rows[i], 1.0, 0.9, 40, forbid, None) for i in range(len(rows))]
        assert dev.tolist() == ref


def test_sampler_temperature(rt, oracle_mod):
    # temperature != 1 is off the reference's live path (phases hard-code T=1, B2); the device powf
    # is double-precision, so parity is token-level with rare last-ulp differences allowed.
    rows = _rows("normal", 4096, 32, seed=9)
    seeds = list(range(32))
    dev = rt.sample(rows, 0.7, 0.95, 50, None, [rwkvtts.StdRng.seed_from_u64(s) for s in seeds])
    ref = [oracle_mod.sample(rows[i], 0.7, 0.95, 50, None, oracle_mod.Rng(seeds[i])) for i in range(32)]
    assert sum(int(a != b) for a, b in zip(dev.tolist(), ref)) <= 1


def _debug_sums(rt, rows, T=1.0, p=0.95, k=80):
    import ctypes
    from rwkvtts import _ffi
    L = _ffi.lib()
    f = L.rwkvtts_debug_sample
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_ffi.SampleArgs),
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    out = np.zeros(len(rows), np.int32)
    dbg = np.zeros(len(rows) * 34, np.float32)  # (sum, r) per row + 16 uint64 stamps per row
    args = _ffi.SampleArgs(T, p, k, -1)
    rc = f(rt.handle, rows.ctypes.data_as(ctypes.c_void_p), len(rows), rows.shape[1], ctypes.byref(args), None,
           out.ctypes.data_as(ctypes.c_void_p), dbg.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out, dbg[:2 * len(rows)].reshape(len(rows), 2)


@pytest.mark.parametrize("n", [17, 64, 1000, 4096, 8193, 16384])
def test_softmax_sum_bit_exact(rt, oracle_mod, n):
    """The parallel emulation of the sequential f32 softmax denominator (sampler.hip
    exact_seq_sum) equals the oracle's left-to-right sum bit for bit, including rows built to
    stress ties at half-ulp, binade crossings, subnormal terms and wide dynamic range."""
    rs = np.random.RandomState(n)
    rows = [rs.randn(n) * s for s in (0.05, 0.6, 1.6, 4.0, 12.0, 40.0)]
    rows.append(np.round(rs.randn(n) * 8) / 8)              # exact binary fractions -> many ties
    rows.append(np.where(rs.rand(n) < 0.5, 0.0, -np.log(2.0) * rs.randint(1, 30, n)))  # powers of two
    x = rs.randn(n) * 2
    x[rs.rand(n) < 0.3] = -np.inf
    rows.append(x)
    rows.append(np.linspace(0, -110, n))                     # down to subnormal/zero exp
    rows.append(np.zeros(n))                                 # all equal: sum == n exactly
    rows = np.stack(rows).astype(np.float32)
    tok, dbg = _debug_sums(rt, rows)
    for i, row in enumerate(rows):
        o_idx, o_sum, _ = oracle_mod.sample(row, 1.0, 0.95, 80, None, None, debug=True)
        assert np.float32(dbg[i, 0]).view(np.uint32) == np.float32(o_sum).view(np.uint32), (i, dbg[i, 0], o_sum)
        assert tok[i] == o_idx, i


@pytest.mark.parametrize("k,p", [(80, 0.95), (20, 0.95), (80, 1.0), (256, 0.5), (7, 0.999)])
def test_sampler_certified_path_sweep(rt, oracle_mod, k, p):
    """sample_cert (the token without the exact sequential sum whenever the decision holds for
    every S in the rigorous interval) against the oracle over many rows: near-uniform rows (the
    benchmark's regime: certified), mid-scale and peaked rows (the draw lands inside the kept mass,
    top-p cuts: the exact sum runs), rows whose k-th / (k+1)-th logits are 1 ulp apart or tied."""
    rs = np.random.RandomState(k * 1000 + int(p * 100))
    n = 8193
    rows = []
    for scale in (0.02, 0.2, 1.0, 3.0):
        rows.append((rs.randn(96, n) * scale).astype(np.float32))
    x = rs.randn(64, n).astype(np.float32)
    for i in range(64):  # the k-th and (k+1)-th largest 1 ulp apart (i even) or equal (i odd)
        order = np.argsort(-x[i], kind="stable")
        a, b = order[k - 1], order[k]
        x[i, b] = x[i, a] if i % 2 else np.nextafter(x[i, a], np.float32(-np.inf))
    rows.append(x)
    rows = np.concatenate(rows)
    seeds = [5 + 31 * i for i in range(len(rows))]
    dev = rt.sample(rows, 1.0, p, k, None, [rwkvtts.StdRng.seed_from_u64(s) for s in seeds])
    ref = [oracle_mod.sample(rows[i], 1.0, p, k, None, oracle_mod.Rng(seeds[i])) for i in range(len(rows))]
    assert dev.tolist() == ref
