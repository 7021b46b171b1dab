"""Pins the oracle RNG: ChaCha block function against published known-answer vectors, then the
rand 0.8 StdRng consumption order (CPU-only)."""
import struct


def test_chacha20_rfc8439_2_3_2(oracle_mod):
    # RFC 8439 §2.3.2: key 00..1f, counter 1, nonce 00:00:00:09:00:00:00:4a:00:00:00:00
    words = [0x61707865, 0x3320646e, 0x79622d32, 0x6b206574, *struct.unpack("<8I", bytes(range(32))),
             1, 0x09000000, 0x4a000000, 0]
    out = oracle_mod.chacha_block_raw(words, 20)
    assert out == [0xe4e7f110, 0x15593bd1, 0x1fdd0f50, 0xc47120a3, 0xc7f4d1c7, 0x0368c033, 0x9aaa2204,
                   0x4e6cd4c3, 0x466482d2, 0x09aa9f07, 0x05d7c214, 0xa2028bd9, 0xd19c12b5, 0xb94e16de,
                   0xe883d0cb, 0x4e3c50a2]


def _stream(key, rounds):
    return bytes(struct.pack("<16I", *__import__("oracle").chacha_block(key, 0, 0, rounds))).hex()


def test_chacha_zero_key_vectors(oracle_mod):
    # RFC 8439 A.1 #1 (20 rounds) and the 8/12-round all-zero-key vectors
    # (draft-strombergson-chacha-test-vectors TC1); rand_chacha's own test_chacha_true_values_a
    # uses the 20-round one (first word 0xade0b876).
    z = [0] * 8
    assert _stream(z, 20).startswith("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7")
    assert _stream(z, 12).startswith("9bf49a6a0755f953811fce125f2683d50429c3bb49e074147e0089a52eae155f")
    assert _stream(z, 8).startswith("3e00ef2f895f40d67f5bb8e81f09a5a12c840ec3ce9a7f3b181be188ef711a1e")


def test_stdrng_linear_consumption(oracle_mod):
    r = oracle_mod.Rng(1042)
    key = r.key
    words = oracle_mod.chacha_block(key, 0) + oracle_mod.chacha_block(key, 1)
    assert [r.next_u32() for _ in range(32)] == words
    r2 = oracle_mod.Rng(1042)
    f = r2.gen_f32()
    assert f == (words[0] >> 8) * 2.0 ** -24


def test_pcg32_seed_fill(oracle_mod):
    # rand_core 0.6.4 seed_from_u64: PCG32 steps, output xorshift+rotate (independent python restatement)
    def pcg_key(s):
        out = []
        for _ in range(8):
            s = (s * 6364136223846793005 + 11634580456473284103) & (2**64 - 1)
            xs = (((s >> 18) ^ s) >> 27) & 0xFFFFFFFF
            rot = s >> 59
            out.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF)
        return out
    for seed in (0, 42, 1000, 2**64 - 1):
        assert oracle_mod.Rng(seed).key == pcg_key(seed)
