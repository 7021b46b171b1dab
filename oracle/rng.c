/* rng.c -- TEST INFRASTRUCTURE (see oracle.h).
 * Restates rand 0.8.5 StdRng (= rand_chacha 0.3.1 ChaCha12Rng) and rand_core 0.6.4
 * SeedableRng::seed_from_u64, as used by src/normal_mode_inference.rs:138-174 and
 * src/rwkv_sampler.rs:174-207 (Cargo.lock:2565-2609 pins). Published algorithms:
 *  - seed_from_u64: 8x PCG32 steps (MUL 6364136223846793005, INC 11634580456473284103),
 *    output xorshift/rotate, little-endian fill of the 32-byte seed;
 *  - ChaCha (djb layout): words 0-3 "expand 32-byte k", 4-11 key, 12-13 64-bit block counter,
 *    14-15 64-bit stream id (0 for from_seed); 12 rounds for StdRng; output block added to input;
 *  - BlockRng::next_u32 consumes block words linearly (block 0 w0..w15, block 1 ...);
 *  - Standard f32: (next_u32 >> 8) * 2^-24.
 */
#include <string.h>
#include "oracle.h"

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define QR(a, b, c, d)                 \
  a += b; d ^= a; d = rotl32(d, 16);   \
  c += d; b ^= c; b = rotl32(b, 12);   \
  a += b; d ^= a; d = rotl32(d, 8);    \
  c += d; b ^= c; b = rotl32(b, 7);

void oracle_chacha_block_raw(const uint32_t in[16], int rounds, uint32_t out[16]) {
  uint32_t x[16];
  memcpy(x, in, sizeof(x));
  for (int i = 0; i < rounds; i += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

void oracle_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds,
                         uint32_t out[16]) {
  uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; ++i) in[4 + i] = key[i];
  in[12] = (uint32_t)counter;
  in[13] = (uint32_t)(counter >> 32);
  in[14] = (uint32_t)stream;
  in[15] = (uint32_t)(stream >> 32);
  oracle_chacha_block_raw(in, rounds, out);
}

void oracle_rng_seed_from_u64(uint64_t state, oracle_rng* r) {
  const uint64_t MUL = 6364136223846793005ull, INC = 11634580456473284103ull;
  for (int i = 0; i < 8; ++i) {
    state = state * MUL + INC;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    uint32_t x = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    r->key[i] = x; /* to_le_bytes then read back as LE u32 = identity */
  }
  r->index = 0;
}

uint32_t oracle_rng_next_u32(oracle_rng* r) {
  uint32_t blk[16];
  oracle_chacha_block(r->key, r->index / 16, 0, 12, blk);
  uint32_t v = blk[r->index % 16];
  r->index++;
  return v;
}

float oracle_rng_gen_f32(oracle_rng* r) {
  uint32_t v = oracle_rng_next_u32(r) >> 8;
  return (float)v * (1.0f / 16777216.0f);
}
