// sampler.h -- device sampler (src/rwkv_sampler.rs:55-211) and the on-device phase controller
// (src/normal_mode_inference.rs:222-391, src/zero_shot_inference.rs:128-309).
#pragma once
#include "common.h"

namespace rwkvtts {

constexpr int kSampleMaxN = 16384;       // row length held in LDS (longer rows: global scratch)
constexpr int kSampleMaxSorted = 4096;   // survivors sortable for top-p in LDS
constexpr int kSampleMaxRowLen = 1 << 24;  // generic sampler API row limit

enum SlotPhase : int32_t { kPhGlobal = 0, kPhGFeed = 1, kPhSemantic = 2, kPhDone = 3 };

// Per-slot control block living in device memory.
struct SlotCtrl {
  int32_t mode;        // 0 normal, 1 zero-shot
  int32_t phase;       // SlotPhase
  int32_t n_global;
  int32_t n_sem;
  int32_t sem_limit;
  int32_t hard_min;    // zero-shot: EOS forbidden while n_sem < hard_min
  int32_t fixed;       // benchmark: EOS always masked
  int32_t top_k_g, top_k_s;
  int32_t next_token;  // token fed at the next step
  int32_t win_bits;    // zero-shot EOS window (bit i = non-EOS, newest at bit 0)
  int32_t win_len;
  int32_t status;
  int32_t pad0;
  uint32_t gkey[8];
  uint32_t skey[8];
  uint64_t gdraw;
  uint64_t sdraw;
  int32_t global_out[32];
  // ChaCha12 keystream block cache of each stream (k_advance): 16 consecutive draws share one
  // block, so 15 of 16 draws are a word read instead of a ChaCha12 block on the critical path.
  // *_blk_id = block index + 1 (0: empty -- the host zero-fills a new request's block)
  uint64_t gblk_id;
  uint64_t sblk_id;
  uint32_t gblk[16];
  uint32_t sblk[16];
};

struct SampleRowArgs {
  const float* logits;  // [rows][ld]
  int ld;
  int n;
  float temperature;
  float top_p;
  int top_k;
  int forbid;
  const uint32_t* keys;     // [rows][8] or null (-> StdRng(42), draw 0)
  const uint64_t* draws;    // [rows]
  int32_t* out;             // [rows]
  float* dbg;               // optional [rows][2]: softmax sum, r
  uint64_t* stamps;         // optional [rows][16]: s_memtime at phase boundaries (diagnostics)
  char* scratch;            // n > kSampleMaxN: [rows][scratch_stride] bytes (wide_scratch_bytes(n))
  size_t scratch_stride;
};

struct AdvanceArgs {
  const float* logits;   // [n_part][rows][ld] split-K partial logits (summed in order)
  int ld;
  int n_part;
  int64_t part_stride;
  const int* row_slot;   // step row -> slot (rows of this decode/prefill step with logits)
  SlotCtrl* ctrl;
  int32_t* sem_out;      // [S][2048]
  int n_rows;
  unsigned long long* tl;  // debug timeline slot (null in production)
  int cert;              // set by launch_advance: 1 certified fast path allowed (sample_cert)
  uint64_t* stamps;      // debug: [rows][16] s_memtime phase stamps (RWKVTTS_DEBUG_STAMPS adv=; null in production)
};

size_t wide_scratch_bytes(int n);
void launch_sample_rows(const SampleRowArgs& a, int rows, hipStream_t st);
// cert: 1 = the certified fast path allowed (the default), 0 = the exact walk always
int launch_advance(const AdvanceArgs& a, hipStream_t st, int cert = 1);

}  // namespace rwkvtts
