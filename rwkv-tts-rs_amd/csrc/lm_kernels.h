// lm_kernels.h -- argument blocks and launchers of the RWKV-7 forward kernels.
#pragma once
#include <stddef.h>
#include <string.h>

#include "common.h"

namespace rwkvtts {

constexpr int kMaxPerThread = 8;     // C <= 2048 with 256-thread rows
constexpr int kMaxLoraTotal = 512;   // Dw + Da + Dv + Dg
constexpr int kMaxParts = 8;         // split-K slabs a WKV row sums (r, k, v, LoRA hidden)
constexpr int kRowFirst = 1;         // row flags
constexpr int kRowLast = 2;
constexpr int kRowCtrl = 4;          // the row's token is its slot's SlotCtrl::next_token (decode)
constexpr int kXPlanes = 0;  // gemm X: bf16 hi/lo planes
constexpr int kXRelu2 = 1;   // gemm X: relu(sum of f32 partial slabs)^2

struct LnMixArgs {
  const float* h_in;   // [R][C]
  float* h_out;        // nullable
  const float* part;   // [n_part][R][ldp]
  int n_part;
  int ldp;
  int64_t part_stride;
  const float* ln_w;
  const float* ln_b;
  int n_mix;
  const float* mu[6];
  bf16_t* x_hi;        // [n_mix][rows][ldx]
  bf16_t* x_lo;
  int64_t mix_stride;
  int ldx;
  float* shift;        // [2][S][L][C] or null (ln_out)
  int S, L, layer, C;
  const int4* rows;    // per row: slot, flags, prev_row, parity
  const int* row_map;  // output row -> source row (ln_out) or null
  int n_rows;          // set by the launcher
  int f16;             // planes in f16 (fp16 model) instead of bf16
  unsigned long long* tl;  // debug timeline slot (null in production)
  int wt;              // k_ln1024: write-through (sc1) plane / residual / shift stores
  int inplace;         // decode step (one row per slot): the shift update overwrites the parity it
                       // read (same thread, read before write) and the parity is not flipped
  // layer 0 of a decode step with the embedding fused in (emb != null: k_ln1024's EMB form): the
  // row's token (rows[r] flagged kRowCtrl: emb_ctrl[slot * emb_ctrl_stride], else emb_tok[r]),
  // its embedding row and LN0 (k_embed's arithmetic, bit for bit) replace the h_in load
  const uint32_t* emb_tok;
  const int* emb_ctrl;
  int emb_ctrl_stride;
  const bf16_t* emb;
  const float* ln0_w;
  const float* ln0_b;
  int n_vocab;
};

struct GemmSeg {
  const bf16_t* W;     // packed by launch_pack_frag (ceil(N/16) blocks of 16 x K)
  const bf16_t* Xhi;   // [rows][ldx]
  const bf16_t* Xlo;
  int ldx;
  int N;
  int col_off;         // output column offset
  int tile_start;      // first 64-column tile index of this segment
};

// NSEG_ segments and NTINFO_ tile descriptors (the arrays last)
template <int NSEG_, int NTINFO_>
struct GemmArgsT {
  int nseg;
  int K;
  int M;               // valid rows
  int k_split;
  int kslice;          // K / k_split in {128, 256, 512}
  int xmode;           // kXPlanes / kXRelu2
  const float* x_part; // kXRelu2: [x_nsplit][rows][x_ld] f32 partial slabs
  int x_nsplit;
  int x_ld;
  int64_t x_part_stride;
  float* out;          // [k_split][rows][ldo] f32
  int64_t split_stride;
  int ldo;
  uint64_t* stamps;    // debug: 4 s_memtime stamps per workgroup (null in production)
  int f16;             // weights and activation planes in f16 (fp16 model)
  unsigned long long* tl;  // debug timeline slot (null in production)
  // Multi-segment launches whose segments are packed back to back in 64-column tiles (set by
  // gemm_tile_table): tile t's weights at tw + t * 64 * K and one descriptor word per tile,
  // mix plane (bits 0-2) | valid columns (bits 3-9) | first output column (bits 10-31); X of
  // mix plane m at seg[0].Xhi / Xlo + m * x_mix_stride. Read by blockIdx alone, so the kernel
  // needs no dependent kernel-argument load to find its segment.
  int n_tinfo;         // 0: per-segment lookup
  const bf16_t* tw;
  int64_t x_mix_stride;
  // XCD-aware 1-D grid (set by the launcher for single-row-group launches): workgroups that
  // share a K-slice -- hence the same X slice / key slabs -- run on one XCD (blocks b and b + 8
  // share one), so each XCD's L2 fetches its slices' activations once instead of all eight
  // fetching every slice. xmap 0: grid (tiles, k_split, row groups).
  int xmap;
  int allow_xmap;      // set by the caller: this launch may use the XCD-aware grid
  int wt;              // k_gemm2: write-through (sc1) output stores (common.h store_wt)
  int ntiles;          // column tiles
  int tiles_per_xcd;   // k_split < 8: tiles of one split per XCD (ceil(ntiles * k_split / 8))
  // xmap 2 (consumer-aligned): every split of column tile t runs on XCD (t / xalign) % 8, the
  // XCD whose workgroups consume those columns next (the value GEMM's K-slice, the WKV head), so
  // the consumer reads the partial slabs from its own L2. Set xalign > 0 to request it.
  int xalign;
  // quantised weights (RWKVTTS_QUANT_INT8 / NF4): q_fmt != 0 -> the launch (MS 0) or its tiles
  // whose tinfo bit 31 is set (MS 2) read codes / scales (launch_quant_pack layout, column tiles
  // of 64 back to back) instead of 16-bit fragments, dequantise in registers and split the weight
  // into hi + lo 16-bit planes (three MFMAs per product: ~f32 dequantised weights)
  int q_fmt;
  const uint8_t* qw;
  const void* qs;
  // f16 models: the dequantised weights are split as w * 2^q_shift (brought up to ~2^14 at the
  // matrix's largest |w|) so that the lo half stays a normal f16 number; the product is scaled
  // back by 2^-q_shift in the epilogue (powers of two: exact)
  int q_shift;
  GemmSeg seg[NSEG_];
  uint32_t tinfo[NTINFO_];
};
using GemmArgs = GemmArgsT<8, 128>;
// a single-segment launch's arguments without the segment / descriptor tables (the roles of the
// one-launch-per-layer form, whose kernel arguments must stay under 4 KB)
using GemmArgs1 = GemmArgsT<1, 1>;
inline GemmArgs1 gemm_args1(const GemmArgs& a) {
  GemmArgs1 b;
  static_assert(offsetof(GemmArgs, seg) == offsetof(GemmArgs1, seg), "shared scalar layout");
  memcpy((void*)&b, (const void*)&a, offsetof(GemmArgs, seg));
  b.seg[0] = a.seg[0];
  b.tinfo[0] = 0;
  return b;
}

struct WkvArgs {
  const float* part;   // [n_part][R][ldp]
  int n_part;
  int ldp;
  int64_t part_stride;
  const bf16_t *w2t, *a2t, *v2t, *g2t;  // LoRA-up rows [C][D] (k_wkv1)
  const bf16_t* lup;   // LoRA-up rows packed for k_wkv (launch_pack_lora) or k_wkv4 (launch_pack_lora4)
  const float *w0, *a0, *v0, *k_k, *k_a, *r_k, *lnx_w, *lnx_b;
  float* state;
  int64_t slot_stride;
  int64_t layer_off;
  float* v_first;
  int ldv;
  bf16_t* z_hi;
  bf16_t* z_lo;
  int ldz;
  const int4* segs;    // slot, row_begin, n_rows, _
  int layer, C, Dw, Da, Dv, Dg;
  int n_slots;         // state slots (bounds the speculative slot = segment index)
  int n_seg;           // segments in this step 
  int perm;            // state block layout (wkv_perm_layout): 0 row-major, 1 k_wkv4, 2 k_wkv6
  int xmap;            // k_wkv4 / k_wkv6: 1-D grid, head h's workgroups on one XCD (H % 8 == 0)
  int allow_xmap;      // set by the caller
  int wt;              // k_wkv4 / k_wkv6: write-through (sc1) state stores
  int f16;             // fp16 model: LoRA-up rows and the z planes are f16
  uint64_t* stamps;    // debug: 8 s_memtime stamps per workgroup (null in production)
  int multi_row;       // some segment has > 1 row (prefill / mixed step): a separate kernel
                       // instantiation, so profiles separate decode launches from prefill ones
  unsigned long long* tl;  // debug timeline slot (null in production)
};

// tokens: per-row ids; a row flagged kRowCtrl (decode) reads ctrl_tok[rows[r].x * ctrl_stride]
void launch_embed(const uint32_t* tokens, const int4* rows, const int* ctrl_tok, int ctrl_stride,
                  const bf16_t* emb, const float* w, const float* b, float* h, int R, int C, int f16, hipStream_t st,
                  unsigned long long* tl, int n_vocab);
// Launchers return the workgroup count of the launch.
int launch_ln_mix(const LnMixArgs& a, int n_out_rows, hipStream_t st);
int launch_gemm(const GemmArgs& a, hipStream_t st);
// a one-row step's head GEMM with ln_out folded in (k_gemm2_lnrow); false if not covered
bool launch_gemm_lnrow(const GemmArgs& a, const LnMixArgs& lo, hipStream_t st);
// The FFN half of a decode step (LN2 + mix, key GEMM, relu^2, value GEMM) as ONE persistent launch
// with in-launch hand-offs (k_ffn_persist); false if the shapes are not covered.
constexpr int kFfnSyncInts = 24 * 64;  // counter block per layer: (8 LN replicas + 16 K-slices) x 256 B
// row-fused form (no LayerNorm rows): key workgroups done (the shift writer waits), in LN replica 1's
// counter. (A 25th counter staggered every later device allocation: 2 % slower decode at 32 rows.)
constexpr int kFfnKeyDone = 1;
// ---- persistent launches: hand-off counters and their arguments (lm_kernels.hip) ----------
// Inter-workgroup hand-offs of the persistent FFN launch (k_ffn_persist): counters kSyncStride
// ints (256 B) apart (see lm_kernels.hip for each launch's layout).
constexpr int kSyncStride = 64;
constexpr int kLnReplicas = 8;
constexpr int kFfnSlices = 16;  // value K-slices (F / 256 at the 0.4B shape)
// counter blocks (kSyncStride-int units) of the persistent attention launch (k_att_persist)
constexpr int kAttLn = 0;      // kLnReplicas: LayerNorm rows published
constexpr int kAttHead = 8;    // 16: head h's r / k / v tiles published (3 tiles x the K-splits)
constexpr int kAttLora = 24;   // kLnReplicas: the LoRA-down tiles published
constexpr int kAttWkv = 32;    // 16: WKV workgroups of head h done (one per row)
constexpr int kAttCounters = 48;
constexpr int kAttRkvDone = kAttLn + 1;  // row-fused form (no LayerNorm rows): rkv workgroups done
struct FfnSync {     // (both persistent launches)
  int* cnt;          // this layer's counters (zero at launch)
  int* cnt_prev;     // the counters of the layer launched before this one: zeroed by block 0
  int n_prev;        // counters to zero there
  int* err;          // give-up word: a bounded wait that timed out ORs its code in
  int n_ln_blocks;   // LayerNorm blocks (rows rounded up to 8: the GEMM blocks keep their XCD order)
  int ln_rows;       // LayerNorm rows the GEMM workgroups wait for
  int n_key;         // FFN: key workgroups; attention: rkv workgroups
  int key_group;     // FFN: key column tiles per value K-slice
  int key_per_slice; // FFN: key workgroups per value K-slice (key_group x key splits)
  int n_wkv;         // attention: WKV workgroups
  int n_val;         // FFN: value workgroups
  int rkv_tiles;     // attention: column tiles of the rkv launch (its grid is tiles x splits)
  int head_target;   // attention: rkv workgroups per head (3 tiles x splits)
  int lora_target;   // attention: LoRA-down workgroups (tiles x splits)
  int C;             // attention: channels (r / k / v columns [0, 3C), LoRA-down beyond)
  int opts;          // bit 0: value workgroups request their weights only once the LN rows are
                     // published (not at dispatch); bit 1: longer sleep between polls; bit 2: key
                     // workgroups request their weights after the LN wait (with their X)
  uint64_t* stamps;  // debug (RWKVTTS_FFN_STAMPS): [block][4] s_memrealtime: start, wait done, work
                     // done, end (null in production)
  // dispatch-time prefetches held back by a fixed time (s_memrealtime ticks of 10 ns; 0 = none),
  // so the LayerNorm rows at the head of the launch run with less traffic beside them:
  // d_w the rkv / key weight streams, d_late the Wo weights, d_s the WKV state + LoRA-up, d_v the
  // FFN value weights
  int d_w, d_late, d_s, d_v;
  int d_k;  // the FFN key weight streams (d_w: the rkv ones)

  // test hook (RWKVTTS_TEST_DROP_ARRIVE, null in production): the first rkv workgroup to find *drop
  // set clears it and skips its head arrival (a hand-off that never completes: the waits time out)
  int* drop;

  // Data-tagged granule hand-off (row-fused FFN form, one decode row; null: partial slabs +
  // counters). A key workgroup stores each output element of the row as ONE 8-byte {f32 bits, tag}
  // granule (sc1 store) at gran[split * gran_ld + column]; a value workgroup polls the granules of
  // its K-slice itself until every tag matches -- no store drain, no counter, no separate payload
  // load behind a poll (MI355X_MICROARCH.md price list: handoff-1to1 vs handoff-flag).
  // tag = (*epoch * 64 + layer) with bit 31 set (lm_kernels.hip gran_tag): never 0, so a zeroed
  // granule never matches. *epoch is bumped once per one-row forward pass by the layer-0 attention
  // launch (epoch_bump) and once by Engine::reset_persistent (which also zeroes every granule), so
  // no granule of an earlier pass matches: every one-row pass rewrites all of them, and a pass
  // that failed part-way is followed by that reset.
  uint64_t* gran;
  const int* epoch;
  int gran_ld;
  int layer;
  // attention (one row): WKV -> Wo granules at zgran[channel] (the z split hi | lo << 16)
  uint64_t* zgran;
  int* epoch_bump;  // (attention launch of layer 0) one lane adds 1 to it
};

// The attention half of a decode step (LN1 + mixes, rkv + LoRA-down, WKV, Wo) as ONE persistent
// launch (k_att_persist); false if the shapes are not covered.
constexpr int kAttSyncInts = kAttCounters * kSyncStride;  // counter block per layer (lm_kernels.hip kAtt*)
// fused_ln (one decode row, no embedding form): the row-fused form -- no LayerNorm blocks; every
// rkv / key workgroup computes the row's LayerNorm itself from the residual and the partial slabs
// (68 / 36 KB) and stages only its K-slice's mix, and one trailing workgroup stores the residual
// and the new token-shift row once every GEMM workgroup has read the old one (kAttRkvDone /
// kFfnKeyDone). Replaces the LayerNorm phase and its hand-off at batch 1.
bool launch_att_persist(const LnMixArgs& ln, const GemmArgs& rkv, const WkvArgs& wkv, const GemmArgs& wo, int* cnt,
                        int* cnt_prev, int* err, int R, int H, hipStream_t st, uint64_t* stamps, int opts,
                        int* drop = nullptr, bool fused_ln = false, int* epoch_bump = nullptr,
                        uint64_t* gran = nullptr, const int* epoch = nullptr);
// granules of the one-row attention form's WKV -> Wo hand-off (one per channel)
inline int64_t att_gran_count(int C) { return (int64_t)C; }
bool launch_ffn_persist(const LnMixArgs& ln, const GemmArgs& key, const GemmArgs& val, int* cnt, int* cnt_prev,
                        int* err, int R, hipStream_t st, uint64_t* stamps = nullptr, int opts = 0,
                        bool fused_ln = false, uint64_t* gran = nullptr, const int* epoch = nullptr);
// granules the row-fused FFN form's key -> value hand-off needs (FfnSync::gran)
inline int64_t ffn_gran_count(int key_splits, int F) { return (int64_t)key_splits * F; }
// Fills a.tw / a.tinfo / a.n_tinfo when the segments' packed weights are contiguous in 64-column
// tiles and every segment's X is seg[0]'s planes plus a multiple of x_mix_stride; returns whether
// the table applies (otherwise the kernel looks the segment up).
bool gemm_tile_table(GemmArgs& a, int64_t x_mix_stride);
int launch_wkv(const WkvArgs& a, int n_seg, int H, hipStream_t st);
// Which coalesced WKV state layout launch_wkv expects for these LoRA ranks / slab count: 0 none
// (row-major S[i][j], generic kernels), 1 k_wkv4 (two waves per block), 2 k_wkv6 (four waves).
// variant: rwkvtts_engine_desc.wkv_variant (0 auto by slot count).
int wkv_perm_layout(int Dw, int Da, int Dv, int Dg, int n_part, int max_slots, int variant);
// relu(sum of nx f32 slabs [nx][R][ld])^2 -> bf16 hi/lo planes [R][F] (bf16 prefill steps)
void launch_relu2_planes(const float* part, int nx, int64_t pstride, int ld, int F, int R, bf16_t* hi, bf16_t* lo,
                         hipStream_t st);
// Repack a GEMM matrix W [N][K] (K % 32 == 0) into MFMA fragment blocks (k_gemm's layout):
// out holds ceil(N/16)*16*K elements.
void launch_pack_frag(const bf16_t* W, int N, int K, bf16_t* out, hipStream_t st);

// Quantised matrices (RWKVTTS_QUANT_*, web-rwkv Quant restated): W [N][K] 16-bit -> codes in
// launch_pack_frag's fragment order (block (nb, kb) = 16 columns x 32 k, lane 16 g + li holding
// k = 32 kb + 8 g .. + 8 of column 16 nb + li: 8 bytes (int8) or 4 bytes (nf4, low nibble first))
// and per-(column, K-block) scales: int8 [N][K / 128] u32 = f16 min | f16 max << 16; nf4
// [N][K / 64] u16 = f16 absmax.
constexpr int kQ8Block = 128, kQ4Block = 64;
inline size_t quant_code_bytes(int qt, int N, int K) { return (size_t)N * K / (qt == 1 ? 1 : 2); }
inline size_t quant_scale_bytes(int qt, int N, int K) { return qt == 1 ? (size_t)N * (K / kQ8Block) * 4 : (size_t)N * (K / kQ4Block) * 2; }
void launch_quant_pack(const uint16_t* W, int N, int K, int f16, int qt, uint8_t* codes, void* scales, hipStream_t st);
// Repack one layer's LoRA-up rows (0.4B ranks 64/64/32/128) into k_wkv4's coalesced order.
void launch_pack_lora4(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                       bf16_t* out, hipStream_t st);
void launch_pack_lora6(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                       bf16_t* out, hipStream_t st);
// Repack one layer's w2t | a2t | v2t | g2t ([C][D] each) into the per-thread order of k_wkv.
void launch_pack_lora(const bf16_t* w2t, const bf16_t* a2t, const bf16_t* v2t, const bf16_t* g2t, int C,
                      int Dw, int Da, int Dv, int Dg, bf16_t* out, hipStream_t st);

}  // namespace rwkvtts
