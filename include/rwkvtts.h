/*
 * rwkvtts.h -- C-ABI drop-in boundary for the RWKV-TTS inference hot path on MI355X (gfx950).
 *
 * Every entry point here replaces one reference interface of liuzl/rwkv-tts-rs @ 2025-12-05
 * (paths relative to the reference root); the Rust-side binding a maintainer would add is in
 * INTEGRATION.md. Conventions: plain pointers + sizes, opaque handles, int status (0 = OK,
 * negative = error, message via rwkvtts_last_error()), no exceptions across the ABI, all
 * buffers caller-owned. One engine per GPU. Engine entry points serialise on a per-engine
 * lock (concurrent callers queue; they do not share GPU steps); the request manager
 * (rwkvtts_manager_*: DynamicBatchManager) is the thread-safe, batching front door: any number
 * of threads submit, one owner thread per GPU engine runs continuous batching.
 */
#ifndef RWKVTTS_H
#define RWKVTTS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants: src/rwkv_sampler.rs:294-299, src/properties_util.rs:5 ------------------ */
#define RWKVTTS_EOS_TOKEN 8192          /* TTS_EOS_TOKEN */
#define RWKVTTS_TAG_0 8193              /* TTS_TAG_0 */
#define RWKVTTS_TAG_1 8194              /* TTS_TAG_1 */
#define RWKVTTS_TAG_2 8195              /* TTS_TAG_2 */
#define RWKVTTS_GLOBAL_TOKEN_OFFSET 8196 /* GLOBAL_TOKEN_OFFSET */
#define RWKVTTS_SPECIAL_TOKEN_OFFSET 77823 /* TTS_SPECIAL_TOKEN_OFFSET */
#define RWKVTTS_N_GLOBAL 32             /* normal_mode_inference.rs:220 global_tokens_size */
#define RWKVTTS_SEMANTIC_LIMIT 2048     /* normal_mode_inference.rs:316 */
#define RWKVTTS_HOP 320                 /* 参考/C/tts/sparktts.h:55 latent_hop_length */
#define RWKVTTS_SAMPLE_RATE 16000       /* 参考/C/tts/sparktts.h:53 */

/* status codes */
#define RWKVTTS_OK 0
#define RWKVTTS_EINVAL -1
#define RWKVTTS_EHIP -2
#define RWKVTTS_ENOMEM -3
#define RWKVTTS_EUNSUPPORTED -4
#define RWKVTTS_EBUSY -5     /* manager: result not ready yet (poll / wait timeout) */
#define RWKVTTS_ECLOSED -6   /* manager: shut down before the request ran */

/* weight storage dtypes (matrices; vectors are always f32) */
#define RWKVTTS_DTYPE_BF16 0
#define RWKVTTS_DTYPE_F16 1

/* ---- model description ------------------------------------------------------------------ */
/* RWKV-7 "x070" dims (tensor names A.3). web-rwkv ModelInfo analogue. */
typedef struct {
  int32_t n_layer;   /* L */
  int32_t n_embd;    /* C */
  int32_t head_size; /* N (64); H = C / N */
  int32_t n_ffn;     /* F */
  int32_t n_vocab;   /* V */
  int32_t d_decay;   /* w LoRA rank */
  int32_t d_aaa;     /* a LoRA rank */
  int32_t d_mv;      /* v LoRA rank */
  int32_t d_gate;    /* g LoRA rank */
} rwkvtts_dims;

/* Packed weight blob: tensor index -> byte offset. Matrices in [out][in] row-major
 * (the LoRA matrices are stored transposed relative to the checkpoint so that every
 * projection reads contiguous rows of its input dimension). */
enum {
  RWKVTTS_T_EMB = 0, RWKVTTS_T_LN0_W, RWKVTTS_T_LN0_B, RWKVTTS_T_LNOUT_W, RWKVTTS_T_LNOUT_B,
  RWKVTTS_T_HEAD, RWKVTTS_T_GLOBAL_COUNT
};
enum {
  RWKVTTS_L_LN1_W = 0, RWKVTTS_L_LN1_B, RWKVTTS_L_LN2_W, RWKVTTS_L_LN2_B,
  RWKVTTS_L_XR, RWKVTTS_L_XW, RWKVTTS_L_XK, RWKVTTS_L_XV, RWKVTTS_L_XA, RWKVTTS_L_XG,
  RWKVTTS_L_W0, RWKVTTS_L_A0, RWKVTTS_L_V0, RWKVTTS_L_KK, RWKVTTS_L_KA, RWKVTTS_L_RK,
  RWKVTTS_L_LNX_W, RWKVTTS_L_LNX_B, RWKVTTS_L_FFN_XK,
  /* ---- matrices from here on ---- */
  RWKVTTS_L_WR, RWKVTTS_L_WK, RWKVTTS_L_WV, RWKVTTS_L_WO,
  RWKVTTS_L_W1T, RWKVTTS_L_A1T, RWKVTTS_L_V1T, RWKVTTS_L_G1T, /* [D][C] */
  RWKVTTS_L_W2T, RWKVTTS_L_A2T, RWKVTTS_L_V2T, RWKVTTS_L_G2T, /* [C][D] */
  RWKVTTS_L_FFN_K, /* [F][C] */
  RWKVTTS_L_FFN_V, /* [C][F] */
  RWKVTTS_L_COUNT
};
#define RWKVTTS_L_FIRST_MAT RWKVTTS_L_WR

/* Fill rows/cols of one tensor. Returns 1 for a matrix (2-byte dtype), 0 for an f32 vector. */
static inline int rwkvtts_tensor_shape(const rwkvtts_dims* d, int layer, int t, int64_t* rows,
                                       int64_t* cols) {
  const int64_t C = d->n_embd, V = d->n_vocab, F = d->n_ffn;
  if (layer < 0) {
    switch (t) {
      case RWKVTTS_T_EMB: *rows = V; *cols = C; return 1;
      case RWKVTTS_T_HEAD: *rows = V; *cols = C; return 1;
      default: *rows = 1; *cols = C; return 0;
    }
  }
  switch (t) {
    case RWKVTTS_L_WR: case RWKVTTS_L_WK: case RWKVTTS_L_WV: case RWKVTTS_L_WO:
      *rows = C; *cols = C; return 1;
    case RWKVTTS_L_W1T: *rows = d->d_decay; *cols = C; return 1;
    case RWKVTTS_L_A1T: *rows = d->d_aaa; *cols = C; return 1;
    case RWKVTTS_L_V1T: *rows = d->d_mv; *cols = C; return 1;
    case RWKVTTS_L_G1T: *rows = d->d_gate; *cols = C; return 1;
    case RWKVTTS_L_W2T: *rows = C; *cols = d->d_decay; return 1;
    case RWKVTTS_L_A2T: *rows = C; *cols = d->d_aaa; return 1;
    case RWKVTTS_L_V2T: *rows = C; *cols = d->d_mv; return 1;
    case RWKVTTS_L_G2T: *rows = C; *cols = d->d_gate; return 1;
    case RWKVTTS_L_FFN_K: *rows = F; *cols = C; return 1;
    case RWKVTTS_L_FFN_V: *rows = C; *cols = F; return 1;
    default: *rows = 1; *cols = C; return 0;
  }
}

/* Byte offset of tensor t of `layer` (-1 = global tensors) in the packed blob; every tensor
 * starts on a 256-byte boundary. With layer == -2 returns the total blob size. */
static inline int64_t rwkvtts_tensor_offset(const rwkvtts_dims* d, int layer, int t) {
  int64_t off = 256; /* header */
  int64_t r, c;
  for (int l = -1; l < d->n_layer; ++l) {
    const int n = (l < 0) ? RWKVTTS_T_GLOBAL_COUNT : RWKVTTS_L_COUNT;
    for (int i = 0; i < n; ++i) {
      if (l == layer && i == t) return off;
      int m = rwkvtts_tensor_shape(d, l, i, &r, &c);
      int64_t bytes = r * c * (m ? 2 : 4);
      off += (bytes + 255) & ~(int64_t)255;
    }
  }
  return off;
}
static inline int64_t rwkvtts_blob_bytes(const rwkvtts_dims* d) {
  return rwkvtts_tensor_offset(d, -2, 0);
}

/* Blob header (first 256 bytes). */
typedef struct {
  uint32_t magic;   /* 'RWT7' = 0x37545752 */
  uint32_t version; /* 1 */
  int32_t dtype;    /* RWKVTTS_DTYPE_* of the matrices */
  int32_t pad0;
  rwkvtts_dims dims;
} rwkvtts_blob_header;
#define RWKVTTS_BLOB_MAGIC 0x37545752u

/* Deterministic synthetic weights (N(0, 0.02) matrices, decay w0 chosen so that
 * w in (0.3, 0.99), lerp coefficients in [0,1]); counter-based so every tool regenerates the
 * same blob. `out` must hold rwkvtts_blob_bytes(dims) bytes. */
int rwkvtts_synth_weights(const rwkvtts_dims* dims, int dtype, uint64_t seed, void* out);

/* ---- engine: SharedRwkvRuntime::new / v7::Bundle::new (src/shared_runtime.rs:70-208) ---- */
typedef struct rwkvtts_engine rwkvtts_engine;

typedef struct {
  int32_t device;           /* HIP device ordinal */
  int32_t max_slots;        /* state slots = Bundle max_batch (shared_runtime.rs:177) */
  int32_t token_chunk_size; /* prompt rows per forward step, shared by the admitted requests (the
                               reference's per-request RnnInput token_chunk_size, 512 at
                               lightweight_tts_pipeline.rs:799; outputs are chunk-invariant) */
  int32_t use_graphs;       /* capture decode steps in hipGraphs */
  int32_t wkv_variant;      /* 0 auto; 1 k_wkv4 (2 waves per (slot, head)); 2 k_wkv6 (4 waves).
                               0.4B LoRA ranks only; both are tested against the oracle */
  /* web-rwkv ModelBuilder::quant(HashMap<layer, Quant>) as the server builds it from
   * --quant-layers / --quant-type (bin/server.rs:1029-1071, src/shared_runtime.rs:156-160):
   * layers [0, quant_layers) store their r / k / v / o and FFN key / value matrices quantised
   * (the LoRA matrices, embedding and head stay 16-bit). RWKVTTS_QUANT_NONE when 0 layers. */
  int32_t quant_layers;
  int32_t quant_type;       /* RWKVTTS_QUANT_* */
  /* Decode-step forms. 0 (the default) = the shipping forms. Each RWKVTTS_FORM_* bit switches one
   * fused form back to the launches it replaces; tokens and the recurrent state are bitwise equal
   * either way (tests/test_gpu_ffn_persist.py, test_gpu_emb_fusion.py). For verification and A/B
   * timing: no bit makes the engine faster. No reference counterpart (web-rwkv has one form). */
  uint32_t forms;
} rwkvtts_engine_desc;

#define RWKVTTS_FORM_SEPARATE_ATT 1u   /* attention half: LN1 / rkv / WKV / Wo launches, not k_att_persist */
#define RWKVTTS_FORM_SEPARATE_FFN 2u   /* FFN half: LN2 / key / value launches, not k_ffn_persist */
#define RWKVTTS_FORM_LN_ROWS 4u        /* one-row steps: LayerNorm workgroups, not the row-fused LayerNorm */
#define RWKVTTS_FORM_SLAB_HANDOFF 8u   /* one-row steps: partial slabs + counters, not data-tagged granules */
#define RWKVTTS_FORM_SEPARATE_LNOUT 16u /* one-row steps: ln_out launch, not folded into the head GEMM */
#define RWKVTTS_FORM_SEPARATE_EMBED 32u /* decode steps: k_embed launch, not folded into layer 0's LayerNorm */
#define RWKVTTS_FORM_EXACT_SAMPLER 64u /* k_advance: always the exact sequential-sum walk (no certificate) */

#define RWKVTTS_QUANT_NONE 0
#define RWKVTTS_QUANT_INT8 1 /* 128-element blocks along K: f16 (min, max), u8 q; w = min + q (max - min)/255 */
#define RWKVTTS_QUANT_NF4 2  /* 64-element blocks along K: f16 absmax, 4-bit NormalFloat index; w = nf4[q] absmax */
#define RWKVTTS_QUANT_SF4 3  /* rejected (RWKVTTS_EUNSUPPORTED): its code table is not available offline */

/* weights: packed blob (header included). blob_on_device != 0: `weights` is a device pointer
 * on desc->device (e.g. a buffer filled by an RCCL broadcast); it is copied. */
int rwkvtts_engine_create(const rwkvtts_engine_desc* desc, const void* weights, size_t bytes,
                          int blob_on_device, rwkvtts_engine** out);
int rwkvtts_engine_destroy(rwkvtts_engine* e);
const char* rwkvtts_last_error(void);
int rwkvtts_engine_dims(const rwkvtts_engine* e, rwkvtts_dims* out);

/* ---- state: State::init/load/back (normal_mode_inference.rs:66-70) --------------------- */
/* Per-slot state = per layer [att_shift C | wkv H*N*N (value-major S[i][j]) | ffn_shift C] f32. */
int64_t rwkvtts_state_floats(const rwkvtts_engine* e);
int rwkvtts_slot_reset(rwkvtts_engine* e, int slot);                 /* State::load(init, slot) */
int rwkvtts_slot_read(rwkvtts_engine* e, int slot, float* host_out); /* State::back(slot) */
int rwkvtts_slot_write(rwkvtts_engine* e, int slot, const float* host_in);

/* ---- LM runtime: Runtime<Rnn>::infer (normal_mode_inference.rs:62-80) ------------------ */
#define RWKVTTS_OPT_LAST 0 /* RnnOption::Last */
#define RWKVTTS_OPT_FULL 1 /* RnnOption::Full (logits for every token) */
typedef struct {
  int32_t slot;           /* batch index == state slot */
  const uint32_t* tokens; /* pending input tokens of this batch */
  int32_t n_tokens;
  int32_t option;         /* RWKVTTS_OPT_* */
} rwkvtts_input;

/* Consumes up to token_chunk_size tokens in total across `inputs` (each batch advances by
 * consumed[i]). For every batch whose input is exhausted by this call and option == LAST,
 * writes logits of its last token to logits[i * head_rows ... + head_rows) and sets
 * has_logits[i] = 1 (RnnOutput[i].0.size() > 0); otherwise has_logits[i] = 0.
 * head_rows <= n_vocab selects the leading vocabulary rows (all samplers read a prefix).
 * OPT_FULL writes logits for every consumed token at logits[(row) * head_rows], rows in
 * input order. logits is a HOST buffer. */
int rwkvtts_infer(rwkvtts_engine* e, const rwkvtts_input* inputs, int n_inputs, int head_rows,
                  float* logits, int32_t* consumed, int32_t* has_logits);

/* ---- sampler: sample_logits_with_top_p_k (src/rwkv_sampler.rs:55-211) ------------------ */
/* rand 0.8.5 StdRng (ChaCha12, seed_from_u64 via PCG32) is represented statelessly by its
 * 32-byte key and the index of the next u32 draw. */
typedef struct {
  uint32_t key[8];
  uint64_t draw_index;
} rwkvtts_rng;
void rwkvtts_rng_seed_from_u64(uint64_t seed, rwkvtts_rng* out); /* StdRng::seed_from_u64 */

typedef struct {
  float temperature;
  float top_p;
  int32_t top_k;
  int32_t forbid_token; /* -1 = None */
} rwkvtts_sample_args;

/* Samples n_rows rows of `logits` (host, n_rows x row_len f32) on the GPU; rng[i] == NULL
 * mirrors `rng: &mut None` (fixed StdRng(42) draw). rngs advance by one draw per row.
 * Any row_len up to 2^24 and every (temperature, top_p, top_k) of the reference is accepted:
 * rows up to 16384 run in LDS, longer rows (the 77,923-token vocabulary) in a device scratch.
 * out_tokens receives the index per row. */
int rwkvtts_sample(rwkvtts_engine* e, const float* logits, int n_rows, int row_len,
                   const rwkvtts_sample_args* args, rwkvtts_rng* const* rngs, int32_t* out_tokens);

/* ---- phase controllers + scheduler ------------------------------------------------------ */
/* TtsBatchRequest (src/rwkv_sampler.rs:222-231) after tokenisation
 * (dynamic_batch_manager.rs:512-515) and property-token construction (properties_util.rs:76-98). */
#define RWKVTTS_MODE_AUTO 0      /* zero-shot iff both ref token sets present (dbm.rs:526-540) */
typedef struct {
  const int32_t* text_tokens;
  int32_t n_text;
  const int32_t* property_tokens;
  int32_t n_property;
  const int32_t* ref_global;   /* NULL = None */
  int32_t n_ref_global;
  const int32_t* ref_semantic; /* NULL = None */
  int32_t n_ref_semantic;
  int32_t has_seed;
  uint64_t seed;
  int32_t max_tokens;          /* SamplerArgs.max_tokens; normal mode emits at most
                                  min(max_tokens, 2048) semantic tokens (normal_mode_inference.rs:316),
                                  so 0 -> none; must be >= 0 (usize) */
  int32_t fixed_semantic;      /* >0: benchmark mode -- EOS masked, exactly this many semantic tokens */
  int32_t greedy;              /* 1: top_k = 1 for both phases (config 1 plumbing check) */
  /* SamplerArgs.layered_randomness (LayeredRandomnessConfig, rwkv_sampler.rs:251-275) as used
   * by normal_mode_inference.rs:138-174 and zero_shot_inference.rs:204-216.
   * layered_set == 0 selects LayeredRandomnessConfig::default() (independent, 1000 / 2000). */
  int32_t layered_set;
  int32_t use_independent_seeds; /* 1: StdRng(seed + offset); 0: StdRng(seed + 100 / + 200),
                                    zero-shot StdRng(0) (dynamic_batch_manager.rs:491-494) */
  uint64_t global_seed_offset;
  uint64_t semantic_seed_offset;
} rwkvtts_request;

typedef struct {
  int32_t status;         /* 0 ok; <0 this request failed -> (vec![], vec![]) as dbm.rs:466-469
                             (the others of its batch still complete) */
  int32_t n_global;
  int32_t n_semantic;
  int32_t global_tokens[RWKVTTS_N_GLOBAL];
  int32_t* semantic_tokens; /* caller buffer, capacity >= RWKVTTS_SEMANTIC_LIMIT */
} rwkvtts_result;

/* DynamicBatchManager::generate_tts_batch (dynamic_batch_manager.rs:124-164) with real GPU
 * continuous batching: up to max_slots requests decode together, one slot each; a request is
 * admitted as soon as a slot frees, and its prompt rows ride in the same forward steps as the
 * other slots' decode rows. Per-request outputs are identical to running the requests one at a
 * time. Returns RWKVTTS_OK when the batch ran (per-request failures are in results[i].status),
 * or a negative code when the engine itself failed (then every status is that code). */
int rwkvtts_generate_batch(rwkvtts_engine* e, const rwkvtts_request* reqs, int n,
                           rwkvtts_result* results);

/* ---- request manager: DynamicBatchManager (dynamic_batch_manager.rs:22-164,185-405) ------ */
/* The reference collects requests (enqueue_worker: first request, then try_recv up to
 * max_batch_size; a lone request waits >= 10 ms for company, :185-264) and hands each batch to
 * whichever infer worker is free (:350-405), which then runs the batch sequentially on state
 * slot 0. Here one owner thread per engine (one engine per GPU: request-level data parallelism
 * over the node's GPUs) runs continuous batching; each collected batch is routed to
 * the least-loaded engine (fewest requests active + queued), and an engine admits queued
 * requests between forward steps whenever it has free slots. Any thread may submit / wait. */
typedef struct rwkvtts_manager rwkvtts_manager;
#define RWKVTTS_MAX_ENGINES 16
typedef struct {
  int32_t n_engines;                      /* engines (owner threads) */
  int32_t devices[RWKVTTS_MAX_ENGINES];   /* HIP device of each engine (repeats allowed) */
  rwkvtts_engine_desc engine;             /* per-engine settings (its .device is ignored) */
  int32_t max_batch_size;                 /* DynamicBatchConfig.max_batch_size (batch_types.rs:71) */
  int32_t collect_timeout_ms;             /* DynamicBatchConfig.collect_timeout_ms (batch_types.rs:73) */
} rwkvtts_manager_desc;
/* weights: one host blob. It crosses PCIe once, into the first engine's device; the manager then
 * broadcasts it over RCCL (ncclBroadcast over xGMI, one rank per distinct device, ncclCommInitAll)
 * to the other devices, and engines that share a device copy it device-to-device. With a single
 * distinct device RCCL is never loaded; if RCCL is missing or cannot initialise, the blob goes to
 * the other devices by hipMemcpyPeer (stats.bcast_rccl = 0). RWKVTTS_MANAGER_NO_RCCL=1 disables
 * RCCL; RWKVTTS_MANAGER_FORCE_RCCL=1 runs it even for one device (and fails create if it fails).
 * The caller's current HIP device is unchanged on return. This replaces
 * the reference's single model load handed to every infer worker (src/shared_runtime.rs:143-184,
 * src/dynamic_batch_manager.rs:33-87). */
int rwkvtts_manager_create(const rwkvtts_manager_desc* desc, const void* weights, size_t bytes,
                           rwkvtts_manager** out);
/* Stops the collector and the engine threads after the requests already submitted finish.
 * Threads blocked in rwkvtts_manager_wait when destroy starts return (their result, or
 * RWKVTTS_ECLOSED) before destroy frees the handle. No call on the handle may START while
 * destroy runs or after it: the caller serialises destroy against new submit / wait /
 * get_stats calls (as dropping the reference's manager requires no outstanding borrow). */
int rwkvtts_manager_destroy(rwkvtts_manager* m);
/* generate_tts (dynamic_batch_manager.rs:90-121) split in two: submit copies the request
 * (token arrays included) and returns a ticket; wait blocks up to timeout_ms (< 0: forever) and
 * returns RWKVTTS_OK with the result (the ticket is then released), RWKVTTS_EBUSY if the
 * request has not finished yet. out->semantic_tokens must hold RWKVTTS_SEMANTIC_LIMIT ids. */
int rwkvtts_manager_submit(rwkvtts_manager* m, const rwkvtts_request* req, uint64_t* ticket);
int rwkvtts_manager_wait(rwkvtts_manager* m, uint64_t ticket, int timeout_ms, rwkvtts_result* out);
/* generate_tts_batch (dynamic_batch_manager.rs:124-164): submit all, wait all. */
int rwkvtts_manager_generate_batch(rwkvtts_manager* m, const rwkvtts_request* reqs, int n,
                                   rwkvtts_result* results);
typedef struct {
  int64_t submitted;
  int64_t completed;
  int64_t batches;                          /* batches the collector formed */
  int64_t served[RWKVTTS_MAX_ENGINES];      /* requests completed per engine */
  int64_t max_active[RWKVTTS_MAX_ENGINES];  /* most slots an engine had decoding at once */
  int64_t steps[RWKVTTS_MAX_ENGINES];       /* forward steps per engine */
  int32_t bcast_ranks;                      /* distinct devices in the weight broadcast (RCCL ranks) */
  int32_t bcast_rccl;                       /* 1: the weights went out by ncclBroadcast */
  double bcast_ms;                          /* upload + broadcast wall time at create */
  int32_t waiters;                          /* threads blocked in rwkvtts_manager_wait now */
  int32_t reserved;
  int32_t persistent[RWKVTTS_MAX_ENGINES];  /* 1: the engine runs the persistent decode launches (at most
                                               one engine per GPU, across processes: rwkvtts_stats) */
} rwkvtts_manager_stats;
int rwkvtts_manager_get_stats(rwkvtts_manager* m, rwkvtts_manager_stats* out);

/* Step-level statistics of the last generate call (bench / roofline). */
typedef struct {
  int64_t steps;            /* decode steps */
  int64_t prefill_steps;
  double decode_ms;         /* HIP-event time of all decode steps */
  double prefill_ms;
  double sample_ms;         /* sampler kernels inside decode steps */
  int64_t decode_rows;      /* sum over decode steps of active rows */
  int32_t profile_kernel_count;
  int32_t persistent;       /* 1: this engine holds its GPU's persistent-launch slot (the first engine
                               created on the device in any process, RWKVTTS_LOCK_DIR lock file);
                               others run the separate launches (same outputs, bit for bit) */
} rwkvtts_stats;
int rwkvtts_get_stats(rwkvtts_engine* e, rwkvtts_stats* out);

/* Per-kernel timing: rwkvtts_set_profiling(e, 1) = HIP events on eager launches (graphs off);
 * (e, 2) = in-graph timing: the decode graphs are recaptured with launch-timeline slots and the
 * last step of every graph-replayed decode window is sampled (first workgroup start to last
 * workgroup end per launch, the interval rocprofv3 --kernel-trace reports); 0 = off. Calling
 * it again with the same mode clears the accumulated entries. Entries: name, launches, total ms. */
int rwkvtts_set_profiling(rwkvtts_engine* e, int on);
int rwkvtts_profile_entry(rwkvtts_engine* e, int idx, char* name, int name_cap, int64_t* launches,
                          double* total_ms);

/* Test hook, not part of the drop-in surface (no reference counterpart): runs the production
 * decode-step sampler/controller k_advance (sample_logits_with_top_p_k + the phase controllers of
 * normal_mode_inference.rs:222-391 / zero_shot_inference.rs, as the decode graphs run it) on
 * caller-given logit rows [n_rows][8193] and controller states, n_steps launches; exact = 1 forces
 * the exact sequential-sum walk. `rows` points to n_rows records of 72 bytes: int32 mode (0 normal,
 * 1 zero-shot), phase (0 global, 2 semantic), top_k, fixed, n_sem, hard_min, win_bits, win_len;
 * uint32 key[8] (ChaCha12 key of the phase's stream); uint64 draw (next u32 draw index).
 * Outputs out_tok / out_used / out_phase are [n_steps][n_rows]. */
int rwkvtts_debug_advance(rwkvtts_engine* e, const float* logits, int n_rows, const void* rows, int exact,
                          int n_steps, int32_t* out_tok, int32_t* out_used, int32_t* out_phase);

/* ---- codec: BiCodecDetokenize via ORT (lightweight_tts_pipeline.rs:606-622,706-730) ----- */
typedef struct rwkvtts_codec rwkvtts_codec;
typedef struct {
  int32_t codebook_size;  /* 8192 semantic codes */
  int32_t codebook_dim;   /* 8 */
  int32_t latent_dim;     /* 1024 */
  int32_t n_global;       /* 32 speaker tokens */
  int32_t fsq_levels;     /* 4 (per dim) */
  int32_t fsq_dims;       /* 6 -> 4^6 = 4096 codes */
  int32_t spk_dim;        /* d-vector 1024 */
  int32_t prenet_dim;     /* ConvNeXt dim 384 */
  int32_t prenet_inter;   /* 2048 */
  int32_t prenet_layers;  /* 12 */
  int32_t dec_channels;   /* 1536 */
  int32_t n_up;           /* 4 */
  int32_t up_rates[4];    /* 8,5,4,2 */
  int32_t up_kernels[4];  /* 16,11,8,4 */
} rwkvtts_codec_dims;
int64_t rwkvtts_codec_blob_bytes(const rwkvtts_codec_dims* d);
int rwkvtts_codec_synth_weights(const rwkvtts_codec_dims* d, uint64_t seed, float* out);
int rwkvtts_codec_create(int device, const rwkvtts_codec_dims* d, const float* weights,
                         rwkvtts_codec** out);
/* As rwkvtts_codec_create with the conv weight path chosen by the caller:
 * RWKVTTS_CODEC_WEIGHTS_AUTO (what rwkvtts_codec_create does): the weight hi + lo planes (three
 * MFMAs per product) iff some conv weight is not bf16-exact, so f32 checkpoints keep ~2^-16
 * relative weights; _BF16: bf16 weights (two MFMAs; faster, the weights rounded to bf16);
 * _HILO: hi + lo planes always (on bf16-exact weights bitwise the _BF16 PCM, tested). */
#define RWKVTTS_CODEC_WEIGHTS_AUTO 0
#define RWKVTTS_CODEC_WEIGHTS_BF16 1
#define RWKVTTS_CODEC_WEIGHTS_HILO 2
int rwkvtts_codec_create_ex(int device, const rwkvtts_codec_dims* d, const float* weights, int weight_path,
                            rwkvtts_codec** out);
int rwkvtts_codec_destroy(rwkvtts_codec* c);
/* semantic [T] i64, global [n_global] i64 -> pcm [T * 320] f32 (output "wav_rec"). */
int rwkvtts_codec_decode(rwkvtts_codec* c, const int64_t* semantic, int T, const int64_t* global,
                         float* pcm);
/* decode_audio_batch (lightweight_tts_pipeline.rs:625-703): n utterances in one pass. */
int rwkvtts_codec_decode_batch(rwkvtts_codec* c, const int64_t* const* semantic, const int* T,
                               const int64_t* const* global, int n, float* const* pcm);
/* Verification forms of later decode calls (0 = shipping); the PCM is bitwise equal either way
 * (tests/test_gpu_codec.py). No reference counterpart (ORT runs one graph). */
#define RWKVTTS_CODEC_FORM_SEPARATE_RESUNIT 1u /* 96-channel residual units as conv7 + conv1 launches */
#define RWKVTTS_CODEC_FORM_CHANNEL_LAST 2u     /* WaveGenerator planes [t][c] instead of [c / 32][t][32] */
int rwkvtts_codec_set_forms(rwkvtts_codec* c, uint32_t forms);
/* Per-stage HIP-event timing of later decode calls (profiling on): name, launches, total ms. */
int rwkvtts_codec_set_profiling(rwkvtts_codec* c, int on);
int rwkvtts_codec_profile_count(rwkvtts_codec* c);
int rwkvtts_codec_profile_entry(rwkvtts_codec* c, int idx, char* name, int name_cap, int64_t* launches,
                                double* total_ms);

/* ---- text tokenizer: web-rwkv Tokenizer::new / encode (src/shared_runtime.rs:187-192,
 * src/dynamic_batch_manager.rs:512-515) over assets/model/tokenizer.json -------------------- */
typedef struct rwkvtts_tokenizer rwkvtts_tokenizer;
/* vocab_json: the vocabulary file's bytes ({"id": "token" | [bytes], ...}). */
int rwkvtts_tokenizer_create(const char* vocab_json, size_t len, rwkvtts_tokenizer** out);
int rwkvtts_tokenizer_destroy(rwkvtts_tokenizer* t);
/* Greedy longest match over UTF-8 bytes. ids == NULL (or cap too small) only counts: *n_ids is
 * always the full count. A byte position no token matches -> RWKVTTS_EINVAL
 * (TokenizerError::NoMatchingTokenFound). */
int rwkvtts_tokenizer_encode(const rwkvtts_tokenizer* t, const uint8_t* text, size_t n, uint32_t* ids,
                             size_t cap, size_t* n_ids);
int rwkvtts_tokenizer_decode(const rwkvtts_tokenizer* t, const uint32_t* ids, size_t n, uint8_t* text,
                             size_t cap, size_t* n_bytes);
int64_t rwkvtts_tokenizer_vocab_size(const rwkvtts_tokenizer* t); /* max id + 1 */

/* ---- zero-shot reference mel (src/tts_pipeline_fixes.rs:12-159) ------------------------- */
/* wav [n] f32 @16 kHz -> mel [128][n_frames] (n_frames = (n + 1024 - 1024) / 320 + 1). */
int rwkvtts_mel(int device, const float* wav, int n, float* mel, int* n_frames);

#ifdef __cplusplus
}
#endif
#endif /* RWKVTTS_H */
