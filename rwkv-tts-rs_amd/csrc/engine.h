// engine.h -- MI355X engine: SharedRwkvRuntime + v7::Bundle + TokioRuntime<Rnn> of the
// reference (src/shared_runtime.rs:23-284) re-designed as one owner thread per GPU with
// device-resident state slots, ragged-batch forward steps and hipGraph-replayed decode steps.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "lm_kernels.h"
#include "sampler.h"

namespace rwkvtts {

// one row of the k_advance test hook (plain layout, mirrored by tests/test_gpu_advance.py)
struct DebugAdvanceRow {
  int32_t mode;      // 0 normal, 1 zero-shot
  int32_t phase;     // 0 global, 2 semantic
  int32_t top_k;
  int32_t fixed;     // EOS always masked
  int32_t n_sem;     // semantic tokens already emitted
  int32_t hard_min;  // zero-shot: EOS masked while n_sem < hard_min
  int32_t win_bits;  // zero-shot EOS window (newest at bit 0)
  int32_t win_len;
  uint32_t key[8];   // ChaCha12 key of the phase's stream
  uint64_t draw;     // index of the next u32 draw
};

struct LayerW {
  const float *ln1_w, *ln1_b, *ln2_w, *ln2_b;
  const float* mu[6];  // x_r x_w x_k x_v x_a x_g
  const float *w0, *a0, *v0, *k_k, *k_a, *r_k, *lnx_w, *lnx_b, *ffn_xk;
  const bf16_t *wr, *wk, *wv, *wo, *w1t, *a1t, *v1t, *g1t, *w2t, *a2t, *v2t, *g2t, *ffn_k, *ffn_v;
  const bf16_t* lup;  // LoRA-up rows repacked for k_wkv
  // RWKVTTS_QUANT_* of this layer's r / k / v / o / FFN matrices (0: 16-bit fragments) and their
  // codes / scales (launch_quant_pack layout; r, k, v back to back as the rkv launch's tiles 0..)
  int quant = 0;
  const uint8_t *q_rkv = nullptr, *q_o = nullptr, *q_fk = nullptr, *q_fv = nullptr;
  const void *s_rkv = nullptr, *s_o = nullptr, *s_fk = nullptr, *s_fv = nullptr;
  int qs_rkv = 0, qs_o = 0, qs_fk = 0, qs_fv = 0;  // f16 models: GemmArgs::q_shift per launch
};

// One forward step description (host side).
struct StepPlan {
  std::vector<uint32_t> tok;   // per row
  std::vector<int4> rows;      // slot, flags, prev_row, 0
  std::vector<int4> segs;      // slot, row_begin, n_rows, 0
  std::vector<int> lg_rows;    // rows whose logits are produced
  std::vector<int> lg_slot;    // slot of each logits row (advance)
  int head_rows = 0;
  bool tok_from_ctrl = false;  // decode: token = ctrl[slot].next_token
  bool advance = false;        // run the phase controller on the logits rows
};

constexpr int kLookahead = 8;  // decode steps queued per host poll of the control blocks

// One request in flight through Engine::serve. The request's arrays stay valid until finish().
struct Job {
  rwkvtts_request req{};
  rwkvtts_result* res = nullptr;
  void* user = nullptr;
};

class Engine;

// Where Engine::serve gets requests and returns results (a fixed list for generate_batch, the
// manager's per-engine inbox for rwkvtts_manager_*). Called only from the engine's owner thread.
class JobSource {
 public:
  virtual ~JobSource() = default;
  // Appends up to `max` new jobs to `out`. wait: block until at least one job is available or the
  // source is closed. Returns false once the source is closed and drained (no job will follow).
  virtual bool next(int max, bool wait, std::vector<Job*>& out) = 0;
  virtual void finish(Job* j) = 0;  // j->res is filled
  // called by the owner thread after every unit of work (live statistics)
  virtual void progress(const Engine&) {}
};

struct Active;  // a request decoding in a state slot (engine.hip, Engine::serve)

struct ProfEntry {
  std::string name;
  int64_t launches = 0;
  double ms = 0.0;
};

class Engine {
 public:
  Engine() = default;
  ~Engine();
  int init(const rwkvtts_engine_desc& desc, const void* weights, size_t bytes, int on_device);

  int slot_reset(int slot, bool sync = true);  // sync = false: stream-ordered only (admission)
  int slot_read(int slot, float* out);
  int slot_write(int slot, const float* in);
  int64_t state_floats() const;

  int infer(const rwkvtts_input* in, int n, int head_rows, float* logits, int32_t* consumed,
            int32_t* has_logits);
  int sample(const float* logits, int n_rows, int row_len, const rwkvtts_sample_args* args,
             rwkvtts_rng* const* rngs, int32_t* out, float* dbg_host = nullptr);
  int generate(const rwkvtts_request* reqs, int n, rwkvtts_result* res);
  // Test hook (rwkvtts_debug_advance): k_advance itself -- advance_prep + the prepped
  // sample_block, the certified fast path or the exact walk -- on caller-given logit rows and
  // per-row controller states, for n_steps consecutive launches on the same rows.
  int debug_advance(const float* logits, int n_rows, const struct DebugAdvanceRow* rows, int exact, int n_steps,
                    int32_t* out_tok, int32_t* out_used, int32_t* out_phase);
  // Continuous batching until `src` is closed and every admitted job has finished.
  int serve(JobSource& src);
  // Checks a request before admission; fills `why` and returns false for a bad one.
  bool validate(const rwkvtts_request& q, std::string& why) const;
  int max_slots() const { return S_; }
  // whether this engine holds its device's persistent-launch slot (claim_persistent)
  bool persistent() const { return att_persist_ != 0 || ffn_persist_ != 0; }
  // true once after serve() returned an error because a persistent hand-off wait timed out: the
  // unit's jobs failed, the give-up word, every hand-off counter block and the failed slots were
  // reset, and the engine serves again (the manager keeps it; the next batch runs normally)
  bool take_recovered() {
    const bool r = recovered_;
    recovered_ = false;
    return r;
  }
  int64_t max_active = 0;  // most slots decoding at once (serve)
  int64_t admissions_ = 0;  // requests admitted over the engine's life (test hook counter)

  rwkvtts_dims dims{};
  rwkvtts_stats stats{};
  bool profiling = false;
  std::vector<ProfEntry> prof;
  // In-graph kernel timing (rwkvtts_set_profiling(e, 2)): the decode graphs are (re)captured with
  // launch-timeline slots; after every graph-replayed decode window the last step's per-launch
  // (first workgroup start, last workgroup end) stamps are copied back with the control snapshot
  // and accumulated into `prof` by launch name -- the kernels' own durations inside the graphs,
  // as rocprofv3 --kernel-trace reports them, without eager launches or per-step syncs.
  int set_graph_timing(bool on);
  bool graph_timing() const { return d_gt_ != nullptr && gtime_; }

 private:
  int run_step(const StepPlan& p, bool upload);
  int finish_unit(int b, bool prefill, std::vector<Active>& act, std::vector<int>& free_slots, JobSource& src,
                  hipEvent_t* ev0, hipEvent_t* ev1);
  int launch_forward(int R, int n_seg, int n_lg, int head_rows, bool tok_from_ctrl, bool advance);
  int upload_plan(const StepPlan& p);
  void prof_begin(hipEvent_t* ev);
  void prof_end(const char* name, hipEvent_t ev);
  int flush_prof();
  int dump_stamps();
  // after a timed-out persistent hand-off: zero the give-up word and every persistent counter block
  // on the engine's stream and wait for it (the jobs of the failed units have already been failed;
  // their slots are reset at their next admission, slot_reset)
  int reset_persistent();
  // after a second timed-out hand-off within kDegradeWindow units: the separate launches from now on
  // (persistent forms off, cached graphs dropped, the device's persistent slot released)
  int degrade_persistent();
  static constexpr int64_t kDegradeWindow = 1024;
  int64_t units_ = 0;             // units finished (finish_unit)
  int64_t last_fault_unit_ = -1;  // units_ at the last timed-out hand-off
  int lock_fd_ = -1;          // the cross-process lock of the persistent slot (claim_persistent)
  int persist_fault_ = 0;     // give-up code of the last failed unit (finish_unit), 0 if none
  bool recovered_ = false;
  std::vector<std::pair<int*, size_t>> sync_bufs_;  // every persistent counter block (reset_persistent)
  // RWKVTTS_TEST_DROP_ARRIVE=n at creation (test hook, not a deployment knob): a device word set to
  // 1; the rkv workgroup of a persistent attention launch that takes it (take_drop) skips its head
  // arrival, so that head's WKV workgroups time out and the unit fails; the word is re-armed after
  // each recovery until n units have failed (tests/test_gpu_persist_recovery.py)
  int* d_drop_ = nullptr;
  int test_drops_left_ = 0;

  void state_permute(const float* std_block, float* dev_block);
  void state_unpermute(const float* dev_block, float* std_block);
  int state_perm_ = 0;  // WKV state block layout (wkv_perm_layout; engine.hip perm_index)
  // XCD-aware grids per launch class: bit 0 rkv, 1 Wo, 2 ffn key, 3 ffn value, 4 head, 5 wkv
  static constexpr int kXmapMask = 0x28;  // measured (timeline A/B): value GEMM and WKV gain, rkv loses
  // write-through (sc1) output stores per launch class, same bit order as kXmapMask, plus
  // bit 6 ln_att, bit 7 ln_ffn
  static constexpr int kWtMask = 0xFF;
  // GemmArgs::xalign per class: bit 0 rkv (-> WKV heads; within noise, off), bit 2 ffn key (-> value K-slices)
  static constexpr int kXalignMask = 4;
  // The decode-step forms (rwkvtts_engine_desc.forms, RWKVTTS_FORM_*; the defaults are the shipping
  // forms, each measured faster than the launches it replaces):
  // one-row decode steps: the row-fused persistent form (each GEMM workgroup computes the row's
  // LayerNorm itself; lm_kernels.h launch_att_persist). RWKVTTS_FORM_LN_ROWS turns it off.
  bool fuse_ln1_ = true;
  // one-row forms: the FFN key -> value and the WKV -> Wo hand-offs as data-tagged granules
  // (FfnSync::gran; d_epoch_ is bumped by each pass's layer-0 attention launch and by
  // reset_persistent). RWKVTTS_FORM_SLAB_HANDOFF turns it off.
  bool gran_ = true;
  uint64_t* d_gran_ = nullptr;
  uint64_t* d_gran_att_ = nullptr;  // the attention form's (WKV -> Wo)
  // one-row steps: ln_out folded into the head GEMM (launch_gemm_lnrow). RWKVTTS_FORM_SEPARATE_LNOUT off.
  bool lnrow_ = true;
  bool exact_sampler_ = false;  // RWKVTTS_FORM_EXACT_SAMPLER: k_advance without the certified fast path
  int* d_epoch_ = nullptr;
  // decode steps' FFN / attention half as one persistent launch (k_ffn_persist / k_att_persist):
  // 0 off (RWKVTTS_FORM_SEPARATE_FFN / _ATT), else 1 + 2 x launch options (opts 2: the longer poll
  // sleep, the measured best)
  static constexpr int kPersistOn = 5;
  int ffn_persist_ = kPersistOn;
  int* ffn_sync_ = nullptr; // its hand-off counters: [L][kFfnSyncInts] (give-up code: d_ctrl_[S_])
  int att_persist_ = kPersistOn;
  int* att_sync_ = nullptr; // its hand-off counters: [L][kAttSyncInts]
  int device_ = 0;
  int f16_ = 0;  // fp16 matrices (else bf16): MFMA f16 and f16 activation planes
  hipStream_t stream_ = nullptr;
  int S_ = 0, Rmax_ = 0, chunk_ = 0, H_ = 0, Vpad_ = 0, Dtot_ = 0, ldA_ = 0;
  int splitA_ = 1, splitO_ = 1, splitK_ = 1, splitF_ = 1, splitH_ = 1;
  bool use_graphs_ = true;
  uint8_t* wblob_ = nullptr;
  // debug timeline (RWKVTTS_DEBUG_STAMPS "timeline=path"): per launch of a decode step, earliest WG start and
  // latest WG end (s_memrealtime); accumulated over steps and written at the end of generate()
  unsigned long long* d_tl_ = nullptr;  // [kTlMax][kTlStride]
  unsigned long long* d_gt_ = nullptr;  // in-graph timing slots [kTlMax][kTlStride]
  unsigned long long* h_gt_ = nullptr;  // pinned: 2 snapshots of them (one per unit buffer)
  bool gtime_ = false;
  std::map<std::pair<int, int>, std::vector<std::string>> graph_names_;  // launch names per graph
  std::pair<int, int> last_graph_ = {-1, -1};  // key of the graph the last run_step replayed
  std::pair<int, int> unit_graph_[2] = {{-1, -1}, {-1, -1}};  // per unit buffer (decode windows)
  unsigned long long* tl_base() const { return d_tl_ ? d_tl_ : (gtime_ ? d_gt_ : nullptr); }
  std::string tl_path_;
  std::vector<std::string> tl_names_;
  std::vector<double> tl_start_, tl_dur_;
  int tl_steps_ = 0;
  int tl_n_ = 0;
  unsigned long long* tl_next(const char* name) {
    unsigned long long* base = tl_base();
    if (!base || tl_n_ >= kTlMax) return nullptr;
    if ((int)tl_names_.size() <= tl_n_) tl_names_.push_back(name);
    unsigned long long* p = base + (size_t)kTlStride * tl_n_;
    ++tl_n_;
    return p;
  }
  static constexpr int kTlMax = 1024;
  bf16_t* wpack_ = nullptr;      // GEMM matrices in MFMA fragment blocks (launch_pack_frag)
  bf16_t* lora_pack_ = nullptr;  // [L][C][Dtot] LoRA-up rows in k_wkv's per-thread order
  const bf16_t* emb_ = nullptr;
  const bf16_t* head_ = nullptr;
  const float *ln0_w_ = nullptr, *ln0_b_ = nullptr, *lnout_w_ = nullptr, *lnout_b_ = nullptr;
  std::vector<LayerW> L_;
  // state
  float* wkv_ = nullptr;     // [S][L][H][N][N]
  float* att_sh_ = nullptr;  // [2][S][L][C]
  float* ffn_sh_ = nullptr;  // [2][S][L][C]
  int* slot_par_ = nullptr;  // [S]
  std::vector<int> par_host_;
  std::vector<SlotCtrl> ctrl_stage_;  // [S] host copy of each admitted slot's initial control block
  // per-step tables
  uint32_t* d_tok_ = nullptr;
  int4* d_rows_ = nullptr;
  int4* d_segs_ = nullptr;
  int* d_lg_rows_ = nullptr;
  int* d_lg_slot_ = nullptr;
  // scratch
  float *h0_ = nullptr, *h1_ = nullptr, *partA_ = nullptr, *partO_ = nullptr, *partF_ = nullptr,
        *partK_ = nullptr,
        *vfirst_ = nullptr, *logits_ = nullptr;
  bf16_t *xm_hi_ = nullptr, *xm_lo_ = nullptr, *z_hi_ = nullptr, *z_lo_ = nullptr,
         *xf_hi_ = nullptr, *xf_lo_ = nullptr, *xk_hi_ = nullptr, *xk_lo_ = nullptr,
         *xo_hi_ = nullptr, *xo_lo_ = nullptr;
  // controller
  SlotCtrl* d_ctrl_ = nullptr;
  int32_t* d_sem_ = nullptr;
  SlotCtrl* h_ctrl_ = nullptr;  // pinned mirror
  // sampler API scratch
  float* d_samp_logits_ = nullptr;
  size_t samp_cap_ = 0;     // logits elements
  int samp_rows_cap_ = 0;   // rows of d_keys_ / d_draws_ / d_out_
  void* d_wide_ = nullptr;  // rows longer than kSampleMaxN: per-row p / keys / list scratch
  size_t wide_cap_ = 0;
  uint32_t* d_keys_ = nullptr;
  uint64_t* d_draws_ = nullptr;
  int32_t* d_out_ = nullptr;
  // graphs keyed by (R, head_rows)
  std::map<std::pair<int, int>, hipGraphExec_t> graphs_;
  std::vector<std::pair<std::string, hipEvent_t>> pending_prof_;
  std::vector<void*> allocs_;
  // debug stamps (RWKVTTS_DEBUG_STAMPS "kind=path", null in production):
  uint64_t* dbg_stamps_ = nullptr;  // wkv: layer-5 WKV phase stamps
  std::string dbg_stamp_path_;
  bool no_emb_fuse_ = false;  // RWKVTTS_FORM_SEPARATE_EMBED: decode steps launch k_embed separately
  uint64_t* dbg_astamps_ = nullptr;  // adv: k_advance phase stamps, [rows][16]
  std::string dbg_astamp_path_;
  uint64_t* dbg_astamps2_ = nullptr;  // att: layer-5 k_att_persist block stamps
  std::string dbg_astamp2_path_;
  uint64_t* dbg_fstamps_ = nullptr;  // ffn: layer-5 k_ffn_persist block stamps
  std::string dbg_fstamp_path_;
  uint64_t* dbg_gstamps_ = nullptr;  // gemm: layer-5 rkv / ffn_value GEMM stamps
  std::string dbg_gstamp_path_;
  template <typename T>
  int alloc(T** p, size_t count);
};

}  // namespace rwkvtts
