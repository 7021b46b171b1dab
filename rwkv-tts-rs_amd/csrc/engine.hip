// engine.cpp -- device memory layout, forward-step launcher, hipGraph cache, LM runtime API
// (Runtime<Rnn>::infer semantics) and the continuous-batching scheduler that replaces
// DynamicBatchManager's sequential slot-0 loop (src/dynamic_batch_manager.rs:409-551).
#include "engine.h"

#include <fcntl.h>
#include <string.h>
#include <sys/file.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <deque>
#include <map>
#include <mutex>
#include <random>

namespace rwkvtts {

template <typename T>
int Engine::alloc(T** p, size_t count) {
  void* q = nullptr;
  RT_HIP(hipMalloc(&q, std::max<size_t>(count * sizeof(T), 256)));
  RT_HIP(hipMemset(q, 0, std::max<size_t>(count * sizeof(T), 256)));
  allocs_.push_back(q);
  *p = (T*)q;
  return RWKVTTS_OK;
}

// At most ONE engine per device runs the persistent launches. Two persistent launches in flight
// on one GPU can deadlock: workgroups are dealt to the 8 XCDs round-robin and each XCD dispatches
// its share in order, so when another launch fills one XCD, a launch's consumers may be resident
// on other XCDs while producers they wait for are not -- and the other launch's consumers may
// wait the same way. Separate launches never wait on one another, so one persistent engine beside
// any number of others (and the vocoder) always makes progress. The first engine created on a
// device takes the slot; it is released when that engine is destroyed. Within a process a map
// guards it; across processes an exclusive flock on a file named by the device's PCI bus id
// (RWKVTTS_LOCK_DIR, default /tmp): a second process on the same GPU finds the lock held and runs
// the separate launches. (Processes that do not share the lock directory -- separate containers on
// one GPU -- are not covered: there the bounded waits turn a deadlock into failed units, which the
// engine recovers from, Engine::reset_persistent.)
namespace {
std::mutex g_persist_mu;
std::map<int, const void*> g_persist_owner;  // device -> the engine holding the persistent slot

// -1: held by another process; -2: no lock file (no cross-process guard); else the locked fd
int lock_device_file(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device) != hipSuccess || !bus[0])
    snprintf(bus, sizeof(bus), "device%d", device);
  for (char* c = bus; *c; ++c)
    if (*c == '/' || *c == ' ') *c = '_';
  const char* dir = getenv("RWKVTTS_LOCK_DIR");
  const std::string path = std::string(dir && dir[0] ? dir : "/tmp") + "/rwkvtts_persist_" + bus + ".lock";
  int fd = open(path.c_str(), O_RDONLY | O_CREAT | O_CLOEXEC, 0666);
  // another user's lock file in a sticky world-writable directory: O_CREAT is refused under
  // fs.protected_regular (EACCES) although the file itself may be readable -- open it as it is
  if (fd < 0) fd = open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    if (access(path.c_str(), F_OK) == 0) {  // it exists but cannot be opened: assume it is held
      fprintf(stderr, "rwkvtts: cannot open the persistent-launch lock %s; running the separate launches\n",
              path.c_str());
      return -1;
    }
    fprintf(stderr, "rwkvtts: cannot create the persistent-launch lock %s: no cross-process guard "
            "(set RWKVTTS_LOCK_DIR to a directory every process on this GPU shares)\n", path.c_str());
    return -2;
  }
  if (flock(fd, LOCK_EX | LOCK_NB) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}
}  // namespace

static bool claim_persistent(int device, const void* who, int* lock_fd) {
  std::lock_guard<std::mutex> lk(g_persist_mu);
  auto it = g_persist_owner.find(device);
  if (it != g_persist_owner.end() && it->second != who) return false;
  if (it == g_persist_owner.end()) {
    const int fd = lock_device_file(device);
    if (fd == -1) return false;  // another process on this GPU holds it
    *lock_fd = fd;
  }
  g_persist_owner[device] = who;
  return true;
}
static void release_persistent(int device, const void* who, int* lock_fd) {
  std::lock_guard<std::mutex> lk(g_persist_mu);
  auto it = g_persist_owner.find(device);
  if (it != g_persist_owner.end() && it->second == who) {
    g_persist_owner.erase(it);
    if (*lock_fd >= 0) close(*lock_fd);  // (closing the descriptor releases the flock)
    *lock_fd = -1;
  }
}

Engine::~Engine() {
  release_persistent(device_, this, &lock_fd_);
  hipSetDevice(device_);
  if (stream_) hipStreamSynchronize(stream_);
  for (auto& g : graphs_) hipGraphExecDestroy(g.second);
  for (auto& e : pending_prof_) hipEventDestroy(e.second);
  for (void* p : allocs_) hipFree(p);
  for (void* p : {(void*)d_samp_logits_, (void*)d_keys_, (void*)d_draws_, (void*)d_out_, d_wide_})
    if (p) hipFree(p);
  if (h_ctrl_) hipHostFree(h_ctrl_);
  if (h_gt_) hipHostFree(h_gt_);
  if (stream_) hipStreamDestroy(stream_);
}

#define RT_OK(x)                      \
  do {                                \
    int _r = (x);                     \
    if (_r != RWKVTTS_OK) return _r;  \
  } while (0)

int Engine::init(const rwkvtts_engine_desc& desc, const void* weights, size_t bytes, int on_device) {
  device_ = desc.device;
  RT_HIP(hipSetDevice(device_));
  {  // the token generator's latency-bound launch chain gets the highest queue priority, so a
     // vocoder sharing the GPU (codec.hip: lowest) fills the CUs it leaves idle
    int least = 0, greatest = 0;
    RT_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    RT_HIP(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest));
  }

  rwkvtts_blob_header hdr;
  if (on_device) {
    RT_HIP(hipMemcpy(&hdr, weights, sizeof(hdr), hipMemcpyDeviceToHost));
  } else {
    memcpy(&hdr, weights, sizeof(hdr));
  }
  RT_CHECK(hdr.magic == RWKVTTS_BLOB_MAGIC, RWKVTTS_EINVAL, "weight blob: bad magic");
  RT_CHECK(hdr.dtype == RWKVTTS_DTYPE_BF16 || hdr.dtype == RWKVTTS_DTYPE_F16, RWKVTTS_EUNSUPPORTED,
           "weight blob: matrices must be bf16 or f16");
  f16_ = hdr.dtype == RWKVTTS_DTYPE_F16 ? 1 : 0;
  dims = hdr.dims;
  const int C = dims.n_embd, F = dims.n_ffn;
  RT_CHECK(dims.head_size == 64, RWKVTTS_EUNSUPPORTED, "head_size must be 64");
  RT_CHECK(C % 128 == 0 && C <= 256 * kMaxPerThread, RWKVTTS_EUNSUPPORTED, "n_embd must be a multiple of 128, <= 2048");
  RT_CHECK(F % 128 == 0, RWKVTTS_EUNSUPPORTED, "n_ffn must be a multiple of 128");
  Dtot_ = dims.d_decay + dims.d_aaa + dims.d_mv + dims.d_gate;
  RT_CHECK(Dtot_ <= kMaxLoraTotal && dims.d_decay % 16 == 0 && dims.d_aaa % 16 == 0 &&
               dims.d_mv % 16 == 0 && dims.d_gate % 16 == 0,
           RWKVTTS_EUNSUPPORTED, "LoRA ranks must be multiples of 16, total <= 512");
  RT_CHECK((size_t)rwkvtts_blob_bytes(&dims) <= bytes, RWKVTTS_EINVAL, "weight blob too small");
  H_ = C / 64;
  Vpad_ = (int)align_up(dims.n_vocab, 16);
  ldA_ = 3 * C + Dtot_;
  S_ = std::max(1, desc.max_slots);
  chunk_ = desc.token_chunk_size > 0 ? desc.token_chunk_size : 512;
  Rmax_ = (int)align_up(std::max(chunk_, S_), 64);
  use_graphs_ = desc.use_graphs != 0;
  // split-K so that every GEMM slice is 128/256/512 deep and the grids fill the 256 CUs
  auto pick = [](int K, int want) {  // K slices of 128 / 256 / 512 (the GEMM kernels' shapes)
    int ks = std::max(128, std::min(std::min(want, 512), K));
    while (ks > 128 && K % ks) ks >>= 1;
    return K / ks;
  };
  // (K-slice depths measured at B = 32 and B = 1: twice or half the slices of any projection are
  // equal or slower, DESIGN.md §7.0 / §12, profiles/r04b1_splitk_ab.txt)
  splitA_ = pick(C, 256);  // r,k,v,LoRA-down: 53 col tiles x 4
  splitO_ = pick(C, 128);  // Wo: 16 col tiles x 8
  splitK_ = pick(C, 256);  // ffn key: 64 col tiles x 4
  splitF_ = pick(F, 256);  // ffn value: 16 col tiles x 16
  splitH_ = pick(C, 512);  // head: 129 col tiles x 2
  RT_CHECK(C % 128 == 0 && F % 128 == 0, RWKVTTS_EUNSUPPORTED, "K dims must be multiples of 128");
  RT_CHECK(splitA_ <= kMaxParts, RWKVTTS_EUNSUPPORTED, "n_embd too large for the WKV partial sum (raise kMaxParts)");
  state_perm_ = wkv_perm_layout(dims.d_decay, dims.d_aaa, dims.d_mv, dims.d_gate, splitA_, S_, desc.wkv_variant);
  // decode-step forms (rwkvtts_engine_desc.forms; 0 = the shipping forms, every bit bitwise-equal)
  constexpr uint32_t kKnownForms = RWKVTTS_FORM_SEPARATE_ATT | RWKVTTS_FORM_SEPARATE_FFN | RWKVTTS_FORM_LN_ROWS |
                                   RWKVTTS_FORM_SLAB_HANDOFF | RWKVTTS_FORM_SEPARATE_LNOUT |
                                   RWKVTTS_FORM_SEPARATE_EMBED | RWKVTTS_FORM_EXACT_SAMPLER;
  RT_CHECK((desc.forms & ~kKnownForms) == 0, RWKVTTS_EINVAL, "engine desc: unknown forms bits");
  att_persist_ = (desc.forms & RWKVTTS_FORM_SEPARATE_ATT) ? 0 : kPersistOn;
  ffn_persist_ = (desc.forms & RWKVTTS_FORM_SEPARATE_FFN) ? 0 : kPersistOn;
  fuse_ln1_ = !(desc.forms & RWKVTTS_FORM_LN_ROWS);
  gran_ = !(desc.forms & RWKVTTS_FORM_SLAB_HANDOFF);
  lnrow_ = !(desc.forms & RWKVTTS_FORM_SEPARATE_LNOUT);
  no_emb_fuse_ = (desc.forms & RWKVTTS_FORM_SEPARATE_EMBED) != 0;
  exact_sampler_ = (desc.forms & RWKVTTS_FORM_EXACT_SAMPLER) != 0;
  if ((ffn_persist_ || att_persist_) && !claim_persistent(desc.device, this, &lock_fd_)) ffn_persist_ = att_persist_ = 0;
  // debug instrumentation (tools/: stamps of one layer's launches, the launch timeline), off in
  // production: RWKVTTS_DEBUG_STAMPS="kind=path[;kind=path...]", kind one of gemm (layer-5 rkv /
  // value GEMM), ffn / att (layer-5 persistent-launch block stamps), timeline (per-launch start /
  // end of every decode step), adv (k_advance phases), wkv (layer-5 WKV phases)
  if (const char* ds = getenv("RWKVTTS_DEBUG_STAMPS")) {
    std::string spec(ds);
    size_t pos = 0;
    while (pos < spec.size()) {
      size_t end = spec.find(';', pos);
      if (end == std::string::npos) end = spec.size();
      const std::string item = spec.substr(pos, end - pos);
      pos = end + 1;
      const size_t eq = item.find('=');
      if (eq == std::string::npos) continue;
      const std::string kind = item.substr(0, eq), path = item.substr(eq + 1);
      if (kind == "gemm") {
        dbg_gstamp_path_ = path;
        RT_OK(alloc(&dbg_gstamps_, 2 * 4096 * 4));
      } else if (kind == "ffn") {
        dbg_fstamp_path_ = path;
        RT_OK(alloc(&dbg_fstamps_, 1024 * 4));
      } else if (kind == "att") {
        dbg_astamp2_path_ = path;
        RT_OK(alloc(&dbg_astamps2_, 2048 * 4));
      } else if (kind == "timeline") {
        tl_path_ = path;
        RT_OK(alloc(&d_tl_, (size_t)kTlStride * kTlMax));
      } else if (kind == "adv") {
        dbg_astamp_path_ = path;
        RT_OK(alloc(&dbg_astamps_, 256 * 16));
      } else if (kind == "wkv") {
        dbg_stamp_path_ = path;
        RT_OK(alloc(&dbg_stamps_, 4096 * 8));
      }
    }
  }

  // weights
  const size_t wbytes = (size_t)rwkvtts_blob_bytes(&dims);
  RT_OK(alloc(&wblob_, wbytes));
  RT_HIP(hipMemcpy(wblob_, weights, wbytes, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice));
  auto T = [&](int l, int t) { return (const void*)(wblob_ + rwkvtts_tensor_offset(&dims, l, t)); };
  emb_ = (const bf16_t*)T(-1, RWKVTTS_T_EMB);
  head_ = (const bf16_t*)T(-1, RWKVTTS_T_HEAD);
  ln0_w_ = (const float*)T(-1, RWKVTTS_T_LN0_W);
  ln0_b_ = (const float*)T(-1, RWKVTTS_T_LN0_B);
  lnout_w_ = (const float*)T(-1, RWKVTTS_T_LNOUT_W);
  lnout_b_ = (const float*)T(-1, RWKVTTS_T_LNOUT_B);
  L_.resize(dims.n_layer);
  for (int l = 0; l < dims.n_layer; ++l) {
    LayerW& w = L_[l];
    auto Fv = [&](int t) { return (const float*)T(l, t); };
    auto Mv = [&](int t) { return (const bf16_t*)T(l, t); };
    w.ln1_w = Fv(RWKVTTS_L_LN1_W); w.ln1_b = Fv(RWKVTTS_L_LN1_B);
    w.ln2_w = Fv(RWKVTTS_L_LN2_W); w.ln2_b = Fv(RWKVTTS_L_LN2_B);
    w.mu[0] = Fv(RWKVTTS_L_XR); w.mu[1] = Fv(RWKVTTS_L_XW); w.mu[2] = Fv(RWKVTTS_L_XK);
    w.mu[3] = Fv(RWKVTTS_L_XV); w.mu[4] = Fv(RWKVTTS_L_XA); w.mu[5] = Fv(RWKVTTS_L_XG);
    w.w0 = Fv(RWKVTTS_L_W0); w.a0 = Fv(RWKVTTS_L_A0); w.v0 = Fv(RWKVTTS_L_V0);
    w.k_k = Fv(RWKVTTS_L_KK); w.k_a = Fv(RWKVTTS_L_KA); w.r_k = Fv(RWKVTTS_L_RK);
    w.lnx_w = Fv(RWKVTTS_L_LNX_W); w.lnx_b = Fv(RWKVTTS_L_LNX_B); w.ffn_xk = Fv(RWKVTTS_L_FFN_XK);
    w.wr = Mv(RWKVTTS_L_WR); w.wk = Mv(RWKVTTS_L_WK); w.wv = Mv(RWKVTTS_L_WV); w.wo = Mv(RWKVTTS_L_WO);
    w.w1t = Mv(RWKVTTS_L_W1T); w.a1t = Mv(RWKVTTS_L_A1T); w.v1t = Mv(RWKVTTS_L_V1T); w.g1t = Mv(RWKVTTS_L_G1T);
    w.w2t = Mv(RWKVTTS_L_W2T); w.a2t = Mv(RWKVTTS_L_A2T); w.v2t = Mv(RWKVTTS_L_V2T); w.g2t = Mv(RWKVTTS_L_G2T);
    w.ffn_k = Mv(RWKVTTS_L_FFN_K); w.ffn_v = Mv(RWKVTTS_L_FFN_V);
  }
  RT_OK(alloc(&lora_pack_, (size_t)dims.n_layer * C * Dtot_));
  RT_HIP(hipDeviceSynchronize());  // alloc's memset runs on the null stream; stream_ is non-blocking
  for (int l = 0; l < dims.n_layer; ++l) {
    LayerW& w = L_[l];
    bf16_t* dst = lora_pack_ + (size_t)l * C * Dtot_;
    if (state_perm_ == 2)  // k_wkv6 (0.4B LoRA ranks): its coalesced register order
      launch_pack_lora6(w.w2t, w.a2t, w.v2t, w.g2t, C, dst, stream_);
    else if (state_perm_ == 1)  // k_wkv4
      launch_pack_lora4(w.w2t, w.a2t, w.v2t, w.g2t, C, dst, stream_);
    else
      launch_pack_lora(w.w2t, w.a2t, w.v2t, w.g2t, C, dims.d_decay, dims.d_aaa, dims.d_mv, dims.d_gate, dst, stream_);
    RT_HIP(hipGetLastError());
    w.lup = dst;
  }
  // quantised layers (web-rwkv ModelBuilder::quant, bin/server.rs:1029-1071): codes + scales of
  // the r / k / v / o / FFN matrices from the blob's row-major 16-bit copies
  {
    const int qt = desc.quant_type, ql = std::min(std::max(desc.quant_layers, 0), (int)dims.n_layer);
    RT_CHECK(qt >= RWKVTTS_QUANT_NONE && qt <= RWKVTTS_QUANT_SF4, RWKVTTS_EINVAL, "unknown quant_type");
    RT_CHECK(!(qt == RWKVTTS_QUANT_SF4 && ql > 0), RWKVTTS_EUNSUPPORTED,
             "quant_type sf4: its code table is not available (web-rwkv not vendored)");
    if (qt != RWKVTTS_QUANT_NONE && ql > 0) {
      RT_CHECK(C % kQ8Block == 0 && F % kQ8Block == 0, RWKVTTS_EUNSUPPORTED, "quantisation needs K % 128 == 0");
      const size_t cb_cc = quant_code_bytes(qt, C, C), sb_cc = quant_scale_bytes(qt, C, C);
      const size_t cb_fc = quant_code_bytes(qt, F, C), sb_fc = quant_scale_bytes(qt, F, C);
      const size_t per_layer = 4 * cb_cc + 2 * cb_fc + 4 * sb_cc + 2 * sb_fc;
      uint8_t* qbuf = nullptr;
      RT_OK(alloc(&qbuf, per_layer * ql));
      RT_HIP(hipDeviceSynchronize());  // alloc's memset runs on the null stream
      for (int l = 0; l < ql; ++l) {
        LayerW& w = L_[l];
        uint8_t* q = qbuf + per_layer * l;
        uint8_t* sc = q + 4 * cb_cc + 2 * cb_fc;
        w.quant = qt;
        w.q_rkv = q; w.s_rkv = sc;
        for (int j = 0; j < 3; ++j)
          launch_quant_pack((const uint16_t*)(j == 0 ? w.wr : j == 1 ? w.wk : w.wv), C, C, f16_, qt,
                            q + j * cb_cc, sc + j * sb_cc, stream_);
        w.q_o = q + 3 * cb_cc; w.s_o = sc + 3 * sb_cc;
        launch_quant_pack((const uint16_t*)w.wo, C, C, f16_, qt, (uint8_t*)w.q_o, (void*)w.s_o, stream_);
        w.q_fk = q + 4 * cb_cc; w.s_fk = sc + 4 * sb_cc;
        launch_quant_pack((const uint16_t*)w.ffn_k, F, C, f16_, qt, (uint8_t*)w.q_fk, (void*)w.s_fk, stream_);
        w.q_fv = q + 4 * cb_cc + cb_fc; w.s_fv = sc + 4 * sb_cc + sb_fc;
        launch_quant_pack((const uint16_t*)w.ffn_v, C, F, f16_, qt, (uint8_t*)w.q_fv, (void*)w.s_fv, stream_);
      }
      RT_HIP(hipGetLastError());
      RT_HIP(hipStreamSynchronize(stream_));
      // f16 models: per launch, the shift that brings the largest dequantised |w| to ~2^14
      // (int8: max(|min|, |max|) of the blocks; nf4: the largest block absmax)
      auto shift_of = [&](const void* scales, size_t bytes) -> int {
        std::vector<uint16_t> h(bytes / 2);
        if (hipMemcpy(h.data(), scales, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 0;
        float mx = 0.0f;
        for (uint16_t v : h) mx = std::max(mx, std::fabs(f16_to_f32(v)));
        if (!(mx > 0.0f) || !std::isfinite(mx)) return 0;
        return std::max(0, std::min(24, 14 - (int)std::ceil(std::log2(mx))));
      };
      if (f16_)
        for (int l = 0; l < ql; ++l) {
          LayerW& w = L_[l];
          w.qs_rkv = shift_of(w.s_rkv, 3 * sb_cc);
          w.qs_o = shift_of(w.s_o, sb_cc);
          w.qs_fk = shift_of(w.s_fk, sb_fc);
          w.qs_fv = shift_of(w.s_fv, sb_fc);
        }
    }
  }
  // GEMM matrices -> MFMA fragment blocks (k_gemm streams each wave's weights as contiguous 1 KB
  // blocks); the blob's row-major copies stay for the embedding gather and the oracle layout
  {
    auto packed_elems = [](int N, int K) { return (size_t)((N + 15) / 16) * 16 * K; };
    const int Dw = dims.d_decay, Da = dims.d_aaa, Dv = dims.d_mv, Dg = dims.d_gate;
    // the r, k, v and LoRA-down matrices are padded to 64-column tiles, back to back, so the
    // rkv launch finds tile t's weights at a fixed stride (gemm_tile_table)
    auto packed64 = [](int N, int K) { return (size_t)((N + 63) / 64) * 64 * K; };
    size_t per_layer = 3 * packed64(C, C) + packed64(Dw, C) + packed64(Da, C) + packed64(Dv, C) +
                       packed64(Dg, C) + packed_elems(C, C) + packed_elems(F, C) + packed_elems(C, F);
    size_t total = per_layer * dims.n_layer + packed_elems(dims.n_vocab, C);
    RT_OK(alloc(&wpack_, total));
    RT_HIP(hipDeviceSynchronize());  // alloc's memset runs on the null stream; stream_ is non-blocking
    bf16_t* dst = wpack_;
    auto pack = [&](const bf16_t*& Wm, int N, int K, bool tile64 = false) {
      launch_pack_frag(Wm, N, K, dst, stream_);
      Wm = dst;
      dst += tile64 ? packed64(N, K) : packed_elems(N, K);
    };
    for (int l = 0; l < dims.n_layer; ++l) {
      LayerW& w = L_[l];
      pack(w.wr, C, C, true); pack(w.wk, C, C, true); pack(w.wv, C, C, true);
      pack(w.w1t, Dw, C, true); pack(w.a1t, Da, C, true); pack(w.v1t, Dv, C, true); pack(w.g1t, Dg, C, true);
      pack(w.wo, C, C); pack(w.ffn_k, F, C); pack(w.ffn_v, C, F);
    }
    pack(head_, dims.n_vocab, C);
    RT_HIP(hipGetLastError());
  }
  RT_HIP(hipStreamSynchronize(stream_));
  // state
  const int64_t Lc = dims.n_layer;
  RT_OK(alloc(&wkv_, (size_t)S_ * Lc * H_ * 64 * 64));
  RT_OK(alloc(&att_sh_, (size_t)2 * S_ * Lc * C));
  RT_OK(alloc(&ffn_sh_, (size_t)2 * S_ * Lc * C));
  RT_OK(alloc(&slot_par_, (size_t)S_));
  par_host_.assign(S_, 0);
  ctrl_stage_.assign(S_, SlotCtrl{});
  // tables
  RT_OK(alloc(&d_tok_, (size_t)Rmax_));
  RT_OK(alloc(&d_rows_, (size_t)Rmax_));
  RT_OK(alloc(&d_segs_, (size_t)std::max(Rmax_, S_)));
  RT_OK(alloc(&d_lg_rows_, (size_t)Rmax_));
  RT_OK(alloc(&d_lg_slot_, (size_t)Rmax_));
  // scratch
  const size_t RC = (size_t)Rmax_ * C;
  RT_OK(alloc(&h0_, RC));
  RT_OK(alloc(&h1_, RC));
  RT_OK(alloc(&xm_hi_, 6 * RC));
  RT_OK(alloc(&xm_lo_, 6 * RC));
  RT_OK(alloc(&partA_, (size_t)splitA_ * Rmax_ * ldA_));
  RT_OK(alloc(&z_hi_, RC));
  RT_OK(alloc(&z_lo_, RC));
  RT_OK(alloc(&partO_, (size_t)splitO_ * RC));
  RT_OK(alloc(&xf_hi_, RC));
  RT_OK(alloc(&xf_lo_, RC));
  if (!f16_) {  // relu(k)^2 planes of bf16 prefill steps (launch_relu2_planes)
    RT_OK(alloc(&xk_hi_, (size_t)Rmax_ * F));
    RT_OK(alloc(&xk_lo_, (size_t)Rmax_ * F));
  }
  RT_OK(alloc(&partK_, (size_t)splitK_ * Rmax_ * F));
  RT_OK(alloc(&partF_, (size_t)splitF_ * RC));
  // k_ffn_persist hand-off counters: one block per layer (zeroed here; each launch zeroes the
  // previous layer's block)
  RT_OK(alloc(&ffn_sync_, (size_t)Lc * kFfnSyncInts));
  RT_OK(alloc(&att_sync_, (size_t)Lc * kAttSyncInts));  // k_att_persist's, the same scheme
  sync_bufs_ = {{ffn_sync_, (size_t)Lc * kFfnSyncInts * sizeof(int)},
                {att_sync_, (size_t)Lc * kAttSyncInts * sizeof(int)}};
  for (auto& b : sync_bufs_) RT_HIP(hipMemset(b.first, 0, b.second));
  if (const char* dr = getenv("RWKVTTS_TEST_DROP_ARRIVE")) {  // test hook: n units with a dropped arrival
    RT_OK(alloc(&d_drop_, 64));
    const int one = 1;
    RT_HIP(hipMemcpy(d_drop_, &one, sizeof(int), hipMemcpyHostToDevice));
    test_drops_left_ = std::max(1, atoi(dr)) - 1;  // re-armed after each recovery
  }
  RT_OK(alloc(&vfirst_, RC));
  RT_OK(alloc(&xo_hi_, RC));
  RT_OK(alloc(&xo_lo_, RC));
  RT_OK(alloc(&logits_, (size_t)splitH_ * Rmax_ * Vpad_));
  // S_ slot control blocks + one block whose first word is the persistent FFN give-up code
  // (snapshotted with the slots, so a timed-out hand-off fails the unit that ran it)
  RT_OK(alloc(&d_ctrl_, (size_t)S_ + 1));
  RT_HIP(hipMemset(d_ctrl_ + S_, 0, sizeof(SlotCtrl)));
  RT_OK(alloc(&d_sem_, (size_t)S_ * RWKVTTS_SEMANTIC_LIMIT));
  RT_HIP(hipHostMalloc((void**)&h_ctrl_, sizeof(SlotCtrl) * 2 * (S_ + 1), hipHostMallocDefault));  // 2 snapshots
  // granule hand-off of the one-row FFN form (FfnSync::gran): four key splits x F granules, and the
  // pass counter that tags them (starts at 1: a zeroed granule never carries a live tag)
  if (gran_) {
    RT_OK(alloc(&d_gran_, (size_t)ffn_gran_count(4, dims.n_ffn)));
    RT_OK(alloc(&d_epoch_, 64));
    const int one = 1;
    RT_HIP(hipMemcpy(d_epoch_, &one, sizeof(int), hipMemcpyHostToDevice));
    sync_bufs_.push_back({(int*)d_gran_, (size_t)ffn_gran_count(4, dims.n_ffn) * sizeof(uint64_t)});
    const int64_t ng = att_gran_count((int)dims.n_embd);
    RT_OK(alloc(&d_gran_att_, (size_t)ng));
    sync_bufs_.push_back({(int*)d_gran_att_, (size_t)ng * sizeof(uint64_t)});
  }

  RT_HIP(hipDeviceSynchronize());
  return RWKVTTS_OK;
}

int64_t Engine::state_floats() const {
  const int64_t C = dims.n_embd;
  return (int64_t)dims.n_layer * (2 * C + (int64_t)H_ * 64 * 64);
}

int Engine::slot_reset(int slot, bool sync) {
  RT_CHECK(slot >= 0 && slot < S_, RWKVTTS_EINVAL, "slot out of range");
  RT_HIP(hipSetDevice(device_));
  const int64_t C = dims.n_embd, Lc = dims.n_layer, per = Lc * H_ * 64 * 64;
  RT_HIP(hipMemsetAsync(wkv_ + slot * per, 0, per * 4, stream_));
  for (int p = 0; p < 2; ++p) {
    RT_HIP(hipMemsetAsync(att_sh_ + ((int64_t)p * S_ + slot) * Lc * C, 0, Lc * C * 4, stream_));
    RT_HIP(hipMemsetAsync(ffn_sh_ + ((int64_t)p * S_ + slot) * Lc * C, 0, Lc * C * 4, stream_));
  }
  par_host_[slot] = 0;
  RT_HIP(hipMemcpyAsync(slot_par_ + slot, &par_host_[slot], 4, hipMemcpyHostToDevice, stream_));
  if (sync) RT_HIP(hipStreamSynchronize(stream_));
  return RWKVTTS_OK;
}

// Coalesced state layouts of one (slot, layer, head) block, in the WKV kernel's register order:
// layout 1 (k_wkv4): thread t = 2 i + (j >> 5) owns row i, half j >> 5; its q-th float4 (columns
// 32 hf + 4 q .. + 3) lives at float4 index q * 128 + t. Layout 2 (k_wkv6): t = 4 i + (j >> 4),
// q-th float4 at q * 256 + t. Either way each wave-wide load / store is 1 KB contiguous.
static inline int64_t perm_index(int kind, int i, int j) {
  if (kind == 1) {
    const int t = 2 * i + (j >> 5), q = (j & 31) >> 2, e = j & 3;
    return ((int64_t)q * 128 + t) * 4 + e;
  }
  const int t = 4 * i + (j >> 4), q = (j & 15) >> 2, e = j & 3;
  return ((int64_t)q * 256 + t) * 4 + e;
}
void Engine::state_permute(const float* std_block, float* dev_block) {
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) dev_block[perm_index(state_perm_, i, j)] = std_block[i * 64 + j];
}
void Engine::state_unpermute(const float* dev_block, float* std_block) {
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) std_block[i * 64 + j] = dev_block[perm_index(state_perm_, i, j)];
}

int Engine::slot_read(int slot, float* out) {
  RT_CHECK(slot >= 0 && slot < S_, RWKVTTS_EINVAL, "slot out of range");
  RT_HIP(hipSetDevice(device_));
  RT_HIP(hipStreamSynchronize(stream_));
  const int64_t C = dims.n_embd, Lc = dims.n_layer, HNN = (int64_t)H_ * 64 * 64;
  int par = 0;
  RT_HIP(hipMemcpy(&par, slot_par_ + slot, 4, hipMemcpyDeviceToHost));
  for (int64_t l = 0; l < Lc; ++l) {
    float* o = out + l * (2 * C + HNN);
    RT_HIP(hipMemcpy(o, att_sh_ + (((int64_t)par * S_ + slot) * Lc + l) * C, C * 4, hipMemcpyDeviceToHost));
    RT_HIP(hipMemcpy(o + C, wkv_ + ((int64_t)slot * Lc + l) * HNN, HNN * 4, hipMemcpyDeviceToHost));
    if (state_perm_) {  // device layout -> S[i][j] per head
      std::vector<float> tmp(o + C, o + C + HNN);
      for (int h = 0; h < H_; ++h) state_unpermute(tmp.data() + (int64_t)h * 4096, o + C + (int64_t)h * 4096);
    }
    RT_HIP(hipMemcpy(o + C + HNN, ffn_sh_ + (((int64_t)par * S_ + slot) * Lc + l) * C, C * 4, hipMemcpyDeviceToHost));
  }
  return RWKVTTS_OK;
}

int Engine::slot_write(int slot, const float* in) {
  RT_CHECK(slot >= 0 && slot < S_, RWKVTTS_EINVAL, "slot out of range");
  RT_HIP(hipSetDevice(device_));
  RT_HIP(hipStreamSynchronize(stream_));
  const int64_t C = dims.n_embd, Lc = dims.n_layer, HNN = (int64_t)H_ * 64 * 64;
  par_host_[slot] = 0;
  RT_HIP(hipMemcpy(slot_par_ + slot, &par_host_[slot], 4, hipMemcpyHostToDevice));
  for (int64_t l = 0; l < Lc; ++l) {
    const float* o = in + l * (2 * C + HNN);
    RT_HIP(hipMemcpy(att_sh_ + (((int64_t)0 * S_ + slot) * Lc + l) * C, o, C * 4, hipMemcpyHostToDevice));
    if (state_perm_) {  // S[i][j] per head -> device layout
      std::vector<float> tmp(HNN);
      for (int h = 0; h < H_; ++h) state_permute(o + C + (int64_t)h * 4096, tmp.data() + (int64_t)h * 4096);
      RT_HIP(hipMemcpy(wkv_ + ((int64_t)slot * Lc + l) * HNN, tmp.data(), HNN * 4, hipMemcpyHostToDevice));
    } else {
      RT_HIP(hipMemcpy(wkv_ + ((int64_t)slot * Lc + l) * HNN, o + C, HNN * 4, hipMemcpyHostToDevice));
    }
    RT_HIP(hipMemcpy(ffn_sh_ + (((int64_t)0 * S_ + slot) * Lc + l) * C, o + C + HNN, C * 4, hipMemcpyHostToDevice));
  }
  return RWKVTTS_OK;
}

// ------------------------------------------------------------------------------------------
// forward step
// ------------------------------------------------------------------------------------------
__global__ void k_rows_parity(int4* rows, const int* slot_par, int R) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) rows[r].w = slot_par[rows[r].x];
}
__global__ void k_sum_partials(float* p, int64_t part_stride, int n_part, int ld, int rows, int cols) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * cols) return;
  const int64_t o = (i / cols) * ld + (i % cols);
  float v = p[o];
  for (int q = 1; q < n_part; ++q) v += p[q * part_stride + o];
  p[o] = v;
}
__global__ void k_flip_parity(const int4* segs, int* slot_par, int n_seg) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n_seg) slot_par[segs[s].x] ^= 1;
}

// Profiling window around one launcher call: the launches inside stamp the two events with
// their own start / end (RT_LAUNCH, common.h). A window whose launcher issued nothing (an
// ablated kernel) gets plain markers.
void Engine::prof_begin(hipEvent_t* ev) {
  *ev = nullptr;
  if (!profiling) return;
  hipEvent_t e2;
  hipEventCreate(ev);
  hipEventCreate(&e2);
  launch_timing() = LaunchTiming{*ev, e2, 0};
}
void Engine::prof_end(const char* name, hipEvent_t ev) {
  if (!profiling || !ev) return;
  LaunchTiming& lt = launch_timing();
  if (lt.launches == 0) {
    hipEventRecord(lt.start, stream_);
    hipEventRecord(lt.stop, stream_);
  }
  pending_prof_.push_back({std::string(name) + "#begin", lt.start});
  pending_prof_.push_back({name, lt.stop});
  lt = LaunchTiming{};
}
int Engine::flush_prof() {
  if (pending_prof_.empty()) return RWKVTTS_OK;
  RT_HIP(hipStreamSynchronize(stream_));
  for (size_t i = 0; i + 1 < pending_prof_.size(); i += 2) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, pending_prof_[i].second, pending_prof_[i + 1].second);
    const std::string& nm = pending_prof_[i + 1].first;
    auto it = std::find_if(prof.begin(), prof.end(), [&](const ProfEntry& e) { return e.name == nm; });
    if (it == prof.end()) {
      prof.push_back({nm, 0, 0.0});
      it = prof.end() - 1;
    }
    it->launches++;
    it->ms += ms;
    hipEventDestroy(pending_prof_[i].second);
    hipEventDestroy(pending_prof_[i + 1].second);
  }
  pending_prof_.clear();
  return RWKVTTS_OK;
}

// prefill steps with more rows than this take the relu^2-plane route for the FFN value GEMM
static constexpr int kPlaneRows = 64;

int Engine::launch_forward(int R, int n_seg, int n_lg, int head_rows, bool tok_from_ctrl, bool advance) {
  const int C = dims.n_embd, F = dims.n_ffn, Lc = dims.n_layer;
  hipEvent_t ev;
  const int nb = (R + 255) / 256;
  // decode steps (tokens from the control blocks, one row per slot) keep each slot's shift
  // state in place: no parity refresh / flip kernels (rows[].w was set once at upload)
  const bool inplace = tok_from_ctrl;
  if (!inplace) hipLaunchKernelGGL(k_rows_parity, dim3(nb), dim3(256), 0, stream_, d_rows_, slot_par_, R);
  tl_n_ = 0;
  if (tl_base()) tl_names_.clear();  // the names of this forward's launches (decode steps have one fewer)
  // decode steps: the embedding (token -> row -> LN0) runs inside layer 0's LayerNorm launch (one
  // launch and one boundary fewer per step; k_embed's arithmetic, bit for bit). Prefill steps keep
  // k_embed (their token-shift rows need the previous token's embedding as well).
  const bool emb_fused = inplace && C == 1024 && !no_emb_fuse_;
  // persistent launches (k_att_persist / k_ffn_persist) run for EVERY layer of a decode forward or
  // for none: each launch zeroes the previous layer's hand-off counters, so a layer that fell back
  // to the separate launches would leave its successor's counters dirty. Quantised layers and the
  // debug paths take the separate launches; the attention form needs layer 0's embedding fusion
  // (its LayerNorm reads no slabs otherwise). Layer 0 tries; if its shapes are not covered, the
  // whole forward falls back.
  bool any_quant = false;
  for (const LayerW& lw : L_) any_quant = any_quant || lw.quant != 0;
  // (every row count: with the 1-us weight-stream hold the persistent halves win at B = 1, 8 and 32,
  // profiles/r04h7_small_batch_ab.txt)
  bool use_att = att_persist_ && inplace && Lc >= 2 && !dbg_stamps_ && !dbg_gstamps_ && !any_quant && emb_fused;
  bool use_ffn = ffn_persist_ && inplace && Lc >= 2 && !dbg_gstamps_ && !any_quant;
  // one-row passes: the FFN key -> value hand-off as granules, live once the layer-0 attention
  // launch (which bumps the pass epoch) has been issued
  const bool gran_pass = gran_ && d_gran_ && fuse_ln1_ && R == 1 && use_att && use_ffn;
  bool gran_live = false;
  if (!emb_fused) {
    prof_begin(&ev);
    launch_embed(d_tok_, d_rows_, &d_ctrl_[0].next_token, (int)(sizeof(SlotCtrl) / 4), emb_,
                 ln0_w_, ln0_b_, h0_, R, C, f16_, stream_, tl_next("embed"), dims.n_vocab);
    prof_end("embed", ev);
  }
  const int64_t RC = (int64_t)Rmax_ * C;
  // ---- att: residual (+ previous layer's ffn partials) -> LN1 -> 6 mixes (layer l's arguments)
  auto ln_att_args = [&](int l) {
    const LayerW& w = L_[l];
    LnMixArgs m{};
    m.f16 = f16_;
    m.h_in = h0_;
    m.h_out = h1_;
    m.part = partF_;
    m.n_part = l == 0 ? 0 : splitF_;
    m.ldp = C;
    m.part_stride = RC;
    m.ln_w = w.ln1_w;
    m.ln_b = w.ln1_b;
    m.n_mix = 6;
    for (int i = 0; i < 6; ++i) m.mu[i] = w.mu[i];
    m.x_hi = xm_hi_;
    m.x_lo = xm_lo_;
    m.mix_stride = RC;
    m.ldx = C;
    m.shift = att_sh_;
    m.S = S_;
    m.L = Lc;
    m.layer = l;
    m.C = C;
    m.rows = d_rows_;
    m.row_map = nullptr;
    m.inplace = inplace ? 1 : 0;
    m.wt = (kWtMask >> 6) & 1;
    if (l == 0 && emb_fused) {
      m.emb_tok = d_tok_;
      m.emb_ctrl = &d_ctrl_[0].next_token;
      m.emb_ctrl_stride = (int)(sizeof(SlotCtrl) / 4);
      m.emb = emb_;
      m.ln0_w = ln0_w_;
      m.ln0_b = ln0_b_;
      m.n_vocab = dims.n_vocab;
    }
    return m;
  };
  // ---- the final LayerNorm of the logits rows
  auto ln_out_args = [&]() {
    LnMixArgs o{};
    o.f16 = f16_;
    o.h_in = h0_;
    o.h_out = nullptr;
    o.part = partF_;
    o.n_part = splitF_;
    o.ldp = C;
    o.part_stride = RC;
    o.ln_w = lnout_w_;
    o.ln_b = lnout_b_;
    o.n_mix = 1;
    o.x_hi = xo_hi_;
    o.x_lo = xo_lo_;
    o.mix_stride = RC;
    o.ldx = C;
    o.shift = nullptr;
    o.C = C;
    o.row_map = d_lg_rows_;
    return o;
  };
  for (int l = 0; l < Lc; ++l) {
    const LayerW& w = L_[l];
    LnMixArgs m = ln_att_args(l);
    // ---- r, k, v and the LoRA-down projections (w, a, v, g) in one launch (7 segments)
    GemmArgs g{};
    g.f16 = f16_;
    int tiles = 0;
    auto seg = [&](int idx, const bf16_t* W, int mix, int N, int col_off) {
      g.seg[idx] = {W, xm_hi_ + mix * RC, xm_lo_ + mix * RC, C, N, col_off, tiles};
      tiles += (N + 63) / 64;
    };
    g.nseg = 7;
    seg(0, w.wr, 0, C, 0);
    seg(1, w.wk, 2, C, C);
    seg(2, w.wv, 3, C, 2 * C);
    seg(3, w.w1t, 1, dims.d_decay, 3 * C);
    seg(4, w.a1t, 4, dims.d_aaa, 3 * C + dims.d_decay);
    seg(5, w.v1t, 3, dims.d_mv, 3 * C + dims.d_decay + dims.d_aaa);
    seg(6, w.g1t, 5, dims.d_gate, 3 * C + dims.d_decay + dims.d_aaa + dims.d_mv);
    g.K = C; g.M = R; g.k_split = splitA_; g.kslice = C / splitA_;
    gemm_tile_table(g, RC);
    if (w.quant) {  // r, k, v (tiles of segments 0-2) quantised; the LoRA-down tiles stay 16-bit
      RT_CHECK(g.n_tinfo > 0, RWKVTTS_EUNSUPPORTED, "quantised rkv launch needs the per-tile table");
      g.q_fmt = w.quant; g.qw = w.q_rkv; g.qs = w.s_rkv; g.q_shift = w.qs_rkv;
      for (int t = 0; t < 3 * C / 64; ++t) g.tinfo[t] |= 1u << 31;
    }
    g.xmode = kXPlanes; g.out = partA_; g.split_stride = (int64_t)Rmax_ * ldA_; g.ldo = ldA_;
    g.allow_xmap = kXmapMask & 1;
    g.xalign = (kXalignMask & 1) ? 1 : 0;  // r / k / v tile h (head h) on the XCD of WKV head h
    g.wt = kWtMask & 1;
    g.stamps = (l == 5 && dbg_gstamps_) ? dbg_gstamps_ : nullptr;
    // ---- WKV + LoRA-up + GroupNorm + bonus + gate
    WkvArgs k{};
    k.f16 = f16_;
    k.part = partA_; k.n_part = splitA_; k.ldp = ldA_; k.part_stride = (int64_t)Rmax_ * ldA_;
    k.lup = w.lup;
    k.w2t = w.w2t; k.a2t = w.a2t; k.v2t = w.v2t; k.g2t = w.g2t;
    k.w0 = w.w0; k.a0 = w.a0; k.v0 = w.v0; k.k_k = w.k_k; k.k_a = w.k_a; k.r_k = w.r_k;
    k.lnx_w = w.lnx_w; k.lnx_b = w.lnx_b;
    k.state = wkv_; k.slot_stride = (int64_t)Lc * H_ * 64 * 64; k.layer_off = (int64_t)l * H_ * 64 * 64;
    k.v_first = vfirst_; k.ldv = C; k.z_hi = z_hi_; k.z_lo = z_lo_; k.ldz = C;
    k.segs = d_segs_; k.layer = l; k.C = C; k.n_slots = S_; k.n_seg = n_seg; k.multi_row = R > n_seg;
    k.perm = state_perm_;
    k.allow_xmap = (kXmapMask >> 5) & 1;
    k.wt = (kWtMask >> 5) & 1;
    k.Dw = dims.d_decay; k.Da = dims.d_aaa; k.Dv = dims.d_mv; k.Dg = dims.d_gate;
    k.stamps = (l == 5) ? dbg_stamps_ : nullptr;
    // ---- output projection (split-K partials)
    GemmArgs go{};
    go.f16 = f16_;
    go.nseg = 1;
    go.seg[0] = {w.wo, z_hi_, z_lo_, C, C, 0, 0};
    go.K = C; go.M = R; go.k_split = splitO_; go.kslice = C / splitO_;
    go.xmode = kXPlanes; go.out = partO_; go.split_stride = RC; go.ldo = C;
    go.allow_xmap = (kXmapMask >> 1) & 1;
    if (w.quant) { go.q_fmt = w.quant; go.qw = w.q_o; go.qs = w.s_o; go.q_shift = w.qs_o; }
    go.wt = (kWtMask >> 1) & 1;
    // ---- ffn: residual + Wo partials -> LN2 -> mix
    LnMixArgs f = m;
    f.emb = nullptr;  // (layer 0's embedding fusion belongs to the attention LayerNorm only)
    f.h_in = h1_;
    f.h_out = h0_;
    f.part = partO_;
    f.n_part = splitO_;
    f.ln_w = w.ln2_w;
    f.ln_b = w.ln2_b;
    f.n_mix = 1;
    f.mu[0] = w.ffn_xk;
    f.x_hi = xf_hi_;
    f.x_lo = xf_lo_;
    f.shift = ffn_sh_;
    f.wt = (kWtMask >> 7) & 1;
    // decode steps: the attention half as ONE persistent launch (k_att_persist: LN1 + mixes, rkv +
    // LoRA-down, WKV, Wo with in-launch hand-offs; bit-identical outputs) where the shapes allow it
    bool att_persisted = false;
    if (use_att) {
      m.tl = g.tl = k.tl = go.tl = tl_next("att_persist");
      prof_begin(&ev);
      att_persisted = launch_att_persist(m, g, k, go, att_sync_ + (size_t)l * kAttSyncInts,
                                         att_sync_ + (size_t)((l + Lc - 1) % Lc) * kAttSyncInts, (int*)(d_ctrl_ + S_),
                                         R, H_, stream_, l == 5 ? dbg_astamps2_ : nullptr, att_persist_ >> 1, d_drop_,
                                         fuse_ln1_, l == 0 && gran_pass ? d_epoch_ : nullptr,
                                         gran_live ? d_gran_att_ : nullptr, d_epoch_);
      if (att_persisted) {
        prof_end("att_persist", ev);
        if (l == 0 && gran_pass) gran_live = true;  // this pass's epoch is bumped
      } else {
        RT_CHECK(l == 0, RWKVTTS_EHIP, "persistent attention launch: a layer after layer 0 fell back");
        use_att = false;  // not covered: the separate launches for this whole forward
        if (tl_base() && tl_n_ > 0) {
          --tl_n_;
          if ((int)tl_names_.size() > tl_n_) tl_names_.resize(tl_n_);
        }
      }
    }
    if (!att_persisted) {
      m.tl = tl_next("ln_att");
      prof_begin(&ev);
      RT_CHECK(launch_ln_mix(m, R, stream_) >= 0, RWKVTTS_EUNSUPPORTED, "layer-0 embedding fusion: unsupported shape");
      prof_end("ln_mix_att", ev);
      g.tl = tl_next("gemm_rkv");
      prof_begin(&ev);
      launch_gemm(g, stream_);
      prof_end("gemm_rkv_lora", ev);
      k.tl = tl_next("wkv");
      prof_begin(&ev);
      launch_wkv(k, n_seg, H_, stream_);
      prof_end("wkv", ev);
      go.tl = tl_next("gemm_wo");
      prof_begin(&ev);
      launch_gemm(go, stream_);
      prof_end("gemm_wo", ev);
    }
    GemmArgs gk{};
    gk.f16 = f16_;
    gk.nseg = 1;
    gk.seg[0] = {w.ffn_k, xf_hi_, xf_lo_, C, F, 0, 0};
    gk.K = C; gk.M = R; gk.k_split = splitK_; gk.kslice = C / splitK_;
    gk.xmode = kXPlanes; gk.out = partK_; gk.split_stride = (int64_t)Rmax_ * F; gk.ldo = F;
    gk.allow_xmap = (kXmapMask >> 2) & 1;
    if (w.quant) { gk.q_fmt = w.quant; gk.qw = w.q_fk; gk.qs = w.s_fk; gk.q_shift = w.qs_fk; }
    // key tiles of value K-slice s on the XCD that runs slice s (value xmap: split = xcd + 8 j)
    if ((kXalignMask >> 2) & 1) gk.xalign = std::max(1, (F / splitF_) / 64);
    gk.wt = (kWtMask >> 2) & 1;
    GemmArgs gv{};
    gv.f16 = f16_;
    gv.nseg = 1;
    gv.seg[0] = {w.ffn_v, nullptr, nullptr, F, C, 0, 0};
    gv.K = F; gv.M = R; gv.k_split = splitF_; gv.kslice = F / splitF_;
    gv.xmode = kXRelu2; gv.x_part = partK_; gv.x_nsplit = splitK_; gv.x_ld = F;
    gv.x_part_stride = (int64_t)Rmax_ * F;
    const bool planes = xk_hi_ && R > kPlaneRows;
    if (planes) {
      // prefill steps: relu^2 planes once (every value column tile would otherwise re-read the
      // NX f32 key slabs of its K-slice); decode steps keep the fused staging (one launch fewer)
      gv.seg[0] = {w.ffn_v, xk_hi_, xk_lo_, F, C, 0, 0};
      gv.xmode = kXPlanes;
    }
    gv.out = partF_; gv.split_stride = RC; gv.ldo = C;
    gv.allow_xmap = (kXmapMask >> 3) & 1;
    if (w.quant) { gv.q_fmt = w.quant; gv.qw = w.q_fv; gv.qs = w.s_fv; gv.q_shift = w.qs_fv; }
    gv.wt = (kWtMask >> 3) & 1;
    gv.stamps = (l == 5 && dbg_gstamps_) ? dbg_gstamps_ + 4096 * 4 : nullptr;
    // decode steps: the whole FFN half as ONE persistent launch (k_ffn_persist, in-launch
    // hand-offs; bit-identical outputs) where the shapes allow it
    bool persisted = false;
    if (use_ffn) {
      f.tl = gk.tl = gv.tl = tl_next("ffn_persist");
      prof_begin(&ev);
      persisted = launch_ffn_persist(f, gk, gv, ffn_sync_ + (size_t)l * kFfnSyncInts,
                                     ffn_sync_ + (size_t)((l + Lc - 1) % Lc) * kFfnSyncInts,
                                     (int*)(d_ctrl_ + S_), R, stream_, l == 5 ? dbg_fstamps_ : nullptr,
                                     ffn_persist_ >> 1, fuse_ln1_, gran_live ? d_gran_ : nullptr, d_epoch_);
      if (persisted) {
        prof_end("ffn_persist", ev);
      } else {
        RT_CHECK(l == 0, RWKVTTS_EHIP, "persistent FFN launch: a layer after layer 0 fell back");
        use_ffn = false;
        if (tl_base() && tl_n_ > 0) {  // (the timeline slot goes to the three launches below)
          --tl_n_;
          if ((int)tl_names_.size() > tl_n_) tl_names_.resize(tl_n_);
        }
      }
    }
    if (!persisted) {
      f.tl = tl_next("ln_ffn");
      prof_begin(&ev);
      launch_ln_mix(f, R, stream_);
      prof_end("ln_mix_ffn", ev);
      prof_begin(&ev);
      gk.tl = tl_next("gemm_key");
      launch_gemm(gk, stream_);
      prof_end("gemm_ffn_key", ev);
      if (planes) launch_relu2_planes(partK_, splitK_, (int64_t)Rmax_ * F, F, F, R, xk_hi_, xk_lo_, stream_);
      prof_begin(&ev);
      gv.tl = tl_next("gemm_value");
      launch_gemm(gv, stream_);
      prof_end("gemm_ffn_value", ev);
    }
  }
  if (n_lg > 0) {
    LnMixArgs o = ln_out_args();
    // one-row steps: ln_out folded into the head GEMM (launch_gemm_lnrow) where covered
    const bool lnrow = lnrow_ && n_lg == 1 && R == 1;
    if (!lnrow) {
      o.tl = tl_next("ln_out");
      prof_begin(&ev);
      launch_ln_mix(o, n_lg, stream_);
      prof_end("ln_out", ev);
    }
    GemmArgs gh{};
    gh.f16 = f16_;
    gh.nseg = 1;
    gh.seg[0] = {head_, xo_hi_, xo_lo_, C, head_rows, 0, 0};
    gh.K = C; gh.M = n_lg; gh.k_split = splitH_; gh.kslice = C / splitH_;
    gh.xmode = kXPlanes; gh.out = logits_; gh.split_stride = (int64_t)Rmax_ * Vpad_; gh.ldo = Vpad_;
    gh.allow_xmap = (kXmapMask >> 4) & 1;
    gh.wt = (kWtMask >> 4) & 1;
    prof_begin(&ev);
    gh.tl = tl_next("gemm_head");
    bool headed = false;
    if (lnrow) {
      o.n_rows = 1;
      headed = launch_gemm_lnrow(gh, o, stream_);
      if (!headed) {  // not covered: the two launches
        prof_end("gemm_head", ev);
        o.tl = tl_next("ln_out");
        prof_begin(&ev);
        launch_ln_mix(o, n_lg, stream_);
        prof_end("ln_out", ev);
        prof_begin(&ev);
      }
    }
    if (!headed) launch_gemm(gh, stream_);
    prof_end("gemm_head", ev);
    if (advance) {
      AdvanceArgs a{};
      a.logits = logits_;
      a.ld = Vpad_;
      a.n_part = splitH_;
      a.part_stride = (int64_t)Rmax_ * Vpad_;
      a.row_slot = d_lg_slot_;
      a.ctrl = d_ctrl_;
      a.sem_out = d_sem_;
      a.n_rows = n_lg;
      a.tl = tl_next("advance");
      a.stamps = dbg_astamps_;
      prof_begin(&ev);
      launch_advance(a, stream_, exact_sampler_ ? 0 : 1);
      prof_end("sample_advance", ev);
    }
  }
  if (!inplace)
    hipLaunchKernelGGL(k_flip_parity, dim3((n_seg + 255) / 256), dim3(256), 0, stream_, d_segs_, slot_par_, n_seg);
  RT_HIP(hipGetLastError());
  return RWKVTTS_OK;
}

int Engine::upload_plan(const StepPlan& p) {
  const int R = (int)p.rows.size();
  if (!p.tok_from_ctrl) RT_HIP(hipMemcpyAsync(d_tok_, p.tok.data(), R * 4, hipMemcpyHostToDevice, stream_));
  RT_HIP(hipMemcpyAsync(d_rows_, p.rows.data(), R * sizeof(int4), hipMemcpyHostToDevice, stream_));
  RT_HIP(hipMemcpyAsync(d_segs_, p.segs.data(), p.segs.size() * sizeof(int4), hipMemcpyHostToDevice, stream_));
  if (!p.lg_rows.empty()) {
    RT_HIP(hipMemcpyAsync(d_lg_rows_, p.lg_rows.data(), p.lg_rows.size() * 4, hipMemcpyHostToDevice, stream_));
    RT_HIP(hipMemcpyAsync(d_lg_slot_, p.lg_slot.data(), p.lg_slot.size() * 4, hipMemcpyHostToDevice, stream_));
  }
  if (p.tok_from_ctrl)  // decode steps keep the parity fixed: set rows[].w once here
    hipLaunchKernelGGL(k_rows_parity, dim3((R + 255) / 256), dim3(256), 0, stream_, d_rows_, slot_par_, R);
  return RWKVTTS_OK;
}

// Runs one forward step. Decode steps (tok_from_ctrl) replay a cached hipGraph.
int Engine::set_graph_timing(bool on) {
  RT_HIP(hipSetDevice(device_));
  if (on && !d_gt_) {
    RT_OK(alloc(&d_gt_, (size_t)kTlStride * kTlMax));
    RT_HIP(hipHostMalloc((void**)&h_gt_, sizeof(unsigned long long) * 2 * kTlStride * kTlMax, hipHostMallocDefault));
  }
  if (on != gtime_) {  // the decode graphs carry (or drop) the timeline slots: recapture
    RT_HIP(hipStreamSynchronize(stream_));
    for (auto& g : graphs_) hipGraphExecDestroy(g.second);
    graphs_.clear();
    graph_names_.clear();
    gtime_ = on;
  }
  prof.clear();
  return RWKVTTS_OK;
}

int Engine::run_step(const StepPlan& p, bool upload) {
  const int R = (int)p.rows.size();
  RT_CHECK(R > 0 && R <= Rmax_, RWKVTTS_EINVAL, "step rows out of range");
  RT_CHECK(p.head_rows <= Vpad_, RWKVTTS_EINVAL, "head_rows > n_vocab");
  if (upload) RT_OK(upload_plan(p));
  const int n_seg = (int)p.segs.size(), n_lg = (int)p.lg_rows.size();
  if (p.tok_from_ctrl && use_graphs_ && !profiling) {
    auto key = std::make_pair(R, p.head_rows * 2 + (p.advance ? 1 : 0));
    auto it = graphs_.find(key);
    if (it == graphs_.end()) {
      // the one-launch step's argument table is uploaded before the capture (no synchronous copy
      // may happen inside it)
      // one capture at a time per process: engines owned by different threads (the manager's
      // workers) never capture / instantiate concurrently
      static std::mutex capture_mu;
      std::unique_lock<std::mutex> cap_lock(capture_mu);
      hipGraph_t graph;
      RT_HIP(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
      int rc = launch_forward(R, n_seg, n_lg, p.head_rows, true, p.advance);
      hipError_t ce = hipStreamEndCapture(stream_, &graph);
      RT_OK(rc);
      RT_HIP(ce);
      hipGraphExec_t exec;
      RT_HIP(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
      RT_HIP(hipGraphDestroy(graph));
      it = graphs_.emplace(key, exec).first;
      if (tl_base()) graph_names_[key] = tl_names_;
    }
    RT_HIP(hipGraphLaunch(it->second, stream_));
    last_graph_ = key;
    return RWKVTTS_OK;
  }
  last_graph_ = {-1, -1};
  RT_OK(launch_forward(R, n_seg, n_lg, p.head_rows, p.tok_from_ctrl, p.advance));
  return RWKVTTS_OK;
}

// ------------------------------------------------------------------------------------------
// Runtime<Rnn>::infer
// ------------------------------------------------------------------------------------------
int Engine::infer(const rwkvtts_input* in, int n, int head_rows, float* logits, int32_t* consumed,
                  int32_t* has_logits) {
  RT_HIP(hipSetDevice(device_));
  RT_CHECK(head_rows > 0 && head_rows <= dims.n_vocab, RWKVTTS_EINVAL, "head_rows out of range");
  StepPlan p;
  p.head_rows = head_rows;
  int budget = chunk_;
  std::vector<std::pair<int, int>> out_map;  // (input index, logits row index)
  for (int i = 0; i < n; ++i) {
    consumed[i] = 0;
    has_logits[i] = 0;
    const rwkvtts_input& b = in[i];
    RT_CHECK(b.slot >= 0 && b.slot < S_, RWKVTTS_EINVAL, "input slot out of range");
    for (int j = 0; j < i; ++j)
      RT_CHECK(in[j].slot != b.slot, RWKVTTS_EINVAL, "two inputs share a slot");
    const int take = std::min(b.n_tokens, budget);
    if (take <= 0) continue;
    const int r0 = (int)p.rows.size();
    for (int t = 0; t < take; ++t) {
      RT_CHECK(b.tokens[t] < (uint32_t)dims.n_vocab, RWKVTTS_EINVAL, "token id >= n_vocab");
      int flags = (t == 0 ? kRowFirst : 0) | (t == take - 1 ? kRowLast : 0);
      p.rows.push_back(make_int4(b.slot, flags, t == 0 ? -1 : r0 + t - 1, 0));
      p.tok.push_back(b.tokens[t]);
      if (b.option == RWKVTTS_OPT_FULL) {
        p.lg_rows.push_back(r0 + t);
        p.lg_slot.push_back(b.slot);
      }
    }
    p.segs.push_back(make_int4(b.slot, r0, take, 0));
    consumed[i] = take;
    budget -= take;
    if (b.option == RWKVTTS_OPT_LAST && take == b.n_tokens) {
      p.lg_rows.push_back(r0 + take - 1);
      p.lg_slot.push_back(b.slot);
      out_map.push_back({i, (int)p.lg_rows.size() - 1});
    } else if (b.option == RWKVTTS_OPT_FULL) {
      has_logits[i] = 1;
    }
  }
  if (p.rows.empty()) return RWKVTTS_OK;
  RT_OK(run_step(p, true));
  const int n_lg = (int)p.lg_rows.size();
  if (n_lg > 0 && logits) {
    if (splitH_ > 1) {
      const int64_t tot = (int64_t)n_lg * head_rows;
      hipLaunchKernelGGL(k_sum_partials, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream_, logits_,
                         (int64_t)Rmax_ * Vpad_, splitH_, Vpad_, n_lg, head_rows);
    }
    RT_HIP(hipMemcpy2DAsync(logits, (size_t)head_rows * 4, logits_, (size_t)Vpad_ * 4,
                            (size_t)head_rows * 4, n_lg, hipMemcpyDeviceToHost, stream_));
  }
  RT_HIP(hipStreamSynchronize(stream_));
  for (auto& om : out_map) has_logits[om.first] = 1;
  RT_OK(flush_prof());
  return dump_stamps();
}

// ------------------------------------------------------------------------------------------
// sample_logits_with_top_p_k on the device
// ------------------------------------------------------------------------------------------
// Test hook: k_advance on caller-given rows (see engine.h). Each row gets its own slot control
// block; logits are [n_rows][8193] host floats (one partial). Per step and row: out_tok = the
// token the step emitted (global or semantic; -1 if it emitted none: finished or stopped),
// out_used = draws the step consumed, out_phase = the phase after the step.
int Engine::debug_advance(const float* logits, int n_rows, const DebugAdvanceRow* rows, int exact, int n_steps,
                          int32_t* out_tok, int32_t* out_used, int32_t* out_phase) {
  RT_HIP(hipSetDevice(device_));
  RT_CHECK(n_rows > 0 && n_rows <= 4096 && n_steps > 0 && n_steps <= 64, RWKVTTS_EINVAL, "debug_advance: bad sizes");
  constexpr int LD = RWKVTTS_EOS_TOKEN + 1;
  std::vector<SlotCtrl> c(n_rows);
  for (int i = 0; i < n_rows; ++i) {
    const DebugAdvanceRow& r = rows[i];
    RT_CHECK((r.phase == kPhGlobal || r.phase == kPhSemantic) && r.top_k > 0 && r.n_sem >= 0 &&
                 r.n_sem + n_steps <= RWKVTTS_SEMANTIC_LIMIT && (r.mode == 0 || r.mode == 1),
             RWKVTTS_EINVAL, "debug_advance: bad row");
    SlotCtrl& x = c[i];
    memset(&x, 0, sizeof(x));
    x.mode = r.mode;
    x.phase = r.phase;
    x.n_sem = r.n_sem;
    x.sem_limit = RWKVTTS_SEMANTIC_LIMIT;
    x.hard_min = r.hard_min;
    x.fixed = r.fixed;
    x.top_k_g = x.top_k_s = r.top_k;
    x.win_bits = r.win_bits;
    x.win_len = r.win_len;
    memcpy(x.gkey, r.key, 32);
    memcpy(x.skey, r.key, 32);
    x.gdraw = x.sdraw = r.draw;
  }
  float* d_lg = nullptr;
  SlotCtrl* d_c = nullptr;
  int32_t *d_slot = nullptr, *d_sem = nullptr;
  auto cleanup = [&] {
    for (void* p : {(void*)d_lg, (void*)d_c, (void*)d_slot, (void*)d_sem})
      if (p) hipFree(p);
  };
  int rc = RWKVTTS_OK;
  do {
    if (hipMalloc(&d_lg, (size_t)n_rows * LD * 4) != hipSuccess || hipMalloc(&d_c, sizeof(SlotCtrl) * n_rows) != hipSuccess ||
        hipMalloc(&d_slot, 4 * (size_t)n_rows) != hipSuccess ||
        hipMalloc(&d_sem, 4 * (size_t)n_rows * RWKVTTS_SEMANTIC_LIMIT) != hipSuccess) {
      set_error("debug_advance: allocation");
      rc = RWKVTTS_ENOMEM;
      break;
    }
    std::vector<int32_t> slot(n_rows);
    for (int i = 0; i < n_rows; ++i) slot[i] = i;
    if (hipMemcpy(d_lg, logits, (size_t)n_rows * LD * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_c, c.data(), sizeof(SlotCtrl) * n_rows, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_slot, slot.data(), 4 * (size_t)n_rows, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d_sem, 0xFF, 4 * (size_t)n_rows * RWKVTTS_SEMANTIC_LIMIT) != hipSuccess) {
      set_error("debug_advance: upload");
      rc = RWKVTTS_EHIP;
      break;
    }
    AdvanceArgs a{};
    a.logits = d_lg;
    a.ld = LD;
    a.n_part = 1;
    a.part_stride = 0;
    a.row_slot = d_slot;
    a.ctrl = d_c;
    a.sem_out = d_sem;
    a.n_rows = n_rows;
    std::vector<SlotCtrl> prev = c, now(n_rows);
    for (int s = 0; s < n_steps && rc == RWKVTTS_OK; ++s) {
      launch_advance(a, stream_, exact ? 0 : 1);
      if (hipStreamSynchronize(stream_) != hipSuccess ||
          hipMemcpy(now.data(), d_c, sizeof(SlotCtrl) * n_rows, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("debug_advance: launch");
        rc = RWKVTTS_EHIP;
        break;
      }
      for (int i = 0; i < n_rows; ++i) {
        const SlotCtrl &p = prev[i], &q = now[i];
        const int64_t o = (int64_t)s * n_rows + i;
        out_phase[o] = q.phase;
        if (p.phase == kPhGlobal) {
          out_tok[o] = q.n_global > p.n_global ? q.global_out[p.n_global] : -1;
          out_used[o] = (int32_t)(q.gdraw - p.gdraw);
        } else {
          out_used[o] = (int32_t)(q.sdraw - p.sdraw);
          out_tok[o] = -1;
          if (q.n_sem > p.n_sem) {
            int32_t t = -1;
            if (hipMemcpy(&t, d_sem + (int64_t)i * RWKVTTS_SEMANTIC_LIMIT + p.n_sem, 4, hipMemcpyDeviceToHost) != hipSuccess) {
              set_error("debug_advance: read-back");
              rc = RWKVTTS_EHIP;
            }
            out_tok[o] = t;
          }
        }
      }
      prev = now;
    }
  } while (false);
  cleanup();
  return rc;
}

int Engine::sample(const float* logits, int n_rows, int row_len, const rwkvtts_sample_args* args,
                   rwkvtts_rng* const* rngs, int32_t* out, float* dbg_host) {
  RT_HIP(hipSetDevice(device_));
  RT_CHECK(n_rows > 0 && row_len >= 0 && row_len <= kSampleMaxRowLen, RWKVTTS_EINVAL,
           "sample: row_len must be <= 2^24");
  const size_t need = (size_t)n_rows * std::max(row_len, 1);
  if (need > samp_cap_) {
    if (d_samp_logits_) hipFree(d_samp_logits_);
    d_samp_logits_ = nullptr;
    samp_cap_ = 0;
    RT_HIP(hipMalloc(&d_samp_logits_, need * 4));
    samp_cap_ = need;
  }
  if (n_rows > samp_rows_cap_) {
    for (void* p : {(void*)d_keys_, (void*)d_draws_, (void*)d_out_})
      if (p) hipFree(p);
    d_keys_ = nullptr;
    d_draws_ = nullptr;
    d_out_ = nullptr;
    samp_rows_cap_ = 0;
    RT_HIP(hipMalloc(&d_keys_, (size_t)n_rows * 32 + 256));
    RT_HIP(hipMalloc(&d_draws_, (size_t)n_rows * 8 + 256));
    RT_HIP(hipMalloc(&d_out_, (size_t)n_rows * 4 + 256));
    samp_rows_cap_ = n_rows;
  }
  std::vector<uint32_t> keys((size_t)n_rows * 8, 0);
  std::vector<uint64_t> draws(n_rows, 0);
  bool any_null = false, all_null = true;
  for (int i = 0; i < n_rows; ++i) {
    if (rngs && rngs[i]) {
      memcpy(&keys[(size_t)i * 8], rngs[i]->key, 32);
      draws[i] = rngs[i]->draw_index;
      all_null = false;
    } else {
      any_null = true;
    }
  }
  RT_CHECK(all_null || !any_null, RWKVTTS_EINVAL, "sample: mix of NULL and non-NULL rngs");
  RT_HIP(hipMemcpyAsync(d_samp_logits_, logits, need * 4, hipMemcpyHostToDevice, stream_));
  RT_HIP(hipMemcpyAsync(d_keys_, keys.data(), keys.size() * 4, hipMemcpyHostToDevice, stream_));
  RT_HIP(hipMemcpyAsync(d_draws_, draws.data(), draws.size() * 8, hipMemcpyHostToDevice, stream_));
  SampleRowArgs a{};
  a.logits = d_samp_logits_;
  a.ld = row_len;
  a.n = row_len;
  a.temperature = args->temperature;
  a.top_p = args->top_p;
  a.top_k = args->top_k;
  a.forbid = args->forbid_token;
  a.keys = all_null ? nullptr : d_keys_;
  a.draws = all_null ? nullptr : d_draws_;
  a.out = d_out_;
  if (row_len > kSampleMaxN) {  // long rows: per-row global scratch for p, sort keys and list
    const size_t stride = wide_scratch_bytes(row_len), bytes = stride * (size_t)n_rows;
    if (bytes > wide_cap_) {
      if (d_wide_) hipFree(d_wide_);
      d_wide_ = nullptr;
      wide_cap_ = 0;
      RT_HIP(hipMalloc(&d_wide_, bytes));
      wide_cap_ = bytes;
    }
    a.scratch = (char*)d_wide_;
    a.scratch_stride = stride;
  }
  a.dbg = nullptr;
  float* d_dbg = nullptr;
  if (dbg_host) {
    RT_HIP(hipMalloc(&d_dbg, (size_t)n_rows * (8 + 128)));
    RT_HIP(hipMemset(d_dbg, 0, (size_t)n_rows * (8 + 128)));
    a.dbg = d_dbg;
    a.stamps = (uint64_t*)(d_dbg + 2 * n_rows);
  }
  launch_sample_rows(a, n_rows, stream_);
  RT_HIP(hipGetLastError());
  if (dbg_host) {
    RT_HIP(hipMemcpyAsync(dbg_host, d_dbg, (size_t)n_rows * (8 + 128), hipMemcpyDeviceToHost, stream_));
    RT_HIP(hipStreamSynchronize(stream_));
    hipFree(d_dbg);
  }
  RT_HIP(hipMemcpyAsync(out, d_out_, (size_t)n_rows * 4, hipMemcpyDeviceToHost, stream_));
  RT_HIP(hipStreamSynchronize(stream_));
  for (int i = 0; i < n_rows; ++i) {
    RT_CHECK(out[i] >= 0, out[i], "sample: device sampler failed");
    if (rngs && rngs[i]) rngs[i]->draw_index++;
  }
  return RWKVTTS_OK;
}

// ------------------------------------------------------------------------------------------
// Continuous-batching scheduler (DynamicBatchManager semantics, src/dynamic_batch_manager.rs)
// ------------------------------------------------------------------------------------------
struct Active {
  Job* job;
  int slot;
  std::vector<uint32_t> prompt;
  int prefilled = 0;
  int advances = 0;  // phase-controller invocations so far
  int total = 0;     // advances after which the request is certainly done (its step limit)
  bool zero_shot = false;
};

namespace {

// generate_batch: a fixed list of requests
class ListSource : public JobSource {
 public:
  ListSource(const rwkvtts_request* reqs, int n, rwkvtts_result* res) : jobs_(n) {
    for (int i = 0; i < n; ++i) {
      jobs_[i].req = reqs[i];
      jobs_[i].res = &res[i];
    }
  }
  bool next(int max, bool, std::vector<Job*>& out) override {
    while (max-- > 0 && pos_ < jobs_.size()) out.push_back(&jobs_[pos_++]);
    return pos_ < jobs_.size();
  }
  void finish(Job*) override {}

 private:
  std::vector<Job> jobs_;
  size_t pos_ = 0;
};
}  // namespace

bool Engine::validate(const rwkvtts_request& q, std::string& why) const {
  auto ids_ok = [&](const int32_t* p, int n, int lo, int hi, const char* what) {
    if (n < 0 || (n > 0 && !p)) {
      why = std::string(what) + ": bad array";
      return false;
    }
    for (int i = 0; i < n; ++i)
      if (p[i] < lo || p[i] >= hi) {
        why = std::string(what) + ": id " + std::to_string(p[i]) + " out of range";
        return false;
      }
    return true;
  };
  const int V = dims.n_vocab;
  if (!ids_ok(q.text_tokens, q.n_text, 0, V, "text_tokens")) return false;
  if (!ids_ok(q.property_tokens, q.n_property, 0, V, "property_tokens")) return false;
  if ((q.ref_global && q.n_ref_global < 0) || (q.ref_semantic && q.n_ref_semantic < 0)) {
    why = "reference token counts must be >= 0";
    return false;
  }
  if (q.max_tokens < 0 || q.fixed_semantic < 0) {
    why = "max_tokens / fixed_semantic must be >= 0";
    return false;
  }
  const bool zero_shot = q.ref_global != nullptr && q.ref_semantic != nullptr;
  if (V <= RWKVTTS_TAG_2 || (!zero_shot && V <= RWKVTTS_GLOBAL_TOKEN_OFFSET + 4095) ||
      (zero_shot && q.n_ref_global > 0 && V <= RWKVTTS_GLOBAL_TOKEN_OFFSET + 4095)) {
    why = "model vocabulary too small for the TTS tags / global tokens";
    return false;
  }
  return true;
}

// Semantic-step limit and RNG seeds of a request, as the reference derives them.
static int sem_limit_of(const rwkvtts_request& q) {
  const bool zero_shot = q.ref_global != nullptr && q.ref_semantic != nullptr;
  if (q.fixed_semantic > 0) return std::min(q.fixed_semantic, RWKVTTS_SEMANTIC_LIMIT);
  if (zero_shot) return RWKVTTS_SEMANTIC_LIMIT;                  // zero_shot_inference.rs:128-142
  return std::min(std::max(q.max_tokens, 0), RWKVTTS_SEMANTIC_LIMIT);  // normal_mode_inference.rs:316
}

int Engine::generate(const rwkvtts_request* reqs, int n, rwkvtts_result* res) {
  stats = rwkvtts_stats{};
  max_active = 0;
  ListSource src(reqs, n, res);
  return serve(src);
}

// Waits for a unit's end event (polling: a blocking wait adds its wake-up latency to the GPU's
// idle gap), accounts its time, and retires the slots its control-block snapshot shows done.
int Engine::finish_unit(int b, bool prefill, std::vector<Active>& act, std::vector<int>& free_slots, JobSource& src,
                        hipEvent_t* ev0, hipEvent_t* ev1) {
  {
    hipError_t q;
    while ((q = hipEventQuery(ev1[b])) == hipErrorNotReady) __builtin_ia32_pause();
    RT_HIP(q);
  }
  float ms = 0;
  hipEventElapsedTime(&ms, ev0[b], ev1[b]);
  (prefill ? stats.prefill_ms : stats.decode_ms) += ms;
  RT_OK(flush_prof());
  if (graph_timing() && unit_graph_[b].first >= 0) {
    const std::vector<std::string>& names = graph_names_[unit_graph_[b]];
    const unsigned long long* h = h_gt_ + (size_t)b * kTlStride * kTlMax;
    for (size_t i = 0; i < names.size(); ++i) {
      const unsigned long long* q = h + (size_t)kTlStride * i;
      unsigned long long e = 0;
      for (int j = 2; j < kTlStride; ++j) e = std::max(e, q[j]);
      if (e <= q[0]) continue;
      auto it = std::find_if(prof.begin(), prof.end(), [&](const ProfEntry& x) { return x.name == names[i]; });
      if (it == prof.end()) {
        prof.push_back({names[i], 0, 0.0});
        it = prof.end() - 1;
      }
      it->launches++;
      it->ms += (double)(e - q[0]) * 1e-5;  // 100 MHz ticks -> ms
    }
  }
  if (d_tl_ && !prefill && stats.steps > 40) {  // semantic-phase steps only
    std::vector<unsigned long long> h((size_t)kTlStride * kTlMax);
    RT_HIP(hipMemcpy(h.data(), d_tl_, h.size() * 8, hipMemcpyDeviceToHost));
    const int n = (int)tl_names_.size();
    tl_start_.resize(n, 0.0);
    tl_dur_.resize(n, 0.0);
    for (int i = 0; i < n; ++i) {
      const unsigned long long* q = h.data() + (size_t)kTlStride * i;
      unsigned long long e = 0;
      for (int j = 2; j < kTlStride; ++j) e = std::max(e, q[j]);
      tl_start_[i] += (double)(q[0] - h[0]) * 0.01;  // us
      tl_dur_[i] += (double)(e - q[0]) * 0.01;
    }
    tl_steps_++;
  }
  ++units_;
  // retire finished slots: every finished slot's tokens copied on the engine's stream (no
  // null-stream sync), one synchronisation, then the jobs are handed back
  const SlotCtrl* snap = h_ctrl_ + (size_t)b * (S_ + 1);
  if (const int code = *(const int*)(snap + S_)) {
    // the unit's outputs are garbage: its jobs fail (serve), the persistent state is reset there
    persist_fault_ = code;
    set_error("persistent decode launch: a hand-off wait timed out (code " + std::to_string(code) + ")");
    return RWKVTTS_EHIP;
  }
  bool copied = false;
  for (auto& a : act) {
    const SlotCtrl& c = snap[a.slot];
    if (a.prefilled < (int)a.prompt.size() || c.phase != kPhDone) continue;
    rwkvtts_result& r = *a.job->res;
    if (r.semantic_tokens && c.n_sem > 0) {
      RT_HIP(hipMemcpyAsync(r.semantic_tokens, d_sem_ + (int64_t)a.slot * RWKVTTS_SEMANTIC_LIMIT,
                            sizeof(int32_t) * c.n_sem, hipMemcpyDeviceToHost, stream_));
      copied = true;
    }
  }
  if (copied) RT_HIP(hipStreamSynchronize(stream_));
  src.progress(*this);
  for (size_t i = 0; i < act.size();) {
    Active& a = act[i];
    const SlotCtrl& c = snap[a.slot];
    if (a.prefilled < (int)a.prompt.size() || c.phase != kPhDone) {
      ++i;
      continue;
    }
    rwkvtts_result& r = *a.job->res;
    r.status = 0;
    r.n_global = c.n_global;
    memcpy(r.global_tokens, c.global_out, sizeof(int32_t) * RWKVTTS_N_GLOBAL);
    r.n_semantic = c.n_sem;
    src.finish(a.job);
    free_slots.push_back(a.slot);
    act.erase(act.begin() + i);
  }
  return RWKVTTS_OK;
}

int Engine::serve(JobSource& src) {
  RT_HIP(hipSetDevice(device_));
  std::vector<int> free_slots;
  for (int s = S_ - 1; s >= 0; --s) free_slots.push_back(s);
  std::vector<Active> act;
  std::random_device rd;
  // Each unit of work (a mixed step or a decode window) ends with a control-block snapshot into
  // its own pinned buffer and an end event. In steady decode (no admission possible, no prompt
  // rows, the plan uploaded earlier, no slot able to pass its step limit) the next window is
  // launched before the host reads the previous one's snapshot, so the GPU does not idle while
  // the host polls, retires and relaunches. A slot that finished inside the older window idles
  // (k_advance skips it) through the newer one; every later operation on it is stream-ordered.
  hipEvent_t ev0[2], ev1[2];
  for (int i = 0; i < 2; ++i) {
    RT_HIP(hipEventCreate(&ev0[i]));
    RT_HIP(hipEventCreate(&ev1[i]));
  }
  struct Unit {
    bool valid = false, prefill = false;
    int buf = 0;
  } pending;
  bool open = true, decode_plan_valid = false;
  StepPlan dp;  // the decode plan (all active slots, tokens from the control blocks)
  std::vector<Job*> fresh;

  auto admit = [&](Job* j) -> int {
    const rwkvtts_request& q = j->req;
    rwkvtts_result& r = *j->res;
    r.status = 0;
    r.n_global = r.n_semantic = 0;
    std::string why;
    if (!validate(q, why)) {  // dynamic_batch_manager.rs:466-469: this request fails alone
      r.status = RWKVTTS_EINVAL;
      set_error("request rejected: " + why);
      src.finish(j);
      return RWKVTTS_OK;
    }
    // test hook: RWKVTTS_TEST_FAIL_ADMIT=k fails this engine's k-th admission as a HIP error would
    if (const char* fa = getenv("RWKVTTS_TEST_FAIL_ADMIT")) {
      if (++admissions_ == atoi(fa)) {
        set_error("injected admission failure (RWKVTTS_TEST_FAIL_ADMIT)");
        return RWKVTTS_EHIP;
      }
    }
    const int slot = free_slots.back();
    free_slots.pop_back();
    Active a;
    a.job = j;
    a.slot = slot;
    a.zero_shot = q.ref_global != nullptr && q.ref_semantic != nullptr;
    for (int i = 0; i < q.n_property; ++i) a.prompt.push_back((uint32_t)q.property_tokens[i]);
    a.prompt.push_back(RWKVTTS_TAG_2);
    for (int i = 0; i < q.n_text; ++i) a.prompt.push_back((uint32_t)q.text_tokens[i]);
    a.prompt.push_back(RWKVTTS_TAG_0);
    SlotCtrl c;
    memset(&c, 0, sizeof(c));
    // RNG streams: normal_mode_inference.rs:138-174, zero_shot_inference.rs:204-216,
    // dynamic_batch_manager.rs:491-499 (no seed -> from_entropy)
    const uint64_t seed = q.has_seed ? q.seed : (((uint64_t)rd() << 32) ^ rd());
    const bool indep = q.layered_set ? q.use_independent_seeds != 0 : true;
    const uint64_t goff = q.layered_set ? q.global_seed_offset : 1000, soff = q.layered_set ? q.semantic_seed_offset : 2000;
    uint64_t gseed = indep ? seed + goff : seed + 100, sseed = indep ? seed + soff : seed + 200;
    if (a.zero_shot && !indep) sseed = 0;  // StdRng::seed_from_u64(0) handed to the zero-shot path
    rwkvtts_rng rg, rs;
    rwkvtts_rng_seed_from_u64(gseed, &rg);
    rwkvtts_rng_seed_from_u64(sseed, &rs);
    memcpy(c.gkey, rg.key, 32);
    memcpy(c.skey, rs.key, 32);
    c.top_k_g = q.greedy ? 1 : 20;
    c.top_k_s = q.greedy ? 1 : 80;
    c.fixed = q.fixed_semantic > 0;
    c.sem_limit = sem_limit_of(q);
    if (a.zero_shot) {
      c.mode = 1;
      c.phase = kPhSemantic;
      for (int i = 0; i < q.n_ref_global; ++i) {
        const int g = std::min(std::max(q.ref_global[i], 0), 4095);
        a.prompt.push_back((uint32_t)(g + RWKVTTS_GLOBAL_TOKEN_OFFSET));
        if (i < RWKVTTS_N_GLOBAL) c.global_out[c.n_global++] = g;
      }
      a.prompt.push_back(RWKVTTS_TAG_1);
      const int tlen = q.n_text;
      const int min_sem = std::min(std::max(tlen / 4, 8), 64);
      const int est = (int)ceilf((float)tlen * 1.8f);
      const int upper = (int)floorf((float)RWKVTTS_SEMANTIC_LIMIT * 0.9f);
      c.hard_min = std::min(upper, std::max(min_sem, est));
      a.total = std::max(c.sem_limit, 1);
    } else {
      c.mode = 0;
      c.phase = kPhGlobal;
      a.total = RWKVTTS_N_GLOBAL + 1 + c.sem_limit;
    }
    RT_OK(slot_reset(slot, false));  // ordered before the slot's first step on stream_
    // from per-slot host storage: admissions are not synchronised, so the source must outlive the
    // stream-ordered copy (the slot's entry is rewritten only after the slot retires)
    ctrl_stage_[slot] = c;
    RT_HIP(hipMemcpyAsync(d_ctrl_ + slot, &ctrl_stage_[slot], sizeof(c), hipMemcpyHostToDevice, stream_));
    act.push_back(std::move(a));
    decode_plan_valid = false;
    return RWKVTTS_OK;
  };

  int rc = RWKVTTS_OK;
  while (true) {
    // ---- admission: new requests take free slots between forward steps
    if (open && !free_slots.empty()) {
      fresh.clear();
      open = src.next((int)free_slots.size(), act.empty(), fresh);
      size_t n_admitted = 0;
      for (; n_admitted < fresh.size(); ++n_admitted)
        if ((rc = admit(fresh[n_admitted])) != RWKVTTS_OK) break;
      if (rc != RWKVTTS_OK) {
        // the failing job and every later one were taken from the source but never reached
        // `act`: they fail with the engine (the failure fan-out below covers `act` only)
        for (size_t i = n_admitted; i < fresh.size(); ++i) {
          Job* j = fresh[i];
          if (std::any_of(act.begin(), act.end(), [&](const Active& a) { return a.job == j; })) continue;
          j->res->status = rc;
          j->res->n_global = j->res->n_semantic = 0;
          src.finish(j);
        }
        break;
      }
    }
    if (act.empty()) {
      if (!open) break;
      continue;
    }
    std::sort(act.begin(), act.end(), [](const Active& x, const Active& y) { return x.slot < y.slot; });
    bool any_prefill = false;
    for (auto& a : act) any_prefill |= a.prefilled < (int)a.prompt.size();
    int K = 1;
    bool all_global = true, uploaded = false;
    const int b = pending.valid ? pending.buf ^ 1 : 0;  // this unit's snapshot buffer / events
    RT_HIP(hipEventRecord(ev0[b], stream_));
    if (any_prefill) {
      // ---- mixed step: every decoding slot's row (token from its control block) plus prompt
      // rows of the admitted slots, up to token_chunk_size rows; the decoding slots never stall
      StepPlan p;
      p.advance = true;
      int budget = chunk_;
      for (auto& a : act) {
        if (a.prefilled < (int)a.prompt.size()) continue;
        const int r = (int)p.rows.size();
        p.rows.push_back(make_int4(a.slot, kRowFirst | kRowLast | kRowCtrl, -1, 0));
        p.tok.push_back(0);
        p.segs.push_back(make_int4(a.slot, r, 1, 0));
        p.lg_rows.push_back(r);
        p.lg_slot.push_back(a.slot);
        all_global &= !a.zero_shot && a.advances <= RWKVTTS_N_GLOBAL;
        a.advances++;
        --budget;
      }
      budget = std::max(budget, 1);
      for (auto& a : act) {
        const int left = (int)a.prompt.size() - a.prefilled;
        if (left <= 0 || budget <= 0) continue;
        const int take = std::min(left, budget);
        const int r0 = (int)p.rows.size();
        for (int t = 0; t < take; ++t) {
          const int flags = (t == 0 ? kRowFirst : 0) | (t == take - 1 ? kRowLast : 0);
          p.rows.push_back(make_int4(a.slot, flags, t == 0 ? -1 : r0 + t - 1, 0));
          p.tok.push_back(a.prompt[a.prefilled + t]);
        }
        p.segs.push_back(make_int4(a.slot, r0, take, 0));
        a.prefilled += take;
        budget -= take;
        if (a.prefilled == (int)a.prompt.size()) {
          p.lg_rows.push_back(r0 + take - 1);
          p.lg_slot.push_back(a.slot);
          all_global &= !a.zero_shot;
          a.advances++;
        }
      }
      p.head_rows = std::min(all_global ? 4096 : 8193, dims.n_vocab);
      if ((rc = run_step(p, true)) != RWKVTTS_OK) break;
      decode_plan_valid = false;
      stats.prefill_steps++;
    } else {
      // ---- decode window: up to kLookahead steps queued back to back before the host reads
      // the control blocks; no slot can pass its step limit inside the window (EOS may end a
      // request earlier: its slot then idles through the rest of the window, k_advance skips it)
      if (!decode_plan_valid) {
        dp = StepPlan();
        dp.tok_from_ctrl = true;
        dp.advance = true;
        for (auto& a : act) {
          const int r = (int)dp.rows.size();
          dp.rows.push_back(make_int4(a.slot, kRowFirst | kRowLast | kRowCtrl, -1, 0));
          dp.segs.push_back(make_int4(a.slot, r, 1, 0));
          dp.lg_rows.push_back(r);
          dp.lg_slot.push_back(a.slot);
        }
        if ((rc = upload_plan(dp)) != RWKVTTS_OK) break;
        decode_plan_valid = true;
        uploaded = true;
      }
      K = (profiling || d_tl_) ? 1 : kLookahead;
      for (auto& a : act) K = std::min(K, std::max(1, a.total - a.advances));
      if (d_tl_) RT_HIP(hipMemsetAsync(d_tl_, 0, (size_t)kTlStride * kTlMax * 8, stream_));
      for (int k = 0; k < K && rc == RWKVTTS_OK; ++k) {
        // head rows: 4096 while every slot samples global tokens (or feeds g31), else 8193
        all_global = true;
        for (auto& a : act) all_global &= !a.zero_shot && a.advances <= RWKVTTS_N_GLOBAL;
        dp.head_rows = std::min(all_global ? 4096 : 8193, dims.n_vocab);
        rc = run_step(dp, false);
        for (auto& a : act) a.advances++;
      }
      if (rc != RWKVTTS_OK) break;
      stats.steps += K;
      stats.decode_rows += (int64_t)dp.rows.size() * K;
      max_active = std::max<int64_t>(max_active, (int64_t)dp.rows.size());
    }
    RT_HIP(hipMemcpyAsync(h_ctrl_ + (size_t)b * (S_ + 1), d_ctrl_, sizeof(SlotCtrl) * (S_ + 1), hipMemcpyDeviceToHost, stream_));
    unit_graph_[b] = {-1, -1};
    if (graph_timing() && !any_prefill && last_graph_.first >= 0) {  // the window's last step's stamps
      const size_t n = graph_names_[last_graph_].size();
      RT_HIP(hipMemcpyAsync(h_gt_ + (size_t)b * kTlStride * kTlMax, d_gt_, n * kTlStride * 8, hipMemcpyDeviceToHost,
                            stream_));
      unit_graph_[b] = last_graph_;
    }
    RT_HIP(hipEventRecord(ev1[b], stream_));
    Unit now;
    now.valid = true;
    now.prefill = any_prefill;
    now.buf = b;
    // the older unit first (its retirements are stream-ordered after this one), then this one
    // unless the next window may go out before its snapshot is read
    if (pending.valid) {
      const Unit u = pending;
      pending.valid = false;
      if ((rc = finish_unit(u.buf, u.prefill, act, free_slots, src, ev0, ev1)) != RWKVTTS_OK) break;
      if (act.size() != dp.rows.size()) decode_plan_valid = false;
    }
    bool ahead = !any_prefill && !uploaded && use_graphs_ && !profiling && !d_tl_ &&
                 (!open || free_slots.empty());
    for (auto& a : act) ahead &= a.total - a.advances >= 1;
    if (ahead) {
      pending = now;
    } else {
      if ((rc = finish_unit(now.buf, now.prefill, act, free_slots, src, ev0, ev1)) != RWKVTTS_OK) break;
      if (act.size() != dp.rows.size()) decode_plan_valid = false;
    }
  }
  if (pending.valid || rc != RWKVTTS_OK) (void)hipStreamSynchronize(stream_);
  if (persist_fault_) {  // a timed-out hand-off: the engine recovers and keeps serving
    const int code = persist_fault_;
    persist_fault_ = 0;
    // a second timeout within kDegradeWindow units of the last one (e.g. another process
    // running persistent launches on this GPU without sharing the lock directory, so the deadlock
    // condition recurs): leave the persistent forms for good -- separate launches never wait on
    // one another -- instead of failing unit after unit
    const bool degrade = last_fault_unit_ >= 0 && units_ - last_fault_unit_ <= kDegradeWindow;
    last_fault_unit_ = units_;
    recovered_ = reset_persistent() == RWKVTTS_OK && (!degrade || degrade_persistent() == RWKVTTS_OK);
    if (recovered_ && d_drop_ && test_drops_left_ > 0) {  // (test hook: the next dropped arrival)
      --test_drops_left_;
      const int one = 1;
      recovered_ = hipMemcpy(d_drop_, &one, sizeof(int), hipMemcpyHostToDevice) == hipSuccess;
    }
    set_error("persistent decode launch: a hand-off wait timed out (code " + std::to_string(code) +
              "); the unit's requests failed, the engine was reset" +
              (degrade ? " and now runs the separate launches (second timeout)" : ""));
  }
  for (int i = 0; i < 2; ++i) {
    hipEventDestroy(ev0[i]);
    hipEventDestroy(ev1[i]);
  }
  if (rc != RWKVTTS_OK) {  // engine failure: every job still in flight fails with it
    for (auto& a : act) {
      a.job->res->status = rc;
      a.job->res->n_global = a.job->res->n_semantic = 0;
      src.finish(a.job);
    }
    return rc;
  }
  return dump_stamps();
}

int Engine::reset_persistent() {
  RT_HIP(hipSetDevice(device_));
  RT_HIP(hipMemsetAsync(d_ctrl_ + S_, 0, sizeof(SlotCtrl), stream_));
  for (auto& b : sync_bufs_) RT_HIP(hipMemsetAsync(b.first, 0, b.second, stream_));
  if (d_epoch_) {  // a new granule pass tag as well (the zeroed granules match no tag anyway)
    int ep = 0;
    RT_HIP(hipMemcpyAsync(&ep, d_epoch_, sizeof(int), hipMemcpyDeviceToHost, stream_));
    RT_HIP(hipStreamSynchronize(stream_));
    ++ep;
    RT_HIP(hipMemcpyAsync(d_epoch_, &ep, sizeof(int), hipMemcpyHostToDevice, stream_));
  }
  RT_HIP(hipStreamSynchronize(stream_));
  return RWKVTTS_OK;
}

int Engine::degrade_persistent() {
  RT_HIP(hipSetDevice(device_));
  RT_HIP(hipStreamSynchronize(stream_));
  att_persist_ = ffn_persist_ = 0;
  for (auto& g : graphs_) hipGraphExecDestroy(g.second);  // they hold persistent launches
  graphs_.clear();
  graph_names_.clear();
  release_persistent(device_, this, &lock_fd_);
  return RWKVTTS_OK;
}

int Engine::dump_stamps() {
  if (d_tl_ && tl_steps_ > 0) {
    FILE* f = fopen(tl_path_.c_str(), "w");
    if (f) {
      fprintf(f, "# steps %d: launch index, name, mean start (us from the step's first launch), mean duration (us)\n", tl_steps_);
      for (size_t i = 0; i < tl_dur_.size(); ++i)
        fprintf(f, "%zu %s %.3f %.3f\n", i, tl_names_[i].c_str(), tl_start_[i] / tl_steps_, tl_dur_[i] / tl_steps_);
      fclose(f);
    }
  }
  if (dbg_astamps_) {
    std::vector<uint64_t> ha(256 * 16);
    RT_HIP(hipMemcpy(ha.data(), dbg_astamps_, ha.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen(dbg_astamp_path_.c_str(), "wb");
    if (f) {
      fwrite(ha.data(), 8, ha.size(), f);
      fclose(f);
    }
  }
  if (dbg_astamps2_) {
    std::vector<uint64_t> hf(2048 * 4);
    RT_HIP(hipMemcpy(hf.data(), dbg_astamps2_, hf.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen(dbg_astamp2_path_.c_str(), "wb");
    if (f) {
      fwrite(hf.data(), 8, hf.size(), f);
      fclose(f);
    }
  }
  if (dbg_fstamps_) {
    std::vector<uint64_t> hf(1024 * 4);
    RT_HIP(hipMemcpy(hf.data(), dbg_fstamps_, hf.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen(dbg_fstamp_path_.c_str(), "wb");
    if (f) {
      fwrite(hf.data(), 8, hf.size(), f);
      fclose(f);
    }
  }
  if (dbg_gstamps_) {
    std::vector<uint64_t> hg(2 * 4096 * 4);
    RT_HIP(hipMemcpy(hg.data(), dbg_gstamps_, hg.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = fopen(dbg_gstamp_path_.c_str(), "wb");
    if (f) {
      fwrite(hg.data(), 8, hg.size(), f);
      fclose(f);
    }
  }
  if (!dbg_stamps_) return RWKVTTS_OK;
  std::vector<uint64_t> hs(4096 * 8);  // debug: layer-5 WKV stamps of the last step -> file
  RT_HIP(hipMemcpy(hs.data(), dbg_stamps_, hs.size() * 8, hipMemcpyDeviceToHost));
  FILE* f = fopen(dbg_stamp_path_.c_str(), "wb");
  if (f) {
    fwrite(hs.data(), 8, hs.size(), f);
    fclose(f);
  }
  return RWKVTTS_OK;
}

}  // namespace rwkvtts
