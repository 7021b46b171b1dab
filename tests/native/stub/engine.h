// TEST INFRASTRUCTURE (tests/test_sanitizers.py): a host-only stand-in for csrc/engine.h so that
// csrc/manager.cpp -- the collector, routing, tickets, wait and destroy logic -- compiles unchanged
// with g++ -fsanitize=thread and runs against a stub engine on the CPU. The stub keeps
// Engine::serve's contract (continuous batching over a JobSource, per-job finish, a recoverable
// failure that fails the in-flight jobs and keeps serving) with sleeps in place of GPU steps.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/rwkvtts.h"

// ---- the HIP runtime calls manager.cpp makes (host memory) ----
typedef int hipError_t;
typedef void* hipStream_t;
constexpr hipError_t hipSuccess = 0;
enum { hipMemcpyHostToDevice = 1, hipStreamNonBlocking = 1 };
inline const char* hipGetErrorString(hipError_t) { return "stub"; }
inline hipError_t hipGetDevice(int* d) { *d = 0; return hipSuccess; }
inline hipError_t hipSetDevice(int) { return hipSuccess; }
inline hipError_t hipMalloc(void** p, size_t n) { *p = malloc(n ? n : 1); return *p ? hipSuccess : 2; }
inline hipError_t hipFree(void* p) { free(p); return hipSuccess; }
inline hipError_t hipMemcpy(void* d, const void* s, size_t n, int) { memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipMemcpyPeer(void* d, int, const void* s, int, size_t n) { memcpy(d, s, n); return hipSuccess; }
inline hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned) { *s = nullptr; return hipSuccess; }
inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
inline hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }

namespace rwkvtts {
void set_error(const std::string& msg);
#define RT_HIP(expr)                                          \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) {                                  \
      ::rwkvtts::set_error(std::string(#expr) + ": stub");   \
      return RWKVTTS_EHIP;                                   \
    }                                                        \
  } while (0)
#define RT_CHECK(cond, code, msg) \
  do {                            \
    if (!(cond)) {                \
      ::rwkvtts::set_error(msg);  \
      return code;                \
    }                             \
  } while (0)

struct Job {
  rwkvtts_request req{};
  rwkvtts_result* res = nullptr;
  void* user = nullptr;
};
class Engine;
class JobSource {
 public:
  virtual ~JobSource() = default;
  virtual bool next(int max, bool wait, std::vector<Job*>& out) = 0;
  virtual void finish(Job* j) = 0;
  virtual void progress(const Engine&) {}
};

// STUB_FAIL_EVERY (env, read at init): every n-th serve() call of engine 1 fails its in-flight
// jobs with a recoverable error after one step; STUB_DEAD_ENGINE=k: engine on device k fails
// unrecoverably at its first serve().
class Engine {
 public:
  int init(const rwkvtts_engine_desc& desc, const void* w, size_t bytes, int) {
    RT_CHECK(w && bytes > 0, RWKVTTS_EINVAL, "stub: no weights");
    // the blob every engine receives (after the manager's broadcast) is the caller's, byte for byte
    // (manager_tsan_main.cpp fills it with (i * 31 + 7) & 255)
    for (size_t i = 0; i < bytes; ++i)
      RT_CHECK(((const uint8_t*)w)[i] == (uint8_t)((i * 31 + 7) & 255), RWKVTTS_EINVAL,
               "stub: an engine's weights differ from the caller's blob");
    device_ = desc.device;
    S_ = desc.max_slots > 0 ? desc.max_slots : 4;
    if (const char* e = getenv("STUB_FAIL_EVERY")) fail_every_ = atoi(e);
    if (const char* e = getenv("STUB_DEAD_ENGINE")) dead_ = atoi(e) == device_;
    return RWKVTTS_OK;
  }
  bool persistent() const { return device_ == 0; }
  bool take_recovered() {
    const bool r = recovered_;
    recovered_ = false;
    return r;
  }
  int serve(JobSource& src) {
    struct A {
      Job* j;
      int left;
    };
    std::vector<A> act;
    bool open = true;
    ++calls_;
    const bool fail_now = fail_every_ > 0 && device_ == 1 && calls_ % fail_every_ == 0;
    int steps_here = 0;
    while (true) {
      if (open && (int)act.size() < S_) {
        std::vector<Job*> fresh;
        open = src.next(S_ - (int)act.size(), act.empty(), fresh);
        for (Job* j : fresh) act.push_back({j, 1 + (int)(j->req.seed % 3)});
      }
      if (act.empty()) {
        if (!open) return RWKVTTS_OK;
        continue;
      }
      if (dead_) {
        for (A& a : act) {
          a.j->res->status = RWKVTTS_EHIP;
          src.finish(a.j);
        }
        set_error("stub: engine dead");
        return RWKVTTS_EHIP;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(300));  // one "decode step"
      ++steps_here;
      stats.steps++;
      max_active = std::max<int64_t>(max_active, (int64_t)act.size());
      if (fail_now && steps_here == 1) {  // a timed-out hand-off: the unit's jobs fail, engine resets
        for (A& a : act) {
          a.j->res->status = RWKVTTS_EHIP;
          a.j->res->n_global = a.j->res->n_semantic = 0;
          src.finish(a.j);
        }
        recovered_ = true;
        set_error("stub: recoverable fault");
        return RWKVTTS_EHIP;
      }
      for (size_t i = 0; i < act.size();) {
        if (--act[i].left > 0) {
          ++i;
          continue;
        }
        Job* j = act[i].j;
        rwkvtts_result& r = *j->res;
        r.status = 0;
        r.n_global = RWKVTTS_N_GLOBAL;
        for (int g = 0; g < RWKVTTS_N_GLOBAL; ++g) r.global_tokens[g] = (int32_t)((j->req.seed + g) % 4096);
        r.n_semantic = j->req.fixed_semantic;
        for (int s = 0; s < r.n_semantic; ++s) r.semantic_tokens[s] = (int32_t)((j->req.seed * 7 + s) % 8192);
        src.finish(j);
        act.erase(act.begin() + i);
      }
      src.progress(*this);
    }
  }
  rwkvtts_stats stats{};
  int64_t max_active = 0;

 private:
  int device_ = 0, S_ = 4, fail_every_ = 0, calls_ = 0;
  bool dead_ = false, recovered_ = false;
};
}  // namespace rwkvtts
