// manager.cpp -- rwkvtts_manager_*: the DynamicBatchManager of the reference
// (src/dynamic_batch_manager.rs:22-405, src/batch_types.rs:67-97) as native host code.
//
// Reference structure: generate_tts sends the request over a flume channel and waits on a
// oneshot (:90-121); one enqueue_worker collects requests into batches (:185-264) and hands each
// batch to whichever of max_concurrent_batches infer workers is free (:267-405), which then runs
// the batch's requests one after another on state slot 0.
//
// Here: submit() copies the request and queues it; the collector thread forms batches with the
// same rules (first request, then try_recv up to max_batch_size with at most 50 quick pulls; go
// once more than one request is pending or a lone request has waited 10 ms, or when
// collect_timeout_ms passes with requests pending) and routes every request of a batch to the
// least-loaded engine (fewest requests queued or decoding; ties -> lowest index). Each engine
// has one owner thread running Engine::serve, which admits queued requests into free state slots
// between forward steps (continuous batching). One engine per GPU = request-level data
// parallelism over the node; no collective is needed on this path.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>

#include <dlfcn.h>
#include <rccl/rccl.h>

#include "engine.h"

namespace rwkvtts {

namespace {

#define RT_OK(x)                      \
  do {                                \
    int _r = (x);                     \
    if (_r != RWKVTTS_OK) return _r;  \
  } while (0)

using Clock = std::chrono::steady_clock;

// RCCL is opened when a manager broadcasts its weights (dlopen), not linked into the library:
// single-engine users never load it, and tools that intercept it (profilers) only see it in
// processes that use the manager.
struct Rccl {
  decltype(&ncclCommInitAll) CommInitAll = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclBroadcast) Broadcast = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.CommInitAll = (decltype(x.CommInitAll))dlsym(h, "ncclCommInitAll");
    x.CommDestroy = (decltype(x.CommDestroy))dlsym(h, "ncclCommDestroy");
    x.Broadcast = (decltype(x.Broadcast))dlsym(h, "ncclBroadcast");
    x.GroupStart = (decltype(x.GroupStart))dlsym(h, "ncclGroupStart");
    x.GroupEnd = (decltype(x.GroupEnd))dlsym(h, "ncclGroupEnd");
    x.GetErrorString = (decltype(x.GetErrorString))dlsym(h, "ncclGetErrorString");
    x.ok = x.CommInitAll && x.CommDestroy && x.Broadcast && x.GroupStart && x.GroupEnd && x.GetErrorString;
    return x;
  }();
  return r;
}

struct MJob : Job {
  uint64_t ticket = 0;
  std::vector<int32_t> text, props, ref_g, ref_s;  // owned copies of the request arrays
  std::vector<int32_t> sem;                        // semantic token buffer
  rwkvtts_result out{};
  bool done = false;
  bool claimed = false;  // a wait() is in progress on this ticket (a second waiter is refused)
  int engine = -1;
};

class Manager;

class Worker : public JobSource {
 public:
  Worker(Manager* m, int idx) : m_(m), idx_(idx) {}
  bool next(int max, bool wait, std::vector<Job*>& out) override {
    std::unique_lock<std::mutex> lk(mu_);
    if (wait) cv_.wait(lk, [&] { return !inbox_.empty() || closing_; });
    while (max > 0 && !inbox_.empty()) {
      out.push_back(inbox_.front());
      inbox_.pop_front();
      --max;
    }
    return !(closing_ && inbox_.empty());
  }
  void finish(Job* j) override;
  // live statistics, published by the owner thread after every unit of work
  void progress(const Engine& e) override {
    steps = e.stats.steps + e.stats.prefill_steps;
    max_active = e.max_active;
  }
  void push(MJob* j) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      inbox_.push_back(j);
    }
    cv_.notify_one();
  }
  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      closing_ = true;
    }
    cv_.notify_one();
  }
  void run(rwkvtts_engine_desc desc, const void* w, size_t bytes);

  Engine eng;
  std::thread th;
  std::atomic<int> load{0};  // requests routed here and not finished
  std::atomic<bool> dead{false};
  std::atomic<int64_t> served{0}, max_active{0}, steps{0};
  std::atomic<int> persistent{0};
  int init_rc = 1;  // 1 = initialising
  std::string init_err;

 private:
  Manager* m_;
  int idx_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<MJob*> inbox_;
  bool closing_ = false;
};

class Manager {
 public:
  ~Manager() { free_dev_blobs(); }
  int create(const rwkvtts_manager_desc& d, const void* w, size_t bytes) {
    desc_ = d;
    RT_CHECK(d.n_engines >= 1 && d.n_engines <= RWKVTTS_MAX_ENGINES, RWKVTTS_EINVAL, "manager: 1..16 engines");
    RT_OK(broadcast_weights(d, w, bytes));
    for (int i = 0; i < d.n_engines; ++i) workers_.emplace_back(new Worker(this, i));
    for (int i = 0; i < d.n_engines; ++i) {
      rwkvtts_engine_desc ed = d.engine;
      ed.device = d.devices[i];
      Worker* wk = workers_[i].get();
      const void* dw = dev_blob_[rank_of_[i]];  // this engine's device's copy of the blob
      wk->th = std::thread([wk, ed, dw, bytes] { wk->run(ed, dw, bytes); });
    }
    // engines upload their weights in parallel; create() returns once all are ready
    int rc = RWKVTTS_OK;
    {
      std::unique_lock<std::mutex> lk(init_mu_);
      init_cv_.wait(lk, [&] {
        for (auto& wk : workers_)
          if (wk->init_rc == 1) return false;
        return true;
      });
      for (auto& wk : workers_)
        if (wk->init_rc != RWKVTTS_OK && rc == RWKVTTS_OK) {
          rc = wk->init_rc;
          set_error("manager: engine init failed: " + wk->init_err);
        }
    }
    free_dev_blobs();  // every engine holds its own copy now
    collector_ = std::thread([this] { collect_loop(); });
    return rc;
  }

  // The weight blob crosses PCIe once (host -> the first device), then goes to every other
  // distinct device by ncclBroadcast over xGMI (RCCL, one rank per device in one process:
  // ncclCommInitAll). With a single distinct device there is nothing to broadcast: RCCL is not
  // loaded at all (RWKVTTS_MANAGER_FORCE_RCCL=1 still runs the one-rank call, so the RCCL code
  // path can be exercised on a one-GPU box). If RCCL is missing or fails to initialise with
  // several devices, the blob goes out by hipMemcpyPeer instead (bcast_rccl = 0 then; the
  // reason is kept in bcast_note_). Engines sharing a device read that device's copy.
  // The caller's current device is restored on return, and every device blob is freed on any
  // error path.
  int broadcast_weights(const rwkvtts_manager_desc& d, const void* w, size_t bytes) {
    const auto t0 = Clock::now();
    int prev_dev = 0;
    RT_HIP(hipGetDevice(&prev_dev));
    struct Restore {
      int dev;
      ~Restore() { hipSetDevice(dev); }
    } restore{prev_dev};
    struct FreeOnError {
      Manager* m;
      bool armed = true;
      ~FreeOnError() {
        if (armed) m->free_dev_blobs();
      }
    } guard{this};
    std::vector<int> devs;
    rank_of_.assign(d.n_engines, 0);
    for (int i = 0; i < d.n_engines; ++i) {
      auto it = std::find(devs.begin(), devs.end(), d.devices[i]);
      rank_of_[i] = (int)(it - devs.begin());
      if (it == devs.end()) devs.push_back(d.devices[i]);
    }
    const int n = (int)devs.size();
    dev_blob_.assign(n, nullptr);
    dev_of_ = devs;
    for (int r = 0; r < n; ++r) {
      RT_HIP(hipSetDevice(devs[r]));
      RT_HIP(hipMalloc(&dev_blob_[r], bytes));
    }
    RT_HIP(hipSetDevice(devs[0]));
    RT_HIP(hipMemcpy(dev_blob_[0], w, bytes, hipMemcpyHostToDevice));
    const bool no_rccl = env_flag("RWKVTTS_MANAGER_NO_RCCL");
    const bool force_rccl = env_flag("RWKVTTS_MANAGER_FORCE_RCCL");
    bcast_rccl_ = 0;
    if (!no_rccl && (n > 1 || force_rccl)) {
      const int rc = rccl_broadcast(devs, bytes);
      if (rc == RWKVTTS_OK) bcast_rccl_ = 1;
      else if (force_rccl) return rc;  // asked for RCCL explicitly: report why it failed
    } else if (n > 1) {
      bcast_note_ = "RCCL disabled (RWKVTTS_MANAGER_NO_RCCL)";
    }
    if (!bcast_rccl_)
      for (int r = 1; r < n; ++r)
        RT_HIP(hipMemcpyPeer(dev_blob_[r], devs[r], dev_blob_[0], devs[0], bytes));
    guard.armed = false;
    bcast_ranks_ = n;
    bcast_ms_ = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    return RWKVTTS_OK;
  }

  // One grouped ncclBroadcast from dev_blob_[0] to every distinct device's buffer. On failure
  // returns an error code with the reason in bcast_note_ (and last_error); nothing is freed here.
  int rccl_broadcast(const std::vector<int>& devs, size_t bytes) {
    const int n = (int)devs.size();
    const Rccl& R = rccl();
    if (!R.ok) {
      bcast_note_ = "RCCL (librccl.so.1) not available";
      set_error("manager: " + bcast_note_);
      return RWKVTTS_EUNSUPPORTED;
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    std::vector<hipStream_t> streams(n, nullptr);
    auto nccl_ok = [&](ncclResult_t r, const char* what) {
      if (r == ncclSuccess) return true;
      bcast_note_ = std::string(what) + ": " + R.GetErrorString(r);
      set_error("manager: " + bcast_note_);
      return false;
    };
    int rc = RWKVTTS_OK;
    if (!nccl_ok(R.CommInitAll(comms.data(), n, devs.data()), "ncclCommInitAll")) rc = RWKVTTS_EHIP;
    for (int r = 0; r < n && rc == RWKVTTS_OK; ++r) {
      if (hipSetDevice(devs[r]) != hipSuccess || hipStreamCreateWithFlags(&streams[r], hipStreamNonBlocking) != hipSuccess) {
        bcast_note_ = "broadcast stream";
        set_error("manager: broadcast stream");
        rc = RWKVTTS_EHIP;
      }
    }
    if (rc == RWKVTTS_OK) {
      bool ok = nccl_ok(R.GroupStart(), "ncclGroupStart");
      for (int r = 0; r < n && ok; ++r)
        ok = nccl_ok(R.Broadcast(dev_blob_[0], dev_blob_[r], bytes, ncclUint8, 0, comms[r], streams[r]), "ncclBroadcast");
      ok = nccl_ok(R.GroupEnd(), "ncclGroupEnd") && ok;
      for (int r = 0; r < n && ok; ++r) {
        hipSetDevice(devs[r]);
        ok = hipStreamSynchronize(streams[r]) == hipSuccess;
        if (!ok) {
          bcast_note_ = "broadcast synchronisation";
          set_error("manager: broadcast synchronisation");
        }
      }
      if (!ok) rc = RWKVTTS_EHIP;
    }
    for (int r = 0; r < n; ++r) {
      if (streams[r]) {
        hipSetDevice(devs[r]);
        hipStreamDestroy(streams[r]);
      }
      if (comms[r]) R.CommDestroy(comms[r]);
    }
    return rc;
  }

  static bool env_flag(const char* name) {
    const char* v = getenv(name);
    return v && *v && strcmp(v, "0") != 0;
  }

  void free_dev_blobs() {
    for (size_t r = 0; r < dev_blob_.size(); ++r)
      if (dev_blob_[r]) {
        hipSetDevice(dev_of_[r]);
        hipFree(dev_blob_[r]);
        dev_blob_[r] = nullptr;
      }
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      closing_ = true;
    }
    q_cv_.notify_all();
    if (collector_.joinable()) collector_.join();
    for (auto& wk : workers_) wk->close();
    for (auto& wk : workers_)
      if (wk->th.joinable()) wk->th.join();
    // every job has completed (the workers drain their inboxes); wake any waiter still blocked
    // and free the jobs only once no thread is inside wait() -- the caller may destroy the
    // manager (its mutexes and condition variables) right after this returns
    std::unique_lock<std::mutex> lk(t_mu_);
    t_closed_ = true;
    t_cv_.notify_all();
    t_cv_.wait(lk, [&] { return waiters_ == 0; });
    for (auto& kv : jobs_) delete kv.second;
    jobs_.clear();
  }

  int submit(const rwkvtts_request& q, uint64_t* ticket) {
    MJob* j = new MJob();
    auto copy = [](const int32_t* p, int n, std::vector<int32_t>& v) {
      if (p && n > 0) v.assign(p, p + n);
    };
    copy(q.text_tokens, q.n_text, j->text);
    copy(q.property_tokens, q.n_property, j->props);
    copy(q.ref_global, q.n_ref_global, j->ref_g);
    copy(q.ref_semantic, q.n_ref_semantic, j->ref_s);
    j->req = q;
    j->req.text_tokens = j->text.empty() ? nullptr : j->text.data();
    j->req.property_tokens = j->props.empty() ? nullptr : j->props.data();
    // presence (Some / None) of the reference token sets is part of the request's meaning
    static const int32_t kEmpty[1] = {0};
    j->req.ref_global = q.ref_global ? (j->ref_g.empty() ? kEmpty : j->ref_g.data()) : nullptr;
    j->req.ref_semantic = q.ref_semantic ? (j->ref_s.empty() ? kEmpty : j->ref_s.data()) : nullptr;
    j->sem.assign(RWKVTTS_SEMANTIC_LIMIT, 0);
    j->out.semantic_tokens = j->sem.data();
    j->res = &j->out;
    {
      std::lock_guard<std::mutex> lk(t_mu_);
      j->ticket = ++next_ticket_;
      jobs_[j->ticket] = j;
      submitted_++;
    }
    *ticket = j->ticket;
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      if (closing_) {
        fail(j, RWKVTTS_ECLOSED);
        return RWKVTTS_OK;
      }
      queue_.push_back(j);
    }
    q_cv_.notify_one();
    return RWKVTTS_OK;
  }

  int wait(uint64_t ticket, int timeout_ms, rwkvtts_result* out) {
    std::unique_lock<std::mutex> lk(t_mu_);
    RT_CHECK(!t_closed_, RWKVTTS_ECLOSED, "manager_wait: manager is shutting down");
    auto it = jobs_.find(ticket);
    RT_CHECK(it != jobs_.end(), RWKVTTS_EINVAL, "manager_wait: unknown ticket");
    MJob* j = it->second;
    RT_CHECK(!j->claimed, RWKVTTS_EINVAL, "manager_wait: another thread is already waiting on this ticket");
    j->claimed = true;
    ++waiters_;
    auto ready = [&] { return j->done || t_closed_; };
    bool got = true;
    if (timeout_ms < 0)
      t_cv_.wait(lk, ready);
    else
      got = t_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready);
    int rc = RWKVTTS_OK;
    if (!got) {
      j->claimed = false;  // may be waited on again
      rc = RWKVTTS_EBUSY;
    } else if (!j->done) {  // shutdown woke us before the job completed
      rc = RWKVTTS_ECLOSED;
      set_error("manager_wait: manager shut down");
    } else {
      int32_t* sem = out->semantic_tokens;
      *out = j->out;
      out->semantic_tokens = sem;
      if (sem && j->out.n_semantic > 0) memcpy(sem, j->sem.data(), sizeof(int32_t) * j->out.n_semantic);
      jobs_.erase(it);
      delete j;
    }
    if (--waiters_ == 0 && t_closed_) t_cv_.notify_all();  // shutdown waits for the last waiter
    return rc;
  }

  void complete(MJob* j, int engine) {
    {
      std::lock_guard<std::mutex> lk(t_mu_);
      j->done = true;
      j->engine = engine;
      completed_++;
    }
    t_cv_.notify_all();
  }

  void stats(rwkvtts_manager_stats* s) {
    memset(s, 0, sizeof(*s));
    {
      std::lock_guard<std::mutex> lk(t_mu_);
      s->submitted = submitted_;
      s->completed = completed_;
    }
    s->batches = batches_.load();
    s->bcast_ranks = bcast_ranks_;
    s->bcast_rccl = bcast_rccl_;
    s->bcast_ms = bcast_ms_;
    {
      std::lock_guard<std::mutex> lk(t_mu_);
      s->waiters = waiters_;
    }
    for (size_t i = 0; i < workers_.size(); ++i) {
      s->served[i] = workers_[i]->served.load();
      s->max_active[i] = workers_[i]->max_active.load();
      s->steps[i] = workers_[i]->steps.load();
      s->persistent[i] = workers_[i]->persistent.load();
    }
  }

  void init_done() { init_cv_.notify_all(); }
  std::mutex init_mu_;

 private:
  void fail(MJob* j, int code) {
    j->out.status = code;
    j->out.n_global = j->out.n_semantic = 0;
    complete(j, -1);
  }

  // enqueue_worker (dynamic_batch_manager.rs:185-264)
  void collect_loop() {
    const int max_batch = std::max(1, desc_.max_batch_size);
    const auto tmo = std::chrono::milliseconds(std::max(0, desc_.collect_timeout_ms));
    std::vector<MJob*> pending;
    std::unique_lock<std::mutex> lk(q_mu_);
    while (true) {
      const auto collect_start = Clock::now();
      pending.clear();
      while (true) {
        // (a zero collect timeout with nothing pending would spin, as the reference's
        // timeout(0) does; wait for the first request without a timeout instead -- same batches)
        const auto ready = [&] { return !queue_.empty() || closing_; };
        bool got;
        if (pending.empty() && tmo.count() == 0) {
          q_cv_.wait(lk, ready);
          got = !queue_.empty();
        } else {
          got = q_cv_.wait_for(lk, tmo, ready) && !queue_.empty();
        }
        if (got) {
          pending.push_back(queue_.front());
          queue_.pop_front();
          int quick = 0;  // take whatever is immediately available
          while ((int)pending.size() < max_batch && quick < 50 && !queue_.empty()) {
            pending.push_back(queue_.front());
            queue_.pop_front();
            ++quick;
          }
          if (pending.size() > 1) break;
          if (Clock::now() - collect_start >= std::chrono::milliseconds(10)) break;
        } else if (!pending.empty() || closing_) {
          break;
        }
      }
      if (pending.empty() && closing_ && queue_.empty()) return;
      lk.unlock();
      route(pending);
      lk.lock();
    }
  }

  void route(const std::vector<MJob*>& batch) {
    if (batch.empty()) return;
    batches_++;
    for (MJob* j : batch) {
      Worker* best = nullptr;
      for (auto& wk : workers_) {
        if (wk->dead || wk->init_rc != RWKVTTS_OK) continue;
        if (!best || wk->load.load() < best->load.load()) best = wk.get();
      }
      if (!best) {
        fail(j, RWKVTTS_EHIP);
        continue;
      }
      best->load++;
      best->push(j);
    }
  }

  rwkvtts_manager_desc desc_{};
  std::vector<void*> dev_blob_;  // per distinct device: the broadcast weight blob (freed after init)
  std::vector<int> dev_of_;      // distinct devices, RCCL rank order
  std::vector<int> rank_of_;     // engine -> its device's rank
  int bcast_ranks_ = 0;
  int bcast_rccl_ = 0;       // 1 only when ncclBroadcast actually moved the blob
  std::string bcast_note_;   // why RCCL was not used (when it was not)
  double bcast_ms_ = 0.0;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::thread collector_;
  std::condition_variable init_cv_;
  // request queue (flume channel of the reference)
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<MJob*> queue_;
  bool closing_ = false;
  // tickets (oneshot channels of the reference)
  std::mutex t_mu_;
  std::condition_variable t_cv_;
  std::map<uint64_t, MJob*> jobs_;
  int waiters_ = 0;        // threads inside wait()
  bool t_closed_ = false;  // shutdown: no new waits, blocked waiters wake
  uint64_t next_ticket_ = 0;
  int64_t submitted_ = 0, completed_ = 0;
  std::atomic<int64_t> batches_{0};
};

void Worker::finish(Job* j) {
  served++;
  load--;
  m_->complete(static_cast<MJob*>(j), idx_);
}

void Worker::run(rwkvtts_engine_desc desc, const void* w, size_t bytes) {
  int rc = eng.init(desc, w, bytes, 1);  // w: the broadcast copy on this engine's device
  {
    std::lock_guard<std::mutex> lk(m_->init_mu_);
    persistent = rc == RWKVTTS_OK && eng.persistent() ? 1 : 0;  // (published before init_rc)
    init_rc = rc;
    if (rc != RWKVTTS_OK) init_err = "device " + std::to_string(desc.device);
  }
  m_->init_done();
  if (rc != RWKVTTS_OK) return;
  while (true) {
    rc = eng.serve(*this);
    progress(eng);
    if (rc != RWKVTTS_OK && eng.take_recovered()) {
      persistent = eng.persistent() ? 1 : 0;  // (0 once the engine left the persistent forms)
      // a persistent hand-off timed out: serve failed the unit's jobs (dynamic_batch_manager.rs:387-392:
      // a failed inference fails its own requests) and reset the engine, which keeps serving its inbox
      fprintf(stderr, "rwkvtts manager: engine %d (device %d): %s\n", idx_, desc.device, rwkvtts_last_error());
      continue;
    }
    if (rc != RWKVTTS_OK) {
      // the error text lives in this (engine) thread: log it, callers only see the status code
      fprintf(stderr, "rwkvtts manager: engine %d (device %d) failed (%d): %s\n", idx_, desc.device, rc,
              rwkvtts_last_error());
      dead = true;  // an engine failure fails its in-flight jobs (serve) and everything queued here
      std::vector<Job*> rest;
      bool open = true;
      while (open) {
        rest.clear();
        open = next(1 << 30, true, rest);
        for (Job* j : rest) {
          j->res->status = rc;
          j->res->n_global = j->res->n_semantic = 0;
          finish(j);
        }
      }
      return;
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (closing_ && inbox_.empty()) return;
  }
}

}  // namespace
}  // namespace rwkvtts

using namespace rwkvtts;

struct rwkvtts_manager {
  Manager m;
};

extern "C" {

int rwkvtts_manager_create(const rwkvtts_manager_desc* desc, const void* weights, size_t bytes,
                           rwkvtts_manager** out) {
  RT_CHECK(desc && weights && out, RWKVTTS_EINVAL, "manager_create: null argument");
  *out = nullptr;
  try {
    rwkvtts_manager* m = new rwkvtts_manager();
    const int rc = m->m.create(*desc, weights, bytes);
    if (rc != RWKVTTS_OK) {
      m->m.shutdown();
      delete m;
      return rc;
    }
    *out = m;
    return RWKVTTS_OK;
  } catch (const std::exception& ex) {
    set_error(ex.what());
    return RWKVTTS_ENOMEM;
  }
}

int rwkvtts_manager_destroy(rwkvtts_manager* m) {
  if (!m) return RWKVTTS_OK;
  m->m.shutdown();
  delete m;
  return RWKVTTS_OK;
}

int rwkvtts_manager_submit(rwkvtts_manager* m, const rwkvtts_request* req, uint64_t* ticket) {
  RT_CHECK(m && req && ticket, RWKVTTS_EINVAL, "manager_submit: null argument");
  try {
    return m->m.submit(*req, ticket);
  } catch (const std::exception& ex) {
    set_error(ex.what());
    return RWKVTTS_ENOMEM;
  }
}

int rwkvtts_manager_wait(rwkvtts_manager* m, uint64_t ticket, int timeout_ms, rwkvtts_result* out) {
  RT_CHECK(m && out, RWKVTTS_EINVAL, "manager_wait: null argument");
  return m->m.wait(ticket, timeout_ms, out);
}

int rwkvtts_manager_generate_batch(rwkvtts_manager* m, const rwkvtts_request* reqs, int n,
                                   rwkvtts_result* results) {
  RT_CHECK(m && (n == 0 || (reqs && results)) && n >= 0, RWKVTTS_EINVAL, "manager_generate_batch: bad arguments");
  std::vector<uint64_t> t(n);
  for (int i = 0; i < n; ++i) {
    const int rc = rwkvtts_manager_submit(m, &reqs[i], &t[i]);
    if (rc != RWKVTTS_OK) return rc;
  }
  for (int i = 0; i < n; ++i) {
    const int rc = m->m.wait(t[i], -1, &results[i]);
    if (rc != RWKVTTS_OK) return rc;
  }
  return RWKVTTS_OK;
}

int rwkvtts_manager_get_stats(rwkvtts_manager* m, rwkvtts_manager_stats* out) {
  RT_CHECK(m && out, RWKVTTS_EINVAL, "manager_get_stats: null argument");
  m->m.stats(out);
  return RWKVTTS_OK;
}

}  // extern "C"
