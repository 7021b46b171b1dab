// TEST INFRASTRUCTURE (tests/test_sanitizers.py): csrc/manager.cpp's C ABI (rwkvtts_manager_*)
// driven from many threads under ThreadSanitizer, against the stub engine of stub/engine.h --
// the round-2 hang class (submit / collect / route / wait / destroy) and the round-3
// use-after-free class (a waiter blocked while destroy frees the tickets) checked by a tool.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rwkvtts.h"

namespace rwkvtts {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
}  // namespace rwkvtts
extern "C" const char* rwkvtts_last_error(void) { return rwkvtts::g_err.c_str(); }

static int fails = 0;
#define EXPECT(c)                                                            \
  do {                                                                       \
    if (!(c)) {                                                              \
      fprintf(stderr, "expectation failed at line %d: %s\n", __LINE__, #c); \
      ++fails;                                                               \
    }                                                                        \
  } while (0)

static rwkvtts_manager* make(int n_engines, int slots, int collect_ms) {
  rwkvtts_manager_desc d;
  memset(&d, 0, sizeof(d));
  d.n_engines = n_engines;
  for (int i = 0; i < n_engines; ++i) d.devices[i] = i;
  d.engine.max_slots = slots;
  d.max_batch_size = 8;
  d.collect_timeout_ms = collect_ms;
  static char w[4096];
  for (size_t i = 0; i < sizeof(w); ++i) w[i] = (char)((i * 31 + 7) & 255);  // checked by every stub engine
  rwkvtts_manager* m = nullptr;
  EXPECT(rwkvtts_manager_create(&d, w, sizeof(w), &m) == RWKVTTS_OK);
  return m;
}

static rwkvtts_request req(uint64_t seed, int fixed) {
  static const int32_t text[4] = {12300, 12301, 12302, 12303};
  rwkvtts_request q;
  memset(&q, 0, sizeof(q));
  q.text_tokens = text;
  q.n_text = 4;
  q.has_seed = 1;
  q.seed = seed;
  q.max_tokens = 64;
  q.fixed_semantic = fixed;
  return q;
}

// many submitters and waiters on three engines; every result is the stub's function of the seed
static void scenario_concurrent(bool faults) {
  rwkvtts_manager* m = make(3, 6, 2);
  std::atomic<int> ok{0}, failed{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      std::vector<uint64_t> tk;
      for (int i = 0; i < 24; ++i) {
        uint64_t id = 0;
        rwkvtts_request q = req(1000 * t + i, 3 + i % 5);
        EXPECT(rwkvtts_manager_submit(m, &q, &id) == RWKVTTS_OK);
        tk.push_back(id);
        if (i % 7 == 3) {  // a stats poll from a client thread while everything runs
          rwkvtts_manager_stats s;
          EXPECT(rwkvtts_manager_get_stats(m, &s) == RWKVTTS_OK);
        }
      }
      for (int i = 0; i < 24; ++i) {
        int32_t sem[RWKVTTS_SEMANTIC_LIMIT];
        rwkvtts_result r;
        memset(&r, 0, sizeof(r));
        r.semantic_tokens = sem;
        int rc;
        while ((rc = rwkvtts_manager_wait(m, tk[i], 5, &r)) == RWKVTTS_EBUSY) {
        }
        EXPECT(rc == RWKVTTS_OK);
        const uint64_t seed = 1000 * t + i;
        if (r.status == 0) {
          EXPECT(r.n_semantic == 3 + i % 5 && r.global_tokens[5] == (int32_t)((seed + 5) % 4096));
          EXPECT(r.n_semantic == 0 || sem[r.n_semantic - 1] == (int32_t)((seed * 7 + r.n_semantic - 1) % 8192));
          ++ok;
        } else {
          EXPECT(faults && r.status == RWKVTTS_EHIP && r.n_semantic == 0);
          ++failed;
        }
      }
    });
  for (auto& x : th) x.join();
  EXPECT(ok + failed == 8 * 24);
  if (!faults) EXPECT(failed == 0);
  rwkvtts_manager_stats s;
  EXPECT(rwkvtts_manager_get_stats(m, &s) == RWKVTTS_OK);
  EXPECT(s.completed == 8 * 24 && s.persistent[0] == 1 && s.persistent[1] == 0);
  EXPECT(rwkvtts_manager_destroy(m) == RWKVTTS_OK);
}

// destroy while waiters are blocked and requests are still queued: every waiter returns
static void scenario_destroy_with_waiters() {
  rwkvtts_manager* m = make(2, 2, 1);
  std::vector<uint64_t> tk(40);
  for (int i = 0; i < 40; ++i) {
    rwkvtts_request q = req(i, 4);
    EXPECT(rwkvtts_manager_submit(m, &q, &tk[i]) == RWKVTTS_OK);
  }
  std::atomic<int> returned{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      int32_t sem[RWKVTTS_SEMANTIC_LIMIT];
      rwkvtts_result r;
      memset(&r, 0, sizeof(r));
      r.semantic_tokens = sem;
      const int rc = rwkvtts_manager_wait(m, tk[39 - t], -1, &r);
      EXPECT(rc == RWKVTTS_OK || rc == RWKVTTS_ECLOSED);
      ++returned;
    });
  // a second waiter on a ticket someone is blocked on is refused (spin until the first holds it)
  std::this_thread::sleep_for(std::chrono::milliseconds(2));
  EXPECT(rwkvtts_manager_destroy(m) == RWKVTTS_OK);
  for (auto& x : th) x.join();
  EXPECT(returned == 4);
}

// an engine that fails unrecoverably: its jobs fail, later batches route to the others
static void scenario_dead_engine() {
  setenv("STUB_DEAD_ENGINE", "1", 1);
  rwkvtts_manager* m = make(3, 4, 1);
  unsetenv("STUB_DEAD_ENGINE");
  int ok = 0, bad = 0;
  for (int round = 0; round < 3; ++round) {
    std::vector<uint64_t> tk(12);
    for (int i = 0; i < 12; ++i) {
      rwkvtts_request q = req(round * 100 + i, 2);
      EXPECT(rwkvtts_manager_submit(m, &q, &tk[i]) == RWKVTTS_OK);
    }
    for (int i = 0; i < 12; ++i) {
      int32_t sem[RWKVTTS_SEMANTIC_LIMIT];
      rwkvtts_result r;
      memset(&r, 0, sizeof(r));
      r.semantic_tokens = sem;
      EXPECT(rwkvtts_manager_wait(m, tk[i], -1, &r) == RWKVTTS_OK);
      (r.status == 0 ? ok : bad)++;
    }
  }
  EXPECT(ok > 0 && ok + bad == 36);
  EXPECT(rwkvtts_manager_destroy(m) == RWKVTTS_OK);
}

// weight distribution over distinct devices: by the RCCL broadcast when a librccl.so.1 is loadable
// (the stub of tests/native/stub/rccl: STUB_EXPECT_RCCL=1) and RCCL is not disabled, else by peer
// copies; every engine checks its copy (stub/engine.h)
static void scenario_broadcast() {
  const bool want = getenv("STUB_EXPECT_RCCL") != nullptr;
  rwkvtts_manager* m = make(4, 2, 2);
  if (!m) return;
  rwkvtts_manager_stats st;
  EXPECT(rwkvtts_manager_get_stats(m, &st) == RWKVTTS_OK);
  EXPECT(st.bcast_ranks == 4);
  EXPECT(st.bcast_rccl == (want ? 1 : 0));
  std::vector<uint64_t> tk(8);
  for (int i = 0; i < 8; ++i) {
    rwkvtts_request q = req(500 + i, 3);
    EXPECT(rwkvtts_manager_submit(m, &q, &tk[i]) == RWKVTTS_OK);
  }
  std::vector<int32_t> sem(RWKVTTS_SEMANTIC_LIMIT);
  for (int i = 0; i < 8; ++i) {
    rwkvtts_result r;
    memset(&r, 0, sizeof(r));
    r.semantic_tokens = sem.data();
    EXPECT(rwkvtts_manager_wait(m, tk[i], -1, &r) == RWKVTTS_OK && r.status == 0);
  }
  EXPECT(rwkvtts_manager_destroy(m) == RWKVTTS_OK);
}

int main() {
  scenario_broadcast();
  scenario_concurrent(false);
  setenv("STUB_FAIL_EVERY", "2", 1);
  scenario_concurrent(true);
  unsetenv("STUB_FAIL_EVERY");
  scenario_destroy_with_waiters();
  scenario_dead_engine();
  if (fails) {
    fprintf(stderr, "%d expectations failed\n", fails);
    return 1;
  }
  printf("manager_tsan: ok\n");
  return 0;
}
