// api.cpp -- the extern "C" boundary (include/rwkvtts.h). Each entry point wraps one engine
// method; errors become status codes + a thread-local message, never C++ exceptions.
#include <string.h>

#include <mutex>
#include <new>

#include "engine.h"

namespace rwkvtts {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace rwkvtts

using namespace rwkvtts;

// Every entry point on an engine holds its lock: concurrent host threads serialise (the engine
// owns one stream, one set of step tables and the slot map). Batching across callers is the
// manager's job (manager.cpp).
struct rwkvtts_engine {
  std::mutex mu;
  Engine eng;
};
#define LOCK(e) std::lock_guard<std::mutex> lock_((e)->mu)

#define GUARD(body)                                      \
  try {                                                  \
    body                                                 \
  } catch (const std::bad_alloc&) {                      \
    set_error("out of host memory");                     \
    return RWKVTTS_ENOMEM;                               \
  } catch (const std::exception& ex) {                   \
    set_error(ex.what());                                \
    return RWKVTTS_EINVAL;                               \
  }

extern "C" {

const char* rwkvtts_last_error(void) { return g_last_error.c_str(); }

int rwkvtts_engine_create(const rwkvtts_engine_desc* desc, const void* weights, size_t bytes,
                          int blob_on_device, rwkvtts_engine** out) {
  GUARD({
    RT_CHECK(desc && weights && out, RWKVTTS_EINVAL, "engine_create: null argument");
    *out = nullptr;
    rwkvtts_engine* e = new rwkvtts_engine();
    const int rc = e->eng.init(*desc, weights, bytes, blob_on_device);
    if (rc != RWKVTTS_OK) {
      delete e;
      return rc;
    }
    *out = e;
    return RWKVTTS_OK;
  })
}

int rwkvtts_engine_destroy(rwkvtts_engine* e) {
  if (e) {
    std::lock_guard<std::mutex> lk(e->mu);  // wait for a call still running on another thread
  }
  delete e;
  return RWKVTTS_OK;
}

int rwkvtts_engine_dims(const rwkvtts_engine* e, rwkvtts_dims* out) {
  RT_CHECK(e && out, RWKVTTS_EINVAL, "null argument");
  *out = e->eng.dims;
  return RWKVTTS_OK;
}

int64_t rwkvtts_state_floats(const rwkvtts_engine* e) { return e ? e->eng.state_floats() : -1; }

int rwkvtts_slot_reset(rwkvtts_engine* e, int slot) {
  RT_CHECK(e, RWKVTTS_EINVAL, "null engine");
  LOCK(e);
  GUARD({ return e->eng.slot_reset(slot); })
}
int rwkvtts_slot_read(rwkvtts_engine* e, int slot, float* out) {
  RT_CHECK(e && out, RWKVTTS_EINVAL, "null argument");
  LOCK(e);
  GUARD({ return e->eng.slot_read(slot, out); })
}
int rwkvtts_slot_write(rwkvtts_engine* e, int slot, const float* in) {
  RT_CHECK(e && in, RWKVTTS_EINVAL, "null argument");
  LOCK(e);
  GUARD({ return e->eng.slot_write(slot, in); })
}

int rwkvtts_infer(rwkvtts_engine* e, const rwkvtts_input* inputs, int n_inputs, int head_rows,
                  float* logits, int32_t* consumed, int32_t* has_logits) {
  RT_CHECK(e && inputs && consumed && has_logits && n_inputs > 0, RWKVTTS_EINVAL, "infer: bad arguments");
  LOCK(e);
  GUARD({ return e->eng.infer(inputs, n_inputs, head_rows, logits, consumed, has_logits); })
}

int rwkvtts_sample(rwkvtts_engine* e, const float* logits, int n_rows, int row_len,
                   const rwkvtts_sample_args* args, rwkvtts_rng* const* rngs, int32_t* out_tokens) {
  RT_CHECK(e && logits && args && out_tokens, RWKVTTS_EINVAL, "sample: bad arguments");
  LOCK(e);
  GUARD({ return e->eng.sample(logits, n_rows, row_len, args, rngs, out_tokens); })
}

// Test hook (not part of the drop-in surface): same as rwkvtts_sample, also returns the softmax
// denominator and the uniform draw of every row in dbg[2*i], dbg[2*i+1], followed by
// n_rows x 16 uint64 phase stamps (dbg must hold n_rows * 34 floats).
int rwkvtts_debug_sample(rwkvtts_engine* e, const float* logits, int n_rows, int row_len,
                         const rwkvtts_sample_args* args, rwkvtts_rng* const* rngs, int32_t* out_tokens,
                         float* dbg) {
  RT_CHECK(e && logits && args && out_tokens && dbg, RWKVTTS_EINVAL, "debug_sample: bad arguments");
  LOCK(e);
  GUARD({ return e->eng.sample(logits, n_rows, row_len, args, rngs, out_tokens, dbg); })
}

// Test hook (not part of the drop-in surface): the production decode-step sampler k_advance
// (advance_prep + the prepped sample_block; exact = 1 forces the exact sequential-sum walk) on
// caller-given logit rows [n_rows][8193] and controller states (engine.h DebugAdvanceRow), for
// n_steps launches; outputs are [n_steps][n_rows].
int rwkvtts_debug_advance(rwkvtts_engine* e, const float* logits, int n_rows, const void* rows, int exact,
                          int n_steps, int32_t* out_tok, int32_t* out_used, int32_t* out_phase) {
  RT_CHECK(e && logits && rows && out_tok && out_used && out_phase, RWKVTTS_EINVAL, "debug_advance: bad arguments");
  LOCK(e);
  GUARD({
    return e->eng.debug_advance(logits, n_rows, (const DebugAdvanceRow*)rows, exact, n_steps, out_tok, out_used,
                                out_phase);
  })
}

int rwkvtts_generate_batch(rwkvtts_engine* e, const rwkvtts_request* reqs, int n,
                           rwkvtts_result* results) {
  RT_CHECK(e && reqs && results && n >= 0, RWKVTTS_EINVAL, "generate_batch: bad arguments");
  LOCK(e);
  GUARD({
    const int rc = e->eng.generate(reqs, n, results);
    if (rc != RWKVTTS_OK)
      for (int i = 0; i < n; ++i) {  // dynamic_batch_manager.rs:387-392: errors -> empty results
        results[i].status = rc;
        results[i].n_global = results[i].n_semantic = 0;
      }
    return rc;
  })
}

int rwkvtts_get_stats(rwkvtts_engine* e, rwkvtts_stats* out) {
  RT_CHECK(e && out, RWKVTTS_EINVAL, "null argument");
  LOCK(e);
  *out = e->eng.stats;
  out->profile_kernel_count = (int32_t)e->eng.prof.size();
  out->persistent = e->eng.persistent() ? 1 : 0;
  return RWKVTTS_OK;
}

int rwkvtts_set_profiling(rwkvtts_engine* e, int on) {
  RT_CHECK(e, RWKVTTS_EINVAL, "null engine");
  RT_CHECK(on >= 0 && on <= 2, RWKVTTS_EINVAL, "set_profiling: 0, 1 or 2");
  LOCK(e);
  GUARD({
    e->eng.profiling = on == 1;
    return e->eng.set_graph_timing(on == 2);
  })
}

int rwkvtts_profile_entry(rwkvtts_engine* e, int idx, char* name, int name_cap, int64_t* launches,
                          double* total_ms) {
  RT_CHECK(e, RWKVTTS_EINVAL, "null engine");
  LOCK(e);
  RT_CHECK(idx >= 0 && idx < (int)e->eng.prof.size(), RWKVTTS_EINVAL, "profile index out of range");
  const ProfEntry& p = e->eng.prof[idx];
  if (name && name_cap > 0) {
    strncpy(name, p.name.c_str(), name_cap - 1);
    name[name_cap - 1] = 0;
  }
  if (launches) *launches = p.launches;
  if (total_ms) *total_ms = p.ms;
  return RWKVTTS_OK;
}

}  // extern "C"
