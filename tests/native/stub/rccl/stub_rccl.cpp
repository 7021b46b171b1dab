// TEST INFRASTRUCTURE (tests/test_sanitizers.py): a host-memory stand-in for RCCL's single-process
// multi-device API, built as librccl.so.1 and found by csrc/manager.cpp's dlopen through
// LD_LIBRARY_PATH, so the manager's multi-rank weight broadcast (ncclCommInitAll over distinct devices,
// one grouped ncclBroadcast per rank, rccl_broadcast) runs on the CPU under ThreadSanitizer. It
// checks the call pattern RCCL requires -- every rank of the communicator set calls ncclBroadcast once
// inside one ncclGroupStart / ncclGroupEnd with the same count and root -- and performs the copies at
// ncclGroupEnd (root's send buffer to every rank's receive buffer).
#include <stdio.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "rccl.h"

struct ncclComm {
  int rank, nranks;
};
namespace {
enum { kInvalidUsage = 5 };
struct Op {
  const void* send;
  void* recv;
  size_t count;
  int root, rank, nranks;
};
std::mutex mu;
int depth = 0;
std::vector<Op> ops;
}  // namespace

extern "C" {
ncclResult_t ncclCommInitAll(ncclComm_t* comms, int n, const int* devs) {
  if (!comms || n < 1 || !devs) return (ncclResult_t)kInvalidUsage;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j)
      if (devs[i] == devs[j]) return (ncclResult_t)kInvalidUsage;  // RCCL: one rank per distinct device
  for (int i = 0; i < n; ++i) comms[i] = new ncclComm{i, n};
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t c) {
  delete c;
  return ncclSuccess;
}
ncclResult_t ncclGroupStart(void) {
  std::lock_guard<std::mutex> lk(mu);
  ++depth;
  return ncclSuccess;
}
ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, ncclDataType_t t, int root, ncclComm_t c, hipStream_t) {
  std::lock_guard<std::mutex> lk(mu);
  // the manager's broadcast is always grouped (several ranks from one thread would deadlock otherwise)
  if (depth == 0 || !c || !r || t != ncclUint8 || root < 0 || root >= c->nranks) return (ncclResult_t)kInvalidUsage;
  ops.push_back({s, r, n, root, c->rank, c->nranks});
  return ncclSuccess;
}
ncclResult_t ncclGroupEnd(void) {
  std::lock_guard<std::mutex> lk(mu);
  if (depth == 0) return (ncclResult_t)kInvalidUsage;
  if (--depth > 0) return ncclSuccess;
  std::vector<Op> g;
  g.swap(ops);
  if (g.empty()) return ncclSuccess;
  const int n = g[0].nranks;
  std::vector<int> seen(n, 0);
  const void* src = nullptr;
  for (const Op& o : g) {
    if (o.nranks != n || o.count != g[0].count || o.root != g[0].root) return (ncclResult_t)kInvalidUsage;
    seen[o.rank]++;
    if (o.rank == o.root) src = o.send;
  }
  for (int r = 0; r < n; ++r)
    if (seen[r] != 1) return (ncclResult_t)kInvalidUsage;
  if (!src) return (ncclResult_t)kInvalidUsage;
  for (const Op& o : g)
    if (o.recv != src) memmove(o.recv, src, o.count);
  fprintf(stderr, "stub_rccl: grouped broadcast of %zu bytes to %d ranks\n", g[0].count, n);
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "stub_rccl: invalid usage"; }
}
