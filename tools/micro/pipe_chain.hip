// Pipelined launch chain: 172 dependent launches, each 256 WGs, that wait on the previous launch's
// arrival counter (bounded spin) after an independent prologue. Modes: plain graph (no waits),
// two-stream graph, single-stream hipExtLaunchKernel(anyOrder) in a graph, and eager anyOrder.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
struct PS {
  int* wait;
  int wait_n;
  int* post;
  int* err;
};
__global__ void k_step(PS p, float* buf, int work) {
  float a = threadIdx.x;
  for (int i = 0; i < work; ++i) a = a * 0.999f + 1.f;  // independent prologue
  if (p.wait) {
    if (threadIdx.x == 0) {
      int spins = 0;
      while (__hip_atomic_load(p.wait, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < p.wait_n) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1 << 20)) {
          __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  for (int i = 0; i < work; ++i) a = a * 0.999f + 1.f;  // dependent body
  buf[blockIdx.x * 256 + threadIdx.x] = a;
  if (p.post) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(p.post, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
int main() {
  const int nk = 172, nwg = 256;
  int work = 600;
  float* buf;
  int *cnt, *err;
  (void)hipMalloc(&buf, nwg * 256 * 4);
  (void)hipMalloc(&cnt, 4096);
  (void)hipMalloc(&err, 64);
  (void)hipMemset(err, 0, 64);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1, fork, join;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&join, hipEventDisableTiming);
  const char* nm[] = {"graph, one stream, no waits", "graph, two streams + waits", "graph, anyOrder + waits",
                      "eager, anyOrder + waits", "graph, anyOrder, no waits (racy)"};
  for (int wi = 0; wi < 2; ++wi)
  for (int mode = 0; mode < 5; ++mode) {
    work = wi == 0 ? 600 : 60;
    if (mode == 1) continue;  // two forked streams with waits deadlock in a graph (measured)
    auto build = [&](hipStream_t st) {
      (void)hipMemsetAsync(cnt, 0, 4096, st);
      if (mode == 1) {
        (void)hipEventRecord(fork, st);
        (void)hipStreamWaitEvent(s2, fork, 0);
      }
      for (int i = 0; i < nk; ++i) {
        const bool nw = mode == 0 || mode == 4;
        PS p{nw ? nullptr : (i ? cnt + i - 1 : nullptr), nwg, nw ? nullptr : cnt + i, err};
        hipStream_t ks = (mode == 1 && (i & 1)) ? s2 : st;
        if (mode >= 2 && i > 0) {
          void* args[] = {&p, &buf, &work};
          (void)hipExtLaunchKernel((const void*)k_step, dim3(nwg), dim3(256), args, 0, ks, nullptr, nullptr,
                                   hipExtAnyOrderLaunch);
        } else {
          hipLaunchKernelGGL(k_step, dim3(nwg), dim3(256), 0, ks, p, buf, work);
        }
      }
      if (mode == 1) {
        (void)hipEventRecord(join, s2);
        (void)hipStreamWaitEvent(st, join, 0);
      }
    };
    float ms = 0;
    if (mode != 3) {
      hipGraph_t g;
      hipGraphExec_t ge;
      (void)hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
      build(s1);
      hipError_t ce = hipStreamEndCapture(s1, &g);
      if (ce != hipSuccess) {
        printf("mode %d capture failed: %s\n", mode, hipGetErrorString(ce));
        continue;
      }
      (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipGraphLaunch(ge, s1);
      (void)hipStreamSynchronize(s1);
      (void)hipEventRecord(e0, s1);
      for (int r = 0; r < 5; ++r) (void)hipGraphLaunch(ge, s1);
      (void)hipEventRecord(e1, s1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
    } else {
      build(s1);
      (void)hipStreamSynchronize(s1);
      (void)hipEventRecord(e0, s1);
      for (int r = 0; r < 5; ++r) build(s1);
      (void)hipEventRecord(e1, s1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
    }
    int herr = 0;
    (void)hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
    (void)hipMemset(err, 0, 64);
    printf("work %d mode %d (%s): %.2f us per launch, timeout flag %d\n", work, mode, nm[mode], ms * 1000 / nk, herr);
  }
  return 0;
}
