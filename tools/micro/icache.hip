// Calibration: is the instruction cache cold at every kernel launch? Kernels of N fully
// unrolled independent VALU ops (straight-line code, N static instructions) vs the same dynamic
// op count in a loop (tiny code), 168 dependent launches in a hipGraph.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int N>
__global__ void k_straight(float* p, float s) {
  float a = threadIdx.x * 1.0001f, b = a + 1.f, c = a + 2.f, d = a + 3.f;
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    a = a * s + 1.f; b = b * s + 2.f; c = c * s + 3.f; d = d * s + 4.f;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  if (a + b + c + d == 1234.5f) p[0] = a;
}
__global__ void k_loop(float* p, float s, int n) {
  float a = threadIdx.x * 1.0001f, b = a + 1.f, c = a + 2.f, d = a + 3.f;
  for (int i = 0; i < n / 4; ++i) {
    a = a * s + 1.f; b = b * s + 2.f; c = c * s + 3.f; d = d * s + 4.f;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  }
  if (a + b + c + d == 1234.5f) p[0] = a;
}
int main() {
  const int nk = 168;
  float* buf;
  (void)hipMalloc(&buf, 1 << 20);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time_graph = [&](auto launch, const char* name) {
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < nk; ++i) launch(i);
    (void)hipStreamEndCapture(st, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, st);
    (void)hipStreamSynchronize(st);
    (void)hipEventRecord(e0, st);
    for (int r = 0; r < 10; ++r) (void)hipGraphLaunch(ge, st);
    (void)hipEventRecord(e1, st);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %.2f us per kernel\n", name, ms * 1000 / 10 / nk);
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
  };
#define ST(N) time_graph([&](int) { hipLaunchKernelGGL(k_straight<N>, dim3(256), dim3(256), 0, st, buf, 0.999f); }, "straight " #N);
#define LP(N) time_graph([&](int) { hipLaunchKernelGGL(k_loop, dim3(256), dim3(256), 0, st, buf, 0.999f, N); }, "loop " #N);
  ST(256) ST(1024) ST(2048) ST(4096) ST(8192)
  LP(256) LP(1024) LP(2048) LP(4096) LP(8192)
  // alternating two different straight kernels (each launch's code differs from the previous)
  time_graph([&](int i) {
    if (i & 1) hipLaunchKernelGGL(k_straight<2048>, dim3(256), dim3(256), 0, st, buf, 0.999f);
    else hipLaunchKernelGGL(k_straight<2052>, dim3(256), dim3(256), 0, st, buf, 0.999f);
  }, "alternating straight 2048/2052");
  return 0;
}
