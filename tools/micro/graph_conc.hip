// Does a hipGraph run two independent branches (captured from two forked streams) concurrently?
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k_spin(float* p, int iters) {
  float a = threadIdx.x;
  for (int i = 0; i < iters; ++i) a = a * 0.999f + 1.f;
  if (a == 1234.5f) p[0] = a;
}
int main() {
  float* buf;
  (void)hipMalloc(&buf, 1 << 20);
  hipStream_t s1, s2;
  (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t e0, e1, fork, join;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  (void)hipEventCreateWithFlags(&join, hipEventDisableTiming);
  const int iters = 20000;
  for (int mode = 0; mode < 3; ++mode) {
    hipGraph_t g; hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
    if (mode == 0) {  // serial: two kernels on one stream
      hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s1, buf, iters);
      hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s1, buf, iters);
    } else if (mode == 1) {  // forked branches
      (void)hipEventRecord(fork, s1);
      (void)hipStreamWaitEvent(s2, fork, 0);
      hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s1, buf, iters);
      hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s2, buf, iters);
      (void)hipEventRecord(join, s2);
      (void)hipStreamWaitEvent(s1, join, 0);
    } else {  // one kernel only
      hipLaunchKernelGGL(k_spin, dim3(64), dim3(256), 0, s1, buf, iters);
    }
    (void)hipStreamEndCapture(s1, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s1);
    (void)hipStreamSynchronize(s1);
    (void)hipEventRecord(e0, s1);
    for (int r = 0; r < 20; ++r) (void)hipGraphLaunch(ge, s1);
    (void)hipEventRecord(e1, s1);
    (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    printf("mode %d (%s): %.1f us per graph\n", mode, mode == 0 ? "serial x2" : mode == 1 ? "forked x2" : "single", ms * 1000 / 20);
  }
  return 0;
}
