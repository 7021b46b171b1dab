// Calibration: per-kernel floor of dependent launches in a hipGraph on this box.
// k_empty: 256 WGs x 256 threads doing nothing; k_store: the same grid writing `bytes` (f32).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void k_empty(float* p) { if (p == nullptr && threadIdx.x == 9999) p[0] = 1.f; }
__global__ void k_store(float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}
__global__ void k_load(const float* p, float* out, int n) {
  float s = 0.f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += p[i];
  if (s == 12345.f) out[0] = s;
}
int main(int argc, char** argv) {
  const int nk = 168;
  float* buf; hipMalloc(&buf, 64 << 20);
  hipStream_t st; hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, int grid, int mode, int n) {
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < nk; ++i) {
      if (mode == 0) hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, st, buf);
      else if (mode == 1) hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, st, buf, n);
      else hipLaunchKernelGGL(k_load, dim3(grid), dim3(256), 0, st, buf + (i % 2) * (16 << 20), buf + (60 << 20), n);
    }
    hipStreamEndCapture(st, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int w = 0; w < 3; ++w) hipGraphLaunch(ge, st);
    hipStreamSynchronize(st);
    hipEventRecord(e0, st);
    for (int r = 0; r < 10; ++r) hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-28s grid %5d: %.2f us per kernel\n", name, grid, ms * 1000 / 10 / nk);
    hipGraphExecDestroy(ge); hipGraphDestroy(g);
  };
  run("empty", 32, 0, 0);
  run("empty", 256, 0, 0);
  run("empty", 512, 0, 0);
  run("store 8 KB", 32, 1, 2048);
  run("store 1.7 MB", 256, 1, 1700000 / 4);
  run("store 8 MB", 256, 1, 2 << 20);
  run("load 1.7 MB", 256, 2, 1700000 / 4);
  run("load 8 MB", 256, 2, 2 << 20);
  run("load 8 MB", 1024, 2, 2 << 20);
  return 0;
}
