// stage_bench.hip -- how fast can a workgroup stage the vocoder's 7-tap chunks into LDS?
// Reproduces k_conv<64, 7, false, 8>'s staging pattern at the 192-channel stage (32 x 81920 rows,
// 6 chunks of 32 channels, 256-row time tiles x 3 column tiles, XCD-aware order) without MFMAs:
//   mode 0: LDS-DMA (buffer_load ... lds, 16 B per lane), double-buffered, barrier per chunk (k_conv)
//   mode 1: global_load_dwordx4 into VGPRs, ds_write_b128, barrier per chunk
//   mode 2: LDS-DMA, every chunk issued up front, one wait (raw DMA throughput)
//   mode 3: VGPR loads, every chunk issued up front (raw load throughput)
//   mode 4: mode 0 + k_conv's per-chunk MFMA work (7 taps x 2 x 4 x hi/lo, fragments from LDS)
//   mode 5: the MFMA work alone (no staging: every chunk computes on buffer 0)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/experiments/stage_bench.bin tools/experiments/stage_bench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int NWV = 8, TM = 256, TN = 64, MAXB = 16;

struct Args {
  const uint16_t* xh;
  const uint16_t* xl;
  const uint16_t* w;
  int64_t x_bs, x_cs;
  int rows, nck, K, Ci, Co, span, gx, gy;
  float* sink;
};

__device__ inline int swz(int row, int piece) { return row * 64 + ((piece ^ ((row >> 1) & 3)) << 4); }

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_stage(Args a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int k = blockIdx.x >> 3;
  const int by = k % a.gy, bx = (blockIdx.x & 7) + 8 * (k / a.gy);
  if (bx >= a.gx) return;
  const int tiles_per_utt = a.rows / TM;
  const int req = bx / tiles_per_utt, q0 = (bx % tiles_per_utt) * TM;
  const int co0 = by * TN;
  const int WRp = (TM + a.span + 15) & ~15;
  const int wstart = q0 - a.span / 2;
  const int nWblk = 7 * (TN / 16), nAblk = 2 * WRp / 16, nblk = nAblk + nWblk;
  const int buf_bytes = nblk * 1024;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane >> 2, lslot = lane & 3;
  const int64_t xoff = req * a.x_bs;
  auto rsrc = [](const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rxh = rsrc(a.xh + xoff), rxl = rsrc(a.xl + xoff), rwh = rsrc(a.w);
  uint32_t voff[MAXB];
#pragma unroll
  for (int u = 0; u < MAXB; ++u) {
    const int b = wave + NWV * u;
    uint32_t o = 0x80000000u;
    if (b < nAblk) {
      const int plane = b >= WRp / 16, row = (b - plane * (WRp / 16)) * 16 + lrow;
      const int piece = lslot ^ ((row >> 1) & 3), pos = wstart + row;
      if (pos >= 0 && pos < a.rows) o = (uint32_t)(pos * 32 + piece * 8) * 2u;
    } else if (b < nblk) {
      const int wb = b - nAblk;
      const int tap = wb / (TN / 16), co = (wb % (TN / 16)) * 16 + lrow;
      const int piece = lslot ^ ((co >> 1) & 3);
      o = (uint32_t)((((co0 + co) * a.K + tap) * a.Ci + piece * 8) * 2);
    }
    voff[u] = o;
  }
  auto issue_dma = [&](int ck, uint8_t* buf) {
    const int aso = (int)(ck * a.x_cs * 2), wso = ck * 64;
#pragma unroll
    for (int u = 0; u < MAXB; ++u) {
      const int b = __builtin_amdgcn_readfirstlane(wave + NWV * u);
      if (b >= nblk) continue;
      auto* dst = (__attribute__((address_space(3))) void*)(buf + b * 1024);
      if (b < nAblk) {
        if (b >= WRp / 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rxl, dst, 16, voff[u], aso, 0, 0);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rxh, dst, 16, voff[u], aso, 0, 0);
      } else {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rwh, dst, 16, voff[u], wso, 0, 0);
      }
    }
  };
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  auto load_regs = [&](int ck, u32x4* r) {
    const int aso = (int)(ck * a.x_cs * 2), wso = ck * 64;
#pragma unroll
    for (int u = 0; u < MAXB; ++u) {
      const int b = __builtin_amdgcn_readfirstlane(wave + NWV * u);
      if (b >= nblk) continue;
      if (b < nAblk) {
        if (b >= WRp / 16) r[u] = __builtin_amdgcn_raw_buffer_load_b128(rxl, voff[u], aso, 0);
        else r[u] = __builtin_amdgcn_raw_buffer_load_b128(rxh, voff[u], aso, 0);
      } else {
        r[u] = __builtin_amdgcn_raw_buffer_load_b128(rwh, voff[u], wso, 0);
      }
    }
  };
  auto store_regs = [&](const u32x4* r, uint8_t* buf) {
#pragma unroll
    for (int u = 0; u < MAXB; ++u) {
      const int b = __builtin_amdgcn_readfirstlane(wave + NWV * u);
      if (b >= nblk) continue;
      *(u32x4*)(buf + b * 1024 + lane * 16) = r[u];
    }
  };
  float acc = 0.f;
  typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
  typedef short sh8 __attribute__((ext_vector_type(8)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 macc[2][4];
  for (int m = 0; m < 2; ++m)
    for (int n = 0; n < 4; ++n) macc[m][n] = (f4){0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, g = lane >> 4;
  auto compute = [&](const uint8_t* cur) {
    const uint8_t* sW = cur + nAblk * 1024;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      sh8 bw[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) bw[n] = *(const sh8*)(sW + j * TN * 64 + swz(n * 16 + li, g));
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int wr = wave * 32 + m * 16 + li + j;
        const sh8 ah = *(const sh8*)(cur + swz(wr, g));
        const sh8 al = *(const sh8*)(cur + WRp * 64 + swz(wr, g));
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          macc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, ah), __builtin_bit_cast(bf8, bw[n]), macc[m][n], 0, 0, 0);
          macc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf8, al), __builtin_bit_cast(bf8, bw[n]), macc[m][n], 0, 0, 0);
        }
      }
    }
  };
  if (MODE == 4) {
    issue_dma(0, lds);
    for (int ck = 0; ck < a.nck; ++ck) {
      __syncthreads();
      const uint8_t* cur = lds + (ck & 1) * buf_bytes;
      if (ck + 1 < a.nck) issue_dma(ck + 1, lds + ((ck + 1) & 1) * buf_bytes);
      compute(cur);
    }
  } else if (MODE == 5) {
    for (int ck = 0; ck < a.nck; ++ck) {
      __syncthreads();
      compute(lds);
    }
  }
  for (int m = 0; m < 2; ++m)
    for (int n = 0; n < 4; ++n) acc += macc[m][n][0] + macc[m][n][3];
  if (MODE == 0) {
    issue_dma(0, lds);
    for (int ck = 0; ck < a.nck; ++ck) {
      __syncthreads();
      const uint8_t* cur = lds + (ck & 1) * buf_bytes;
      if (ck + 1 < a.nck) issue_dma(ck + 1, lds + ((ck + 1) & 1) * buf_bytes);
      acc += *(const float*)(cur + swz(tid & 255, lane & 3));
    }
  } else if (MODE == 1) {
    u32x4 r[MAXB];
    load_regs(0, r);
    for (int ck = 0; ck < a.nck; ++ck) {
      uint8_t* cur = lds + (ck & 1) * buf_bytes;
      store_regs(r, cur);
      if (ck + 1 < a.nck) load_regs(ck + 1, r);
      __syncthreads();
      acc += *(const float*)(cur + swz(tid & 255, lane & 3));
    }
  } else if (MODE == 2) {
    for (int ck = 0; ck < a.nck; ++ck) issue_dma(ck, lds + (ck & 1) * buf_bytes);
    __syncthreads();
    acc += *(const float*)(lds + swz(tid & 255, lane & 3));
  } else if (MODE == 3) {
    for (int ck = 0; ck < a.nck; ++ck) {
      u32x4 r[MAXB];
      load_regs(ck, r);
#pragma unroll
      for (int u = 0; u < MAXB; ++u) acc += __builtin_bit_cast(float, r[u].x ^ r[u].w);
    }
  }
  if (acc == 12345.678f) a.sink[tid] = acc;
}

int main(int argc, char** argv) {
  const int nutt = 32, rows = 81920, C = 192, K = 7, span = 6;
  const int nck = C / 32;
  const int64_t x_cs = (int64_t)rows * 32, x_bs = x_cs * nck;
  const size_t plane = (size_t)nutt * x_bs * 2;
  uint16_t *xh, *xl, *w;
  float* sink;
  CK(hipMalloc(&xh, plane));
  CK(hipMalloc(&xl, plane));
  CK(hipMalloc(&w, (size_t)C * K * C * 2));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(xh, 0, plane));
  CK(hipMemset(xl, 0, plane));
  CK(hipMemset(w, 0, (size_t)C * K * C * 2));
  Args a{xh, xl, w, x_bs, x_cs, rows, nck, K, C, C, span, nutt * rows / TM, C / TN, sink};
  const int WRp = (TM + span + 15) & ~15, nblk = 2 * WRp / 16 + 7 * (TN / 16);
  const int lds_bytes = 2 * nblk * 1024;
  const int grid = ((a.gx + 7) / 8) * 8 * a.gy;
  const double bytes_per_wg = (double)nblk * 1024 * nck;
  printf("grid %d WGs, %d blocks per chunk, LDS %d B, %.1f KB staged per WG\n", grid, nblk, lds_bytes, bytes_per_wg / 1024);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  void (*kern[6])(Args) = {k_stage<0>, k_stage<1>, k_stage<2>, k_stage<3>, k_stage<4>, k_stage<5>};
  const char* names[6] = {"dma double-buffered", "vgpr double-buffered", "dma all-up-front", "vgpr loads only",
                          "dma + mfma", "mfma only"};
  for (int m = 0; m < 6; ++m) {
    CK(hipFuncSetAttribute((const void*)kern[m], hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
    for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(kern[m], dim3(grid), dim3(512), lds_bytes, 0, a);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    const int reps = 5;
    for (int rep = 0; rep < reps; ++rep) hipLaunchKernelGGL(kern[m], dim3(grid), dim3(512), lds_bytes, 0, a);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const double tot = bytes_per_wg * grid;
    printf("mode %d %-22s %8.3f ms  %7.2f TB/s staged (L2->CU)  %.2f us per WG slot\n", m, names[m], ms,
           tot / ms / 1e9, ms * 1e3 / (grid / 256.0));
  }
  return 0;
}
