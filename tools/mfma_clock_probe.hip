// MFMA loops vs the clock the chip holds under them (measurement only; not part of the product library).
// Round 5 form (verdict r4 item 3a): every wave issues v_mfma_f32_16x16x32_bf16 with 8 independent accumulators
// on 4 workgroups of 4 waves per CU; per wave s_memtime (core clock) and s_memrealtime (100 MHz) deltas around
// the loop go to a stamp buffer of their own.  Each variant runs >= 2 s of back-to-back launches before the
// measured launch (MI355X_MICROARCH.md 'DVFS give-back' item 6), every launch is checked for a HIP error and the
// program stops at the first one.
//   reg        operands held in registers
//   lds        operands re-read from LDS every 4 MFMAs: one ds_read_b128 per 4 MFMAs, as the w4 GEMM loop reads
//              its fragments, rotating over 8 slots of 2 KiB so consecutive reads return different data
//   lds+l2     lds, plus 16 B per lane per 8 MFMAs streamed from a 2-MiB (L2-resident) window
//   lds+hbm    lds, plus the same stream from a 1-GiB window (beyond the 256-MB Infinity Cache)
// each on random bf16 in [-1, 1) (a hash of lane / slot / element) and on all-zero operands.  Question: is the
// w4 GEMM's 1.65-1.76 GHz the MFMA data energy (random vs zero) or the staging traffic (lds+l2 / lds+hbm)?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_clock_probe tools/mfma_clock_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                         \
  do {                                                                                   \
    hipError_t e__ = (x);                                                                \
    if (e__ != hipSuccess) {                                                             \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e__), __FILE__, __LINE__);    \
      fflush(stdout);                                                                    \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

__device__ __forceinline__ __bf16 rand_bf16(unsigned x, bool zero) {
  x *= 0x9E3779B1u;
  x ^= x >> 15;
  x *= 0x85EBCA77u;
  x ^= x >> 13;
  const float f = (float)(x >> 8) * (1.0f / 8388608.0f) - 1.0f;  // [-1, 1)
  return (__bf16)(zero ? 0.0f : f);
}

// MODE 0 reg, 1 lds, 2 lds+l2, 3 lds+hbm
template <int MODE, bool ZERO>
__global__ __launch_bounds__(256) void mfma_burn(int iters, float* out, unsigned long long* st, const void* gsrc) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = rand_bf16(threadIdx.x * 16 + i, ZERO);
    b[i] = rand_bf16(threadIdx.x * 16 + 8 + i, ZERO);
  }
  f32x4 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float sink = 0.f;
  unsigned long long t0, r0;
  if constexpr (MODE == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j)  // inline asm: the builtin form's accumulators were shuffled through VGPRs
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
    }
  } else {
    __shared__ __attribute__((aligned(16))) __bf16 lds[8192];  // 16 KiB: 8 slots x (a 1 KiB | b 1 KiB) per wave group
    for (int e = threadIdx.x; e < 8192; e += 256) lds[e] = rand_bf16(0x1000u + e, ZERO);
    __syncthreads();
    const unsigned la = (unsigned)(uintptr_t)((__attribute__((address_space(3))) __bf16*)lds) + lane * 16;
    const long nglob = MODE == 3 ? (1L << 26) : (1L << 17);  // 16-B elements: 1 GiB / 2 MiB
    // index step reduced mod nglob: gi, gstride < nglob, so gi + gstride < 2 nglob and one conditional
    // subtraction keeps gi in [0, nglob)
    const long gstride = ((long)gridDim.x * 256) % nglob;
    const u32x4_t* gp = reinterpret_cast<const u32x4_t*>(gsrc);
    long gi = ((long)blockIdx.x * 256 + threadIdx.x) % nglob;
    u32x4_t gv[4] = {};
    unsigned gx = 0;
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it += 4) {
      const unsigned half = (unsigned)((it >> 2) & 1) * 8192u;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bf16x8 a2, b2;
        const unsigned addr = la + half + (unsigned)u * 2048u;
        asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(a2) : "v"(addr));
        asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(b2) : "v"(addr));
        if constexpr (MODE >= 2) {
          gx ^= gv[u][0] ^ gv[u][1] ^ gv[u][2] ^ gv[u][3];
          gv[u] = __builtin_nontemporal_load(gp + gi);
          gi += gstride;
          gi = gi >= nglob ? gi - nglob : gi;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a2), "+v"(b2));
        a = a2;
        b = b2;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) gx ^= gv[u][0] ^ gv[u][1] ^ gv[u][2] ^ gv[u][3];
    sink += (float)(gx & 1);
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // asm MFMA results: wait out their latency
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int j = 0; j < 8; ++j) sink += acc[j][0];
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  out[(long)blockIdx.x * 256 + threadIdx.x] = sink;
  if (lane < 2) st[w * 2 + lane] = lane == 0 ? t1 - t0 : r1 - r0;
}

static const char* kNames[4] = {"reg", "lds", "lds+l2", "lds+hbm"};

template <int MODE, bool ZERO>
static void run(int cus, int iters, float* out, unsigned long long* st, void* g) {
  const int grid = cus * 4;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // >= 2 s of back-to-back launches, then the measured one
  for (int w = 0; w < 4; ++w) {
    hipLaunchKernelGGL((mfma_burn<MODE, ZERO>), dim3(grid), dim3(256), 0, 0, iters, out, st, g);
    CHECK(hipGetLastError());
  }
  CHECK(hipEventRecord(e0, 0));
  hipLaunchKernelGGL((mfma_burn<MODE, ZERO>), dim3(grid), dim3(256), 0, 0, iters, out, st, g);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e1, 0));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipDeviceSynchronize());
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h((size_t)grid * 4 * 2);
  CHECK(hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  std::vector<double> clk;
  for (size_t w = 0; w < h.size() / 2; ++w)
    if (h[2 * w + 1]) clk.push_back((double)h[2 * w] / (double)h[2 * w + 1] * 0.1);
  std::sort(clk.begin(), clk.end());
  const double flops = (double)grid * 4 * iters * 8 * 16384.0;  // 8 MFMAs x 2*16*16*32 per iteration
  const double cyc_per_mfma = clk.empty() ? 0.0 : ms * 1e-3 * clk[clk.size() / 2] * 1e9 / ((double)iters * 8 * 4);
  printf("{\"variant\": \"%s\", \"data\": \"%s\", \"ms\": %.1f, \"tflops\": %.1f, \"clock_ghz_p10_p50_p90\": [%.3f, %.3f, %.3f], "
         "\"cycles_per_mfma_per_simd\": %.2f}\n",
         kNames[MODE], ZERO ? "zero" : "random", ms, flops / (ms * 1e-3) / 1e12, clk[clk.size() / 10],
         clk[clk.size() / 2], clk[clk.size() * 9 / 10], cyc_per_mfma);
  fflush(stdout);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = cus * 4;
  float* out;
  unsigned long long* st;
  void* g = nullptr;
  CHECK(hipMalloc(&out, (size_t)grid * 256 * sizeof(float)));
  CHECK(hipMalloc(&st, (size_t)grid * 4 * 2 * sizeof(unsigned long long)));
  CHECK(hipMalloc(&g, 1UL << 30));
  CHECK(hipMemset(g, 0x5a, 1UL << 30));
  CHECK(hipDeviceSynchronize());
  const int iters = 2000000;  // ~0.5 s per launch
  run<0, false>(cus, iters, out, st, g);
  run<0, true>(cus, iters, out, st, g);
  run<1, false>(cus, iters, out, st, g);
  run<1, true>(cus, iters, out, st, g);
  run<2, false>(cus, iters, out, st, g);
  run<2, true>(cus, iters, out, st, g);
  run<3, false>(cus, iters, out, st, g);
  run<3, true>(cus, iters, out, st, g);
  CHECK(hipFree(out));
  CHECK(hipFree(st));
  CHECK(hipFree(g));
  return 0;
}
