// MFMA shape vs sustained clock (measurement only; not part of the product library).
// Every wave issues bf16 MFMAs on register operands with 8 (16x16x32) or 4 (32x32x16) independent accumulators
// -- the same flops per iteration -- on 4 workgroups of 4 waves per CU for ~1 s, and records per wave
// s_memtime (core clock) and s_memrealtime (100 MHz constant) deltas with vector stores.  Prints achieved
// TFLOP/s and the mean core clock for each shape: does the 32x32 form (half the instructions and operand reads
// per flop) hold a higher clock under the power limit than the 16x16 form the GEMM loop uses?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_clock_probe tools/mfma_clock_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_burn(int iters, float* out, unsigned long long* st, const void* gsrc) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (float)((lane + i) & 7));
    b[i] = (__bf16)(0.001f * (float)((lane * 3 + i) & 7));
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  if constexpr (SHAPE == 16) {
    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j)  // inline asm: the builtin form's accumulators were shuffled through VGPRs
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sink += acc[j][0];
  } else if constexpr (SHAPE >= 17 && SHAPE <= 19) {
    // 16x16x32 at the GEMM loop's operand rates: one ds_read_b128 per 4 MFMAs (the w4 wave reads 32 KiB of
    // fragments per 128 MFMAs); 18 / 19 also load 16 B per lane per 8 MFMAs (~the w4 workgroup's 64 KiB of
    // LDS-DMA per K-tile and CU) from a 2-MiB (L2-resident) / 1-GiB (HBM) buffer, 4 iterations in flight
    typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
    __shared__ __attribute__((aligned(16))) char lds[16384];
    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    reinterpret_cast<bf16x8*>(lds)[threadIdx.x] = a;
    reinterpret_cast<bf16x8*>(lds)[256 + threadIdx.x] = b;
    __syncthreads();
    const unsigned la = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char*)lds) + threadIdx.x * 16;
    const long nglob = SHAPE == 19 ? (1L << 26) : (1L << 17);  // 16-B elements: 1 GiB / 2 MiB
    // index step reduced mod nglob: gi + gs < 2 nglob, so one conditional subtraction keeps gi in range (the
    // unreduced step, 256 x grid 16-B elements, exceeds the 2-MiB window: that form walked off the buffer)
    const long gstride = ((long)gridDim.x * 256) % nglob;
    const u32x4_t* gp = reinterpret_cast<const u32x4_t*>(gsrc);
    long gi = ((long)blockIdx.x * 256 + threadIdx.x) % nglob;
    u32x4_t gv[4] = {};
    unsigned gx = 0;
    for (int it = 0; it < iters; it += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bf16x8 a2, b2;
        asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(a2) : "v"(la));
        asm volatile("ds_read_b128 %0, %1 offset:4096" : "=v"(b2) : "v"(la));
        if constexpr (SHAPE >= 18) {
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
    for (int j = 0; j < 8; ++j) sink += acc[j][0];
#pragma unroll
    for (int u = 0; u < 4; ++u) gx ^= gv[u][0] ^ gv[u][1] ^ gv[u][2] ^ gv[u][3];
    sink += (float)(gx & 1);
  } else {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) sink += acc[j][0];
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // asm MFMA results: wait out their latency
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  out[(long)blockIdx.x * 256 + threadIdx.x] = sink;
  if (lane < 2) st[w * 2 + lane] = lane == 0 ? t1 - t0 : r1 - r0;
}

template <int SHAPE>
static void run(int cus, int iters) {
  const int grid = cus * 4;
  float* out;
  unsigned long long* st;
  if (hipMalloc(&out, (size_t)grid * 256 * sizeof(float)) != hipSuccess ||
      hipMalloc(&st, (size_t)grid * 4 * 2 * sizeof(unsigned long long)) != hipSuccess) {
    printf("alloc failed\n");
    exit(1);
  }
  void* g = nullptr;
  if (hipMalloc(&g, 1UL << 30) != hipSuccess || hipMemset(g, 1, 1UL << 30) != hipSuccess) {
    printf("alloc failed\n");
    exit(1);
  }
  hipLaunchKernelGGL(mfma_burn<SHAPE>, dim3(grid), dim3(256), 0, 0, iters / 10, out, st, g);  // warm-up
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(mfma_burn<SHAPE>, dim3(grid), dim3(256), 0, 0, iters, out, st, g);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h((size_t)grid * 4 * 2);
  hipMemcpy(h.data(), st, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double core = 0, real = 0;
  for (size_t w = 0; w < h.size() / 2; ++w) {
    core += (double)h[2 * w];
    real += (double)h[2 * w + 1];
  }
  const double flops = (double)grid * 4 * iters * 131072.0;
  const char* nm = SHAPE == 16 ? "16x16x32" : SHAPE == 32 ? "32x32x16" : SHAPE == 17 ? "16x16x32+lds"
                   : SHAPE == 18 ? "16x16x32+lds+l2" : "16x16x32+lds+hbm";
  printf("{\"variant\": \"%s\", \"ms\": %.1f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n", nm, ms,
         flops / (ms * 1e-3) / 1e12, core / real * 0.1);
  fflush(stdout);
  hipFree(out);
  hipFree(st);
  hipFree(g);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int iters = 4000000;
  for (int r = 0; r < 2; ++r) {
    run<16>(cus, iters);
    run<32>(cus, iters);
    run<17>(cus, iters);
    run<18>(cus, iters);
    run<19>(cus, iters);
  }
  return 0;
}
