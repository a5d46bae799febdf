// MFMA shape vs sustained clock (measurement only; not part of the product library).
// Every wave issues bf16 MFMAs on register operands with 8 (16x16x32) or 4 (32x32x16) independent accumulators
// -- the same flops per iteration -- on 4 workgroups of 4 waves per CU for ~1 s, and records per wave
// s_memtime (core clock) and s_memrealtime (100 MHz constant) deltas with vector stores.  Prints achieved
// TFLOP/s and the mean core clock for each shape: does the 32x32 form (half the instructions and operand reads
// per flop) hold a higher clock under the power limit than the 16x16 form the GEMM loop uses?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_clock_probe tools/mfma_clock_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE>
__global__ __launch_bounds__(256) void mfma_burn(int iters, float* out, unsigned long long* st) {
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
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) sink += acc[j][0];
  } else {
    f32x16 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) sink += acc[j][0];
  }
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
  hipMalloc(&out, (size_t)grid * 256 * sizeof(float));
  hipMalloc(&st, (size_t)grid * 4 * 2 * sizeof(unsigned long long));
  hipLaunchKernelGGL(mfma_burn<SHAPE>, dim3(grid), dim3(256), 0, 0, iters / 10, out, st);  // warm-up
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(mfma_burn<SHAPE>, dim3(grid), dim3(256), 0, 0, iters, out, st);
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
  printf("{\"shape\": \"%dx%d\", \"ms\": %.1f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n", SHAPE, SHAPE, ms,
         flops / (ms * 1e-3) / 1e12, core / real * 0.1);
  fflush(stdout);
  hipFree(out);
  hipFree(st);
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int iters = 4000000;
  for (int r = 0; r < 2; ++r) {
    run<16>(cus, iters);
    run<32>(cus, iters);
  }
  return 0;
}
