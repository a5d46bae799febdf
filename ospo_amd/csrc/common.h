// Shared device helpers for the OSPO MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ospo_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short i16x4;
typedef __attribute__((ext_vector_type(8))) short i16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

#define LDS_AS __attribute__((address_space(3)))
#define WAVE 64

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
__device__ __forceinline__ float round_bf(float x) { return (float)(bf16)x; }

// LoRA dropout mask (counter-based; ospo_amd/dropout.py restates it bit for bit):
// element idx = row * ncols + col of the adapter input, kept iff drop_keep(idx) (below);
// kept values become bf16(x / (1 - p)).
// Multiply rounds on 24-bit multiplies (v_mad_u32_u24, full rate; a 32-bit v_mul_lo_u32 is quarter rate).
// Round 5: every step is a bijection of all 32 bits, so the hash is a permutation of the pair index for each
// seed and no two pairs of any mask (up to 2^32 pairs) share a hash.  The round-4 form multiplied only the low
// 24 bits and dropped the top byte (x = (x & 0xFFFFFF) * c): pairs p and p ^ 0x01000100 collided for every
// seed, so masks beyond 2^24 pairs (the down adapter's [4800, 11008] input) repeated ~36 % of themselves
// ~3048 rows later.  A round is now x + lo24(x) * c with c even -- ONE v_mad_u32_u24 (x, c, x), as cheap as the
// old multiply: the low 24 bits of the result are lo24(x) * (c + 1) mod 2^24 (c + 1 odd: invertible), and
// x = result - lo24(x) * c recovers the top byte.  The seed enters after the first multiply + xorshift rather
// than as idx ^ seed, so the masks of two seeds are not one table re-indexed by an XOR.  Statistics
// (tools/hash_stats.py 'h6'): keep rate, both halves of a hash, row / column lags (incl. the old collision
// lag), cross-seed re-indexing and single-bit avalanche all at sampling noise.
__host__ __device__ __forceinline__ uint32_t drop_mad24(uint32_t x, uint32_t c) {
  return (x & 0xFFFFFFu) * c + x;
}
__host__ __device__ __forceinline__ uint32_t drop_hash(uint32_t idx, uint32_t seed) {
  uint32_t x = drop_mad24(idx, 0xED5AD4u);
  x ^= x >> 16;
  x ^= seed;
  x = drop_mad24(x, 0xAC4C1Au);
  x ^= x >> 15;
  x = drop_mad24(x, 0x9E3778u);
  x ^= x >> 13;
  x = drop_mad24(x, 0xC2B2AEu);
  x ^= x >> 16;
  return x;
}

// Keep decision of mask element idx: the 16-bit half (idx & 1) of drop_hash(idx >> 1), kept iff it is
// >= thr = p * 2^16 -- one hash per two adjacent elements of a row (since round 3 the forward's u product
// hashes each adapter input once per step and writes keep bits that the backward reads).  Callers that decide 2n consecutive elements start
// at an even index (row widths are even: the launchers check) and hash n times.
__host__ __device__ __forceinline__ bool drop_keep(uint32_t idx, uint32_t seed, uint32_t thr) {
  const uint32_t h = drop_hash(idx >> 1, seed);
  return ((idx & 1u) ? (h >> 16) : (h & 0xffffu)) >= thr;
}
// keep bits of elements idx0 .. idx0 + 2N - 1, idx0 even
template <int N>
__device__ __forceinline__ void drop_keep_pairs(uint32_t idx0, uint32_t seed, uint32_t thr, bool (&keep)[2 * N]) {
#pragma unroll
  for (int q = 0; q < N; ++q) {
    const uint32_t h = drop_hash((idx0 >> 1) + (uint32_t)q, seed);
    keep[2 * q] = (h & 0xffffu) >= thr;
    keep[2 * q + 1] = (h >> 16) >= thr;
  }
}
static inline uint32_t drop_threshold(double p) { return (uint32_t)(p * 65536.0); }

__device__ __forceinline__ float bits2f(unsigned short b) { return __uint_as_float(((unsigned)b) << 16); }
__device__ __forceinline__ unsigned short f2bits(float x) {
  bf16 h = (bf16)x;
  return *reinterpret_cast<unsigned short*>(&h);
}
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  return (unsigned)f2bits(lo) | ((unsigned)f2bits(hi) << 16);
}

__device__ __forceinline__ void unpack8(const u32x4& v, float* f) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = bits2f(v[q] & 0xffff);
    f[2 * q + 1] = bits2f(v[q] >> 16);
  }
}
__device__ __forceinline__ u32x4 pack8(const float* f) {
  u32x4 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = pack2(f[2 * q], f[2 * q + 1]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// GELU, exact erf form (torch.nn.GELU() default, projector.py / modeling_vlm.py).
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
// silu / sigmoid with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of the ~9-instruction IEEE divide:
// the results are rounded to bf16 next, where a 1-ulp fp32 difference flips a rounding on ~2e-5 of the
// elements; every kernel of the SwiGLU forward / backward (standalone, fused, decode) shares these.
__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// SwiGLU backward of 8 columns: d = dh (bf16 values), g / u = gate / up -> dg, du (fp32, rounded by the
// caller's pack).  h = bf16(silu(g)) * u, as HF's act_fn(gate) * up with a bf16 activation.
// Shared by swiglu_bwd_kernel and the GEMM epilogue that fuses it (bit-identical by construction).
__device__ __forceinline__ void swiglu_bwd8(const float* d, const float* g, const float* u, float* dg, float* du) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-g[q]));
    const float a = round_bf(g[q] * sg);
    du[q] = d[q] * a;
    const float da = round_bf(d[q] * u[q]);
    dg[q] = da * sg * (1.f + g[q] * (1.f - sg));
  }
}

#define OSPO_CHECK_LAUNCH()                                  \
  do {                                                       \
    hipError_t e__ = hipGetLastError();                      \
    if (e__ != hipSuccess) return OSPO_ERR_HIP;              \
  } while (0)

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
