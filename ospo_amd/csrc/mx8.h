// MXFP8 block quantization helpers shared by the standalone quantizer (mx8.hip) and the producer
// kernels that emit an MXFP8 copy of their output directly (ops.hip: RMSNorm fwd/bwd, SwiGLU
// fwd/bwd of the fp8 variant), so both produce the same bytes.  Format and scale layout: mx8.hip.
#pragma once
#include "common.h"

// E8M0 scale byte of a 32-block from its amax (round-up rule) and the matching 1 / X
__device__ __forceinline__ int mx8_scale_byte(float amax) {
  const uint32_t abits = __float_as_uint(amax);
  const int ebits = (int)((abits >> 23) & 0xff);
  return min(max(ebits - 8 + ((abits & 0x7fffffu) > 0x600000u ? 1 : 0), 0), 254);
}
__device__ __forceinline__ float mx8_inv_scale(int sbyte) { return __uint_as_float((uint32_t)(254 - sbyte) << 23); }
// 4 values -> 4 e4m3 bytes (clamped to +-448 first: v_cvt_pk_fp8_f32 is RNE below, NaN beyond)
__device__ __forceinline__ uint32_t mx8_pack4(float a, float b, float c, float d, float inv) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(a * inv, -448.f), 448.f), fminf(fmaxf(b * inv, -448.f), 448.f),
                                          0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(c * inv, -448.f), 448.f), fminf(fmaxf(d * inv, -448.f), 448.f), r,
                                      true);
  return (uint32_t)r;
}
// byte offset of the scale of (row, 32-block b) in the GEMM's tile layout, KT = K / 128
__device__ __forceinline__ long mx8_scale_index(long row, int b, int KT) {
  return (((row >> 6) * KT + (b >> 2)) * 64 + (b & 3) * 16 + (row & 15)) * 4 + ((row & 63) >> 4);
}

// An MXFP8 output of a producer kernel (q == nullptr: none)
struct Mx8Out {
  uint8_t* q;
  int ldq;
  uint8_t* s;
  int K;
};

// Quantize the 8 consecutive (already bf16-valued) outputs v of row `row`, columns 8 c8 .. 8 c8 + 7.
// The 4 lanes 4k .. 4k+3 of the wave must hold one 32-block (c8 = 4 b .. 4 b + 3), all active.
__device__ __forceinline__ void mx8_store8(const Mx8Out& mo, long row, int c8, const float (&v)[8]) {
  float amax = 0.f;
#pragma unroll
  for (int q = 0; q < 8; ++q) amax = fmaxf(amax, fabsf(v[q]));
  amax = fmaxf(amax, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(amax), 0xb1, 0xf, 0xf, false)));
  amax = fmaxf(amax, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(amax), 0x4e, 0xf, 0xf, false)));
  const int sbyte = mx8_scale_byte(amax);
  const float inv = mx8_inv_scale(sbyte);
  uint2 o;
  o.x = mx8_pack4(v[0], v[1], v[2], v[3], inv);
  o.y = mx8_pack4(v[4], v[5], v[6], v[7], inv);
  *reinterpret_cast<uint2*>(mo.q + row * mo.ldq + 8 * c8) = o;
  if ((c8 & 3) == 0) mo.s[mx8_scale_index(row, c8 >> 2, mo.K >> 7)] = (uint8_t)sbyte;
}
