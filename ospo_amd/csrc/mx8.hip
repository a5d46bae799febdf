// MXFP8 (OCP MX, e4m3 elements, E8M0 scale per 32-element block along K) quantization of the
// operands of the fp8 SimPO variant (BASELINE config 5).
//
// Per block of 32 values along K (OCP MX v1.0 element/scale formats): X = the smallest power of two
// with amax / X <= 448 (round-up scale; the spec's floor rule would clip block maxima by up to
// 12.5 %), q = e4m3_rne(clamp(x / X, -448, 448)).  With amax = m * 2^E: scale byte = E + 127 - 8,
// +1 when m > 1.75, clamped to [0, 254] (amax = 0 -> byte 0) -- read off the f32 bits exactly;
// x / X is an exact power-of-two multiply, and v_cvt_pk_fp8_f32 is RNE on |x| <= 448
// (tools/mx8_probe.hip; beyond it the hardware returns NaN, hence the clamp).  oracle/mx8_ref.py
// restates this and the tests compare the bytes exactly.
//
// Scale layout (what gemm_nt_v5_kernel<.., MX> streams into LDS, one 256-B line per wave):
//   u32 index ((row / 64) * (K / 128) + k / 128) * 64 + ((k % 128) / 32) * 16 + row % 16,
//   byte (row % 64) / 16
// so lane l of a 16-row MFMA fragment finds the scale of (row l & 15, k-block l >> 4) in one
// dword, with OPSEL picking the fragment's 16-row group.  Rows are padded to a multiple of 256
// (the GEMM tile); the padding's scales are written as 0.
#include "mx8.h"

namespace {

__global__ __launch_bounds__(256) void quant_mx8_kernel(const bf16* __restrict__ X, int ldx, int M, int Mp, int K,
                                                        uint8_t* __restrict__ Q, int ldq, uint8_t* __restrict__ S) {
  const int nb = K >> 5;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)Mp * nb) return;
  const int row = (int)(idx / nb), b = (int)(idx % nb);
  const int KT = K >> 7;
  const long sidx = mx8_scale_index(row, b, KT);
  if (row >= M) {
    S[sidx] = 0;
    return;
  }
  const bf16* src = X + (long)row * ldx + b * 32;
  u32x4 w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = *reinterpret_cast<const u32x4*>(src + 8 * i);
  float v[32];
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[8 * i + 2 * q] = __uint_as_float(w[i][q] << 16);
      v[8 * i + 2 * q + 1] = __uint_as_float(w[i][q] & 0xffff0000u);
      amax = fmaxf(amax, fmaxf(fabsf(v[8 * i + 2 * q]), fabsf(v[8 * i + 2 * q + 1])));
    }
  const int sbyte = mx8_scale_byte(amax);
  const float inv = mx8_inv_scale(sbyte);
  uint32_t o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = mx8_pack4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3], inv);
  uint8_t* dst = Q + (long)row * ldq + b * 32;
  *reinterpret_cast<u32x4*>(dst) = u32x4{o[0], o[1], o[2], o[3]};
  *reinterpret_cast<u32x4*>(dst + 16) = u32x4{o[4], o[5], o[6], o[7]};
  S[sidx] = (uint8_t)sbyte;
}

}  // namespace

extern "C" size_t ospo_mx8_scale_bytes(int M, int K) {
  if (M <= 0 || K <= 0 || K % 128) return 0;
  return (size_t)((M + 255) / 256) * 4 * (size_t)(K / 128) * 256;
}

extern "C" int ospo_quant_mx8(const void* X, int ldx, int M, int K, void* Q, int ldq, void* S, hipStream_t stream) {
  if (!X || !Q || !S) return OSPO_ERR_ARG;
  if (M <= 0 || K <= 0 || K % 128) return OSPO_ERR_SHAPE;
  if (ldx < K || ldx % 8 || ldq < K || ldq % 16) return OSPO_ERR_SHAPE;
  if (!aligned16(X) || !aligned16(Q) || !aligned16(S)) return OSPO_ERR_ALIGN;
  const int Mp = (M + 255) / 256 * 256;
  const long n = (long)Mp * (K / 32);
  hipLaunchKernelGGL(quant_mx8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const bf16*)X, ldx, M,
                     Mp, K, (uint8_t*)Q, ldq, (uint8_t*)S);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
