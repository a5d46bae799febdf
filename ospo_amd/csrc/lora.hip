// Skinny LoRA products on MFMA for the PEFT adapters of the Janus-Pro decoder
// (peft 0.9 lora.Linear, y += s * B(A x); reached from ospo/wrapper/train.py:352
// through every q/k/v/o/gate/up/down projection).
//
//   u = s * x . A_cat^T    [M, 16*nt]   (forward; the GEMM's K-extension operand)
//   g = s * dy . B         [M, 16*nt]   (backward; block-diagonal over modules)
//
// Both are [M, <=64] outputs reducing over a long K (4096 .. 22016): pure HBM
// streams of the activation (x or dy), the adapter operand is L2-resident.  A
// workgroup owns 16 rows; its waves split K (interleaved 32-wide steps) with
// operands loaded straight into MFMA fragments (no LDS staging: every element
// of the row block is used exactly once per n-tile), partial sums are reduced
// through LDS and written as bf16 -- no fp32 atomics, no zero-fill, no
// separate convert pass.  Any permutation of k is legal as long as A and B
// agree, so each lane streams its own 16-B chunk of the row.
#include "common.h"

namespace {

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

constexpr int SK_WAVES = 8;
constexpr int SK_U = 4;  // k-steps per register batch; two batches in flight per wave

// One wave's share of the reduction: steps s = wave + i*SK_WAVES, i < n_i.
// Register double-buffered batches keep 2*SK_U*(1+NTL) 1-KiB loads in flight
// (addresses clamped, tail steps zeroed in A), no branches in the loop.
template <int NTL>
__device__ __forceinline__ void sk_loop(const bf16* arow, const bf16* const (&bp)[NTL], const bool (&bok)[NTL],
                                        int wave, int n_i, f32x4 (&acc)[NTL]) {
  if (n_i <= 0) return;
  bf16x8 a0[SK_U], b0[SK_U][NTL], a1[SK_U], b1[SK_U][NTL];
  auto load = [&](int batch, bf16x8 (&a)[SK_U], bf16x8 (&b)[SK_U][NTL]) {
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      int i = batch * SK_U + u;
      i = i < n_i ? i : n_i - 1;
      const int off = 32 * (wave + i * SK_WAVES);
      a[u] = *reinterpret_cast<const bf16x8*>(arow + off);
#pragma unroll
      for (int j = 0; j < NTL; ++j) b[u][j] = *reinterpret_cast<const bf16x8*>(bp[j] + off);
    }
  };
  auto consume = [&](int batch, const bf16x8 (&a)[SK_U], const bf16x8 (&b)[SK_U][NTL]) {
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const bf16x8 av = (batch * SK_U + u < n_i) ? a[u] : bf16x8{};
#pragma unroll
      for (int j = 0; j < NTL; ++j)
        acc[j] = MFMA(bok[j] ? b[u][j] : bf16x8{}, av, acc[j]);  // D[n][m]: lane m = l16, n = 4g..4g+3
    }
  };
  const int nb = (n_i + SK_U - 1) / SK_U;
  load(0, a0, b0);
  for (int bt = 0; bt < nb; bt += 2) {
    load(bt + 1, a1, b1);
    consume(bt, a0, b0);
    if (bt + 1 >= nb) break;
    load(bt + 2, a0, b0);
    consume(bt + 1, a1, b1);
  }
}

// out[m][16j + c] = scale * sum_k A[m][j*a_koff + k] * Bt[16j + c][k]
template <int NT>
__global__ __launch_bounds__(64 * SK_WAVES) void skinny_kernel(const bf16* __restrict__ A, int lda,
                                                               const bf16* __restrict__ Bt, int ldb, int b_rows,
                                                               int M, int M_out, int K, int a_koff, float scale,
                                                               bf16* __restrict__ out, int ldo, int out_cols) {
  __shared__ f32x4 red[SK_WAVES][NT][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int m0 = blockIdx.x * 16;
  int row = m0 + l16;
  row = row < M ? row : M - 1;
  const int nsteps = K >> 5;
  const int n_i = (nsteps - wave + SK_WAVES - 1) / SK_WAVES;  // this wave's steps

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* arow = A + (long)row * lda + 8 * g;
  if (a_koff == 0) {  // dense: one A fragment feeds every n-tile
    const bf16* bp[NT];
    bool bok[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int br = 16 * j + l16;
      bok[j] = br < b_rows;
      bp[j] = Bt + (long)(bok[j] ? br : 0) * ldb + 8 * g;
    }
    sk_loop<NT>(arow, bp, bok, wave, n_i, acc);
  } else {  // block-diagonal: n-tile j reduces over its own K block of A
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int br = 16 * j + l16;
      const bool ok1[1] = {br < b_rows};
      const bf16* const bp1[1] = {Bt + (long)(ok1[0] ? br : 0) * ldb + 8 * g};
      f32x4 acc1[1] = {acc[j]};
      sk_loop<1>(arow + (long)j * a_koff, bp1, ok1, wave, n_i, acc1);
      acc[j] = acc1[0];
    }
  }

#pragma unroll
  for (int j = 0; j < NT; ++j) red[wave][j][lane] = acc[j];
  __syncthreads();
  const int m = m0 + l16;
  for (int j = wave; j < NT; j += SK_WAVES) {
    f32x4 v = red[0][j][lane];
#pragma unroll
    for (int w = 1; w < SK_WAVES; ++w) v += red[w][j][lane];
    if (m < M_out) {
      uint2 pk;
      if (m < M) {
        pk.x = pack2(v[0] * scale, v[1] * scale);
        pk.y = pack2(v[2] * scale, v[3] * scale);
      } else {
        pk.x = pk.y = 0u;
      }
      *reinterpret_cast<uint2*>(out + (long)m * ldo + 16 * j + 4 * g) = pk;
    }
  }
  // zero padding columns 16*NT .. out_cols-1 of this row block
  const int pad = out_cols - 16 * NT;
  for (int i = threadIdx.x; i < 16 * pad; i += 64 * SK_WAVES) {
    const int r = m0 + i / pad;
    if (r < M_out) out[(long)r * ldo + 16 * NT + i % pad] = f2bf(0.f);
  }
}

}  // namespace

extern "C" int ospo_lora_skinny(const void* A, int lda, const void* Bt, int ldb, int b_rows, int M, int M_out, int K,
                                int n_tiles, int a_koff, float scale, void* out, int ldo, int out_cols,
                                hipStream_t stream) {
  if (!A || !Bt || !out) return OSPO_ERR_ARG;
  if (M <= 0 || M_out < M || K <= 0 || n_tiles < 1 || n_tiles > 4 || b_rows <= 0 || a_koff < 0) return OSPO_ERR_SHAPE;
  if (K % 32 || lda % 8 || ldb % 8 || a_koff % 8 || ldo % 4 || out_cols < 16 * n_tiles || ldo < out_cols)
    return OSPO_ERR_SHAPE;
  if (ldb < K || (a_koff == 0 && lda < K) || (a_koff > 0 && lda < (n_tiles - 1) * a_koff + K)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(Bt) || ((uintptr_t)out & 7)) return OSPO_ERR_ALIGN;
  const dim3 grid((M_out + 15) / 16), block(64 * SK_WAVES);
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)Bt;
  bf16* o = (bf16*)out;
  switch (n_tiles) {
    case 1: hipLaunchKernelGGL(skinny_kernel<1>, grid, block, 0, stream, a, lda, b, ldb, b_rows, M, M_out, K, a_koff, scale, o, ldo, out_cols); break;
    case 2: hipLaunchKernelGGL(skinny_kernel<2>, grid, block, 0, stream, a, lda, b, ldb, b_rows, M, M_out, K, a_koff, scale, o, ldo, out_cols); break;
    case 3: hipLaunchKernelGGL(skinny_kernel<3>, grid, block, 0, stream, a, lda, b, ldb, b_rows, M, M_out, K, a_koff, scale, o, ldo, out_cols); break;
    default: hipLaunchKernelGGL(skinny_kernel<4>, grid, block, 0, stream, a, lda, b, ldb, b_rows, M, M_out, K, a_koff, scale, o, ldo, out_cols); break;
  }
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
