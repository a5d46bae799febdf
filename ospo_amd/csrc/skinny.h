// Register-direct skinny MFMA reduction loop shared by the LoRA products (lora.hip) and the
// step-3 decode GEMV (decode.hip): a [16-row x long-K] operand streamed straight into
// v_mfma_f32_16x16x32_bf16 fragments against <= 4 small tiles, no LDS staging.
#pragma once
#include "common.h"

namespace {

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

constexpr int SK_WAVES = 4;
constexpr int SK_U = 4;  // k-steps per register batch; two batches in flight per wave

// LoRA dropout on the A operand (the adapter input x), dense mode only: the lane's
// 8 elements of step s sit at columns k0 + 32 s .. +7 of row `row`; the masked
// fragment is also stored to xd (the backward's dA operand) when `xd` is set.
struct SkDrop {
  uint32_t seed, thresh, rowidx;  // rowidx = row * ncols
  float scale;
  int k0;                         // absolute column of the lane at step 0
  bf16* xd;                       // xd + row * ld (nullptr: do not store)
};

// One wave's share of the reduction: steps s = wave + i*SK_WAVES, i < n_i.
// Register double-buffered batches keep 2*SK_U*(1+NTL) 1-KiB loads in flight
// (addresses clamped, tail steps zeroed in A), no branches in the loop.
template <int NTL, bool DROP = false>
__device__ __forceinline__ void sk_loop(const bf16* arow, const bf16* const (&bp)[NTL], const bool (&bok)[NTL],
                                        int wave, int n_i, f32x4 (&acc)[NTL], const SkDrop& dp = SkDrop{}) {
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
      bf16x8 av = (batch * SK_U + u < n_i) ? a[u] : bf16x8{};
      if constexpr (DROP) {
        const int k = dp.k0 + 32 * (wave + (batch * SK_U + u) * SK_WAVES);
        bool keep[8];
        drop_keep_pairs<4>(dp.rowidx + (uint32_t)k, dp.seed, dp.thresh, keep);
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = keep[e] ? f2bf(bf2f(av[e]) * dp.scale) : f2bf(0.f);
        if (dp.xd && batch * SK_U + u < n_i) *reinterpret_cast<bf16x8*>(dp.xd + k) = av;
      }
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

}  // namespace
