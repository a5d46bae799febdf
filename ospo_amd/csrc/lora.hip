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
#include "skinny.h"

namespace {

// out[m][16j + c] = scale * sum_k A[m][j*a_koff + k] * Bt[16j + c][k]
// grid (row blocks of 16, K splits).  Each workgroup reduces its K range; with
// splits > 1 the fp32 partial tile goes to ws and skinny_reduce_kernel sums the
// splits (a cross-workgroup handoff inside one launch would need an agent-scope
// release, i.e. an L2 writeback per workgroup on gfx950 -- far dearer).
template <int NT, bool DROP>
__global__ __launch_bounds__(64 * SK_WAVES) void skinny_kernel(const bf16* __restrict__ A, int lda,
                                                               const bf16* __restrict__ Bt, int ldb, int b_rows,
                                                               int M, int M_out, int K, int a_koff, float scale,
                                                               bf16* __restrict__ out, int ldo, int out_cols,
                                                               f32x4* __restrict__ ws, uint32_t dseed,
                                                               uint32_t dthresh, float dscale, bf16* __restrict__ xd,
                                                               int ldxd) {
  __shared__ f32x4 red[SK_WAVES][NT][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int rb = blockIdx.x, z = blockIdx.y, splits = gridDim.y;
  const int m0 = rb * 16;
  int row = m0 + l16;
  row = row < M ? row : M - 1;
  const int nsteps = K >> 5;
  const int s_begin = (int)((long)nsteps * z / splits), s_end = (int)((long)nsteps * (z + 1) / splits);
  const int n_i = (s_end - s_begin - wave + SK_WAVES - 1) / SK_WAVES;  // this wave's steps

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bf16* arow = A + (long)row * lda + 8 * g + 32 * s_begin;
  if (a_koff == 0) {  // dense: one A fragment feeds every n-tile
    const bf16* bp[NT];
    bool bok[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int br = 16 * j + l16;
      bok[j] = br < b_rows;
      bp[j] = Bt + (long)(bok[j] ? br : 0) * ldb + 8 * g + 32 * s_begin;
    }
    if constexpr (DROP) {
      SkDrop dp;
      dp.seed = dseed;
      dp.thresh = dthresh;
      dp.scale = dscale;
      dp.rowidx = (uint32_t)row * (uint32_t)K;
      dp.k0 = 32 * s_begin + 8 * g;
      dp.xd = (xd && m0 + l16 < M) ? xd + (long)row * ldxd : nullptr;
      sk_loop<NT, true>(arow, bp, bok, wave, n_i, acc, dp);
    } else {
      sk_loop<NT>(arow, bp, bok, wave, n_i, acc);
    }
  } else {  // block-diagonal: n-tile j reduces over its own K block of A
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int br = 16 * j + l16;
      const bool ok1[1] = {br < b_rows};
      const bf16* const bp1[1] = {Bt + (long)(ok1[0] ? br : 0) * ldb + 8 * g + 32 * s_begin};
      f32x4 acc1[1] = {acc[j]};
      sk_loop<1>(arow + (long)j * a_koff, bp1, ok1, wave, n_i, acc1);
      acc[j] = acc1[0];
    }
  }

#pragma unroll
  for (int j = 0; j < NT; ++j) red[wave][j][lane] = acc[j];
  __syncthreads();
  // wave j (< NT) owns n-tile j: sum the waves' partials
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  if (wave < NT) {
#pragma unroll
    for (int w = 0; w < SK_WAVES; ++w) v += red[w][wave][lane];
  }
  if (splits > 1) {  // fp32 partial; skinny_reduce_kernel sums the splits
    if (wave < NT) ws[((long)(z * gridDim.x + rb) * NT + wave) * 64 + lane] = v;
    return;
  }
  const int m = m0 + l16;
  if (wave < NT && m < M_out) {
    uint2 pk;
    if (m < M) {
      pk.x = pack2(v[0] * scale, v[1] * scale);
      pk.y = pack2(v[2] * scale, v[3] * scale);
    } else {
      pk.x = pk.y = 0u;
    }
    *reinterpret_cast<uint2*>(out + (long)m * ldo + 16 * wave + 4 * g) = pk;
  }
  // zero padding columns 16*NT .. out_cols-1 of this row block
  const int pad = out_cols - 16 * NT;
  for (int i = threadIdx.x; i < 16 * pad; i += 64 * SK_WAVES) {
    const int r = m0 + i / pad;
    if (r < M_out) out[(long)r * ldo + 16 * NT + i % pad] = f2bf(0.f);
  }
}

// sum the split partials of one row block: block = NT waves, wave j = n-tile j
template <int NT>
__global__ __launch_bounds__(64 * NT) void skinny_reduce_kernel(const f32x4* __restrict__ ws, int splits, int RB,
                                                               int M, int M_out, float scale, bf16* __restrict__ out,
                                                               int ldo, int out_cols) {
  const int lane = threadIdx.x & 63, j = threadIdx.x >> 6;
  const int rb = blockIdx.x, g = lane >> 4, l16 = lane & 15;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < splits; ++z) v += ws[((long)(z * RB + rb) * NT + j) * 64 + lane];
  const int m = rb * 16 + l16;
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
  const int pad = out_cols - 16 * NT;
  for (int i = threadIdx.x; i < 16 * pad; i += 64 * NT) {
    const int r = rb * 16 + i / pad;
    if (r < M_out) out[(long)r * ldo + 16 * NT + i % pad] = f2bf(0.f);
  }
}

}  // namespace

// K splits: enough workgroups to keep every CU streaming (>= ~4 per CU), each
// split >= 512 k; the workspace holds splits x row_blocks fp32 partial tiles.
static int skinny_splits(int M_out, int K) {
  const int rb = (M_out + 15) / 16;
  int s = 1;
  while (s < 16 && (long)rb * s < 1024 && K / (32 * (s * 2)) >= 16) s *= 2;
  return s;
}

extern "C" size_t ospo_lora_skinny_ws_bytes(int M_out, int K, int n_tiles) {
  const long rb = (M_out + 15) / 16;
  const int sp = skinny_splits(M_out, K);
  return (size_t)(sp > 1 ? sp : 0) * rb * n_tiles * 64 * sizeof(f32x4) + 16;
}

struct SkDropArgs {
  uint32_t seed = 0, thresh = 0;
  float scale = 0.f;  // > 0: dropout on
  bf16* xd = nullptr;
  int ldxd = 0;
};

#define SK_LAUNCH(NTV, DV)                                                                                        \
  hipLaunchKernelGGL((skinny_kernel<NTV, DV>), grid, block, 0, stream, a, lda, b, ldb, b_rows, M, M_out, K, a_koff, \
                     scale, o, ldo, out_cols, part, dr.seed, dr.thresh, dr.scale, dr.xd, dr.ldxd)

static int launch_skinny(const bf16* a, int lda, const bf16* b, int ldb, int b_rows, int M, int M_out, int K,
                         int n_tiles, int a_koff, float scale, bf16* o, int ldo, int out_cols, f32x4* part,
                         hipStream_t stream, const SkDropArgs& dr = SkDropArgs{}) {
  const int rbn = (M_out + 15) / 16;
  const int sp = skinny_splits(M_out, K);
  const dim3 grid(rbn, sp), block(64 * SK_WAVES);
  const bool drop = dr.scale > 0.f;
  switch (n_tiles) {
    case 1: if (drop) SK_LAUNCH(1, true); else SK_LAUNCH(1, false); break;
    case 2: if (drop) SK_LAUNCH(2, true); else SK_LAUNCH(2, false); break;
    case 3: if (drop) SK_LAUNCH(3, true); else SK_LAUNCH(3, false); break;
    default: if (drop) SK_LAUNCH(4, true); else SK_LAUNCH(4, false); break;
  }
  OSPO_CHECK_LAUNCH();
  if (sp > 1) {
    switch (n_tiles) {
      case 1: hipLaunchKernelGGL(skinny_reduce_kernel<1>, dim3(rbn), dim3(64), 0, stream, part, sp, rbn, M, M_out, scale, o, ldo, out_cols); break;
      case 2: hipLaunchKernelGGL(skinny_reduce_kernel<2>, dim3(rbn), dim3(128), 0, stream, part, sp, rbn, M, M_out, scale, o, ldo, out_cols); break;
      case 3: hipLaunchKernelGGL(skinny_reduce_kernel<3>, dim3(rbn), dim3(192), 0, stream, part, sp, rbn, M, M_out, scale, o, ldo, out_cols); break;
      default: hipLaunchKernelGGL(skinny_reduce_kernel<4>, dim3(rbn), dim3(256), 0, stream, part, sp, rbn, M, M_out, scale, o, ldo, out_cols); break;
    }
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}

extern "C" int ospo_lora_skinny(const void* A, int lda, const void* Bt, int ldb, int b_rows, int M, int M_out, int K,
                                int n_tiles, int a_koff, int module_tiles, float scale, void* out, int ldo,
                                int out_cols, void* ws, size_t ws_bytes, unsigned drop_seed, float drop_p, void* xd,
                                int ld_xd, hipStream_t stream) {
  if (!A || !Bt || !out || !ws) return OSPO_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  SkDropArgs dr;
  if (drop_p > 0.f) {
    if (a_koff != 0) return OSPO_ERR_UNSUPPORTED;  // dropout acts on the adapter input (dense u product)
    if ((long)M * K > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
    if (xd && (ld_xd < K || ld_xd % 8 || !aligned16(xd))) return OSPO_ERR_SHAPE;
    dr.seed = drop_seed;
    dr.thresh = (uint32_t)((double)drop_p * 4294967296.0);
    dr.scale = 1.f / (1.f - drop_p);
    dr.xd = (bf16*)xd;
    dr.ldxd = ld_xd;
  }
  if (M <= 0 || M_out < M || K <= 0 || n_tiles < 1 || n_tiles > 16 || b_rows <= 0 || a_koff < 0 || module_tiles < 1)
    return OSPO_ERR_SHAPE;
  if (K % 32 || lda % 8 || ldb % 8 || a_koff % 8 || ldo % 4 || out_cols < 16 * n_tiles || ldo < out_cols)
    return OSPO_ERR_SHAPE;
  if (a_koff > 0 && n_tiles % module_tiles) return OSPO_ERR_SHAPE;
  const int nmods = a_koff > 0 ? n_tiles / module_tiles : 1;
  if (ldb < K || (a_koff == 0 && lda < K) || (a_koff > 0 && lda < (nmods - 1) * a_koff + K)) return OSPO_ERR_SHAPE;
  if (ws_bytes < ospo_lora_skinny_ws_bytes(M_out, K, n_tiles)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(Bt) || !aligned16(ws) || ((uintptr_t)out & 7)) return OSPO_ERR_ALIGN;
  const bf16* a = (const bf16*)A;
  const bf16* b = (const bf16*)Bt;
  bf16* o = (bf16*)out;
  f32x4* part = (f32x4*)ws;
  if (a_koff > 0 && module_tiles == 1 && n_tiles <= 4)  // one launch: n-tile j reduces over block j of A
    return launch_skinny(a, lda, b, ldb, b_rows, M, M_out, K, n_tiles, a_koff, scale, o, ldo, out_cols, part, stream,
                         dr);
  // general form: per module (block-diagonal) or the whole matrix (dense), in chunks of <= 4 n-tiles;
  // each chunk zero-pads only its own columns, the last one also the tail up to out_cols
  for (int mi = 0; mi < nmods; ++mi) {
    const int t0 = a_koff > 0 ? mi * module_tiles : 0, tn = a_koff > 0 ? module_tiles : n_tiles;
    for (int c0 = 0; c0 < tn; c0 += 4) {
      const int nt = tn - c0 < 4 ? tn - c0 : 4;
      const int j0 = t0 + c0;
      const bool last = (mi == nmods - 1) && (c0 + nt == tn);
      const int oc = last ? out_cols - 16 * j0 : 16 * nt;
      const int rc = b_rows - 16 * j0;
      if (rc <= 0) {  // nothing left of B: zero the remaining columns via a chunk with all-zero rows
        const int rs = launch_skinny(a + (a_koff > 0 ? (long)mi * a_koff : 0), lda, b, ldb, 1, M, M_out, K, 1, 0,
                                     0.f, o + 16 * j0, ldo, oc, part, stream);
        if (rs) return rs;
        break;
      }
      const int rs = launch_skinny(a + (a_koff > 0 ? (long)mi * a_koff : 0), lda, b + (long)16 * j0 * ldb, ldb, rc, M,
                                   M_out, K, nt, 0, scale, o + 16 * j0, ldo, oc, part, stream, dr);
      if (rs) return rs;
    }
  }
  return OSPO_OK;
}
