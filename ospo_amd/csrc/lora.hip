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
#include <cstdlib>

#include "common.h"
#include "skinny.h"

namespace {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));  // the buffer intrinsics' 16-B operand

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

// ---------------------------------------------------------------------------------------------
// v2: 64 activation rows per workgroup (wave w: rows 16w..16w+15) streamed with a whole chunk of
// loads in flight per wave, the small LoRA operand (Bt rows of this launch's tiles) staged once
// per chunk in LDS and shared by the four waves -- v1 re-read it from L2 for every 16 rows, which
// was (n_tiles x) the activation traffic.  Dense (u, forward, optional dropout on A) or
// block-diagonal (g, backward: grid z = module, its tiles reduce over its own K block of A).
// Split-K partials: fp32 [split][M_pad][16 * n_tiles] + skinny2_reduce_kernel.
template <int NT>
struct Sk2Cfg {
  static constexpr int KC = NT <= 2 ? 512 : (NT <= 4 ? 256 : 128);  // k per LDS chunk
  static constexpr int PITCH = 2 * KC + 16;                           // 16-row fragment reads hit distinct banks
  static constexpr int STEPS = KC / 32;
};

template <int NT, bool DROP>
__global__ __launch_bounds__(256) void skinny2_kernel(const bf16* __restrict__ A, int lda, const bf16* __restrict__ Bt,
                                                      int ldb, int b_rows, int M, int M_out, int K, int kper,
                                                      int a_koff, int tiles_total, float scale, bf16* __restrict__ out,
                                                      int ldo, int out_cols, float* __restrict__ ws, int M_pad,
                                                      uint32_t dseed, uint32_t dthresh, float dscale,
                                                      bf16* __restrict__ xd, int ldxd) {
  using C = Sk2Cfg<NT>;
  __shared__ __attribute__((aligned(16))) char bs[16 * NT * C::PITCH];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int m = blockIdx.x * 64 + wave * 16 + l16;
  const int mr = m < M ? m : M - 1;
  const int z = blockIdx.y, splits = gridDim.y, mod = blockIdx.z;
  const int tbase = mod * NT;                              // first output tile of this workgroup
  const bf16* arow = A + (long)mr * lda + (long)mod * a_koff;
  const int k_begin = z * kper, k_end = min(K, k_begin + kper);
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = k_begin; kc < k_end; kc += C::KC) {
    const int nsteps = min(C::KC, k_end - kc) >> 5;
    // stage Bt rows [16 tbase, 16 (tbase + NT)) x [kc, kc + KC): one LDS-DMA per (row, 1 KiB piece)
    constexpr int PIECES = C::KC / 512 > 0 ? C::KC / 512 : 1, LANES = C::KC >= 512 ? 64 : C::KC / 8;
    for (int t = wave; t < 16 * NT * PIECES; t += 4) {
      const int r = t / PIECES, pc = t % PIECES;
      const int br = min(16 * tbase + r, b_rows - 1);  // rows >= b_rows are masked at the fragment
      const int col = min(kc + pc * 512 + 8 * lane, K - 8);
      if (LANES == 64 || lane < LANES)  // a row image is 2 KC bytes: lanes past it must not write the next row's
        __builtin_amdgcn_global_load_lds(Bt + (long)br * ldb + col, (LDS_AS void*)(bs + r * C::PITCH + pc * 1024),
                                         16, 0, 0);
    }
    asm volatile("" ::: "memory");  // the Bt DMA is issued before the activation loads (counted below)
    bf16x8 av[C::STEPS];
#pragma unroll
    for (int s = 0; s < C::STEPS; ++s) {
      const int k = kc + 32 * min(s, nsteps - 1) + 8 * g;
      av[s] = *reinterpret_cast<const bf16x8*>(arow + k);
    }
    if constexpr (C::STEPS >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (C::STEPS >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int s = 0; s < C::STEPS; ++s) {
      if (s < nsteps) {
        bf16x8 a = av[s];
        if constexpr (DROP) {
          const int k0 = kc + 32 * s + 8 * g;
          bool keep[8];
          drop_keep_pairs<4>((uint32_t)mr * (uint32_t)K + (uint32_t)k0, dseed, dthresh, keep);
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = keep[e] ? f2bf(bf2f(a[e]) * dscale) : f2bf(0.f);
          if (xd && m < M) *reinterpret_cast<bf16x8*>(xd + (long)m * ldxd + k0) = a;
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 bfr = *reinterpret_cast<const bf16x8*>(bs + (16 * j + l16) * C::PITCH + (32 * s + 8 * g) * 2);
          if (16 * (tbase + j) + l16 >= b_rows) bfr = bf16x8{};
          acc[j] = MFMA(bfr, a, acc[j]);  // D[c = 16 j + 4 g + q][m = l16]
        }
      }
    }
    __syncthreads();
  }
  const int ctot = 16 * tiles_total;
  if (splits > 1) {
    if (m < M_pad) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
        *reinterpret_cast<f32x4*>(ws + ((long)z * M_pad + m) * ctot + 16 * (tbase + j) + 4 * g) = acc[j];
    }
    return;
  }
  if (m < M_out) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      uint2 pk;
      if (m < M) {
        pk.x = pack2(acc[j][0] * scale, acc[j][1] * scale);
        pk.y = pack2(acc[j][2] * scale, acc[j][3] * scale);
      } else {
        pk.x = pk.y = 0u;
      }
      *reinterpret_cast<uint2*>(out + (long)m * ldo + 16 * (tbase + j) + 4 * g) = pk;
    }
    if (mod == gridDim.z - 1 && g == 0) {  // zero the padding columns of this lane's row
      for (int c = ctot; c < out_cols; ++c) out[(long)m * ldo + c] = f2bf(0.f);
    }
  }
}

// out[m][c] = bf16(scale * sum_z ws[z][m][c]) for c < ctot, 0 for ctot <= c < out_cols; rows >= M zero
__global__ void skinny2_reduce_kernel(const float* __restrict__ ws, int splits, int M, int M_out, int M_pad, int ctot,
                                      float scale, bf16* __restrict__ out, int ldo, int out_cols) {
  const unsigned cq = (unsigned)out_cols / 4;  // 32-bit index math: M_out * cq < 2^31 (host check)
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (unsigned)M_out * cq) return;
  const int m = (int)(tid / cq), c = (int)(tid % cq) * 4;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  if (m < M && c < ctot) {
    // 8 splits' partials in flight at a time (a serial load chain was latency-bound), summed in
    // split order as before
    for (int z0 = 0; z0 < splits; z0 += 8) {
      f32x4 p[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (z0 + u < splits) p[u] = *reinterpret_cast<const f32x4*>(ws + ((long)(z0 + u) * M_pad + m) * ctot + c);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (z0 + u < splits) v += p[u];
    }
  }
  uint2 pk;
  pk.x = pack2(v[0] * scale, v[1] * scale);
  pk.y = pack2(v[2] * scale, v[3] * scale);
  *reinterpret_cast<uint2*>(out + (long)m * ldo + c) = pk;
}


// ---------------------------------------------------------------------------------------------
// v3: the activation streamed through LDS in whole 128-B lines.  v2 loaded each lane's 16 B straight
// into its MFMA fragment, so a wave instruction touched 16 rows x 64 B (half lines): the texture path,
// not HBM, set its rate.  Here a workgroup (4 waves, 64 rows) walks its K range in chunks of 64
// (one 128-B line per row): each chunk is 8 LDS-DMA pieces of 8 rows x 128 B (buffer_load ... lds from
// launch-constant per-lane offsets, the K advance in soffset), XOR-swizzled by row so the 16-row
// fragment reads are conflict-free, in an NS-stage ring with NS - 1 chunks in flight.  The Bt rows
// of the workgroup's tiles ride in the same stage (padded to 2 / 4 / 8 tiles so every wave issues the
// same number of pieces and the counted waits are uniform).  Split-K partials as v2.
template <int NT>
struct Sk3Cfg {
  static constexpr int NTP = NT <= 2 ? 2 : (NT <= 4 ? 4 : 8);  // staged Bt tiles
  static constexpr int BPW = NTP / 2;                           // Bt pieces per wave per chunk
  static constexpr int PW = 2 + BPW;                            // pieces per wave per chunk
  static constexpr int NS = 2;                                  // ring stages (the launchers' default)
  static constexpr int STAGE = 8192 + NTP * 2048;               // A 64 x 128 B + Bt 16 NTP x 128 B
};

// (a device function: hipcc's host pass drops the kernel's launch stub when this builtin sits in the
// kernel body itself inside a loop)
template <int AUX = 0>
__device__ __forceinline__ void sk3_lds16(__amdgpu_buffer_rsrc_t rs, char* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)dst, 16, voff, soff, 0, AUX);
}

__device__ __forceinline__ void sk3_wait(int n) {
  switch (n) {  // vmcnt holds 6 bits on gfx950
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    case 23: asm volatile("s_waitcnt vmcnt(23)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 25: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 26: asm volatile("s_waitcnt vmcnt(26)" ::: "memory"); break;
    case 27: asm volatile("s_waitcnt vmcnt(27)" ::: "memory"); break;
    case 28: asm volatile("s_waitcnt vmcnt(28)" ::: "memory"); break;
    case 29: asm volatile("s_waitcnt vmcnt(29)" ::: "memory"); break;
    case 30: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    case 31: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
    case 32: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
    case 33: asm volatile("s_waitcnt vmcnt(33)" ::: "memory"); break;
    case 34: asm volatile("s_waitcnt vmcnt(34)" ::: "memory"); break;
    case 35: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
    case 36: asm volatile("s_waitcnt vmcnt(36)" ::: "memory"); break;
    case 37: asm volatile("s_waitcnt vmcnt(37)" ::: "memory"); break;
    case 38: asm volatile("s_waitcnt vmcnt(38)" ::: "memory"); break;
    case 39: asm volatile("s_waitcnt vmcnt(39)" ::: "memory"); break;
    case 40: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
    case 41: asm volatile("s_waitcnt vmcnt(41)" ::: "memory"); break;
    case 42: asm volatile("s_waitcnt vmcnt(42)" ::: "memory"); break;
    case 43: asm volatile("s_waitcnt vmcnt(43)" ::: "memory"); break;
    case 44: asm volatile("s_waitcnt vmcnt(44)" ::: "memory"); break;
    case 45: asm volatile("s_waitcnt vmcnt(45)" ::: "memory"); break;
    case 46: asm volatile("s_waitcnt vmcnt(46)" ::: "memory"); break;
    case 47: asm volatile("s_waitcnt vmcnt(47)" ::: "memory"); break;
    case 48: asm volatile("s_waitcnt vmcnt(48)" ::: "memory"); break;
    case 49: asm volatile("s_waitcnt vmcnt(49)" ::: "memory"); break;
    case 50: asm volatile("s_waitcnt vmcnt(50)" ::: "memory"); break;
    case 51: asm volatile("s_waitcnt vmcnt(51)" ::: "memory"); break;
    case 52: asm volatile("s_waitcnt vmcnt(52)" ::: "memory"); break;
    case 53: asm volatile("s_waitcnt vmcnt(53)" ::: "memory"); break;
    case 54: asm volatile("s_waitcnt vmcnt(54)" ::: "memory"); break;
    case 55: asm volatile("s_waitcnt vmcnt(55)" ::: "memory"); break;
    case 56: asm volatile("s_waitcnt vmcnt(56)" ::: "memory"); break;
    case 57: asm volatile("s_waitcnt vmcnt(57)" ::: "memory"); break;
    case 58: asm volatile("s_waitcnt vmcnt(58)" ::: "memory"); break;
    case 59: asm volatile("s_waitcnt vmcnt(59)" ::: "memory"); break;
    case 60: asm volatile("s_waitcnt vmcnt(60)" ::: "memory"); break;
    case 61: asm volatile("s_waitcnt vmcnt(61)" ::: "memory"); break;
    case 62: asm volatile("s_waitcnt vmcnt(62)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;  // (more in flight: waiting longer is safe)
  }
}

// one 16-B Bt fragment into registers (a device function for the same reason as sk3_lds16)
__device__ __forceinline__ bf16x8 sk3_ldb(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

// SWG (round 3): the down-projection's u product fused with the SwiGLU forward that makes its input: A is gu
// [M][>= 2F] (gate | up); each chunk stages the gate and the up tile, the fragment's h = bf16(silu(g)) * u is
// formed in registers (swiglu_fwd_kernel's rounding), stored to hout [M][F] (the down GEMM's operand) and
// fed to the MFMAs -- h is never re-read.  K = F, up_off = F * 2 bytes.
// BTR (ablation build, OSPO_SK3_BTREG; 2-stage ring only): the adapter rows' fragments come straight from L2 into
// registers (one chunk ahead, issued before the chunk's LDS-DMA pieces so the counted wait is unchanged) instead
// of being staged with every 64-k chunk: 2 DMA pieces + 2 NT LDS reads fewer per chunk and wave.
template <int NT, bool DROP, bool SWG = false, int NSREQ = 4, bool BTR = false, int AA = 0>  // AA: A-load policy bits
__global__ __launch_bounds__(256) void skinny3_kernel(const bf16* __restrict__ A, int lda, int a_bytes,
                                                      const bf16* __restrict__ Bt, int ldb, int b_rows, int b_bytes,
                                                      int M, int M_out, int K, int kper, int a_koff, int tiles_total,
                                                      float scale, bf16* __restrict__ out, int ldo, int out_cols,
                                                      float* __restrict__ ws, int M_pad, uint32_t dseed,
                                                      uint32_t dthresh, float dscale, uint8_t* __restrict__ kbits,
                                                      bf16* __restrict__ hout = nullptr, int ldh = 0, int up_off = 0,
                                                      unsigned* __restrict__ cnt = nullptr) {
  using C = Sk3Cfg<NT>;
  constexpr int ABYTES = SWG ? 16384 : 8192;        // A image(s): gate and up under SWG
  constexpr int STAGE = BTR ? ABYTES : C::STAGE + ABYTES - 8192;
  constexpr int PW = (BTR ? 2 : C::PW) + (SWG ? 2 : 0);
  constexpr int NS = NSREQ * STAGE <= 163840 ? NSREQ : 163840 / STAGE;  // ring stages (the LDS caps deep rings)
  static_assert(!BTR || NS == 2, "register Bt fragments: the 2-stage ring's counted waits only");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4, r8 = lane >> 3, c8 = lane & 7;
  const int m0 = blockIdx.x * 64;
  const int z = blockIdx.y, splits = gridDim.y, mod = blockIdx.z;
  const int tbase = mod * NT;
  const int k_begin = z * kper, k_end = min(K, k_begin + kper);
  const int nch = (k_end - k_begin + 63) >> 6;  // K % 64 == 0 (host check)

  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bt, 0, b_bytes, 0x00020000);
  // per-lane byte offsets of this wave's pieces (rows clamped; the swizzled 16-B chunk of the row)
  uint32_t va[2], vb[C::BPW];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + r8;
    const int gr = min(m0 + row, M - 1);
    va[i] = ((uint32_t)gr * (uint32_t)lda + (uint32_t)(mod * a_koff) + (uint32_t)k_begin) * 2u + ((c8 ^ r8) << 4);
  }
#pragma unroll
  for (int i = 0; i < C::BPW; ++i) {
    const int row = (wave * C::BPW + i) * 8 + r8;
    const int br = min(16 * tbase + row, b_rows - 1);
    vb[i] = ((uint32_t)br * (uint32_t)ldb + (uint32_t)k_begin) * 2u + ((c8 ^ r8) << 4);
  }
#define SK3_STAGE(cc)                                                                                            \
  {                                                                                                              \
    char* st_ = smem + ((cc) % NS) * STAGE;                                                                  \
    const int kb_ = (cc) * 128;                                                                                  \
    _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                                \
        sk3_lds16<AA>(rsA, st_ + (wave * 2 + i) * 1024, va[i], kb_);                                             \
    if constexpr (SWG) {                                                                                         \
      _Pragma("unroll") for (int i = 0; i < 2; ++i)                                                              \
          sk3_lds16<AA>(rsA, st_ + 8192 + (wave * 2 + i) * 1024, va[i], kb_ + up_off);                           \
    }                                                                                                            \
    if constexpr (!BTR) {                                                                                        \
      _Pragma("unroll") for (int i = 0; i < C::BPW; ++i)                                                         \
          sk3_lds16(rsB, st_ + ABYTES + (wave * C::BPW + i) * 1024, vb[i], kb_);                                 \
    }                                                                                                            \
  }

  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int spi = (SWG ? 2 : 0) + (DROP && kbits ? 2 : 0);  // global stores per chunk per lane
  const int arow_l = wave * 16 + l16;  // this lane's fragment row in the 64-row block
  const uint32_t drow = (uint32_t)min(m0 + arow_l, M - 1) * (uint32_t)K;
  bool bok[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) bok[j] = 16 * (tbase + j) + l16 < b_rows;

  // BTR: this lane's Bt fragment offsets (row 16 (tbase + j) + l16 clamped, k group g), + 64 B per k step s
  uint32_t vbr[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int br = min(16 * (tbase + j) + l16, b_rows - 1);
    vbr[j] = ((uint32_t)br * (uint32_t)ldb + (uint32_t)k_begin + 8u * (uint32_t)g) * 2u;
  }
  bf16x8 bcur[2][NT], bnxt[2][NT];
  if constexpr (BTR) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int j = 0; j < NT; ++j) bcur[s2][j] = sk3_ldb(rsB, vbr[j] + 64u * s2, 0);
  }
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (j < nch) SK3_STAGE(j);
  for (int c = 0; c < nch; ++c) {
    // this wave's pieces of chunk c landed: newer are the pieces of up to NS - 2 later chunks and the stores
    // (h, keep bits; unconditional, so the count is exact) of the up to NS - 1 chunks computed since
    sk3_wait(PW * min(NS - 2, nch - 1 - c) + spi * min(c, NS - 1));
    if constexpr (BTR) {  // chunk c's Bt fragments were issued before its pieces: landed too
      if (c > 0) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < NT; ++j) bcur[s2][j] = bnxt[s2][j];
      }
    }
    __builtin_amdgcn_s_barrier();                    // everyone's; and chunk c-1's slot is free
    asm volatile("" ::: "memory");
    if constexpr (BTR) {
      if (c + 1 < nch) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < NT; ++j) bnxt[s2][j] = sk3_ldb(rsB, vbr[j] + 64u * s2, (c + 1) * 128);
      }
    }
    if (c + NS - 1 < nch) SK3_STAGE(c + NS - 1);
    const char* st = smem + (c % NS) * STAGE;
    bf16x8 a[2], b[2][NT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = 4 * s + g;  // 16-B chunk of the 128-B line
      a[s] = *reinterpret_cast<const bf16x8*>(st + arow_l * 128 + ((q ^ (arow_l & 7)) << 4));
      if constexpr (SWG) {  // h = bf16(silu(gate)) * up of the fragment's 8 elements, rounded; stored once
        const bf16x8 up = *reinterpret_cast<const bf16x8*>(st + 8192 + arow_l * 128 + ((q ^ (arow_l & 7)) << 4));
        float hv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) hv[e] = round_bf(silu(bf2f(a[s][e]))) * bf2f(up[e]);
        const u32x4 pk = pack8(hv);
        a[s] = __builtin_bit_cast(bf16x8, pk);
        // rows >= M hold row M - 1 (clamped staging) and rewrite its h: the store is unconditional
        *reinterpret_cast<u32x4*>(hout + (long)min(m0 + arow_l, M - 1) * ldh + k_begin + 64 * c + 32 * s + 8 * g) = pk;
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (BTR) {
          b[s][j] = bcur[s][j];
        } else {
          const int br = 16 * j + l16;
          b[s][j] = *reinterpret_cast<const bf16x8*>(st + ABYTES + br * 128 + ((q ^ (br & 7)) << 4));
        }
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 av = a[s];
      if constexpr (DROP) {
        const uint32_t k0 = (uint32_t)(k_begin + 64 * c + 32 * s + 8 * g);
        bool keep[8];
        drop_keep_pairs<4>(drow + k0, dseed, dthresh, keep);
#pragma unroll
        for (int e = 0; e < 8; ++e) av[e] = keep[e] ? f2bf(bf2f(av[e]) * dscale) : f2bf(0.f);
        if (kbits) {  // the keep bits, one byte per 8 columns (bit e = column k0 + e); rows >= M rewrite row M - 1's
          uint32_t byte = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) byte |= (keep[e] ? 1u : 0u) << e;
          kbits[(drow + k0) >> 3] = (uint8_t)byte;
        }
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = MFMA(bok[j] ? b[s][j] : bf16x8{}, av, acc[j]);  // D[16j+4g+q][m]
    }
  }
  const int m = m0 + arow_l;
  const int ctot = 16 * tiles_total;
  if (splits > 1 && !cnt) {  // fp32 partials; skinny2_reduce_kernel sums them
    if (m < M_pad) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
        *reinterpret_cast<f32x4*>(ws + ((long)z * M_pad + m) * ctot + 16 * (tbase + j) + 4 * g) = acc[j];
    }
    return;
  }
  if (splits > 1) {
    // The split sum in this launch (round 3; it was a separate reduce launch, ~5.7 us each): every workgroup
    // stores its fp32 partial write-through (sc1) and takes a ticket on its row block's counter; the last of
    // the row block's splits x modules workgroups reads all partials back (sc1 loads), sums them in split order
    // (as skinny2_reduce_kernel, bit-identical), writes the bf16 rows and zeroes the counter for the next call.
    // No release / acquire fence: sc1 stores are visible device-wide once acknowledged (vmcnt(0)), and sc1
    // loads do not hit a stale line (cdna_hip_programming.md, the in-launch split-K hand-off).
    const __amdgpu_buffer_rsrc_t rsW =
        __builtin_amdgcn_make_buffer_rsrc((void*)ws, 0, (int)((long)splits * M_pad * ctot * 4), 0x00020000);
    if (m < M_pad) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[j]), rsW,
                                               (uint32_t)((((long)z * M_pad + m) * ctot + 16 * (tbase + j) + 4 * g) * 4),
                                               0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's partial acknowledged; every wave done with the ring (the flag reuses it)
    unsigned* flag = reinterpret_cast<unsigned*>(smem);
    if (threadIdx.x == 0) {
      const unsigned total = gridDim.y * gridDim.z;
      const unsigned t = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (t == total - 1) ? 1u : 0u;
    }
    __syncthreads();
    if (*flag == 0u) return;
    // no instruction: keeps the sc1 partial loads below the ticket (sc1 stores drained before it, sc1 loads
    // after it: the hand-off Valid form of cdna_hip_programming.md, where this replaces the agent-scope acquire)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int cq = out_cols / 4;
    for (int it = threadIdx.x; it < 64 * cq; it += blockDim.x) {
      const int r = it / cq, c = (it % cq) * 4;
      const int mm = m0 + r;
      if (mm >= M_out) continue;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (mm < M && c < ctot) {
        for (int z0 = 0; z0 < splits; z0 += 8) {  // 8 partials in flight, summed in split order
          u32x4v pv[8];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (z0 + u < splits)
              pv[u] = __builtin_amdgcn_raw_buffer_load_b128(
                  rsW, (uint32_t)((((long)(z0 + u) * M_pad + mm) * ctot + c) * 4), 0, 16);
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (z0 + u < splits) v += __builtin_bit_cast(f32x4, pv[u]);
        }
      }
      uint2 pk;
      pk.x = pack2(v[0] * scale, v[1] * scale);
      pk.y = pack2(v[2] * scale, v[3] * scale);
      *reinterpret_cast<uint2*>(out + (long)mm * ldo + c) = pk;
    }
    if (threadIdx.x == 0) __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (m < M_out) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      uint2 pk;
      if (m < M) {
        pk.x = pack2(acc[j][0] * scale, acc[j][1] * scale);
        pk.y = pack2(acc[j][2] * scale, acc[j][3] * scale);
      } else {
        pk.x = pk.y = 0u;
      }
      *reinterpret_cast<uint2*>(out + (long)m * ldo + 16 * (tbase + j) + 4 * g) = pk;
    }
    if (mod == gridDim.z - 1 && g == 0) {
      for (int cc = ctot; cc < out_cols; ++cc) out[(long)m * ldo + cc] = f2bf(0.f);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused backward over one stream of dy (LoRA r = 16): g = s dy.B (the dX GEMM's K-extension operand)
// and dB += dy^T.u (the adapter B gradient), which before read dy twice (the g product on the main
// stream, dB as a separate f32-atomic GEMM on the side stream).  Workgroup = 4 waves over 64*RSB rows x
// 64*nch columns of one module.  dy sub-tiles of 64 rows x 64 columns stream through a 4-stage LDS ring
// (128-B lines, XOR-swizzled); the module's Bt columns and u rows of the workgroup are staged once.
//   g : row sub-block rb belongs to wave rb & 3 (2 per wave at RSB 8); MFMA D[j][m] (as the skinny kernels),
//       fp32 partials per column block -> gdb_reduce_kernel.
//   dB: wave w owns columns 16w..16w+15 of each 64-column chunk, D[n][j] over the workgroup's rows from
//       transposed reads of the dy image (ds_read_b64_tr_b16) and of u; one f32 atomic add per element
//       and chunk.  u rows >= M are zeroed in the fragment (dy rows are clamped, so finite).
// Transposed LDS reads as inline asm: the builtin makes hipcc drain vmcnt(0) -- every LDS-DMA of the
// prefetched sub-tiles -- before it (it cannot tell them apart); the caller waits lgkmcnt with the
// destinations tied (tr4_wait) and fences the schedule.
__device__ __forceinline__ void tr4_issue(const char* p, i16x4& v) {
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"((uint32_t)(uintptr_t)((LDS_AS const char*)p)));
}
__device__ __forceinline__ void tr4_wait(i16x4& a, i16x4& b, i16x4& c, i16x4& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void tr6_wait(i16x4& a, i16x4& b, i16x4& c, i16x4& d, i16x4& e, i16x4& f) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f)::"memory");
  __builtin_amdgcn_sched_barrier(0);
}

// In-launch sum of the g partials (INL, round 5, ablation A/B: bit-identical, no faster in the step than
// gdb_reduce_kernel's launch, ~7.7 us each, 90 per step):
// every workgroup stores its partials write-through (sc1) and takes a ticket on its row block's counter; once
// all gridDim.y workgroups of the row block have (a bounded wait; the host launches this form only when the whole
// grid fits on the device at once), each sums its share of the row block's output quads in gdb_reduce_kernel's
// order (bit-identical), then takes a second ticket, and the row block's last one zeroes both counters.
struct GdbInl {
  unsigned* cnt;  // [2][1024] row-block counters (zero at allocation, left zero), then a give-up word
  int M_out;
  float scale;
  bf16* out;
  int ldo, out_cols;
};
constexpr int GDB_CNT_BYTES = OSPO_WS_LORA_GDB_CNT_BYTES;
constexpr unsigned GDB_SPIN_LIMIT = 1u << 24;

// HPM (round 6): 16-column halves per module (LoRA r = 16 HPM): one workgroup reads its dy tile once for all
// of them -- HPM Bt / u images and accumulator sets; the partials of half h of module mod are those of the
// "module" mod HPM + h (gdb_reduce_kernel sums nmods HPM of them), the dB block of a module is [Nmod][16 HPM]
template <int RSB, int NS = 4, int YA = 0, bool INL = false, int HPM = 1>  // YA: cache-policy bits of the dy loads
__global__ __launch_bounds__(256) void lora_gdb_kernel(const bf16* __restrict__ dy, int ldy, const bf16* __restrict__ Bt,
                                                       int ldb, const bf16* __restrict__ u, int ldu, int M, int Nmod,
                                                       int nch, float* __restrict__ ws, int Mw,
                                                       float* __restrict__ dB, const GdbInl inl = GdbInl{}) {
  static_assert(!(INL && HPM != 1), "the in-launch sum is r = 16 only");
  // NS-stage ring of 8-KiB dy sub-tiles, NS - 1 in flight (a 6-stage ring measured 10-30 % slower)
  constexpr int STAGE = 8192;
  constexpr int BT_OFF = NS * STAGE, BT_BYTES = 16 * 4 * 128;  // up to nch = 4, per half
  constexpr int ROWS = 64 * RSB;
  constexpr int U_OFF = BT_OFF + HPM * BT_BYTES, U_BYTES = ROWS * 32;  // per half
  __shared__ __attribute__((aligned(16))) char smem[U_OFF + HPM * U_BYTES];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4, r8 = lane >> 3, c8 = lane & 7;
  const int rb0 = blockIdx.x * ROWS;
  const int nsplit = Nmod / (64 * nch);
  // mod: the module (dy columns mod Nmod ..); half h of it: rows 16 (mod HPM + h) of Bt, columns 16 (mod HPM + h)
  // of u and g, columns 16 h of the module's [Nmod][16 HPM] dB block
  const int mod = blockIdx.y / nsplit, sp = blockIdx.y % nsplit;
  const int kc0 = sp * 64 * nch;              // first column of the workgroup within its module
  const long col0 = (long)mod * Nmod + kc0;   // ... within dy
  const int btrow = nch * 128;               // bytes per Bt image row

  // Bt images [16 j][nch*64 k]: 16-B chunk q of row j at physical chunk q ^ j (source-side swizzle)
  {
    const int rpp = 1024 / btrow;  // rows per 1-KiB piece (2 or 4)
#pragma unroll
    for (int h = 0; h < HPM; ++h)
      for (int p = wave; p < 2 * nch; p += 4) {
        const int off = lane * 16;
        const int j = p * rpp + off / btrow, pc = (off % btrow) >> 4;
        const int q = pc ^ j;
        __builtin_amdgcn_global_load_lds(Bt + (long)((mod * HPM + h) * 16 + j) * ldb + kc0 + q * 8,
                                         (LDS_AS void*)(smem + BT_OFF + h * BT_BYTES + p * 1024), 16, 0, 0);
      }
  }
  // u images [ROWS][16] (32 B per row), rows clamped (masked at the fragment)
#pragma unroll
  for (int h = 0; h < HPM; ++h)
#pragma unroll
    for (int p = wave; p < ROWS / 32; p += 4) {
      const int row = min(rb0 + p * 32 + (lane >> 1), M - 1);
      __builtin_amdgcn_global_load_lds(u + (long)row * ldu + (mod * HPM + h) * 16 + (lane & 1) * 8,
                                       (LDS_AS void*)(smem + U_OFF + h * U_BYTES + p * 1024), 16, 0, 0);
    }
  auto stage = [&](int t) {  // sub-tile t = (chunk t / RSB, row sub-block t % RSB): 2 pieces per wave
    char* st = smem + (t % NS) * STAGE;
    const int cc = t / RSB, rb = t % RSB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int p = wave * 2 + i;
      const int row = min(rb0 + rb * 64 + p * 8 + r8, M - 1);
      __builtin_amdgcn_global_load_lds(dy + (long)row * ldy + col0 + cc * 64 + ((c8 ^ r8) << 3),
                                       (LDS_AS void*)(st + p * 1024), 16, 0, YA);
    }
  };
  const int T = nch * RSB;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) stage(t);

  // g: every wave computes its 16-row group (rows 16 wave .. +15) of every 64-row sub-block, 2 MFMAs per
  // sub-tile (the sub-block's 64 rows used to go to one wave, 8 MFMAs while the other three waited at
  // the next barrier); same per-row accumulation order (chunks, then k steps), bit-identical partials
  f32x4 accg[HPM][RSB];
  f32x4 accb[HPM];
#pragma unroll
  for (int h = 0; h < HPM; ++h) {
#pragma unroll
    for (int a = 0; a < RSB; ++a) accg[h][a] = f32x4{0.f, 0.f, 0.f, 0.f};
    accb[h] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int li = l16, q4 = li >> 2, p4 = li & 3;
  const int grow = 16 * wave + l16;  // this lane's row of the g product inside a sub-tile
  for (int cc = 0; cc < nch; ++cc) {
#pragma unroll
    for (int rb = 0; rb < RSB; ++rb) {
      const int t = cc * RSB + rb;
      const int newer = min(NS - 2, T - 1 - t);  // stages issued after t that may stay in flight (2 pieces each)
      switch (newer) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (t + NS - 1 < T) stage(t + NS - 1);
      const char* st = smem + (t % NS) * STAGE;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int qk = cc * 8 + 4 * s2 + g;  // Bt chunk (8 bf16) of this lane's k group
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(st + grow * 128 + (((4 * s2 + g) ^ (grow & 7)) << 4));
#pragma unroll
        for (int h = 0; h < HPM; ++h) {
          const bf16x8 bt =
              *reinterpret_cast<const bf16x8*>(smem + BT_OFF + h * BT_BYTES + l16 * btrow + ((qk ^ l16) << 4));
          accg[h][rb] = MFMA(bt, a, accg[h][rb]);  // D[j = 4g..][m = l16]
        }
      }
      // dB: columns 16 wave .. +15 of the chunk, the sub-block's 64 rows as K
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r1 = 32 * s + 8 * g + q4, r2 = r1 + 4;
        const int x = 2 * wave + (p4 >> 1), h = (p4 & 1) << 3;
        const int ur = rb * 64 + 32 * s + 8 * g;  // u image row of element 0
        i16x4 lo, hi, ulo[HPM], uhi[HPM];
        tr4_issue(st + r1 * 128 + ((x ^ (r1 & 7)) << 4) + h, lo);
        tr4_issue(st + r2 * 128 + ((x ^ (r2 & 7)) << 4) + h, hi);
#pragma unroll
        for (int hh = 0; hh < HPM; ++hh) {
          tr4_issue(smem + U_OFF + hh * U_BYTES + (ur + q4) * 32 + p4 * 8, ulo[hh]);
          tr4_issue(smem + U_OFF + hh * U_BYTES + (ur + 4 + q4) * 32 + p4 * 8, uhi[hh]);
        }
        if constexpr (HPM == 1)
          tr4_wait(lo, hi, ulo[0], uhi[0]);
        else
          tr6_wait(lo, hi, ulo[0], uhi[0], ulo[1], uhi[1]);
        const int mrow = rb0 + ur;  // global row of element 0
        const i16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int hh = 0; hh < HPM; ++hh) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ulo[hh][e] = (mrow + e < M) ? ulo[hh][e] : (short)0;
            uhi[hh][e] = (mrow + 4 + e < M) ? uhi[hh][e] : (short)0;
          }
          const i16x8 bv = {ulo[hh][0], ulo[hh][1], ulo[hh][2], ulo[hh][3],
                            uhi[hh][0], uhi[hh][1], uhi[hh][2], uhi[hh][3]};
          accb[hh] = MFMA(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv), accb[hh]);  // D[n][j]
        }
      }
      if (rb == RSB - 1 && !(INL && cc == nch - 1)) {  // the chunk's dB over the workgroup's rows
        const long n0 = col0 + cc * 64 + 16 * wave + 4 * g;
#pragma unroll
        for (int hh = 0; hh < HPM; ++hh) {
#pragma unroll
          for (int i = 0; i < 4; ++i) atomicAdd(dB + (n0 + i) * (16 * HPM) + 16 * hh + l16, accb[hh][i]);
          accb[hh] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  }
  if constexpr (!INL) {
    // g partials of this column block: ws [mod HPM + h][sp][Mw][16]
#pragma unroll
    for (int hh = 0; hh < HPM; ++hh)
#pragma unroll
      for (int rb = 0; rb < RSB; ++rb) {
        const int m = rb0 + rb * 64 + grow;
        if (m < Mw)
          *reinterpret_cast<f32x4*>(ws + ((((long)mod * HPM + hh) * nsplit + sp) * Mw + m) * 16 + 4 * g) = accg[hh][rb];
      }
  } else {
    const int nmods = gridDim.y / nsplit;
    const __amdgpu_buffer_rsrc_t rsW =
        __builtin_amdgcn_make_buffer_rsrc((void*)ws, 0, (int)((long)nmods * nsplit * Mw * 64), 0x00020000);
#pragma unroll
    for (int rb = 0; rb < RSB; ++rb) {
      const int m = rb0 + rb * 64 + grow;
      if (m < Mw)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, accg[0][rb]), rsW,
                                               (uint32_t)(((((long)mod * nsplit + sp) * Mw + m) * 16 + 4 * g) * 4), 0, 16);
    }
    {  // the last chunk's dB atomics after the partial stores: the wait below leaves them in flight
      const long n0 = col0 + (nch - 1) * 64 + 16 * wave + 4 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(dB + (n0 + i) * 16 + l16, accb[0][i]);
    }
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // this lane's partial stores acknowledged
    __syncthreads();
    const unsigned W = gridDim.y;  // the row block's workgroups
    unsigned* c1 = inl.cnt + blockIdx.x;
    unsigned* c2 = inl.cnt + 1024 + blockIdx.x;
    if (threadIdx.x < 64) {
      if (threadIdx.x == 0) __hip_atomic_fetch_add(c1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      unsigned spins = 0;
      while (__hip_atomic_load(c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < W) {
        if (++spins > GDB_SPIN_LIMIT) {
          if (threadIdx.x == 0) __hip_atomic_store(inl.cnt + 2048, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // this workgroup's share of the row block's output quads (rows up to M_out in the last row block)
    const int rows = (blockIdx.x == gridDim.x - 1) ? inl.M_out - rb0 : min(ROWS, inl.M_out - rb0);
    const int cq = inl.out_cols / 4;
    const int total = rows > 0 ? rows * cq : 0;
    const int per = (total + (int)W - 1) / (int)W;
    const int q0 = (int)blockIdx.y * per, q1 = min(total, q0 + per);
    for (int qq = q0 + (int)threadIdx.x; qq < q1; qq += 256) {
      const int m = rb0 + qq / cq, c = (qq % cq) * 4, md = c / 16;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < M && md < nmods) {
        for (int s0 = 0; s0 < nsplit; s0 += 8) {  // gdb_reduce_kernel's order: ((0 + p_0) + p_1) + ...
          f32x4 pv[8];
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (s0 + k < nsplit) pv[k] = *reinterpret_cast<const f32x4*>(ws + (((long)md * nsplit + s0 + k) * Mw + m) * 16 + (c & 15));
#pragma unroll
          for (int k = 0; k < 8; ++k)
            if (s0 + k < nsplit) v += pv[k];
        }
      }
      uint2 pk;
      pk.x = pack2(v[0] * inl.scale, v[1] * inl.scale);
      pk.y = pack2(v[2] * inl.scale, v[3] * inl.scale);
      *reinterpret_cast<uint2*>(inl.out + (long)m * inl.ldo + c) = pk;
    }
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(c2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == W - 1u) {
      __hip_atomic_store(c1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// SwiGLU backward fused with the gate|up group's g / dB stream (round 4): a workgroup computes
// dgate | dup = swiglu_bwd(dh, gate, up) (swiglu_bwd8, as swiglu_bwd_kernel) over 64*RSB rows x 64*nch
// columns of BOTH modules -- the two share their inputs -- stores them (the A operand of the gate|up dX
// GEMM) and feeds the same tiles to lora_gdb_kernel's g / dB MFMAs, so dgu is written once and never read
// back.  Inputs come to registers by 16-B buffer loads PF sub-tiles ahead (no input ring in LDS); the two
// output tiles of a sub-tile go through one LDS image each, in lora_gdb_kernel's swizzled dy layout, between
// two barriers.  Row sub-blocks outer (runtime loop), the NCH column chunks inner (unrolled): g of a row
// sub-block is complete after its chunks (2 accumulators, stored at once), dB keeps one accumulator per
// chunk -- the fully unrolled chunk-outer order of lora_gdb_kernel held 8x the live registers here.  Same
// nch, per-element MFMA order and partials layout as lora_gdb_kernel over dgu: bit-identical g (and dB up
// to the f32 atomics' order) to ospo_swiglu_bwd + ospo_lora_gdb.
// LAUX / SAUX: cache-policy bits of the input loads / dgu stores.  DBG (measurement only): 1 no MFMA phase,
// 2 no dgu stores.
// HPM (round 6): 16-column halves per module (LoRA r = 16 HPM): 2 HPM Bt / u images and accumulator sets, the
// dB block of a module [F][16 HPM]
template <int RSB, int PF, int NCH, int DBG = 0, int LAUX = 2, int SAUX = 16, int HPM = 1>
__global__ __launch_bounds__(256) void swiglu_gdb_kernel(const bf16* __restrict__ dh, int lddh,
                                                         const bf16* __restrict__ gu, int ldg, bf16* __restrict__ dgu,
                                                         int lddg, const bf16* __restrict__ Bt, int ldb,
                                                         const bf16* __restrict__ u, int ldu, int M, int F,
                                                         float* __restrict__ ws, int Mw, float* __restrict__ dB) {
  static_assert(NCH % PF == 0, "the prefetch slot must be a compile-time index");
  constexpr int nch = NCH;
  constexpr int TILE = 8192;  // a 64 x 64 bf16 image; [dgate | dup] at 0 and TILE
  constexpr int NV = 2 * HPM;  // 16-column halves of the two modules
  constexpr int BT_OFF = 2 * TILE, BT_BYTES = 16 * 4 * 128;  // per half, up to nch = 4
  constexpr int ROWS = 64 * RSB;
  constexpr int U_OFF = BT_OFF + NV * BT_BYTES;  // per half ROWS * 32 B
  __shared__ __attribute__((aligned(16))) char smem[U_OFF + NV * ROWS * 32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int rb0 = blockIdx.x * ROWS;
  const int nsplit = F / (64 * nch);
  const int sp = blockIdx.y;
  const int kc0 = sp * 64 * nch;
  const int btrow = nch * 128;

  // Bt and u images as lora_gdb_kernel's (same swizzle), through registers: no LDS-DMA in this kernel, so
  // the compiler's vmcnt tracking of the register prefetch below stays exact.  All loads first, then the writes.
  {
    const int off = lane * 16, rpp = 1024 / btrow;
    u32x4 bv[NV][2], uv[NV * ROWS / 32 / 4];
#pragma unroll
    for (int mod = 0; mod < NV; ++mod)
#pragma unroll
      for (int k = 0; k < 2; ++k) {  // pieces p = wave + 4k < 2 nch (nch = 2: k = 0 only)
        const int p = min(wave + 4 * k, 2 * nch - 1);
        const int j = p * rpp + off / btrow, pc = (off % btrow) >> 4;
        bv[mod][k] = *reinterpret_cast<const u32x4*>(Bt + (long)(mod * 16 + j) * ldb + kc0 + (pc ^ j) * 8);
      }
#pragma unroll
    for (int k = 0; k < NV * ROWS / 32 / 4; ++k) {  // pieces p = wave + 4k of the halves' u images
      const int p = wave + 4 * k, mod = p / (ROWS / 32), pp = p % (ROWS / 32);
      const int row = min(rb0 + pp * 32 + (lane >> 1), M - 1);
      uv[k] = *reinterpret_cast<const u32x4*>(u + (long)row * ldu + mod * 16 + (lane & 1) * 8);
    }
#pragma unroll
    for (int mod = 0; mod < NV; ++mod)
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (wave + 4 * k < 2 * nch)
          *reinterpret_cast<u32x4*>(smem + BT_OFF + mod * BT_BYTES + (wave + 4 * k) * 1024 + off) = bv[mod][k];
#pragma unroll
    for (int k = 0; k < NV * ROWS / 32 / 4; ++k) {
      const int p = wave + 4 * k, mod = p / (ROWS / 32), pp = p % (ROWS / 32);
      *reinterpret_cast<u32x4*>(smem + U_OFF + mod * ROWS * 32 + pp * 1024 + off) = uv[k];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the images are read after the first barrier

  // this thread's two 16-B chunks of a sub-tile: rows r0, r0 + 32, logical chunk c.  Buffer loads / stores:
  // rows >= M fall outside the ranges, so their loads return 0 (finite dgate / dup: g partials of rows >= M
  // are never read) and their stores drop.
  const int r0 = tid >> 3, c = tid & 7;
  const __amdgpu_buffer_rsrc_t rsG = __builtin_amdgcn_make_buffer_rsrc((void*)gu, 0, (int)((long)M * ldg * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsH = __builtin_amdgcn_make_buffer_rsrc((void*)dh, 0, (int)((long)M * lddh * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsD = __builtin_amdgcn_make_buffer_rsrc((void*)dgu, 0, (int)((long)M * lddg * 2), 0x00020000);
  const uint32_t vg = (uint32_t)((r0 * ldg + c * 8) * 2), vh = (uint32_t)((r0 * lddh + c * 8) * 2);
  const uint32_t vd = (uint32_t)((r0 * lddg + c * 8) * 2);
  u32x4 in[PF][6];  // [slot][gate0, gate1, up0, up1, dh0, dh1]
  auto load = [&](int t, u32x4* v) {  // sub-tile t = (row sub-block t / NCH, chunk t % NCH)
    const int rb = t / NCH, cc = t % NCH;
    const int row = rb0 + rb * 64, col = kc0 + cc * 64;
    // the whole offset in voffset: the range check does not cover soffset
    const uint32_t og = vg + (uint32_t)((row * ldg + col) * 2), oh = vh + (uint32_t)((row * lddh + col) * 2);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      v[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsG, og + i * 64 * ldg, 0, LAUX));
      v[2 + i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsG, og + i * 64 * ldg + 2 * F, 0, LAUX));
      v[4 + i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsH, oh + i * 64 * lddh, 0, LAUX));
    }
  };
  constexpr int T = NCH * RSB;
#pragma unroll
  for (int s = 0; s < PF - 1; ++s) load(s, in[s]);

  f32x4 accb[NV][NCH];
#pragma unroll
  for (int mod = 0; mod < NV; ++mod)
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) accb[mod][cc] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int li = l16, q4 = li >> 2, p4 = li & 3;
  const int grow = 16 * wave + l16;
  for (int rb = 0; rb < RSB; ++rb) {
    f32x4 accg[NV];
#pragma unroll
    for (int mod = 0; mod < NV; ++mod) accg[mod] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
      const int t = rb * NCH + cc;
      load(min(t + PF - 1, T - 1), in[(cc + PF - 1) % PF]);  // unconditional: exact vmcnt, no join
      __builtin_amdgcn_s_barrier();  // every wave is done with the previous sub-tile's images
      asm volatile("" ::: "memory");
      {
        const u32x4* v = in[cc % PF];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = r0 + 32 * i;
          float d[8], gg[8], uu[8], dg[8], du[8];
          unpack8(v[4 + i], d);
          unpack8(v[i], gg);
          unpack8(v[2 + i], uu);
          swiglu_bwd8(d, gg, uu, dg, du);
          const u32x4 pg = pack8(dg), pu = pack8(du);
          const int so = r * 128 + ((c ^ (r & 7)) << 4);
          *reinterpret_cast<u32x4*>(smem + so) = pg;
          *reinterpret_cast<u32x4*>(smem + TILE + so) = pu;
          const uint32_t od = vd + (uint32_t)(((rb0 + rb * 64 + 32 * i) * lddg + kc0 + cc * 64) * 2);
          if (DBG != 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, pg), rsD, od, 0, SAUX);
          if (DBG != 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, pu), rsD, od + 2 * F, 0, SAUX);
        }
      }
      if (DBG == 1) continue;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // both images complete
      asm volatile("" ::: "memory");
#pragma unroll
      for (int mod = 0; mod < NV; ++mod) {
        const char* st = smem + (mod / HPM) * TILE;  // dgate (halves 0 .. HPM - 1) or dup
        const char* bts = smem + BT_OFF + mod * BT_BYTES;
        const char* us = smem + U_OFF + mod * ROWS * 32;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int qk = cc * 8 + 4 * s2 + g;
          const bf16x8 bt = *reinterpret_cast<const bf16x8*>(bts + l16 * btrow + ((qk ^ l16) << 4));
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(st + grow * 128 + (((4 * s2 + g) ^ (grow & 7)) << 4));
          accg[mod] = MFMA(bt, a, accg[mod]);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r1 = 32 * s + 8 * g + q4, r2 = r1 + 4;
          const int x = 2 * wave + (p4 >> 1), h = (p4 & 1) << 3;
          const int ur = rb * 64 + 32 * s + 8 * g;
          // the builtin here (no LDS-DMA in flight to drain): immediate offsets, exact lgkmcnt
          i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(st + r1 * 128 + ((x ^ (r1 & 7)) << 4) + h));
          i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(st + r2 * 128 + ((x ^ (r2 & 7)) << 4) + h));
          i16x4 ulo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(us + (ur + q4) * 32 + p4 * 8));
          i16x4 uhi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(us + (ur + 4 + q4) * 32 + p4 * 8));
          // no row mask on u: the dgate / dup rows >= M are exact zeros (zero inputs), u's clamped rows finite
          const i16x8 av = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const i16x8 bv = {ulo[0], ulo[1], ulo[2], ulo[3], uhi[0], uhi[1], uhi[2], uhi[3]};
          accb[mod][cc] = MFMA(__builtin_bit_cast(bf16x8, av), __builtin_bit_cast(bf16x8, bv), accb[mod][cc]);
        }
      }
    }
    const int m = rb0 + rb * 64 + grow;  // g partials of this row sub-block: ws [half][sp][Mw][16]
#pragma unroll
    for (int mod = 0; mod < NV; ++mod)
      if (m < Mw) *reinterpret_cast<f32x4*>(ws + (((long)mod * nsplit + sp) * Mw + m) * 16 + 4 * g) = accg[mod];
  }
#pragma unroll
  for (int mod = 0; mod < NV; ++mod)
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {  // each chunk's dB over the workgroup's rows
      const long n0 = (long)(mod / HPM) * F + kc0 + cc * 64 + 16 * wave + 4 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(dB + (n0 + i) * (16 * HPM) + 16 * (mod % HPM) + l16, accb[mod][cc][i]);
    }
}


// ---------------------------------------------------------------------------------------------
// dA of one adapter group as ONE stream over its input (round 3; replaces the 64 x 64 f32-atomic tiles):
//   dA[j][n] += sum_m g_s[m][j] * dropout(x)[m][n]        j < s_cols (the used rank rows), n < N
// (peft lora_A.weight.grad; the backward of train.py:352's adapters).  A workgroup owns a 128-column
// stripe of x and a range of 64-row K-tiles (tokens); x [64 x 128] and g_s [64 x 64] tiles stream through
// an NS-stage LDS ring by LDS-DMA from launch-constant per-lane offsets (the K advance in soffset, counted
// vmcnt, raw s_barrier: nothing drains the ring -- the f32-atomic tile kernel's transposed-read builtin made
// hipcc wait vmcnt(0) before every read, serialising its loads).  Both MFMA operands are transposed reads
// (the contraction runs over rows), inline asm with tied waits.  With dropout the x fragments are masked in
// registers by the forward's hash, one hash per two elements: partner lanes (columns n, n ^ 1 share a hash)
// each hash half of the fragment's 8 rows and swap halves by DPP.  Split partials meet in fp32 atomics,
// 64-B segments (D[j][n] with n along the lanes).
constexpr int DA_TN = 128;                 // x columns per workgroup (32 per wave)
constexpr int DA_XB = 64 * DA_TN * 2;      // x tile bytes (64 rows of 256 B)
constexpr int DA_SB = 64 * 128;            // g_s tile bytes (64 rows x 64 rank columns)
constexpr int DA_STG = DA_XB + DA_SB;
constexpr int DA_NS = 3;                   // ring stages (72 KiB: two workgroups per CU)
constexpr int DA_PW = (DA_STG / 1024) / 4; // LDS-DMA pieces per wave per stage (6)

// x image row r (256 B = 16 chunks): logical chunk c at physical c ^ da_swz(r); the 16 rows one
// transposed read touches (8g + q, q < 4) get 16 distinct values
__device__ __forceinline__ int da_swz(int r) { return (r & 3) | (((r >> 3) & 3) << 2); }

template <int AUX = 0>
__device__ __forceinline__ void da_lds16(__amdgpu_buffer_rsrc_t rs, char* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)dst, 16, voff, soff, 0, AUX);
}

__device__ __forceinline__ void da_lds4(__amdgpu_buffer_rsrc_t rs, char* dst, uint32_t voff, int soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)dst, 4, voff, soff, 0, 0);
}

__device__ __forceinline__ void tr2_wait(i16x4& a, i16x4& b) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}

// the keep bits of a lane's x fragment: column n (even lanes n even), rows m0 .. m0 + 7
__device__ __forceinline__ void da_keep8(uint32_t m0, uint32_t n, uint32_t ld, uint32_t seed, uint32_t thr, bool odd,
                                         bool (&keep)[8]) {
  uint32_t mine[4], other[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {  // even lane: rows 0..3, odd lane: rows 4..7 (the pair's shared hashes)
    const uint32_t idx = (m0 + (uint32_t)q + (odd ? 4u : 0u)) * ld + n;
    mine[q] = drop_hash(idx >> 1, seed);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) other[q] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine[q], 0xB1, 0xF, 0xF, false);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const uint32_t h = (e < 4) ? (odd ? other[e] : mine[e]) : (odd ? mine[e - 4] : other[e - 4]);
    keep[e] = (odd ? (h >> 16) : (h & 0xffffu)) >= thr;
  }
}

// DM: 0 no dropout, 1 mask re-hashed, 2 mask from the forward's keep bits (staged with the tile: 64 rows x
// 16 B, one 4-B LDS-DMA per wave)
template <int NJ, int DM, int XA = 0>  // XA: cache-policy bits of the x loads
__global__ __launch_bounds__(256) void lora_da_kernel(const bf16* __restrict__ X, int ldx, int x_bytes,
                                                      const bf16* __restrict__ S, int lds, int s_bytes, int s_cols,
                                                      int nt, float* __restrict__ C, int ldc, uint32_t dseed,
                                                      uint32_t dthresh, float dscale, int drop_ld,
                                                      const uint8_t* __restrict__ kbits, int k_bytes) {
  constexpr int STG = DA_STG + (DM == 2 ? 1024 : 0);
  constexpr int PW = DA_PW + (DM == 2 ? 1 : 0);
  __shared__ __attribute__((aligned(16))) char smem[DA_NS * STG];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4, q4 = l16 >> 2, p4 = l16 & 3;
  const int n0 = blockIdx.x * DA_TN;
  const int t0 = (int)((long)nt * blockIdx.y / gridDim.y), t1 = (int)((long)nt * (blockIdx.y + 1) / gridDim.y);
  const int n_my = t1 - t0;
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)X, 0, x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc((void*)S, 0, s_bytes, 0x00020000);
  // per-lane byte offsets of this wave's pieces at K-tile 0: x pieces = 4 rows x 256 B (4 per wave),
  // g_s pieces = 8 rows x 128 B (2 per wave); the K-tile's 64 rows advance in soffset
  uint32_t vx[4], vs[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (wave * 4 + i) * 4 + (lane >> 4), pc = lane & 15;
    vx[i] = ((uint32_t)row * (uint32_t)ldx + (uint32_t)n0 + (uint32_t)((pc ^ da_swz(row)) * 8)) * 2u;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 8 + (lane >> 3), pc = lane & 7;
    vs[i] = ((uint32_t)row * (uint32_t)lds + (uint32_t)((pc ^ (row & 7)) * 8)) * 2u;
  }
  const int xstep = 64 * ldx * 2, sstep = 64 * lds * 2;  // bytes per K-tile (host: < 2^31 in total)
  // keep bits: row 16 wave + lane / 4, dword lane % 4 of the stripe's 16 bytes
  const __amdgpu_buffer_rsrc_t rsK =
      __builtin_amdgcn_make_buffer_rsrc((void*)kbits, 0, DM == 2 ? k_bytes : 0, 0x00020000);
  const uint32_t vk = (uint32_t)(16 * wave + (lane >> 2)) * (uint32_t)(drop_ld >> 3) + (uint32_t)(n0 >> 3) +
                      (uint32_t)((lane & 3) * 4);
  const int kstep = 64 * (drop_ld >> 3);
  auto stage = [&](int t, int slot) __attribute__((always_inline)) {
    char* st = smem + slot * STG;
#pragma unroll
    for (int i = 0; i < 4; ++i) da_lds16<XA>(rsX, st + (wave * 4 + i) * 1024, vx[i], t * xstep);
#pragma unroll
    for (int i = 0; i < 2; ++i) da_lds16(rsS, st + DA_XB + (wave * 2 + i) * 1024, vs[i], t * sstep);
    if constexpr (DM == 2) da_lds4(rsK, st + DA_STG + wave * 256, vk, t * kstep);
  };
  f32x4 acc[NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int f = 0; f < 2; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < DA_NS - 1; ++i)
    if (i < n_my) stage(t0 + i, i);
  const bool odd = (l16 & 1) != 0;
  for (int i = 0; i < n_my; ++i) {
    // this wave's pieces of stage i landed (NS - 2 newer stages may stay in flight)
    if (i + 1 < n_my) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW * (DA_NS - 2)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's pieces of stage i; every wave done reading stage i - 1
    asm volatile("" ::: "memory");
    if (i + DA_NS - 1 < n_my) stage(t0 + i + DA_NS - 1, (i + DA_NS - 1) % DA_NS);
    const char* xs = smem + (i % DA_NS) * STG;
    const char* ss = xs + DA_XB;
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      const int r1 = 32 * sk + 8 * g + q4, r2 = r1 + 4;
      bf16x8 bx[2], as[NJ];
#pragma unroll
      for (int f = 0; f < 2; ++f) {  // x columns n0 + 32 wave + 16 f + (0..15): chunks 4 wave + 2 f + (0, 1)
        const int x = 4 * wave + 2 * f + (p4 >> 1), h = (p4 & 1) << 3;
        i16x4 lo, hi;
        tr4_issue(xs + r1 * 256 + ((x ^ da_swz(r1)) << 4) + h, lo);
        tr4_issue(xs + r2 * 256 + ((x ^ da_swz(r2)) << 4) + h, hi);
        tr2_wait(lo, hi);
        const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bx[f] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {  // rank columns 16 j + (0..15): chunks 2 j + (0, 1)
        const int x = 2 * j + (p4 >> 1), h = (p4 & 1) << 3;
        i16x4 lo, hi;
        tr4_issue(ss + r1 * 128 + ((x ^ (r1 & 7)) << 4) + h, lo);
        tr4_issue(ss + r2 * 128 + ((x ^ (r2 & 7)) << 4) + h, hi);
        tr2_wait(lo, hi);
        const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        as[j] = __builtin_bit_cast(bf16x8, v);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DM == 1) {  // lane: column n, rows m .. m + 7 of x
        const uint32_t m = (uint32_t)((t0 + i) * 64 + 32 * sk + 8 * g);
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const uint32_t n = (uint32_t)(n0 + 32 * wave + 16 * f + l16);
          bool keep[8];
          da_keep8(m, n, (uint32_t)drop_ld, dseed, dthresh, odd, keep);
#pragma unroll
          for (int e = 0; e < 8; ++e) bx[f][e] = keep[e] ? f2bf(bf2f(bx[f][e]) * dscale) : f2bf(0.f);
        }
      } else if constexpr (DM == 2) {  // the bits of rows 32 sk + 8 g + e, columns 32 wave .. + 31
        const char* kb = xs + DA_STG + (32 * sk + 8 * g) * 16 + wave * 4;
        uint32_t w[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) w[e] = *reinterpret_cast<const uint32_t*>(kb + e * 16);
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            bx[f][e] = ((w[e] >> (16 * f + l16)) & 1u) ? f2bf(bf2f(bx[f][e]) * dscale) : f2bf(0.f);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[j][f] = MFMA(as[j], bx[f], acc[j][f]);  // D[16 j + 4 g + q][n = l16]
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int n = n0 + 32 * wave + 16 * f + l16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jr = 16 * j + 4 * g + q;
        if (jr < s_cols) atomicAdd(C + (long)jr * ldc + n, acc[j][f][q]);
      }
    }
}

// out[m][16 mod + c] = bf16(scale * sum_sp ws[mod][sp][m][c]) (m < M; 0 for M <= m < M_out), pad columns 0
// PB partial loads in flight per thread (the same left-to-right sum for any PB, bit-identical).  16 instead of 8
// measured no faster (kernel + reduce per group within 0.5 us either way, profiles/r06/gdb_reduce_pb_ab.log):
// the product keeps 8, the ablation build's OSPO_GDB_RED16 runs 16
template <int PB = 8>
__global__ void gdb_reduce_kernel(const float* __restrict__ ws, int nmods, int nsplit, int Mw, int M, int M_out,
                                  float scale, bf16* __restrict__ out, int ldo, int out_cols) {
  const unsigned cq = (unsigned)out_cols / 4;  // 32-bit index math: M_out * cq < 2^31 (host check)
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (unsigned)M_out * cq) return;
  const int m = (int)(tid / cq), c = (int)(tid % cq) * 4;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  const int mod = c / 16;
  if (m < M && mod < nmods) {
    for (int s0 = 0; s0 < nsplit; s0 += PB) {
      f32x4 p[PB];
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if (s0 + k < nsplit)  // (non-temporal: each partial is read once)
          p[k] = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>(ws + (((long)mod * nsplit + s0 + k) * Mw + m) * 16 + (c & 15)));
#pragma unroll
      for (int k = 0; k < PB; ++k)
        if (s0 + k < nsplit) v += p[k];
    }
  }
  uint2 pk;
  pk.x = pack2(v[0] * scale, v[1] * scale);
  pk.y = pack2(v[2] * scale, v[3] * scale);
  *reinterpret_cast<uint2*>(out + (long)m * ldo + c) = pk;
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

// skinny workspace head: one counter per 64-row block for the in-launch split sum (M_out <= 65536)
constexpr int SK_CNT_BYTES = OSPO_WS_SKINNY_CNT_BYTES;
#ifdef OSPO_ABLATION
static bool g_sk_reduce_launch = getenv("OSPO_SK_REDUCE_LAUNCH") != nullptr;  // A/B: the separate reduce kernel
#else
constexpr bool g_sk_reduce_launch = false;
#endif

struct SkDropArgs {
  uint32_t seed = 0, thresh = 0;
  float scale = 0.f;  // > 0: dropout on
  bf16* xd = nullptr;
  int ldxd = 0;
  uint8_t* bits = nullptr;  // v3 only: the keep bits of every element (row-major, 8 per byte)
};

#ifdef OSPO_ABLATION
static int g_skinny_variant = 4;  // 1 = 16-row skinny loop, 2 = 64-row LDS-shared, 3 = 2 with whole-chunk splits, 4 = v3 (default)
static int g_sk3_wgs = 0;         // v3: target workgroups per launch (0: sk3_target's rule; A/B knob 100 + W)
#else
constexpr int g_skinny_variant = 4;  // the product library runs v3 (v2 where v3's 32-bit buffer offsets do not reach)
constexpr int g_sk3_wgs = 0;
#endif
// v3 workgroup target: 512 (two per CU) for the 4096-long adapter inputs; 1024 for the 11008-long down input,
// whose 25-chunk workgroups at 512 left the loop latency-bound (SwiGLU + u_d 100.8 / 93.9 / 86.4 / 92.0 us at
// 512 / 768 / 1024 / 1536, profiles/r03/skinny_swg_wgs.json).  At most 1024 (the workspace rule below).
static inline int sk3_target(int K) { return g_sk3_wgs > 0 ? g_sk3_wgs : (K >= 8192 ? 1024 : 512); }

// v2 K split: ~1024 workgroups over (64-row blocks x modules), each split >= one chunk.
// Variant 3: splits own whole KC chunks (kper = a multiple of KC), so no workgroup runs a short
// remainder chunk of its own; only the last split can be shorter.
static int skinny2_kper(int M_out, int K, int nz, int KC, bool whole_chunks) {
  const int blocks = (M_out + 63) / 64 * nz;
  int splits = (1024 + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : splits;
  const int maxs = K / KC > 0 ? K / KC : 1;
  splits = splits > maxs ? maxs : splits;
  if (whole_chunks) {
    const int chunks = (K + KC - 1) / KC;
    const int cpk = (chunks + splits - 1) / splits;
    return cpk * KC;
  }
  const int kper = (K + splits - 1) / splits;
  return (kper + 31) / 32 * 32;
}

extern "C" size_t ospo_lora_skinny_ws_bytes(int M_out, int K, int n_tiles) {
  const long rb = (M_out + 15) / 16;
  const int sp = skinny_splits(M_out, K);
  const size_t v1 = (size_t)(sp > 1 ? sp : 0) * rb * n_tiles * 64 * sizeof(f32x4) + 16;
  // v2: the worst case over its tilings (KC = 128 .. 512, one module or n_tiles modules)
  size_t v2 = 0;
  for (int nz = 1; nz <= n_tiles; nz = nz * 2 > n_tiles && nz < n_tiles ? n_tiles : nz * 2) {
    for (int KC = 128; KC <= 512; KC *= 2) {
      const int kper = skinny2_kper(M_out, K, nz, KC, false);  // the larger split count of the two rules
      const size_t sp2 = (K + kper - 1) / kper;
      const size_t b = sp2 > 1 ? sp2 * (size_t)((M_out + 63) / 64 * 64) * 16 * n_tiles * 4 : 0;
      v2 = b > v2 ? b : v2;
    }
    if (nz == n_tiles) break;
  }
  // v3: at most max(g_sk3_wgs, 1024) workgroups' worth of splits over one module's row blocks
  {
    const long blocks = (M_out + 63) / 64;
    const long wgs = sk3_target(K) > 1024 ? sk3_target(K) : 1024;
    long sp3 = (wgs + blocks - 1) / blocks;
    sp3 = sp3 > K / 64 ? K / 64 : sp3;
    const size_t b = sp3 > 1 ? (size_t)sp3 * (size_t)((M_out + 63) / 64 * 64) * 16 * n_tiles * 4 : 0;
    v2 = b > v2 ? b : v2;
  }
  return (v1 > v2 ? v1 : v2) + 16 + SK_CNT_BYTES;  // + the row-block counters at the head
}

#ifdef OSPO_ABLATION
extern "C" int ospo_set_skinny_variant(int v) {
  if (v >= 100) {  // v3 with a target of v - 100 workgroups per launch
    g_skinny_variant = 4;
    g_sk3_wgs = v - 100;
    return OSPO_OK;
  }
  if (v < 1 || v > 4) return OSPO_ERR_ARG;
  g_skinny_variant = v;
  g_sk3_wgs = 0;  // back to sk3_target's rule
  return OSPO_OK;
}
#endif

template <int NT>
static int launch_skinny2(const bf16* a, int lda, const bf16* b, int ldb, int b_rows, int M, int M_out, int K,
                          int a_koff, int nz, int tiles_total, float scale, bf16* o, int ldo, int out_cols, float* part,
                          size_t ws_bytes, hipStream_t stream, const SkDropArgs& dr) {
  const int kper = skinny2_kper(M_out, K, nz, Sk2Cfg<NT>::KC, g_skinny_variant == 3);
  const int splits = (K + kper - 1) / kper;
  const int M_pad = (M_out + 63) / 64 * 64;
  if (splits > 1 && ws_bytes < (size_t)splits * M_pad * 16 * tiles_total * 4) return OSPO_ERR_SHAPE;
  const dim3 grid(M_pad / 64, splits, nz);
  if (dr.scale > 0.f)
    hipLaunchKernelGGL((skinny2_kernel<NT, true>), grid, dim3(256), 0, stream, a, lda, b, ldb, b_rows, M, M_out, K,
                       kper, a_koff, tiles_total, scale, o, ldo, out_cols, part, M_pad, dr.seed, dr.thresh, dr.scale,
                       dr.xd, dr.ldxd);
  else
    hipLaunchKernelGGL((skinny2_kernel<NT, false>), grid, dim3(256), 0, stream, a, lda, b, ldb, b_rows, M, M_out, K,
                       kper, a_koff, tiles_total, scale, o, ldo, out_cols, part, M_pad, 0u, 0u, 0.f, nullptr, 0);
  OSPO_CHECK_LAUNCH();
  if (splits > 1) {
    const long n = (long)M_out * (out_cols / 4);
    if (n >= (1L << 31)) return OSPO_ERR_SHAPE;  // the reduce's 32-bit index
    hipLaunchKernelGGL(skinny2_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, part, splits,
                       M, M_out, M_pad, 16 * tiles_total, scale, o, ldo, out_cols);
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}


// v3 split: ~2 workgroups per CU over (64-row blocks x modules), whole 64-k chunks per split.
// SWG: a = gu (gate | up, up at column K), the SwiGLU product h written to hout on the way
// ws: [row-block counters: SK_CNT_BYTES][fp32 partials] (the counters are zero between calls)
template <int NT, bool SWG = false>
static int launch_skinny3(const bf16* a, int lda, const bf16* b, int ldb, int b_rows, int M, int M_out, int K,
                          int a_koff, int nz, int tiles_total, float scale, bf16* o, int ldo, int out_cols, float* part,
                          size_t ws_bytes, hipStream_t stream, const SkDropArgs& dr, bf16* hout = nullptr,
                          int ldh = 0, unsigned* cnt = nullptr) {
  const int blocks = (M_out + 63) / 64 * nz;
  const int chunks = K / 64;
  int splits = (sk3_target(K) + blocks - 1) / blocks;
  splits = splits < 1 ? 1 : (splits > chunks ? chunks : splits);
  const int cps = (chunks + splits - 1) / splits;
  const int kper = cps * 64;
  splits = (K + kper - 1) / kper;
  const int M_pad = (M_out + 63) / 64 * 64;
  if (splits > 1 && ws_bytes < (size_t)splits * M_pad * 16 * tiles_total * 4) return OSPO_ERR_SHAPE;
  const long a_bytes = (long)(M - 1) * lda * 2 + (long)((nz - 1) * a_koff + K * (SWG ? 2 : 1)) * 2;
  const long b_bytes = (long)(b_rows - 1) * ldb * 2 + (long)K * 2;
  if (a_bytes >= (1L << 31)) return OSPO_ERR_SHAPE;  // 32-bit buffer offsets
  const dim3 grid(M_pad / 64, splits, nz);
  // the split sum in the launch (last arriver per row block) unless the ablation build asks for the reduce kernel
  unsigned* c = (splits > 1 && M_pad / 64 <= SK_CNT_BYTES / 4 && !g_sk_reduce_launch) ? cnt : nullptr;
  // LDS ring stages: 2 (one chunk in flight beside the one computed).  The loop is issue-bound (per 64-k chunk
  // and wave: the LDS-DMA issue, a barrier, the dropout hash's quarter-rate multiplies), so residency beats
  // depth: per call 19.3 / 17.5 / 93.7 us at 2 stages against 20.3 / 18.7 / 97.1 at 4 and 29.0 / 25.1 / 121.4
  // at 8 (u_qkv / u_o / SwiGLU + u_d, profiles/r03/skinny_ring_depth.jsonl).  Ablation: OSPO_SK3_NS.
  [[maybe_unused]] int ns = 2;
#ifdef OSPO_ABLATION
  static const int ns_env = [] {
    const char* e = getenv("OSPO_SK3_NS");
    return e ? atoi(e) : 2;
  }();
  ns = ns_env;
#endif
#define SK3_LAUNCH3(NS_, BTR_, AA_)                                                                              \
  if (dr.scale > 0.f)                                                                                            \
    hipLaunchKernelGGL((skinny3_kernel<NT, true, SWG, NS_, BTR_, AA_>), grid, dim3(256), 0, stream, a, lda,        \
                       (int)a_bytes, b, ldb, b_rows, (int)b_bytes, M, M_out, K, kper, a_koff, tiles_total, scale, o, \
                       ldo, out_cols, part, M_pad, dr.seed, dr.thresh, dr.scale, dr.bits, hout, ldh, K * 2, c);     \
  else                                                                                                           \
    hipLaunchKernelGGL((skinny3_kernel<NT, false, SWG, NS_, BTR_, AA_>), grid, dim3(256), 0, stream, a, lda,       \
                       (int)a_bytes, b, ldb, b_rows, (int)b_bytes, M, M_out, K, kper, a_koff, tiles_total, scale, o, \
                       ldo, out_cols, part, M_pad, 0u, 0u, 0.f, nullptr, hout, ldh, K * 2, c);
// A loads non-temporal (the activation is not re-read from this CU's caches): same-box step 111.04 / 110.77 ->
// 110.73 / 110.58 ms (profiles/r04/step_skinny_nt_ab.txt); OSPO_SK3_NT=0 (ablation build) restores the default policy
#define SK3_LAUNCH2(NS_, BTR_) SK3_LAUNCH3(NS_, BTR_, 2)
#define SK3_LAUNCH(NS_) SK3_LAUNCH2(NS_, false)
#ifdef OSPO_ABLATION
  static const bool btreg = getenv("OSPO_SK3_BTREG") != nullptr;
  static const int sk_nt = [] {  // A/B: OSPO_SK3_NT=0 restores the default cache policy of the A loads
    const char* e = getenv("OSPO_SK3_NT");
    return e ? atoi(e) : 2;
  }();
  if (ns == 2 && sk_nt == 0) {
    SK3_LAUNCH3(2, false, 0)
  } else if (ns == 2 && btreg) {
    SK3_LAUNCH2(2, true)
  } else if (ns == 2) {
    SK3_LAUNCH(2)
  } else if (ns == 3) {
    SK3_LAUNCH(3)
  } else if (ns == 6) {
    SK3_LAUNCH(6)
  } else if (ns == 8) {
    SK3_LAUNCH(8)
  } else {
    SK3_LAUNCH(4)
  }
#else
  SK3_LAUNCH(2)
#endif
#undef SK3_LAUNCH
#undef SK3_LAUNCH2
#undef SK3_LAUNCH3
  OSPO_CHECK_LAUNCH();
  if (splits > 1 && !c) {
    const long n = (long)M_out * (out_cols / 4);
    if (n >= (1L << 31)) return OSPO_ERR_SHAPE;  // the reduce's 32-bit index
    hipLaunchKernelGGL(skinny2_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, part, splits,
                       M, M_out, M_pad, 16 * tiles_total, scale, o, ldo, out_cols);
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}

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
                                int ld_xd, void* keep_bits, hipStream_t stream) {
  if (!A || !Bt || !out || !ws) return OSPO_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  SkDropArgs dr;
  if (drop_p > 0.f) {
    if (a_koff != 0) return OSPO_ERR_UNSUPPORTED;  // dropout acts on the adapter input (dense u product)
    if ((long)M * K > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
    if (K & 1) return OSPO_ERR_SHAPE;                       // mask pairs (drop_keep) start at even indices
    if (xd && (ld_xd < K || ld_xd % 8 || !aligned16(xd))) return OSPO_ERR_SHAPE;
    dr.seed = drop_seed;
    dr.thresh = drop_threshold(drop_p);
    dr.scale = 1.f / (1.f - drop_p);
    dr.xd = (bf16*)xd;
    dr.ldxd = ld_xd;
    dr.bits = (uint8_t*)keep_bits;
  } else if (keep_bits) {
    return OSPO_ERR_ARG;  // keep bits are a dropout output
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
  // ws head: the skinny kernel's row-block counters (zero between calls); partials after it
  unsigned* cnt = (unsigned*)ws;
  f32x4* part = (f32x4*)((char*)ws + SK_CNT_BYTES);
  ws_bytes -= SK_CNT_BYTES;
  const bool sk3_ok = K % 64 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
                      (long)(M - 1) * lda * 2 + (long)(nmods * (a_koff > 0 ? a_koff : 0) + K) * 2 < (1L << 31) &&
                      (long)b_rows * ldb * 2 < (1L << 31);
  if (dr.bits && !(g_skinny_variant == 4 && sk3_ok && out_cols % 4 == 0 && !dr.xd))
    return OSPO_ERR_UNSUPPORTED;  // the keep-bit output is v3's
  if (g_skinny_variant == 4 && sk3_ok && out_cols % 4 == 0 && !dr.xd) {  // (the masked-copy output is v2's)
    const int nz = a_koff > 0 ? nmods : 1;
    const int nt = a_koff > 0 ? module_tiles : n_tiles;
    float* p2 = (float*)part;
    switch (nt) {
      case 1: return launch_skinny3<1>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      case 2: return launch_skinny3<2>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      case 3: return launch_skinny3<3>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      case 4: return launch_skinny3<4>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      case 6: return launch_skinny3<6>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      case 8: return launch_skinny3<8>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, nullptr, 0, cnt);
      default: break;
    }
  }
  if (dr.bits) return OSPO_ERR_UNSUPPORTED;  // keep bits are written by the v3 cases above only (tile counts 1-4, 6, 8)
  if (g_skinny_variant >= 2 && out_cols % 4 == 0 && K >= 128) {
    // dense: one workgroup column over all n-tiles; block-diagonal: grid z = module
    const int nz = a_koff > 0 ? nmods : 1;
    const int nt = a_koff > 0 ? module_tiles : n_tiles;
    float* p2 = (float*)part;
    switch (nt) {
      case 1: return launch_skinny2<1>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      case 2: return launch_skinny2<2>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      case 3: return launch_skinny2<3>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      case 4: return launch_skinny2<4>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      case 6: return launch_skinny2<6>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      case 8: return launch_skinny2<8>(a, lda, b, ldb, b_rows, M, M_out, K, a_koff, nz, n_tiles, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr);
      default: break;  // other tile counts: v1 below
    }
  }
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

// ---------------------------------------------------------------------------------- lora_gdb
using GdbReduceFn = void (*)(const float*, int, int, int, int, int, float, bf16*, int, int);
static GdbReduceFn gdb_reduce_fn() {
#ifdef OSPO_ABLATION
  if (getenv("OSPO_GDB_RED16")) return gdb_reduce_kernel<16>;  // A/B: 16 partial loads in flight
#endif
  return gdb_reduce_kernel<8>;
}

static int gdb_nch(int M, int nmods, int Nmod, int rows = 512) {  // rows: the workgroup's row block
  const int rbk = (M + rows - 1) / rows;
  int min_wgs = 256;
#ifdef OSPO_ABLATION
  if (const char* e = getenv("OSPO_GDB_MINWG")) min_wgs = atoi(e);  // A/B: grid size below which nch = 2
#endif
  if (Nmod % 256 == 0 && (long)rbk * nmods * (Nmod / 256) >= min_wgs) return 4;
  return 2;
}

extern "C" size_t ospo_lora_gdb_ws_bytes(int M, int nmods, int Nmod) {
  if (M <= 0 || nmods <= 0 || Nmod <= 0 || Nmod % 128) return 0;
  const size_t Mw = (size_t)(M + 63) / 64 * 64;
  // the in-launch sum's counters (head), then the partials (the nch = 2 worst case)
  return GDB_CNT_BYTES + (size_t)nmods * (Nmod / 128) * Mw * 16 * sizeof(float) + 16;
}

#ifdef OSPO_ABLATION
// lora_gdb_kernel's in-launch sum needs every workgroup of the grid resident at once (its row blocks wait for
// all their workgroups): the device's capacity for the kernel, cached per device
static long gdb_inl_capacity() {
  static long cap[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (cap[dev] == 0) {
    int ncu = 0, per = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, lora_gdb_kernel<8, 4, 0, true>, 256, 0) != hipSuccess)
      return 0;
    cap[dev] = (long)ncu * per;
  }
  return cap[dev];
}
#endif

extern "C" int ospo_lora_gdb_r(const void* dy, int ldy, const void* Bt, int ldb, const void* u, int ldu, int M,
                               int M_out, int nmods, int Nmod, int r, float scale, void* out, int ldo, int out_cols,
                               float* dB, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!dy || !Bt || !u || !out || !dB || !ws) return OSPO_ERR_ARG;
  if (r != 16 && r != 32) return OSPO_ERR_UNSUPPORTED;
  const int hpm = r / 16, vm = nmods * hpm;  // 16-column halves: the kernel's "modules"
  if (M <= 0 || M_out < M || nmods < 1 || nmods > 4 || Nmod <= 0 || Nmod % 128) return OSPO_ERR_SHAPE;
  if (ldy < nmods * Nmod || ldb < Nmod || ldu < 16 * vm || ldo < out_cols || out_cols < 16 * vm ||
      out_cols % 4 || ldy % 8 || ldb % 8 || ldu % 8 || ldo % 4)
    return OSPO_ERR_SHAPE;
  if (ws_bytes < ospo_lora_gdb_ws_bytes(M, vm, Nmod)) return OSPO_ERR_SHAPE;
  if (!aligned16(dy) || !aligned16(Bt) || !aligned16(u) || !aligned16(ws) || ((uintptr_t)dB & 3) ||
      ((uintptr_t)out & 7))
    return OSPO_ERR_ALIGN;
  // one workgroup covers all hpm halves of its module's column block (dy read once).  Row blocks of 256 at
  // r = 32 (RSB 4: the two halves' g accumulators of 512 rows left one wave per SIMD) and for one-module groups
  // (o, down: 304 workgroups of 256 columns instead of 320 of 128, half the g partials; 18.5-18.9 against
  // 20.6-21.4 us per call at r = 16, 26-28 against 29-30 at r = 32, profiles/r06/gdb_variant_sweep_*b.log);
  // 512 for the multi-module groups at r = 16 (q|k|v 32.5 against 37.0 us at 256)
  int wrows = (hpm == 2 || nmods == 1) ? 256 : 512;
#ifdef OSPO_ABLATION
  const bool rsb4 = hpm == 1 && getenv("OSPO_GDB_RSB4");  // A/B: 256-row workgroups at r = 16
  const bool ns6r32 = hpm == 2 && getenv("OSPO_GDB_NS6");  // A/B: a 6-stage ring at r = 32
  if (rsb4) wrows = 256;
  if (hpm == 1 && getenv("OSPO_GDB_RSB8")) wrows = 512;  // A/B: the round-5 512-row blocks for every group
#endif
  const int nch = gdb_nch(M, nmods, Nmod, wrows);
  const int nsplit = Nmod / (64 * nch);
  const int Mw = (M + 63) / 64 * 64;
  const dim3 grid((M + wrows - 1) / wrows, nmods * nsplit);
  float* part = (float*)((char*)ws + GDB_CNT_BYTES);
  // A/B (ablation build, OSPO_GDB_INL=1): the partials summed inside the launch where the whole grid fits on the
  // device at once -- bit-identical, and no faster in the step (36.44 / 36.37 against 36.47 / 36.37 pairs/s,
  // profiles/r05/gdb_inlaunch_ab.txt): the product keeps the reduce launch
  bool inl = false;
#ifdef OSPO_ABLATION
  if (getenv("OSPO_GDB_INL") && wrows == 512)
    inl = grid.x <= 1024 && (long)grid.x * grid.y <= gdb_inl_capacity() && (long)M_out * out_cols < (1L << 31);
#endif
  if (inl) {
    const GdbInl gi{(unsigned*)ws, M_out, scale, (bf16*)out, ldo, out_cols};
    hipLaunchKernelGGL((lora_gdb_kernel<8, 4, 0, true>), grid, dim3(256), 0, stream, (const bf16*)dy, ldy,
                       (const bf16*)Bt, ldb, (const bf16*)u, ldu, M, Nmod, nch, part, Mw, dB, gi);
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  auto kfn = hpm == 2 ? lora_gdb_kernel<4, 4, 0, false, 2> : wrows == 256 ? lora_gdb_kernel<4, 4> : lora_gdb_kernel<8, 4>;
#ifdef OSPO_ABLATION
  const bool r8 = hpm == 1 && wrows == 512;
  if (r8 && getenv("OSPO_GDB_NS6")) kfn = lora_gdb_kernel<8, 6>;  // A/B: a 6-stage ring
  if (r8 && getenv("OSPO_GDB_NS2")) kfn = lora_gdb_kernel<8, 2>;  // A/B: 2- and 3-stage rings (more residency)
  if (r8 && getenv("OSPO_GDB_NS3")) kfn = lora_gdb_kernel<8, 3>;
  if (r8 && getenv("OSPO_NT_GDB")) kfn = lora_gdb_kernel<8, 4, 2>;  // A/B: non-temporal dy loads
  if (rsb4) kfn = getenv("OSPO_GDB_NS6") ? lora_gdb_kernel<4, 6> : lora_gdb_kernel<4, 4>;
  if (ns6r32) kfn = lora_gdb_kernel<4, 6, 0, false, 2>;
#endif
  const long n = (long)M_out * (out_cols / 4);
  if (n >= (1L << 31)) return OSPO_ERR_SHAPE;  // the reduce's 32-bit index
  hipLaunchKernelGGL(kfn, grid, dim3(256), 0, stream, (const bf16*)dy, ldy, (const bf16*)Bt, ldb,
                     (const bf16*)u, ldu, M, Nmod, nch, part, Mw, dB, GdbInl{});
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(gdb_reduce_fn(), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const float*)part,
                     vm, nsplit, Mw, M, M_out, scale, (bf16*)out, ldo, out_cols);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_lora_gdb(const void* dy, int ldy, const void* Bt, int ldb, const void* u, int ldu, int M, int M_out,
                             int nmods, int Nmod, float scale, void* out, int ldo, int out_cols, float* dB, void* ws,
                             size_t ws_bytes, hipStream_t stream) {
  return ospo_lora_gdb_r(dy, ldy, Bt, ldb, u, ldu, M, M_out, nmods, Nmod, 16, scale, out, ldo, out_cols, dB, ws,
                         ws_bytes, stream);
}

extern "C" int ospo_swiglu_lora_gdb_r(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu,
                                      const void* Bt, int ldb, const void* u, int ldu, int M, int M_out, int F, int r,
                                      float scale, void* out, int ldo, int out_cols, float* dB, void* ws,
                                      size_t ws_bytes, hipStream_t stream) {
  if (!dh || !gu || !dgu || !Bt || !u || !out || !dB || !ws) return OSPO_ERR_ARG;
  if (r != 16 && r != 32) return OSPO_ERR_UNSUPPORTED;
  const int hpm = r / 16, vm = 2 * hpm;
  if (M <= 0 || M_out < M || F <= 0 || F % 128) return OSPO_ERR_SHAPE;
  if (ld_dh < F || ld_gu < 2 * F || ld_dgu < 2 * F || ldb < F || ldu < 16 * vm || ldo < out_cols ||
      out_cols < 16 * vm || out_cols % 4 || ld_dh % 8 || ld_gu % 8 || ld_dgu % 8 || ldb % 8 || ldu % 8 || ldo % 4)
    return OSPO_ERR_SHAPE;
  if (ws_bytes < ospo_lora_gdb_ws_bytes(M, vm, F)) return OSPO_ERR_SHAPE;
  if (!aligned16(dh) || !aligned16(gu) || !aligned16(dgu) || !aligned16(Bt) || !aligned16(u) || !aligned16(ws) ||
      ((uintptr_t)dB & 3) || ((uintptr_t)out & 7))
    return OSPO_ERR_ALIGN;
  const long Mr = (long)(M + 511) / 512 * 512;  // rows the grid addresses (clamped by the ranges, not the offsets)
  if (Mr * ld_dgu * 2 >= (1L << 31) || Mr * ld_gu * 2 >= (1L << 31) || Mr * ld_dh * 2 >= (1L << 31))
    return OSPO_ERR_UNSUPPORTED;  // the buffer ranges / offsets (32-bit)
  const int nch = gdb_nch(M, 2, F, hpm == 2 ? 256 : 512);  // as ospo_lora_gdb_r on dgu: the same partials
  const int nsplit = F / (64 * nch);
  const int Mw = (M + 63) / 64 * 64;
  // one sub-tile of prefetch, non-temporal input loads (gu, dh are dead after this pass) and sc1 dgu stores:
  // 103.6 us at the step shape against 125.0 with default policies and 150 for the two launches
  // (profiles/r04/swiglu_gdb_variants.log)
  auto kfn = nch == 4 ? swiglu_gdb_kernel<8, 2, 4> : swiglu_gdb_kernel<8, 2, 2>;
  int rows = 512;
  if (hpm == 2) {  // r = 32: four halves' Bt / u images; 256-row workgroups keep two per CU (80 KiB of LDS)
    kfn = nch == 4 ? swiglu_gdb_kernel<4, 2, 4, 0, 2, 16, 2> : swiglu_gdb_kernel<4, 2, 2, 0, 2, 16, 2>;
    rows = 256;
  }
#ifdef OSPO_ABLATION
  if (const char* e = getenv("OSPO_SWGDB"); e && hpm == 1) {  // A/B: prefetch depth, cache policies, phases removed
    const int v = atoi(e);
    if (nch == 4) {
      if (v == 1) kfn = swiglu_gdb_kernel<8, 2, 4, 0, 0, 0>;
      if (v == 2) kfn = swiglu_gdb_kernel<8, 4, 4, 0, 0, 0>;
      if (v == 3) kfn = swiglu_gdb_kernel<8, 2, 4, 0, 2, 0>;
      if (v == 4) kfn = swiglu_gdb_kernel<8, 2, 4, 0, 2, 2>;
      if (v == 5) kfn = swiglu_gdb_kernel<8, 2, 4, 0, 0, 2>;
      if (v == 6) kfn = swiglu_gdb_kernel<8, 4, 4>;
      if (v == 7) kfn = swiglu_gdb_kernel<8, 2, 4, 1>;
      if (v == 8) kfn = swiglu_gdb_kernel<8, 2, 4, 2>;
    }
  }
#endif
  const long n = (long)M_out * (out_cols / 4);
  if (n >= (1L << 31)) return OSPO_ERR_SHAPE;
  float* part = (float*)((char*)ws + GDB_CNT_BYTES);  // (ospo_lora_gdb's layout: the counters' head first)
  hipLaunchKernelGGL(kfn, dim3((M + rows - 1) / rows, nsplit), dim3(256), 0, stream,
                     (const bf16*)dh, ld_dh, (const bf16*)gu, ld_gu, (bf16*)dgu, ld_dgu, (const bf16*)Bt, ldb,
                     (const bf16*)u, ldu, M, F, part, Mw, dB);
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(gdb_reduce_fn(), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const float*)part, vm,
                     nsplit, Mw, M, M_out, scale, (bf16*)out, ldo, out_cols);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_swiglu_lora_gdb(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu,
                                    const void* Bt, int ldb, const void* u, int ldu, int M, int M_out, int F,
                                    float scale, void* out, int ldo, int out_cols, float* dB, void* ws,
                                    size_t ws_bytes, hipStream_t stream) {
  return ospo_swiglu_lora_gdb_r(dh, ld_dh, gu, ld_gu, dgu, ld_dgu, Bt, ldb, u, ldu, M, M_out, F, 16, scale, out, ldo,
                                out_cols, dB, ws, ws_bytes, stream);
}

// dA of one adapter group (lora_da_kernel): C [s_cols][N] fp32 += S^T . dropout(X) over K = nt * 64 rows.
// X [K][N] bf16 (ldx), S [K][lds] bf16 with lds in {64, 128} (the packed g_s; rows the caller zero-padded
// are zero), splits = K-tile ranges per 128-column stripe (1 .. nt).
extern "C" int ospo_lora_da(const void* X, int ldx, int N, const void* S, int lds, int s_cols, int K, float* C,
                            int ldc, int splits, unsigned drop_seed, float drop_p, const void* keep_bits,
                            hipStream_t stream) {
  if (!X || !S || !C) return OSPO_ERR_ARG;
  if (N <= 0 || K <= 0 || K % 64 || N % DA_TN || s_cols <= 0 || s_cols > 64) return OSPO_ERR_SHAPE;
  if (splits < 1 || splits > K / 64) return OSPO_ERR_SHAPE;
  if (ldx < N || ldx % 8 || (lds != 64 && lds != 128) || ldc < N) return OSPO_ERR_SHAPE;
  if ((long)K * ldx * 2 >= (1L << 31) || (long)K * lds * 2 >= (1L << 31)) return OSPO_ERR_SHAPE;  // 32-bit offsets
  if (!aligned16(X) || !aligned16(S)) return OSPO_ERR_ALIGN;
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  const bool drop = drop_p > 0.f;
  if (drop && (N & 1)) return OSPO_ERR_SHAPE;  // mask pairs start at even indices
  if (drop && (long)K * N > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
  const uint32_t thr = drop_threshold(drop_p);
  const float dscale = drop ? 1.f / (1.f - drop_p) : 0.f;
  const int nt = K / 64;
  const int x_bytes = (int)((long)(K - 1) * ldx * 2 + (long)N * 2);
  const int s_bytes = (int)((long)K * lds * 2);
  if (keep_bits && (!drop || (long)K * N / 8 >= (1L << 31))) return OSPO_ERR_ARG;
  const int k_bytes = keep_bits ? (int)((long)K * N / 8) : 0;
  const uint8_t* kb = (const uint8_t*)keep_bits;
  const dim3 grid(N / DA_TN, splits);
  int xa = 2;  // x non-temporal: the saved activation is read once here (same-box step 111.74 / 111.33 -> 111.48 /
               // 111.31 ms, profiles/r04/step_swiglu_gdb_nt_ab.txt)
#ifdef OSPO_ABLATION
  if (getenv("OSPO_DA_DEFAULT_POLICY")) xa = 0;  // A/B: the default cache policy
#endif
#define DA_LAUNCH2(NJV, XAV)                                                                                      \
  do {                                                                                                            \
    if (drop && kb)                                                                                               \
      hipLaunchKernelGGL((lora_da_kernel<NJV, 2, XAV>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, x_bytes, \
                         (const bf16*)S, lds, s_bytes, s_cols, nt, C, ldc, 0u, 0u, dscale, N, kb, k_bytes);       \
    else if (drop)                                                                                                \
      hipLaunchKernelGGL((lora_da_kernel<NJV, 1, XAV>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, x_bytes, \
                         (const bf16*)S, lds, s_bytes, s_cols, nt, C, ldc, drop_seed, thr, dscale, N, nullptr, 0); \
    else                                                                                                          \
      hipLaunchKernelGGL((lora_da_kernel<NJV, 0, XAV>), grid, dim3(256), 0, stream, (const bf16*)X, ldx, x_bytes, \
                         (const bf16*)S, lds, s_bytes, s_cols, nt, C, ldc, 0u, 0u, 0.f, N, nullptr, 0);          \
  } while (0)
#define DA_LAUNCH(NJV)            \
  do {                            \
    if (xa) DA_LAUNCH2(NJV, 2);   \
    else DA_LAUNCH2(NJV, 0);      \
  } while (0)
  switch ((s_cols + 15) / 16) {
    case 1: DA_LAUNCH(1); break;
    case 2: DA_LAUNCH(2); break;
    case 3: DA_LAUNCH(3); break;
    default: DA_LAUNCH(4); break;
  }
#undef DA_LAUNCH2
#undef DA_LAUNCH
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

// The MLP's SwiGLU forward fused with the down adapter's u product (ospo/wrapper/train.py:352 through HF
// LlamaMLP.forward: down_proj(act_fn(gate_proj(x)) * up_proj(x)) with peft's lora_A on the down input):
//   h[m][k]   = bf16(bf16(silu(gu[m][k])) * gu[m][F + k])                 (= ospo_swiglu_fwd, rows < M)
//   out[m][c] = scale * sum_k dropout(h)[m][k] * Bt[c][k]                 (= ospo_lora_skinny on h, dense)
// one stream over gu: h is stored and consumed in registers, never re-read.  K = F % 64 == 0; ws and
// the zero-fill of out rows M..M_out-1 / columns 16 n_tiles.. as ospo_lora_skinny; keep_bits as there.
extern "C" int ospo_swiglu_fwd_lora_down(const void* gu, int ld_gu, void* h, int ld_h, int M, int M_out, int F,
                                         const void* Bt, int ldb, int b_rows, int n_tiles, float scale, void* out,
                                         int ldo, int out_cols, void* ws, size_t ws_bytes, unsigned drop_seed,
                                         float drop_p, void* keep_bits, hipStream_t stream) {
  if (!gu || !h || !Bt || !out || !ws) return OSPO_ERR_ARG;
  if (drop_p < 0.f || drop_p >= 1.f || (keep_bits && drop_p == 0.f)) return OSPO_ERR_ARG;
  if (M <= 0 || M_out < M || F <= 0 || F % 64 || b_rows <= 0 || n_tiles < 1 || n_tiles > 8) return OSPO_ERR_SHAPE;
  if (ld_gu < 2 * F || ld_gu % 8 || ld_h < F || ld_h % 8 || ldb < F || ldb % 8 || ldo % 4 || out_cols % 4 ||
      out_cols < 16 * n_tiles || ldo < out_cols)
    return OSPO_ERR_SHAPE;
  if ((long)b_rows * ldb * 2 >= (1L << 31)) return OSPO_ERR_SHAPE;
  if (drop_p > 0.f && (long)M * F > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
  if (ws_bytes < ospo_lora_skinny_ws_bytes(M_out, F, n_tiles)) return OSPO_ERR_SHAPE;
  if (!aligned16(gu) || !aligned16(h) || !aligned16(Bt) || !aligned16(ws) || ((uintptr_t)out & 7)) return OSPO_ERR_ALIGN;
  SkDropArgs dr;
  if (drop_p > 0.f) {
    dr.seed = drop_seed;
    dr.thresh = drop_threshold(drop_p);
    dr.scale = 1.f / (1.f - drop_p);
    dr.bits = (uint8_t*)keep_bits;
  }
  const bf16* a = (const bf16*)gu;
  const bf16* b = (const bf16*)Bt;
  bf16* o = (bf16*)out;
  unsigned* cnt = (unsigned*)ws;  // ws head: the row-block counters (see ospo_lora_skinny)
  float* p2 = (float*)((char*)ws + SK_CNT_BYTES);
  ws_bytes -= SK_CNT_BYTES;
  bf16* ho = (bf16*)h;
  switch (n_tiles) {
    case 1: return launch_skinny3<1, true>(a, ld_gu, b, ldb, b_rows, M, M_out, F, 0, 1, 1, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, ho, ld_h, cnt);
    case 2: return launch_skinny3<2, true>(a, ld_gu, b, ldb, b_rows, M, M_out, F, 0, 1, 2, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, ho, ld_h, cnt);
    case 3: return launch_skinny3<3, true>(a, ld_gu, b, ldb, b_rows, M, M_out, F, 0, 1, 3, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, ho, ld_h, cnt);
    case 4: return launch_skinny3<4, true>(a, ld_gu, b, ldb, b_rows, M, M_out, F, 0, 1, 4, scale, o, ldo, out_cols, p2, ws_bytes, stream, dr, ho, ld_h, cnt);
    default: return OSPO_ERR_UNSUPPORTED;
  }
}
