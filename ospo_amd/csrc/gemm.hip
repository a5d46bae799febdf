// MFMA bf16 GEMM family for gfx950 (CDNA4): the Linear layers of the Janus-Pro
// decoder with the peft LoRA update fused as a K-extension, and the fp32-atomic
// skinny / transposed GEMMs that produce the LoRA activations and gradients.
//
// Design (MI355X-first, not a translation of any CUDA tiling):
//  * 64-lane waves, v_mfma_f32_16x16x32_bf16, fp32 accumulators in registers.
//  * Operand tiles stream HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA, no
//    VGPR round trip), double buffered; BK = 64.
//  * M/N-major tiles ([rows][64 k], 128-B rows) are XOR-swizzled per 16-B chunk
//    (chunk ^ row&7) on the global SOURCE address so the lane-linear DMA image
//    reads back conflict-free with ds_read_b128.
//  * K-major tiles ([64 k][cols]) are read with ds_read_b64_tr_b16 (hardware
//    transpose) so dA = g^T x and dB = dy^T u need no transpose pass; their
//    chunk swizzle makes the transposed reads conflict-free.
//  * bf16 epilogue stages the tile in LDS and writes 16-B coalesced rows,
//    fusing alpha, bias and the bf16 residual add of the decoder layer.
//  * The LoRA update x.A^T.B^T*s is one more K segment (A2 = s*u, B2 = packed
//    block-diagonal lora_B), so the adapter costs Rp/K extra MFMAs, no pass.
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <type_traits>

#include "common.h"

namespace {

constexpr int BK = 64;

// ---------------------------------------------------------------- swizzles
__device__ __forceinline__ int mmaj_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

template <int ROWB>
__device__ __forceinline__ int kmaj_swz(int row) {
  if constexpr (ROWB == 128)
    return (row & 2) | ((row & 8) >> 1);
  else
    return ((row & 3) << 1) | (row & 8);
}

__device__ __forceinline__ void glds16(const void* gsrc, char* lds_dst_uniform) {
  __builtin_amdgcn_global_load_lds(gsrc, (LDS_AS void*)lds_dst_uniform, 16, 0, 0);
}

// Stage one BK-deep tile of an operand (TM rows of the m/n dim) into LDS.
// Work split: 1-KiB pieces, wave w takes pieces w, w+NW, ...
template <int TM, bool KMAJ, int NW>
__device__ __forceinline__ void stage_tile(const bf16* __restrict__ base, int ld, int row0, int rows_total,
                                           int k0, char* lds, int wave, int lane) {
  constexpr int PIECES = TM * BK * 2 / 1024;
  if constexpr (!KMAJ) {
#pragma unroll
    for (int p = wave; p < PIECES; p += NW) {
      const int row = p * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (row & 7);
      int grow = row0 + row;
      grow = grow < rows_total ? grow : rows_total - 1;
      glds16(base + (long)grow * ld + k0 + c * 8, lds + p * 1024);
    }
  } else {
    constexpr int LPR = TM / 8;     // lanes (16-B chunks) per k-row
    constexpr int RPP = 64 / LPR;   // k-rows per piece
    constexpr int ROWB = TM * 2;
#pragma unroll
    for (int p = wave; p < PIECES; p += NW) {
      const int row = p * RPP + lane / LPR;
      const int x = (lane % LPR) ^ kmaj_swz<ROWB>(row);
      glds16(base + (long)(k0 + row) * ld + row0 + x * 8, lds + p * 1024);
    }
  }
}

// Read the MFMA fragment (16 rows of the m/n dim x 32 k) for k-substep s.
template <int TM, bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int r0, int s, int lane) {
  if constexpr (!KMAJ) {
    const int r = r0 + (lane & 15);
    const int c = 4 * s + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + mmaj_off(r, c));
  } else {
    constexpr int ROWB = TM * 2;
    const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
    const int row = 32 * s + 8 * g + q;
    const int x = (r0 >> 3) + (p >> 1);
    const int o1 = row * ROWB + ((x ^ kmaj_swz<ROWB>(row)) << 4) + ((p & 1) << 3);
    const int o2 = (row + 4) * ROWB + ((x ^ kmaj_swz<ROWB>(row + 4)) << 4) + ((p & 1) << 3);
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + o1));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + o2));
    i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// v_mfma_scale_f32_16x16x128_f8f6f4 on e4m3 operands (cbsz = blgp = 0); OPSEL picks the scale
// byte of each lane's 32-bit scale register and must be an immediate, hence the switch (it folds
// away under the unrolled callers).
template <int OA, int OB>
__device__ __forceinline__ f32x4 mx_mfma_t(const i32x8& a, const i32x8& b, const f32x4& c, uint32_t sa, uint32_t sb) {
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, OA, (int)sa, OB, (int)sb);
}
__device__ __forceinline__ f32x4 mx_mfma(const i32x8& a, const i32x8& b, const f32x4& c, int oa, uint32_t sa, int ob,
                                         uint32_t sb) {
#define MXC(x, y) \
  case x * 4 + y: return mx_mfma_t<x, y>(a, b, c, sa, sb);
  switch (oa * 4 + ob) {
    MXC(0, 0) MXC(0, 1) MXC(0, 2) MXC(0, 3) MXC(1, 0) MXC(1, 1) MXC(1, 2) MXC(1, 3)
    MXC(2, 0) MXC(2, 1) MXC(2, 2) MXC(2, 3) MXC(3, 0) MXC(3, 1) MXC(3, 2) MXC(3, 3)
    default: return c;
  }
#undef MXC
}

enum { EPI_BF16 = 0, EPI_F32_ATOMIC = 1 };

struct GemmArgs {
  const bf16* A; const bf16* B; const bf16* A2; const bf16* B2;
  int lda, ldb, lda2, ldb2;
  int M, N, K, K2;
  float alpha;
  const bf16* bias;
  const bf16* res; int ldr;
  void* C; int ldc;
  int k_splits;
  int diag_nblk, diag_r;
  // fused RoPE (HF rotate-half, head_dim 128) on output columns < rope_cols, position = row % rope_T
  const bf16* rope_cs = nullptr;
  const bf16* rope_sn = nullptr;
  int rope_T = 0, rope_cols = 0;
  // LoRA dropout backward: C = A.B^T + mask (.) (A2.B2^T) / (1 - p), mask over [M, drop_ld]
  uint32_t drop_seed = 0, drop_thresh = 0;
  float drop_scale = 0.f;  // > 0: on
  int drop_ld = 0;
  // MXFP8 main operands (gemm_nt_v5_kernel<.., MX = true>): A / B are e4m3 bytes, lda / ldb
  // in BYTES; sa / sb the E8M0 block scales in ospo_quant_mx8's tile layout (mx8.hip).
  const uint32_t* sa = nullptr;
  const uint32_t* sb = nullptr;
  // fused SwiGLU backward (ospo_gemm_nt_swiglu_bwd_bf16): the bf16 product is dh [M, N = F]; instead of
  // storing it, the epilogue reads gate / up from swg_gu [M, 2F] and writes [dgate | dup] to swg_dgu
  const bf16* swg_gu = nullptr;
  bf16* swg_dgu = nullptr;
  int ld_gu = 0, ld_dgu = 0;
  uint32_t* dbg = nullptr;  // ablation build, DBG 4: per-wave s_memtime stamps of one K-tile
  // LoRA dropout backward with the forward's keep bits (ospo_lora_skinny keep_bits, [M][drop_ld / 8] bytes)
  // instead of re-hashing the mask: the v5 kernel stages the tile's 256 x 32-B block into LDS with tile 0
  const uint8_t* drop_bits = nullptr;
  int epi_var = 0;  // ablation build (OSPO_GEMM_EPI): plain-epilogue store variants, see epi_plain_var
};

// the SwiGLU-backward store of 8 product columns (row m, columns n..n+7 of F = args.N)
__device__ __forceinline__ void swiglu_bwd_store8(const GemmArgs& args, long m, int n, const u32x4& v) {
  float d[8], g[8], u[8], dg[8], du[8];
  unpack8(v, d);
  const bf16* gr = args.swg_gu + m * args.ld_gu + n;
  unpack8(*reinterpret_cast<const u32x4*>(gr), g);
  unpack8(*reinterpret_cast<const u32x4*>(gr + args.N), u);
  swiglu_bwd8(d, g, u, dg, du);
  bf16* o = args.swg_dgu + m * args.ld_dgu + n;
  *reinterpret_cast<u32x4*>(o) = pack8(dg);
  *reinterpret_cast<u32x4*>(o + args.N) = pack8(du);
}

// DBG (A/B decomposition only, results invalid): 1 = no global loads after the
// prologue, 2 = no MFMA, 3 = global loads only (no LDS reads, no MFMA).
template <int WM, int WN, int FM, int FN, bool AK, bool BKM, int EPI, int DBG = 0>
__global__ __launch_bounds__(WM* WN * 64) void gemm_kernel(const GemmArgs args) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16;
  constexpr int BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int CBYTES = (EPI == EPI_BF16) ? BM * CPITCH : 0;
  constexpr int LDS_BYTES = (2 * STAGE > CBYTES) ? 2 * STAGE : CBYTES;
  constexpr bool SWAP = (EPI == EPI_BF16);
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // tile coordinates (blockIdx.x over N tiles, y over M tiles)
  const int n0 = blockIdx.x * BN;
  const int m0 = blockIdx.y * BM;

  const int nt1 = args.K / BK;
  const int nt2 = args.K2 / BK;
  const int nt = nt1 + nt2;
  int t_begin = 0, t_end = nt;
  if (args.k_splits > 1) {
    t_begin = (int)((long)nt * blockIdx.z / args.k_splits);
    t_end = (int)((long)nt * (blockIdx.z + 1) / args.k_splits);
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int t, int buf) {
    char* la = smem + buf * STAGE;
    char* lb = la + A_BYTES;
    if (t < nt1) {
      stage_tile<BM, AK, NW>(args.A, args.lda, m0, args.M, t * BK, la, wave, lane);
      stage_tile<BN, BKM, NW>(args.B, args.ldb, n0, args.N, t * BK, lb, wave, lane);
    } else {
      const int k0 = (t - nt1) * BK;
      stage_tile<BM, false, NW>(args.A2, args.lda2, m0, args.M, k0, la, wave, lane);
      stage_tile<BN, false, NW>(args.B2, args.ldb2, n0, args.N, k0, lb, wave, lane);
    }
  };

  // LoRA dropout recomputed on a K-major B operand (the dA product's activations): the landed tile
  // is masked in LDS, element (m = reduction row, n) kept iff drop_keep(m * drop_ld + n) and
  // scaled by 1/(1-p) with the bf16 rounding of the forward's masked copy -- the same bf16 values the
  // forward's skinny product multiplied, without storing them.
  auto mask_b = [&](int t, int buf) {
    if constexpr (EPI == EPI_F32_ATOMIC && BKM) {
      if (args.drop_scale > 0.f && t < nt1) {
        char* lb = smem + buf * STAGE + A_BYTES;
        constexpr int LPR = BN / 8, RPP = 64 / LPR, ROWB = BN * 2;
        for (int c = threadIdx.x; c < B_BYTES / 16; c += NW * 64) {
          const int p = c >> 6, ln = c & 63;
          const int row = p * RPP + ln / LPR;
          const int x = (ln % LPR) ^ kmaj_swz<ROWB>(row);
          const uint32_t base = (uint32_t)(t * BK + row) * (uint32_t)args.drop_ld + (uint32_t)(n0 + x * 8);
          bf16x8 v = *reinterpret_cast<const bf16x8*>(lb + c * 16);
          bool keep[8];
          if (args.drop_bits) {  // the forward's keep bits: one byte = these 8 columns (base % 8 == 0)
            const uint32_t kb = args.drop_bits[base >> 3];
#pragma unroll
            for (int e = 0; e < 8; ++e) keep[e] = (kb >> e) & 1u;
          } else {
            drop_keep_pairs<4>(base, args.drop_seed, args.drop_thresh, keep);  // base even (drop_ld even)
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = keep[e] ? f2bf(bf2f(v[e]) * args.drop_scale) : f2bf(0.f);
          *reinterpret_cast<bf16x8*>(lb + c * 16) = v;
        }
        __syncthreads();
      }
    }
  };

  if (t_begin < t_end) {
    stage(t_begin, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    mask_b(t_begin, 0);
    for (int t = t_begin; t < t_end; ++t) {
      const int buf = (t - t_begin) & 1;
      if (DBG != 1 && t + 1 < t_end) stage(t + 1, buf ^ 1);
      const char* la = smem + buf * STAGE;
      const char* lb = la + A_BYTES;
      const bool ext = t >= nt1;  // the K-extension tiles are always M/N-major
#pragma unroll
      for (int s = 0; s < 2 && DBG != 3; ++s) {
        bf16x8 af[FM], bfr[FN];
        if (AK && !ext) {
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, AK>(la, wm * FM * 16 + i * 16, s, lane);
        } else {
#pragma unroll
          for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, false>(la, wm * FM * 16 + i * 16, s, lane);
        }
        if (BKM && !ext) {
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, BKM>(lb, wn * FN * 16 + j * 16, s, lane);
        } else {
#pragma unroll
          for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, false>(lb, wn * FN * 16 + j * 16, s, lane);
        }
        if (DBG == 2) {  // keep the reads alive without MFMA
#pragma unroll
          for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
          for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bfr[j]));
          continue;
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (SWAP)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (t + 1 < t_end) mask_b(t + 1, buf ^ 1);
    }
  }

  const int g = lane >> 4, l16 = lane & 15;
  if constexpr (EPI == EPI_BF16) {
    // registers -> LDS tile [BM][BN] (bf16, rounded after alpha/bias)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int nl = wn * FN * 16 + j * 16 + 4 * g;
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
      if (args.bias) {
#pragma unroll
        for (int q = 0; q < 4; ++q) b4[q] = bf2f(args.bias[n0 + nl + q]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int ml = wm * FM * 16 + i * 16 + l16;
        const f32x4 v = acc[i][j];
        uint2 pk;
        pk.x = pack2(v[0] * args.alpha + b4[0], v[1] * args.alpha + b4[1]);
        pk.y = pack2(v[2] * args.alpha + b4[2], v[3] * args.alpha + b4[3]);
        *reinterpret_cast<uint2*>(smem + ml * CPITCH + nl * 2) = pk;
      }
    }
    __syncthreads();
    constexpr int CPR = BN / 8;  // 16-B chunks per row
    bf16* C = reinterpret_cast<bf16*>(args.C);
    for (int c = threadIdx.x; c < BM * CPR; c += NW * 64) {
      const int r = c / CPR, cc = c % CPR;
      const int m = m0 + r;
      if (m >= args.M) continue;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + r * CPITCH + cc * 16);
      if (args.res) {
        const u32x4 rv = *reinterpret_cast<const u32x4*>(args.res + (long)m * args.ldr + n0 + cc * 8);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = bits2f(v[q] & 0xffff) + bits2f(rv[q] & 0xffff);
          const float hi = bits2f(v[q] >> 16) + bits2f(rv[q] >> 16);
          v[q] = pack2(lo, hi);
        }
      }
      *reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + cc * 8) = v;
    }
  } else {
    float* C = reinterpret_cast<float*>(args.C);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * FN * 16 + j * 16 + l16;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = m0 + wm * FM * 16 + i * 16 + 4 * g + q;
          if (m >= args.M) continue;
          const float v = acc[i][j][q] * args.alpha;
          if (args.diag_nblk > 0) {
            if (n / args.diag_r != m / args.diag_nblk) continue;
            atomicAdd(C + (long)m * args.diag_r + (n % args.diag_r), v);
          } else {
            atomicAdd(C + (long)m * args.ldc + n, v);
          }
        }
      }
  }
}

template <int WM, int WN, int FM, int FN, bool AK, bool BKM, int EPI, int DBG = 0>
int launch(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  if (a.N % BN) return OSPO_ERR_SHAPE;
  // K-major A: the tile loads columns up to roundup(M, BM) (must exist), stores are predicated on M
  if (AK && a.lda < ((a.M + BM - 1) / BM) * BM) return OSPO_ERR_SHAPE;
  dim3 grid(a.N / BN, (a.M + BM - 1) / BM, a.k_splits > 1 ? a.k_splits : 1);
  hipLaunchKernelGGL((gemm_kernel<WM, WN, FM, FN, AK, BKM, EPI, DBG>), grid, dim3(WM * WN * 64), 0, s, a);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

// ----------------------------------------------------------------------------
// Pipelined NT GEMM helpers (8 waves 2 x 4, tile BM x 256, BK = 64).
//  * LDS-DMA loads of later tiles stay in flight across a raw s_barrier (counted
//    vmcnt; __syncthreads() would drain them -- guide "Pipelining across barriers");
//  * XCD-aware tile order: block b runs on XCD b % 8 (round-robin dispatch), so each
//    XCD gets a contiguous range of tile ids, grouped GM tile-rows deep so its
//    co-resident tiles share operand panels in its L2 (T1); speed only, never results;
//  * s_setprio(1) around each MFMA cluster (T5).
// Wait until at most n of this wave's vector-memory ops are outstanding.  n is wave-uniform;
// rounding it DOWN to a supported constant only waits longer, so it is always safe.
__device__ __forceinline__ void wait_vmcnt(int n) {
  if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ----------------------------------------------------------------------------
// v3: the barrier sits BETWEEN the two k-substep MFMA clusters of a K-tile, and the
// MFMA fragments are double-buffered in registers, so the cluster after each barrier
// runs on fragments read before it while the next tile's first fragments load:
//   read(t,1)->SB | MFMA(SA) | vmcnt(0) lgkmcnt(0) s_barrier | stage(t+2) | read(t+1,0)->SA | MFMA(SB)
// Two LDS buffers; tile t+2 streams into tile t's buffer right after the barrier that
// certifies every wave finished reading it.  Loads get one K-tile of slack.

// LoRA weight gradients as one stream over the big operand (round 2; replaces the 64 x 64 f32-atomic
// tiles of gemm_kernel for dA / dB):
//   mode 0 (dA):  C[j][n]      += sum_m S[m][j] X[m][n]             j < s_cols (the used rank rows)
//   mode 1 (dB):  C[n][jr]     += sum_m X[m][n] S[m][mod * r + jr]  mod = n / nmod, jr < r (block diagonal)
// X [Mk][N] is the big activation (x_in for dA, dy for dB), S [Mk][>= s_cols] the small LoRA operand
// (g for dA, u for dB).  A workgroup owns a TN-column stripe of X and a range of 64-row K-tiles; the
// stripe and the S rows of a K-tile stream through an NS-deep LDS ring by LDS-DMA (one barrier per
// K-tile, NS - 1 tiles in flight), both MFMA operands are transposed reads (the contraction runs over
// rows), each X fragment feeds every rank tile.  Split partials meet in fp32 atomics.  With dropout
// (dA of a dropped-out adapter input) the X fragments are masked in registers with the forward's hash
// and bf16 rounding.
template <int TN, int TS, int NS, int MODE, bool DROP>
__global__ __launch_bounds__(256) void lora_wgrad_kernel(const bf16* __restrict__ X, int ldx, int N,
                                                         const bf16* __restrict__ S, int lds, int s_cols, int K,
                                                         int nmod, int r, float* __restrict__ C, int ldc,
                                                         uint32_t dseed, uint32_t dthresh, float dscale, int drop_ld) {
  constexpr int XB = TN * BK * 2, SB = TS * BK * 2, STG = XB + SB;
  constexpr int NF = TN / 64;                       // 16-column X fragments per wave
  constexpr int RT = MODE == 0 ? TS / 16 : 2;       // rank tiles of the product (dB: r <= 32)
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = blockIdx.x * TN;
  const int nt = K / BK;
  const int t0 = (int)((long)nt * blockIdx.y / gridDim.y), t1 = (int)((long)nt * (blockIdx.y + 1) / gridDim.y);
  // S columns this stripe needs: all s_cols (dA), or the module's r columns (dB); the S tile holds the
  // whole padded row (TS = its leading dimension), the fragments start at rbase
  const int rbase = MODE == 0 ? 0 : (n0 / nmod) * r;
  const int rt_used = MODE == 0 ? (s_cols + 15) / 16 : r / 16;
  f32x4 acc[RT][NF];
#pragma unroll
  for (int j = 0; j < RT; ++j)
#pragma unroll
    for (int f = 0; f < NF; ++f) acc[j][f] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto stage = [&](int t, int slot) {
    char* xs = smem + slot * STG;
    stage_tile<TN, true, 4>(X, ldx, n0, N, t * BK, xs, wave, lane);
    stage_tile<TS, true, 4>(S, lds, 0, TS, t * BK, xs + XB, wave, lane);
  };
  constexpr int PIECES = STG / 1024 / 4;  // LDS-DMA pieces per wave per stage
  const int n_my = t1 - t0;
  // prologue: NS - 1 stages in flight
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < n_my) stage(t0 + i, i);
  const int g = lane >> 4, l16 = lane & 15;
  for (int i = 0; i < n_my; ++i) {
    // this wave's pieces of stage i have landed (NS - 2 newer stages may still be in flight)
    const int newer = min(NS - 2, n_my - 1 - i);
    if (newer >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PIECES) : "memory");
    else if (newer == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PIECES) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every wave's pieces of stage i visible; every wave done with stage i - 1
    if (i + NS - 1 < n_my) stage(t0 + i + NS - 1, (i + NS - 1) % NS);
    const char* xs = smem + (i % NS) * STG;
    const char* ss = xs + XB;
#pragma unroll
    for (int sk = 0; sk < 2; ++sk) {
      bf16x8 bx[NF], as[RT];
#pragma unroll
      for (int f = 0; f < NF; ++f) bx[f] = read_frag<TN, true>(xs, wave * (TN / 4) + 16 * f, sk, lane);
#pragma unroll
      for (int j = 0; j < RT; ++j) as[j] = read_frag<TS, true>(ss, rbase + 16 * (j < rt_used ? j : 0), sk, lane);
      if constexpr (DROP) {  // element e: row m = 64 t + 32 sk + 8 g + e, column n
        const uint32_t mrow = (uint32_t)((t0 + i) * BK + 32 * sk + 8 * g);
#pragma unroll
        for (int f = 0; f < NF; ++f) {
          const uint32_t n = (uint32_t)(n0 + wave * (TN / 4) + 16 * f + l16);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const bool keep = drop_keep((mrow + e) * (uint32_t)drop_ld + n, dseed, dthresh);
            bx[f][e] = keep ? f2bf(bf2f(bx[f][e]) * dscale) : f2bf(0.f);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < RT; ++j)
        if (j < rt_used)
#pragma unroll
          for (int f = 0; f < NF; ++f)
            acc[j][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as[j], bx[f], acc[j][f], 0, 0, 0);
    }
  }
  // lane holds D[rank row 16 j + 4 g + q][column n0 + wave TN/4 + 16 f + l16]
#pragma unroll
  for (int j = 0; j < RT; ++j) {
    if (j >= rt_used) continue;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int n = n0 + wave * (TN / 4) + 16 * f + l16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jr = 16 * j + 4 * g + q;
        if (MODE == 0) {
          if (jr < s_cols) atomicAdd(C + (long)jr * ldc + n, acc[j][f][q]);
        } else {
          atomicAdd(C + (long)n * r + jr, acc[j][f][q]);
        }
      }
    }
  }
}

template <int TN, int TS, int MODE, bool DROP>
int launch_wgrad(const bf16* X, int ldx, int N, const bf16* S, int lds, int s_cols, int K, int nmod, int r, float* C,
                 int ldc, int splits, uint32_t seed, uint32_t thresh, float scale, int drop_ld, hipStream_t st) {
  constexpr int NS = 3;
  hipLaunchKernelGGL((lora_wgrad_kernel<TN, TS, NS, MODE, DROP>), dim3(N / TN, splits), dim3(256), 0, st, X, ldx, N, S,
                     lds, s_cols, K, nmod, r, C, ldc, seed, thresh, scale, drop_ld);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

}  // namespace

extern "C" int ospo_lora_wgrad(const void* X, int ldx, int N, const void* S, int lds, int s_cols, int K, int mode,
                               int nmod, int r, float* C, int ldc, int splits, uint32_t drop_seed, float drop_p,
                               hipStream_t stream) {
  if (!X || !S || !C) return OSPO_ERR_ARG;
  if (N <= 0 || K <= 0 || K % BK || s_cols <= 0 || splits < 1 || splits > K / BK) return OSPO_ERR_SHAPE;
  if (ldx < N || ldx % 8 || lds % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(X) || !aligned16(S)) return OSPO_ERR_ALIGN;
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  const bool drop = drop_p > 0.f;
  const uint32_t thresh = drop_threshold(drop_p);
  const float dscale = drop ? 1.f / (1.f - drop_p) : 0.f;
  const bf16* x = (const bf16*)X;
  const bf16* sp = (const bf16*)S;
  // S rows are staged whole: lds = the padded rank width (64 or 128 columns)
  if (lds != 64 && lds != 128) return OSPO_ERR_SHAPE;
  if (mode == 0) {  // dA: C[s_cols][N], ldc >= N
    if (ldc < N || N % 256 || s_cols > lds) return OSPO_ERR_SHAPE;
    if (lds == 64)
      return drop ? launch_wgrad<256, 64, 0, true>(x, ldx, N, sp, lds, s_cols, K, 0, 0, C, ldc, splits, drop_seed, thresh,
                                                   dscale, N, stream)
                  : launch_wgrad<256, 64, 0, false>(x, ldx, N, sp, lds, s_cols, K, 0, 0, C, ldc, splits, 0, 0, 0.f, N,
                                                    stream);
    return drop ? launch_wgrad<256, 128, 0, true>(x, ldx, N, sp, lds, s_cols, K, 0, 0, C, ldc, splits, drop_seed, thresh,
                                                  dscale, N, stream)
                : launch_wgrad<256, 128, 0, false>(x, ldx, N, sp, lds, s_cols, K, 0, 0, C, ldc, splits, 0, 0, 0.f, N,
                                                   stream);
  }
  if (mode == 1) {  // dB: C[N][r] block-diagonal, module = n / nmod; S columns mod * r .. + r
    if (drop || r <= 0 || r % 16 || r > 32 || nmod % 256 || N % nmod) return OSPO_ERR_UNSUPPORTED;
    if ((N / nmod) * r > lds) return OSPO_ERR_SHAPE;
    return lds == 64 ? launch_wgrad<256, 64, 1, false>(x, ldx, N, sp, lds, s_cols, K, nmod, r, C, 0, splits, 0, 0, 0.f, 0,
                                                       stream)
                     : launch_wgrad<256, 128, 1, false>(x, ldx, N, sp, lds, s_cols, K, nmod, r, C, 0, splits, 0, 0, 0.f,
                                                        0, stream);
  }
  return OSPO_ERR_ARG;
}

namespace {

template <int FM, int STAGES, bool REMAP, bool PRIO, int WM = 2, int WN = 4, int FN = 4, int DBG = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_nt_v3_kernel(const GemmArgs args, int tiles_m, int tiles_n) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = A_BYTES / 1024, PT = PA + B_BYTES / 1024;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int LDS_BYTES = (STAGES * STAGE > BM * CPITCH) ? STAGES * STAGE : BM * CPITCH;
  static_assert(LDS_BYTES <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ppw = (PT - wave + NW - 1) / NW;  // LDS-DMA pieces this wave issues per tile

  int m0, n0;
  if (REMAP) {
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, slot = wg >> 3, q = nwg >> 3, r = nwg & 7;
    const int tid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    constexpr int GM = 4;
    const int gsize = GM * tiles_n;
    const int first_m = (tid / gsize) * GM;
    const int gm = min(tiles_m - first_m, GM);
    const int within = tid % gsize;
    m0 = (first_m + within % gm) * BM;
    n0 = (within / gm) * BN;
  } else {
    m0 = (blockIdx.x / tiles_n) * BM;
    n0 = (blockIdx.x % tiles_n) * BN;
  }
  const int nt1 = args.K / BK, nt = nt1 + args.K2 / BK;

  const bf16* const pA = args.A;
  const bf16* const pB = args.B;
  const bf16* const pA2 = args.A2;
  const bf16* const pB2 = args.B2;
  const int lda1 = args.lda, ldb1 = args.ldb, lda2 = args.lda2, ldb2 = args.ldb2;
  const int Mlast = args.M - 1, Nlast = args.N - 1;
  const int rr8 = lane >> 3, c8 = lane & 7;
  auto stage = [&](int t, int buf) {
    char* la = smem + buf * STAGE;
    char* lb = la + A_BYTES;
    const bool ext = t >= nt1;
    const bf16* Ab = ext ? pA2 : pA;
    const bf16* Bb = ext ? pB2 : pB;
    const int lda = ext ? lda2 : lda1;
    const int ldb = ext ? ldb2 : ldb1;
    const int k0 = (ext ? t - nt1 : t) * BK;
#pragma unroll
    for (int p = wave; p < PT; p += NW) {
      if (p < PA) {
        const int row = p * 8 + rr8;
        const int g = min(m0 + row, Mlast);
        glds16(Ab + (long)g * lda + k0 + ((c8 ^ (row & 7)) << 3), la + p * 1024);
      } else {
        const int row = (p - PA) * 8 + rr8;
        const int g = min(n0 + row, Nlast);
        glds16(Bb + (long)g * ldb + k0 + ((c8 ^ (row & 7)) << 3), lb + (p - PA) * 1024);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 aA[FM], bA[FN], aB[FM], bB[FN];
  auto rd = [&](const char* buf, int s, bf16x8 (&af)[FM], bf16x8 (&bfr)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = read_frag<BM, false>(buf, wm * FM * 16 + i * 16, s, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = read_frag<BN, false>(buf + A_BYTES, wn * FN * 16 + j * 16, s, lane);
  };
  auto mm = [&](const bf16x8 (&af)[FM], const bf16x8 (&bfr)[FN]) {
    if (DBG == 2) {
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(bfr[j]));
      return;
    }
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: tiles 0 .. STAGES-1 in flight, wait for tile 0
  for (int s0 = 0; s0 < STAGES && s0 < nt; ++s0) stage(s0, s0);
  wait_vmcnt(ppw * (min(STAGES, nt) - 1));
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  rd(smem, 0, aA, bA);
  for (int t = 0; t < nt; ++t) {
    const char* cur = smem + (t % STAGES) * STAGE;
    rd(cur, 1, aB, bB);
    mm(aA, bA);
    __builtin_amdgcn_sched_barrier(0);
    // tile t+1 must have landed; tiles t+2 .. min(t+STAGES, nt)-1 may stay in flight
    wait_vmcnt(ppw * max(0, min(t + STAGES, nt) - t - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // tile t's buffer is free (its fragments are in registers): refill it with tile t+STAGES
    if (DBG != 1 && t + STAGES < nt) stage(t + STAGES, t % STAGES);
    // unconditional (the last iteration re-reads a valid, unused buffer): a branch here
    // makes the loop header merge 0 and 12 pending LDS reads and the waitcnt pass then
    // drains lgkmcnt(0) before the next cluster, serialising the fragment prefetch
    rd(smem + ((t + 1) % STAGES) * STAGE, 0, aA, bA);
    mm(aB, bB);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * FN * 16 + j * 16 + 4 * g;
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (args.bias) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) b4[qq] = bf2f(args.bias[n0 + nl + qq]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = wm * FM * 16 + i * 16 + l16;
      const f32x4 v = acc[i][j];
      uint2 pk;
      pk.x = pack2(v[0] * args.alpha + b4[0], v[1] * args.alpha + b4[1]);
      pk.y = pack2(v[2] * args.alpha + b4[2], v[3] * args.alpha + b4[3]);
      *reinterpret_cast<uint2*>(smem + ml * CPITCH + nl * 2) = pk;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  bf16* C = reinterpret_cast<bf16*>(args.C);
  for (int c = threadIdx.x; c < BM * CPR; c += NW * 64) {
    const int rr = c / CPR, cc = c % CPR;
    const int m = m0 + rr;
    if (m >= args.M) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(smem + rr * CPITCH + cc * 16);
    if (args.res) {
      const u32x4 rv = *reinterpret_cast<const u32x4*>(args.res + (long)m * args.ldr + n0 + cc * 8);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const float lo = bits2f(v[qq] & 0xffff) + bits2f(rv[qq] & 0xffff);
        const float hi = bits2f(v[qq] >> 16) + bits2f(rv[qq] >> 16);
        v[qq] = pack2(lo, hi);
      }
    }
    *reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + cc * 8) = v;
  }
}

// ----------------------------------------------------------------------------
// v4: BK = 32 stages in a deep ring.  The per-CU L2 -> LDS rate grows with the bytes
// in flight (MI355X_MICROARCH.md "gather into LDS": ~70 GB/s/CU L2-resident, ~33 from
// the Infinity Cache at 72 KiB in flight) and a 256 x 256 tile at full MFMA rate needs
// ~77 GB/s/CU.  64-deep stages cap the ring at 2 x 64 KiB (one tile in flight); 32-deep
// stages of 32 KiB give a 4-6 deep ring with 3-5 tiles in flight.
// LDS image [rows][32 k] = 64-B rows; 16-B chunk c of row r lives at c ^ h(r),
// h(r) = (-(r >> 2)) & 3, conflict-free for all four ds_read_b128 lane groups.
constexpr int BK4 = 32;
__device__ __forceinline__ int off32(int r, int c) { return r * 64 + ((c ^ ((-(r >> 2)) & 3)) << 4); }

__device__ __forceinline__ void wait_vmcnt_exact(int n) {
  switch (n) {
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
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;  // n >= 15: waiting for more is safe
  }
}

template <int FM, int STAGES>
__global__ __launch_bounds__(512) void gemm_nt_v4_kernel(const GemmArgs args, int tiles_m, int tiles_n) {
  constexpr int WN = 4, FN = 4, NW = 8;
  constexpr int BM = 2 * FM * 16, BN = WN * FN * 16;
  constexpr int A_BYTES = BM * BK4 * 2, B_BYTES = BN * BK4 * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int PA = A_BYTES / 1024, PT = PA + B_BYTES / 1024;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int LDS_BYTES = (STAGES * STAGE > BM * CPITCH) ? STAGES * STAGE : BM * CPITCH;
  static_assert(LDS_BYTES <= 163840, "LDS");
  static_assert(A_BYTES % 1024 == 0 && B_BYTES % 1024 == 0, "pieces");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int ppw = (PT - wave + NW - 1) / NW;

  int m0, n0;
  {
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int xcd = wg & 7, slot = wg >> 3, q = nwg >> 3, r = nwg & 7;
    const int tid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
    constexpr int GM = 4;
    const int gsize = GM * tiles_n;
    const int first_m = (tid / gsize) * GM;
    const int gm = min(tiles_m - first_m, GM);
    const int within = tid % gsize;
    m0 = (first_m + within % gm) * BM;
    n0 = (within / gm) * BN;
  }
  const int nt1 = args.K / BK4, nt = nt1 + args.K2 / BK4;
  const int Mlast = args.M - 1, Nlast = args.N - 1;
  const int rr = lane >> 2, c4 = lane & 3;
  auto stage = [&](int t, int buf) {
    char* la = smem + buf * STAGE;
    const bool ext = t >= nt1;
    const bf16* Ab = ext ? args.A2 : args.A;
    const bf16* Bb = ext ? args.B2 : args.B;
    const int lda = ext ? args.lda2 : args.lda;
    const int ldb = ext ? args.ldb2 : args.ldb;
    const int k0 = (ext ? t - nt1 : t) * BK4;
#pragma unroll
    for (int p = wave; p < PT; p += NW) {
      if (p < PA) {
        const int row = p * 16 + rr;
        const int g = min(m0 + row, Mlast);
        glds16(Ab + (long)g * lda + k0 + ((c4 ^ ((-(row >> 2)) & 3)) << 3), la + p * 1024);
      } else {
        const int row = (p - PA) * 16 + rr;
        const int g = min(n0 + row, Nlast);
        glds16(Bb + (long)g * ldb + k0 + ((c4 ^ ((-(row >> 2)) & 3)) << 3), la + p * 1024);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < nt) stage(s0, s0);
  const int fr = lane & 15, fc = lane >> 4;
  for (int t = 0; t < nt; ++t) {
    // tile t landed (own pieces), tiles t+1 .. t+STAGES-2 may stay in flight
    wait_vmcnt_exact(ppw * max(0, min(STAGES - 2, nt - 1 - t)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of buffer (t-1) % STAGES retired
    __builtin_amdgcn_s_barrier();  // every wave's pieces of tile t landed; buffer (t-1) % STAGES is free
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nt) stage(t + STAGES - 1, (t + STAGES - 1) % STAGES);
    const char* la = smem + (t % STAGES) * STAGE;
    const char* lb = la + A_BYTES;
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const bf16x8*>(la + off32(wm * FM * 16 + i * 16 + fr, fc));
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(lb + off32(wn * FN * 16 + j * 16 + fr, fc));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int nl = wn * FN * 16 + j * 16 + 4 * g;
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (args.bias) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) b4[qq] = bf2f(args.bias[n0 + nl + qq]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int ml = wm * FM * 16 + i * 16 + l16;
      const f32x4 v = acc[i][j];
      uint2 pk;
      pk.x = pack2(v[0] * args.alpha + b4[0], v[1] * args.alpha + b4[1]);
      pk.y = pack2(v[2] * args.alpha + b4[2], v[3] * args.alpha + b4[3]);
      *reinterpret_cast<uint2*>(smem + ml * CPITCH + nl * 2) = pk;
    }
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  bf16* C = reinterpret_cast<bf16*>(args.C);
  for (int c = threadIdx.x; c < BM * CPR; c += NW * 64) {
    const int r2 = c / CPR, cc = c % CPR;
    const int m = m0 + r2;
    if (m >= args.M) continue;
    u32x4 v = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + cc * 16);
    if (args.res) {
      const u32x4 rv = *reinterpret_cast<const u32x4*>(args.res + (long)m * args.ldr + n0 + cc * 8);
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const float lo = bits2f(v[qq] & 0xffff) + bits2f(rv[qq] & 0xffff);
        const float hi = bits2f(v[qq] >> 16) + bits2f(rv[qq] >> 16);
        v[qq] = pack2(lo, hi);
      }
    }
    *reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + cc * 8) = v;
  }
}

template <int FM, int STAGES>
int launch_v4(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = 2 * FM * 16, BN = 256;
  if (a.N % BN || a.K % BK4 || a.K2 % BK4) return OSPO_ERR_SHAPE;
  const int tm = (a.M + BM - 1) / BM, tn = a.N / BN;
  hipLaunchKernelGGL((gemm_nt_v4_kernel<FM, STAGES>), dim3(tm * tn), dim3(512), 0, s, a, tm, tn);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

// ----------------------------------------------------------------------------
// v5: 256 x 256 x 64 "8-phase" ping-pong (cdna_hip_programming.md, The 256^2 8-phase
// template: T1 XCD remap, T2 swizzle, T3+T4 phases with counted vmcnt, T5 setprio).
//  * Each K-tile = 4 phases; phase j computes one 128 x 128 C-quadrant (A-half ia,
//    B-half ib) in the order (0,0) (0,1) (1,1) (1,0); wave w owns rows 64*(w>>2)
//    and cols 32*(w&3) of every quadrant (16 MFMAs per phase) and reads only the
//    fragments that change (12 / 4 / 8 / 4 ds_read_b128).
//  * Waves 4-7 run one s_barrier behind waves 0-3: on every SIMD one wave's MFMA
//    cluster overlaps the other wave's LDS reads + LDS-DMA issue.
//  * LDS: 2 slots x {A0, A1, B0, B1} half-tiles of 128 rows x 64 k (16 KiB, 128-B
//    rows, chunk ^ row&7).  Phase j of tile T stages one half-tile (2 glds / wave):
//    j=0 B1(T+1), j=1 B0(T+1), j=2 A1(T+1), j=3 A0(T+2) -- each after the last read
//    of the slot it overwrites has been retired (lgkmcnt(0) + a barrier).
//  * Counted vmcnt, never 0 in the loop: before the first read of a half-tile each
//    wave waits for its own DMA of it (vmcnt(2+2) before q0, vmcnt(6) before q2),
//    placed just before the barrier that precedes the first reader.
// Tile order: XCD-contiguous chunks of the data-parallel workgroups, GM = 4 row-tile groups.
#ifdef OSPO_ABLATION
int g_v5_gm = 4;  // row tiles per L2 group (A/B knob, variants 20-23)
#else
constexpr int g_v5_gm = 4;  // row tiles per L2 group
#endif

__device__ __forceinline__ void v5_tile(int L, int tiles_m, int tiles_n, int& m0, int& n0, int GM = 4) {
  const int gsize = GM * tiles_n;
  const int first_m = (L / gsize) * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int within = L % gsize;
  m0 = (first_m + within % gm) * 256;
  n0 = (within / gm) * 256;
}

// Data-parallel + split-K tail: workgroups [0, dp) own whole tiles (XCD-remapped);
// workgroups dp + u (u < tail * split) own K-range u % split of tail tile dp + u / split
// and write an fp32 partial tile to ws (summed + epilogued by splitk_fixup_kernel).
//
// MX = true: the main K-tiles are MXFP8 (e4m3 bytes, 128 k per tile = the same 128-B LDS rows
// as 64 bf16) and run v_mfma_scale_f32_16x16x128_f8f6f4 -- 8 MFMAs per phase at twice the bf16
// rate per clock.  Its operand layout (measured, tools/mx8_probe.hip): lane l holds row l & 15,
// bytes 0-15 = k 16g..16g+15 and bytes 16-31 = k 64+16g.., g = l >> 4 -- i.e. exactly the two
// ds_read_b128 fragments of the bf16 k-substeps s = 0, 1; the scale of lane l is that of
// (row l & 15, 32-k block l >> 4), byte chosen by OPSEL.  The E8M0 scales of K-tile t stream into
// LDS with the data: one 4-B LDS-DMA per wave (waves 0-3: A's four 64-row groups, 4-7: B's),
// issued with B1 of the tile before, so the counted waits cover them.  The LoRA K-extension
// tiles stay bf16 (16 bf16 MFMAs per phase).
// bf16 epilogue, second half: the tile's rounded products staged in LDS as [256][CPITCH] rows ->
// RoPE / residual -> 16-B coalesced global stores (shared by the 256x256 kernels)
// GEMM outputs (bf16 tiles, split-K fp32 partials) are stored plainly.  Non-temporal stores (-DOSPO_GEMM_NT_STORES=1)
// win in isolation -- no later access in the launch re-reads the tile, and 'nt' leaves the L2 to the streamed
// operands (profiles/r05/gemm_epi_ab.log, variant 2: gu_fwd 613 -> 595 us, gh2_fwd 423 -> 413, down_dx 326 -> 320)
// -- but lose 0.65% on the step (profiles/r05/step_ab_r5i.txt: 35.13 vs 35.36 pairs/s, both rounds): the next
// kernel (SwiGLU, the fixup, the norm) re-reads the output, and plain stores leave it in the MALL for it.
#ifndef OSPO_GEMM_NT_STORES
#define OSPO_GEMM_NT_STORES 0
#endif
template <typename T>
__device__ __forceinline__ void gemm_out_store(T* p, const T& v) {
  if constexpr (OSPO_GEMM_NT_STORES) __builtin_nontemporal_store(v, p);
  else *p = v;
}

#ifdef OSPO_ABLATION
// Ablation (round 5): the plain epilogue (no residual, no RoPE) with BATCH LDS reads in flight before their
// stores, and optionally non-temporal stores.  Same values and addresses as epi_rows: bit-identical output.
template <int NTHR, int BATCH, bool NTS>
__device__ __forceinline__ void epi_plain_var(const GemmArgs& args, const char* smem, int m0, int n0, int tid) {
  constexpr int BM = 256, BN = 256, CPITCH = BN * 2 + 16, CPR = BN / 8, ITERS = BM * CPR / NTHR;
  bf16* C = reinterpret_cast<bf16*>(args.C);
#pragma unroll 1
  for (int b0 = 0; b0 < ITERS; b0 += BATCH) {
    u32x4 v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int c = tid + (b0 + u) * NTHR;
      v[u] = *reinterpret_cast<const u32x4*>(smem + (c / CPR) * CPITCH + (c % CPR) * 16);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int c = tid + (b0 + u) * NTHR;
      const int m = m0 + c / CPR;
      u32x4* dst = reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + (c % CPR) * 8);
      if (m < args.M) {
        if constexpr (NTS) __builtin_nontemporal_store(v[u], dst);
        else *dst = v[u];
      }
    }
  }
}
#endif

template <int NTHR>
__device__ __forceinline__ void epi_rows(const GemmArgs& args, const char* smem, int m0, int n0) {
  constexpr int BM = 256, BN = 256, CPITCH = BN * 2 + 16;
  constexpr int CPR = BN / 8;
  constexpr int ITERS = BM * CPR / NTHR;  // 16-B chunks per thread
  constexpr int BATCH = 4;                // chunks whose global loads are in flight together
  static_assert(ITERS % BATCH == 0, "epilogue batch");
  bf16* C = reinterpret_cast<bf16*>(args.C);
  if (args.swg_gu) {  // fused SwiGLU backward: one chunk at a time (reads gate|up, writes dgate|dup)
    for (int c = threadIdx.x; c < BM * CPR; c += NTHR) {
      const int r2 = c / CPR, cc = c % CPR;
      const int m = m0 + r2;
      if (m >= args.M) continue;
      const u32x4 v = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + cc * 16);
      swiglu_bwd_store8(args, m, n0 + cc * 8, v);
    }
    return;
  }
  // The residual and RoPE-table loads of BATCH chunks are issued before any of their stores: a load
  // after a store to C (which the compiler cannot prove disjoint from res) would wait for it, and one
  // chunk at a time the epilogue ran latency-bound (~9 us per 256 x 256 tile with a residual).
  // the epilogue's index math starts here: keeps the compiler from hoisting it above the K loop (registers)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid), "+v"(m0), "+v"(n0));
  const bool rope_tile = n0 < args.rope_cols;  // (rope_cols % 128 == 0: a chunk's partner is in the tile)
#ifdef OSPO_ABLATION
  if (args.epi_var && !rope_tile && !args.res) {
    switch (args.epi_var) {
      case 1: epi_plain_var<NTHR, 8, false>(args, smem, m0, n0, tid); return;
      case 2: epi_plain_var<NTHR, 4, true>(args, smem, m0, n0, tid); return;
      case 3: epi_plain_var<NTHR, 8, true>(args, smem, m0, n0, tid); return;
      case 4: epi_plain_var<NTHR, 16, false>(args, smem, m0, n0, tid); return;
      default: epi_plain_var<NTHR, 4, false>(args, smem, m0, n0, tid); return;
    }
  }
#endif
  if (rope_tile && !args.res) {
    // RoPE tiles: one thread per (row, head, 8-column group j < 8) computes BOTH outputs of the rotate-half
    // pair -- columns 8j.. and 64 + 8j.. -- from one unpack of x1, x2 and of the shared cos / sin entry
    // (HF's tables repeat freqs: cos[d + 64] = cos[d]); the per-chunk form unpacked every value and table
    // entry twice (once per partner) and the epilogue was VALU bound (qkv_fwd: +36 us per launch).  Same
    // roundings, bit-identical.  Heads at or past rope_cols are copied.
    constexpr int UNITS = BM * 2 * 8, PITERS = UNITS / NTHR, PB = 4;
    static_assert(PITERS % PB == 0, "rope epilogue batch");
#pragma unroll 1
    for (int b0 = 0; b0 < PITERS; b0 += PB) {
      u32x4 cw[PB], sw[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int un = tid + (b0 + u) * NTHR;
        const int j = un & 7, r2 = un >> 4;
        const int t = min(m0 + r2, args.M - 1) % args.rope_T;
        cw[u] = *reinterpret_cast<const u32x4*>(args.rope_cs + (long)t * 64 + 8 * j);
        sw[u] = *reinterpret_cast<const u32x4*>(args.rope_sn + (long)t * 64 + 8 * j);
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const int un = tid + (b0 + u) * NTHR;
        const int j = un & 7, hd = (un >> 3) & 1, r2 = un >> 4;
        const int m = m0 + r2;
        const int cl = hd * 16 + j;  // 16-B chunk of columns 8j.. of head hd; its partner is cl + 8
        u32x4 v1 = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + cl * 16);
        u32x4 v2 = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + (cl + 8) * 16);
        if (n0 + hd * 128 < args.rope_cols) {
          u32x4 o1, o2;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            float r1[2], r2v[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const int sh = 16 * hh;
              const float x1 = bits2f((v1[qq] >> sh) & 0xffff), x2 = bits2f((v2[qq] >> sh) & 0xffff);
              const float cf = bits2f((cw[u][qq] >> sh) & 0xffff), sf = bits2f((sw[u][qq] >> sh) & 0xffff);
              r1[hh] = round_bf(x1 * cf) + round_bf(-x2 * sf);
              r2v[hh] = round_bf(x2 * cf) + round_bf(x1 * sf);
            }
            o1[qq] = pack2(r1[0], r1[1]);
            o2[qq] = pack2(r2v[0], r2v[1]);
          }
          v1 = o1;
          v2 = o2;
        }
        if (m < args.M) {
          gemm_out_store(reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + cl * 8), v1);
          gemm_out_store(reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + (cl + 8) * 8), v2);
        }
      }
    }
    return;
  }
#pragma unroll 1
  for (int b0 = 0; b0 < ITERS; b0 += BATCH) {
    u32x4 rv[BATCH], cw[BATCH], sw[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int c = tid + (b0 + u) * NTHR;
      const int r2 = c / CPR, cc = c % CPR;
      const int m = min(m0 + r2, args.M - 1);
      if (args.res) rv[u] = *reinterpret_cast<const u32x4*>(args.res + (long)m * args.ldr + n0 + cc * 8);
      if (rope_tile) {
        const int d = (cc * 8) & 127;
        const int t = m % args.rope_T, dd = d < 64 ? d : d - 64;
        cw[u] = *reinterpret_cast<const u32x4*>(args.rope_cs + (long)t * 64 + dd);
        sw[u] = *reinterpret_cast<const u32x4*>(args.rope_sn + (long)t * 64 + dd);
      }
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int c = tid + (b0 + u) * NTHR;
      const int r2 = c / CPR, cc = c % CPR;
      const int m = m0 + r2;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + cc * 16);
      if (rope_tile && n0 + cc * 8 < args.rope_cols) {
        // RoPE on the bf16-rounded product, rounding per op like HF: x*cos + rotate_half(x)*sin.
        // The tile holds two whole heads, so the partner (+-64 columns) is in the same LDS row.
        const int d = (cc * 8) & 127;
        const bool lo = d < 64;
        const u32x4 pv = *reinterpret_cast<const u32x4*>(smem + r2 * CPITCH + (lo ? cc + 8 : cc - 8) * 16);
        u32x4 o;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          float r[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int sh = 16 * hh;
            const float x = bits2f((v[qq] >> sh) & 0xffff), p = bits2f((pv[qq] >> sh) & 0xffff);
            const float cf = bits2f((cw[u][qq] >> sh) & 0xffff), sf = bits2f((sw[u][qq] >> sh) & 0xffff);
            // lo half: x1*c + (-x2)*s ; hi half: x2*c + x1*s
            r[hh] = lo ? round_bf(x * cf) + round_bf(-p * sf) : round_bf(x * cf) + round_bf(p * sf);
          }
          o[qq] = pack2(r[0], r[1]);
        }
        v = o;
      }
      if (args.res) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float lo = bits2f(v[qq] & 0xffff) + bits2f(rv[u][qq] & 0xffff);
          const float hi = bits2f(v[qq] >> 16) + bits2f(rv[u][qq] >> 16);
          v[qq] = pack2(lo, hi);
        }
      }
      if (m < args.M) gemm_out_store(reinterpret_cast<u32x4*>(C + (long)m * args.ldc + n0 + cc * 8), v);
    }
  }
}

template <int DBG = 0, bool DROP = false, bool MX = false, int SP = 0>
__global__ __launch_bounds__(512) void gemm_nt_v5_kernel(const GemmArgs args, int tiles_m, int tiles_n, int dp,
                                                         int split, float* __restrict__ ws, int GM) {
  constexpr int BM = 256, BN = 256, HALF = 16384, SLOT = 4 * HALF;  // half order in a slot: A0 A1 B0 B1
  constexpr int SC_SLOT = 2048;                                       // MX: 1 KiB A + 1 KiB B scales
  constexpr int SC_BASE = 2 * SLOT;
  constexpr int CPITCH = BN * 2 + 16;
  constexpr int MAIN_BYTES = 2 * SLOT + (MX ? 2 * SC_SLOT : 0);
  constexpr int BITS_BASE = MAIN_BYTES;                      // DROP: the tile's keep bits, 256 rows x 32 B
  constexpr int RING_BYTES = MAIN_BYTES + (DROP ? 8192 : 0);
  constexpr int LDS_BYTES = (RING_BYTES > BM * CPITCH) ? RING_BYTES : BM * CPITCH;
  static_assert(LDS_BYTES <= 163840, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  // DBG 5 (ablation): s_memrealtime (100 MHz) stamps of the workgroup's phases, wave 0
  uint64_t rt[6] = {};
  if constexpr (DBG == 5) rt[0] = __builtin_amdgcn_s_memrealtime();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool g1 = wave >= 4;
  const int wm = wave >> 2, wn = wave & 3;

  int m0, n0, tb, tcount, part = -1;
  const int nt1 = MX ? args.K / 128 : args.K / BK, nt2 = args.K2 / BK, ntot = nt1 + nt2;
  {
    const int wg = blockIdx.x;
    if (wg < dp) {
      const int xcd = wg & 7, slot = wg >> 3, q = dp >> 3, r = dp & 7;
      const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
      v5_tile(L, tiles_m, tiles_n, m0, n0, GM);
      tb = 0;
      tcount = ntot;
    } else {
      const int u = wg - dp, z = u % split;
      part = u;
      v5_tile(dp + u / split, tiles_m, tiles_n, m0, n0, GM);
      tb = (int)((long)ntot * z / split);
      tcount = (int)((long)ntot * (z + 1) / split) - tb;
    }
  }
  const int nt = tcount;  // K-tiles this workgroup runs; absolute tile = tb + local
  const int Mlast = args.M - 1, Nlast = args.N - 1;
  const int rr8 = lane >> 3, c8 = lane & 7;

  // with dropout the LoRA extension tiles run FIRST so their (masked) sum can be scaled alone
  auto abs_tile = [&](int tl) {
    const int q = tb + tl;
    return DROP ? (q < nt2 ? nt1 + q : q - nt2) : q;
  };
  // stage half-tile h (0 A0, 1 A1, 2 B0, 3 B1) of K-tile t: 16 pieces of 8 rows x 128 B, 2 per wave.
  // A K-tile row is 128 bytes in both formats (64 bf16 or 128 e4m3), so staging is byte-generic.
  auto stage_half = [&](int tl, int h) {  // tl: local K-tile index
    if (DBG == 1 && tl >= 2) return;
    char* dst = smem + (tl & 1) * SLOT + h * HALF;
    const int t = abs_tile(tl);
    const bool ext = t >= nt1;
    const bool isA = h < 2;
    const int row0 = (isA ? m0 : n0) + (h & 1) * 128;
    const int last = isA ? Mlast : Nlast;
    if constexpr (MX) {
      const char* base = reinterpret_cast<const char*>(isA ? (ext ? args.A2 : args.A) : (ext ? args.B2 : args.B));
      const int ldB = (isA ? (ext ? args.lda2 : args.lda) : (ext ? args.ldb2 : args.ldb)) * (ext ? 2 : 1);
      const int kb = (ext ? t - nt1 : t) * 128;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = wave * 2 + i;
        const int row = p * 8 + rr8;
        const int g = min(row0 + row, last);
        glds16(base + (long)g * ldB + kb + ((c8 ^ (row & 7)) << 4), dst + p * 1024);
      }
    } else {
      const bf16* base = isA ? (ext ? args.A2 : args.A) : (ext ? args.B2 : args.B);
      const int ld = isA ? (ext ? args.lda2 : args.lda) : (ext ? args.ldb2 : args.ldb);
      const int k0 = (ext ? t - nt1 : t) * BK;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = wave * 2 + i;
        const int row = p * 8 + rr8;
        const int g = min(row0 + row, last);
        glds16(base + (long)g * ld + k0 + ((c8 ^ (row & 7)) << 3), dst + p * 1024);
      }
    }
  };
  // MX: the E8M0 scales of K-tile tl (one 4-B LDS-DMA per wave; extension tiles load a valid, unused tile)
  auto stage_scales = [&](int tl) {
    if constexpr (MX) {
      const int t = min(abs_tile(tl), nt1 - 1);
      const uint32_t* src = wave < 4 ? args.sa + ((long)(m0 / 64 + wave) * nt1 + t) * 64
                                     : args.sb + ((long)(n0 / 64 + wave - 4) * nt1 + t) * 64;
      __builtin_amdgcn_global_load_lds(src + lane, (LDS_AS void*)(smem + SC_BASE + (tl & 1) * SC_SLOT + wave * 256), 4,
                                       0, 0);
    }
  };

  // SP >= 5 (bf16): the main (non-extension) tiles are staged by buffer_load_dwordx4 ... lds from per-lane
  // byte offsets fixed for the whole launch, the K advance riding in the scalar soffset: no VALU address math
  // and no per-piece operand selects in the loop (SP 6: the same schedule with the generic staging, for A/B).
  static_assert(!((SP == 6 || SP == 7 || SP == 9) && MX), "SP 6, 7, 9 are bf16 schedules");
  constexpr bool FAST = (SP == 5 || SP == 7 || SP == 8 || SP == 9);  // buffer-offset staging of the main tiles
  constexpr bool BAL = (SP == 5 || SP == 6 || SP == 8 || SP == 9);  // 4 + 4 refills per K-tile
  constexpr bool UNR2 = (SP == 8 || SP == 9);             // steady loop unrolled by 2 (slot parity constant)
  constexpr bool EARLYB = (SP == 9);                      // B0 of tile t+1 read in R(t,1): 12 + 12 fragment reads
  // main-operand element bytes: 2 (bf16) or 1 (MXFP8: lda / ldb are in bytes, a K-tile row is 128 B either way)
  constexpr int EB = MX ? 1 : 2;
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)args.A, 0, (int)(((long)Mlast * args.lda + args.K) * EB), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)args.B, 0, (int)(((long)Nlast * args.ldb + args.K) * EB), 0x00020000);
  uint32_t voff[4][2] = {};
  if constexpr (FAST) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool isA = h < 2;
        const int row = (h & 1) * 128 + (wave * 2 + i) * 8 + rr8;
        const int g = min((isA ? m0 : n0) + row, isA ? Mlast : Nlast);
        voff[h][i] = (uint32_t)g * (uint32_t)(isA ? args.lda : args.ldb) * (uint32_t)EB + ((c8 ^ rr8) << 4);
      }
  }
  auto is_ext = [&](int tl) { return abs_tile(tl) >= nt1; };
  auto stage_fast = [&](int tl, int h, int par = -1) __attribute__((always_inline)) {
    char* dst = smem + (par >= 0 ? par : (tl & 1)) * SLOT + h * HALF;
    const int kb = abs_tile(tl) * 128;  // one 128-B row per K-tile (64 bf16 or 128 e4m3)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB, (LDS_AS void*)(dst + (wave * 2 + i) * 1024), 16,
                                               voff[h][i], kb, 0, 0);
  };
  auto stage_any = [&](int tl, int h) __attribute__((always_inline)) {
    if (FAST && !is_ext(tl))
      stage_fast(tl, h);
    else
      stage_half(tl, h);
  };

  uint32_t stp[2][5] = {};  // DBG 4
  f32x4 acc[4][4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2];
  bf16x8 bsp[2][2][2];  // SP: [B half][n][k-substep], the whole K-tile's B fragments
  bf16x8 b0n[2][2];     // SP 9: B0 fragments of the next K-tile
  i32x8 a8[4], b8[2];  // MX tiles: both k-halves of a fragment in one 8-register operand
  i32x8 b8sp[2][2];    // SP + MX: [B half][n]

  // dropout with keep bits: the tile's mask block (rows clamped) goes in first, so every wait below covers it
  if constexpr (DROP) {
    if (args.drop_bits && tb == 0 && nt2 > 0) {
      const int p = wave * 64 + lane, row = p >> 1;
      glds16(args.drop_bits + (long)min(m0 + row, Mlast) * (args.drop_ld >> 3) + (n0 >> 3) + 16 * (p & 1),
             smem + BITS_BASE + wave * 1024);
    }
  }
  // prologue: tile 0 complete, A0 of tile 1 in flight (SP: tile 0 only)
  if constexpr (BAL) {  // tile 0 complete; B0 B1 (+ scales) of tile 1 in flight (its A0 A1 are staged in R(0,0))
    if (nt > 0) { stage_scales(0); stage_any(0, 2); stage_any(0, 3); stage_any(0, 0); stage_any(0, 1); }
    if (nt > 1) {
      stage_scales(1); stage_any(1, 2); stage_any(1, 3);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MX ? 5 : 4) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
  if (nt > 0) {
    stage_scales(0);
    stage_any(0, 2); stage_any(0, 3); stage_any(0, 1); stage_any(0, 0);
  }
  if (!SP && nt > 1) stage_half(1, 0);
  if (SP && nt > 1) { stage_scales(1); stage_any(1, 2); stage_any(1, 3); stage_any(1, 0); }
  if (!SP && nt > 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (SP && nt > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(MX ? 7 : 6) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (g1) {  // the ping-pong offset
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if constexpr (DBG == 5) rt[1] = __builtin_amdgcn_s_memrealtime();
  if constexpr (EARLYB) {  // B0 of tile 0 (landed per the prologue wait; retired by the first lgkmcnt(0))
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        b0n[n][s] = *reinterpret_cast<const bf16x8*>(smem + 2 * HALF + mmaj_off(wn * 32 + n * 16 + (lane & 15), 4 * s + (lane >> 4)));
  }

  const int frow = lane & 15, fcol = lane >> 4;
  // one K-tile = 4 phases; a lambda so the dropout variant can peel its extension tiles
  // mxt: an MXFP8 main tile (compile-time, so each loop below keeps one MFMA form and its
  // accumulators in place; a per-phase runtime branch made the compiler copy them)
  // SP ("super-phase") schedule: 2 phases per K-tile of 32 MFMAs per wave (2 C-quadrants), half the
  // barriers of the 8-phase schedule and 24 fragment reads per K-tile instead of 32 (the B fragments
  // of both halves stay in registers across the tile).  Global intervals I (one barrier apart), g1 one
  // interval behind g0:  I 4t..4t+3  g0: R(t,0) M(t,0) R(t,1) M(t,1);  g1: M(t-1,1) R(t,0) M(t,0) R(t,1).
  // A slot half is refilled as soon as both groups have read it, from each wave's R sections:
  //   A1 of tile t+1 in R(t,0), B0 B1 A0 of tile t+2 in R(t,1),
  // and each wave waits for its pieces (vmcnt: 8 newer pieces at steady state) before the barrier
  // that opens g0's first read of them -- 5-6 intervals of load latency per piece.
  // MX: the E8M0 scales of tile t+2 travel with its B0 B1 A0 (7 pieces in that group, 9 newer at steady state)
  constexpr int KB = MX ? 7 : 6;
  auto wait_sp = [&](int n) __attribute__((always_inline)) { wait_vmcnt_exact(n); };
  auto run_tile_sp = [&](int t, auto mxt) __attribute__((always_inline)) {
    constexpr bool mx_tile = MX && decltype(mxt)::value;
    const char* slot = smem + (t & 1) * SLOT;
    const bool n1 = t + 1 < nt, n2 = t + 2 < nt;
    uint32_t scA[2] = {0u, 0u}, scB[2] = {0u, 0u};
    if constexpr (mx_tile) {  // staged with tile t's B0 B1 A0: landed per the same waits
      const char* sc = smem + SC_BASE + (t & 1) * SC_SLOT;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        scA[h] = *reinterpret_cast<const uint32_t*>(sc + (h * 2 + wm) * 256 + lane * 4);
        scB[h] = *reinterpret_cast<const uint32_t*>(sc + 1024 + (h * 2 + (wn >> 1)) * 256 + lane * 4) >>
                 (16 * (wn & 1));
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const char* la = slot + p * HALF;
      if (SP == 3 && p == 0 && n1) stage_any(t + 1, 1);
      if (SP == 3 && p == 1 && n2) { stage_scales(t + 2); stage_any(t + 2, 2); stage_any(t + 2, 3); stage_any(t + 2, 0); }
      if constexpr (mx_tile) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a8[i].lo = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, fcol));
          a8[i].hi = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 + fcol));
        }
        if (p == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const char* lb = slot + (2 + h) * HALF;
              b8sp[h][n].lo = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, fcol));
              b8sp[h][n].hi = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, 4 + fcol));
            }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[i][s] = *reinterpret_cast<const bf16x8*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 * s + fcol));
        if (p == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                bsp[h][n][s] = *reinterpret_cast<const bf16x8*>(slot + (2 + h) * HALF +
                                                                 mmaj_off(wn * 32 + n * 16 + frow, 4 * s + fcol));
        }
      }
      if (SP != 3 && p == 0 && n1) stage_any(t + 1, 1);
      if (SP != 3 && p == 1 && n2) { stage_scales(t + 2); stage_any(t + 2, 2); stage_any(t + 2, 3); stage_any(t + 2, 0); }
      if (g1) {
        if (p == 0) wait_sp(n1 ? KB + 2 : 0);         // A1(t)
        if (p == 1 && n1) wait_sp(n2 ? KB + 2 : 2);   // B0 B1 A0 (+ scales) of t+1
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (DBG != 2 && mx_tile) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = 2 * p + q;
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[j][i][n] = mx_mfma(b8sp[ib][n], a8[i], acc[j][i][n], n, scB[ib], i, scA[p]);
        }
        // keep the scaled MFMAs inside their phase (see the 8-phase loop)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[2 * p + q][i][n]));
        __builtin_amdgcn_s_setprio(0);
      } else if constexpr (DBG != 2) {
        if (SP != 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          // p 0: quadrants j 0 (ia 0, ib 0), 1 (0, 1); p 1: j 2 (1, 1), 3 (1, 0)
          const int j = 2 * p + q;
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                acc[j][i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bsp[ib][n][s], af[i][s], acc[j][i][n], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i][0]), "v"(af[i][1]));
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int n = 0; n < 2; ++n) asm volatile("" ::"v"(bsp[h][n][0]), "v"(bsp[h][n][1]));
      }
      if (!g1) {
        if (p == 0) wait_sp(n1 ? KB + 2 : 0);
        if (p == 1 && n1) wait_sp(n2 ? KB + 2 : 2);
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  // SP 5/6: the SP intervals with the refills balanced 4 + 4 pieces per K-tile: A0 A1 of tile t+1 in R(t,0)
  // (their slot halves were last read in R(t-1,.)), B0 B1 of tile t+2 in R(t,1).  Counted waits (before the
  // barrier that opens g0's first read): A1(t) before R(t,1) -- 8 newer pieces (B(t+1), A(t+1)); A0 B of t+1
  // before R(t+1,0) -- 6 newer (A1(t+1), B(t+2)).  STEADY: t+1 and t+2 exist and are main tiles, so the waits
  // are constants and staging takes the fast path with no branch.
  auto run_tile_sp5 = [&](int t, auto steady, auto parity, auto mxt) __attribute__((always_inline)) {
    constexpr bool ST = decltype(steady)::value;
    constexpr int PAR = decltype(parity)::value;  // slot parity of tile t when known at compile time, else -1
    constexpr bool mx_tile = MX && decltype(mxt)::value;
    constexpr int SC = MX ? 1 : 0;                // MX: the scales of tile t+2 ride with its B0 B1
    const char* slot = smem + (PAR >= 0 ? PAR : (t & 1)) * SLOT;
    const bool n1 = ST || t + 1 < nt, n2 = ST || t + 2 < nt;
    uint32_t scA[2] = {0u, 0u}, scB[2] = {0u, 0u};
    if constexpr (mx_tile) {  // staged with tile t's B0 B1: landed per the waits before R(t,0)
      const char* sc = smem + SC_BASE + (PAR >= 0 ? PAR : (t & 1)) * SC_SLOT;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        scA[h] = *reinterpret_cast<const uint32_t*>(sc + (h * 2 + wm) * 256 + lane * 4);
        scB[h] = *reinterpret_cast<const uint32_t*>(sc + 1024 + (h * 2 + (wn >> 1)) * 256 + lane * 4) >>
                 (16 * (wn & 1));
      }
    }
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t st_raw[5];
#define STAMP(k)                                                       \
  if constexpr (DBG == 4 && ST && PAR == 0) {                           \
    __builtin_amdgcn_sched_barrier(0);                                  \
    st_raw[k] = (uint32_t)__builtin_amdgcn_s_memtime();                 \
    __builtin_amdgcn_sched_barrier(0);                                  \
  }
      STAMP(0);
      const char* la = slot + p * HALF;
      if constexpr (mx_tile) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          a8[i].lo = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, fcol));
          a8[i].hi = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 + fcol));
        }
        if (p == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const char* lb = slot + (2 + h) * HALF;
              b8sp[h][n].lo = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, fcol));
              b8sp[h][n].hi = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, 4 + fcol));
            }
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[i][s] = *reinterpret_cast<const bf16x8*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 * s + fcol));
        if (EARLYB) {
          if (p == 0) {  // B0(t) came with R(t-1,1); B1(t) now
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s) {
                bsp[0][n][s] = b0n[n][s];
                bsp[1][n][s] = *reinterpret_cast<const bf16x8*>(slot + 3 * HALF +
                                                                 mmaj_off(wn * 32 + n * 16 + frow, 4 * s + fcol));
              }
          } else if (n1) {
            const char* nslot = smem + (PAR >= 0 ? 1 - PAR : ((t + 1) & 1)) * SLOT;
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                b0n[n][s] = *reinterpret_cast<const bf16x8*>(nslot + 2 * HALF +
                                                            mmaj_off(wn * 32 + n * 16 + frow, 4 * s + fcol));
          }
        } else if (p == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                bsp[h][n][s] = *reinterpret_cast<const bf16x8*>(slot + (2 + h) * HALF +
                                                                 mmaj_off(wn * 32 + n * 16 + frow, 4 * s + fcol));
        }
      }
      if (ST && FAST) {
        if (p == 0) { stage_fast(t + 1, 0, PAR >= 0 ? 1 - PAR : -1); stage_fast(t + 1, 1, PAR >= 0 ? 1 - PAR : -1); }
        if (p == 1) { stage_scales(t + 2); stage_fast(t + 2, 2, PAR); stage_fast(t + 2, 3, PAR); }
      } else if (ST) {
        if (p == 0) { stage_half(t + 1, 0); stage_half(t + 1, 1); }
        if (p == 1) { stage_scales(t + 2); stage_half(t + 2, 2); stage_half(t + 2, 3); }
      } else {
        if (p == 0 && n1) { stage_any(t + 1, 0); stage_any(t + 1, 1); }
        if (p == 1 && n2) { stage_scales(t + 2); stage_any(t + 2, 2); stage_any(t + 2, 3); }
      }
      // counted waits: p 0 -> A1(t) (+ EARLYB: B0(t+1)); p 1 -> A0 B (+ scales) of t+1
      auto waits = [&]() __attribute__((always_inline)) {
        if (ST) {
          if (p == 0 && !EARLYB) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + SC) : "memory");
          else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 + SC) : "memory");  // EARLYB p 0: A1(t) and B0(t+1)
        } else {
          if (p == 0) wait_vmcnt_exact(n1 ? (EARLYB ? 6 : 8 + SC) : 0);
          if (p == 1 && n1) wait_vmcnt_exact(n2 ? 6 + SC : 2);
        }
      };
      if (g1) waits();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      STAMP(1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      STAMP(2);
      __builtin_amdgcn_s_setprio(1);
      if constexpr (mx_tile) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = 2 * p + q;
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n)
              acc[j][i][n] = mx_mfma(b8sp[ib][n], a8[i], acc[j][i][n], n, scB[ib], i, scA[p]);
        }
        // keep the scaled MFMAs inside their phase (see the 8-phase loop)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[2 * p + q][i][n]));
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = 2 * p + q;
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                acc[j][i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bsp[ib][n][s], af[i][s], acc[j][i][n], 0, 0, 0);
        }
      }
      __builtin_amdgcn_s_setprio(0);
      STAMP(3);
      if (!g1) waits();
      STAMP(4);
      if constexpr (DBG == 4 && ST && PAR == 0) {  // commit (only memtimes are pending here)
        const bool rec = (t == 8);
#pragma unroll
        for (int k = 0; k < 5; ++k) stp[p][k] = rec ? st_raw[k] : stp[p][k];
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  auto run_tile = [&](int t, auto mxt) __attribute__((always_inline)) {
    if constexpr (BAL) {
      run_tile_sp5(t, std::integral_constant<bool, false>{}, std::integral_constant<int, -1>{}, mxt);
      return;
    }
    if constexpr (SP) {
      run_tile_sp(t, mxt);
      return;
    }
    const char* slot = smem + (t & 1) * SLOT;
    constexpr bool mx_tile = MX && decltype(mxt)::value;
    uint32_t scA[2] = {0u, 0u}, scB[2] = {0u, 0u};
    if constexpr (mx_tile) {  // staged with tile t-1's B1 (or in the prologue): landed per the q0 wait + barriers
      const char* sc = smem + SC_BASE + (t & 1) * SC_SLOT;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        scA[h] = *reinterpret_cast<const uint32_t*>(sc + (h * 2 + wm) * 256 + lane * 4);
        scB[h] = *reinterpret_cast<const uint32_t*>(sc + 1024 + (h * 2 + (wn >> 1)) * 256 + lane * 4) >>
                 (16 * (wn & 1));
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ia = (j >= 2) ? 1 : 0;
      const int ib = (j == 1 || j == 2) ? 1 : 0;
      // ---- R: fragments that change this phase, then one half-tile of staging
      if constexpr (mx_tile) {
        if (j == 0 || j == 2) {
          const char* la = slot + ia * HALF;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            a8[i].lo = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, fcol));
            a8[i].hi = *reinterpret_cast<const i32x4*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 + fcol));
          }
        }
        const char* lb = slot + (2 + ib) * HALF;
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          b8[n].lo = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, fcol));
          b8[n].hi = *reinterpret_cast<const i32x4*>(lb + mmaj_off(wn * 32 + n * 16 + frow, 4 + fcol));
        }
      } else {
        if (j == 0 || j == 2) {
          const char* la = slot + ia * HALF;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              af[i][s] = *reinterpret_cast<const bf16x8*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 * s + fcol));
        }
        const char* lb = slot + (2 + ib) * HALF;
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            bfr[n][s] = *reinterpret_cast<const bf16x8*>(lb + mmaj_off(wn * 32 + n * 16 + frow, 4 * s + fcol));
      }
      if (DBG != 1) {
        if (j == 0 && t + 1 < nt) stage_scales(t + 1);
        if (j == 0 && t + 1 < nt) stage_half(t + 1, 3);
        if (j == 1 && t + 1 < nt) stage_half(t + 1, 2);
        if (j == 2 && t + 1 < nt) stage_half(t + 1, 1);
        if (j == 3 && t + 2 < nt) stage_half(t + 2, 0);
      }
      // counted DMA waits before the barrier that precedes the first reader:
      // into q2 of this tile: A1(t) (6 later glds when tile t+1 is staged, +1 scale DMA with MX);
      // into q0 of tile t+1: A0(t+1), B0(t+1) (A1(t+1) + A0(t+2) later)
      const bool wq2 = (j == 1), wq0 = (j == 3) && (t + 1 < nt);
      const int nq2 = (t + 1 < nt) ? (MX ? 7 : 6) : 0;
      const int nq0 = (t + 2 < nt) ? 4 : 2;
      if (g1) {
        if (wq2) wait_vmcnt_exact(nq2);
        if (wq0) wait_vmcnt_exact(nq0);
      }
      asm volatile("" ::: "memory");  // keep this phase's reads / DMA issue above the barrier
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      // ---- M: one C-quadrant x K = 64
      if constexpr (DBG != 2 && mx_tile) {
        // one scaled MFMA per (i, n) over the whole 128-k tile; first operand B (SWAP layout)
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < 2; ++n) acc[j][i][n] = mx_mfma(b8[n], a8[i], acc[j][i][n], n, scB[ib], i, scA[ia]);
        // pin the cluster inside its phase: the scaled-MFMA builtin is not convergent, so without a
        // use here the compiler sinks it past the barriers (merging phases, spilling)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < 2; ++n) asm volatile("" : "+v"(acc[j][i][n]));
        __builtin_amdgcn_s_setprio(0);
      } else if (DBG != 2) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int s = 0; s < 2; ++s)
              acc[j][i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n][s], af[i][s], acc[j][i][n], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i][0]), "v"(af[i][1]));
#pragma unroll
        for (int n = 0; n < 2; ++n) asm volatile("" ::"v"(bfr[n][0]), "v"(bfr[n][1]));
      }
      if (!g1) {
        if (wq2) wait_vmcnt_exact(nq2);
        if (wq0) wait_vmcnt_exact(nq0);
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  };
  // with dropout the LoRA extension tiles come first (stage_half's order); their masked sum is
  // scaled once between the two loops, outside the hot loop's register allocation
  using MXT = std::integral_constant<bool, true>;
  using BFT = std::integral_constant<bool, false>;
  const int pre = (DROP && tb == 0) ? (nt2 < nt ? nt2 : nt) : 0;
  for (int t = 0; t < pre; ++t) run_tile(t, BFT{});
  if (pre > 0) {
    if constexpr (DROP) {
      {  // accumulators hold exactly A2.B2^T: apply the dropout mask.  Per (row, B half) the keep bits of the
         // 32 tile columns ib*128 + wn*32 + 0..31 this wave's lanes hold: from the forward's keep bits (staged in
         // the prologue; landed -- every wait since covers them) or re-hashed (this lane's 8 bits only); one
         // multiply pass either way (two alternative passes over the 128 accumulators spilled)
        const int gq = lane >> 4, lq = lane & 15;
        const bool from_bits = args.drop_bits != nullptr;
#pragma unroll
        for (int ia = 0; ia < 2; ++ia)
#pragma unroll
          for (int ib = 0; ib < 2; ++ib) {
            const int j = ia ? (ib ? 2 : 3) : (ib ? 1 : 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int rl = ia * 128 + wm * 64 + i * 16 + lq;
              uint32_t w;
              if (from_bits) {
                w = *reinterpret_cast<const uint32_t*>(smem + BITS_BASE + rl * 32 + ib * 16 + wn * 4);
              } else {
                w = 0;
                const uint32_t m = (uint32_t)(m0 + rl);
#pragma unroll
                for (int n = 0; n < 2; ++n) {
                  const uint32_t c = (uint32_t)(n0 + ib * 128 + wn * 32 + n * 16 + 4 * gq);
                  bool keep[4];
                  drop_keep_pairs<2>(m * (uint32_t)args.drop_ld + c, args.drop_seed, args.drop_thresh, keep);  // c % 4 == 0
#pragma unroll
                  for (int e = 0; e < 4; ++e) w |= (keep[e] ? 1u : 0u) << (n * 16 + 4 * gq + e);
                }
              }
#pragma unroll
              for (int n = 0; n < 2; ++n) {
                const uint32_t nib = w >> (n * 16 + 4 * gq);
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[j][i][n][e] *= ((nib >> e) & 1u) ? args.drop_scale : 0.f;
              }
            }
          }
      }
    }
  }
  if constexpr (MX && !BAL) {  // main (fp8) tiles, then any bf16 extension tiles of this K-range
    const int main_end = DROP ? nt : min(nt, max(pre, nt1 - tb));
    for (int t = pre; t < main_end; ++t) run_tile(t, MXT{});
    for (int t = main_end; t < nt; ++t) run_tile(t, BFT{});
  } else if constexpr (BAL) {
    // steady tiles: t+1 and t+2 exist and are main tiles (non-dropout: the extension tiles come last)
    const int main_lim = DROP ? nt : min(nt, max(0, nt1 - tb));
    using STT = std::integral_constant<bool, true>;
    using STF = std::integral_constant<bool, false>;
    using PRT = std::integral_constant<int, -1>;
    using MT = std::integral_constant<bool, MX>;  // the main tiles' MFMA form
    int t = pre;
    if constexpr (UNR2) {
      if ((t & 1) && t < main_lim - 2) run_tile_sp5(t++, STT{}, PRT{}, MT{});
      for (; t + 1 < main_lim - 2; t += 2) {
        run_tile_sp5(t, STT{}, std::integral_constant<int, 0>{}, MT{});
        run_tile_sp5(t + 1, STT{}, std::integral_constant<int, 1>{}, MT{});
      }
    }
    for (; t < main_lim - 2; ++t) run_tile_sp5(t, STT{}, PRT{}, MT{});
    for (; t < main_lim; ++t) run_tile_sp5(t, STF{}, PRT{}, MT{});
    for (; t < nt; ++t) run_tile_sp5(t, STF{}, PRT{}, BFT{});  // (non-dropout: the extension tiles come last)
  } else {
    for (int t = pre; t < nt; ++t) run_tile(t, BFT{});
  }
  if (!g1) {  // re-align the barrier count
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (DBG == 5) rt[2] = __builtin_amdgcn_s_memrealtime();
  if constexpr (DBG == 4) {
    if (args.dbg && lane < 10) args.dbg[((long)blockIdx.x * 8 + wave) * 16 + lane] = stp[lane / 5][lane % 5];
  }

  // epilogue: quadrant j, frag (i, n): D[n][m] -> lane holds m = l16, n = 4g..4g+3
  const int g = lane >> 4, l16 = lane & 15;
  if (part >= 0) {  // split-K tail: raw fp32 partial tile [256][256]
    float* wt = ws + (long)part * (BM * BN);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ia = (j >= 2) ? 1 : 0;
      const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ml = ia * 128 + wm * 64 + i * 16 + l16;
          const int nl = ib * 128 + wn * 32 + n * 16 + 4 * g;
          gemm_out_store(reinterpret_cast<f32x4*>(wt + ml * BN + nl), acc[j][i][n]);
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int ia = (j >= 2) ? 1 : 0;
    const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int nl = ib * 128 + wn * 32 + n * 16 + 4 * g;
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
      if (args.bias) {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) b4[qq] = bf2f(args.bias[n0 + nl + qq]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ml = ia * 128 + wm * 64 + i * 16 + l16;
        const f32x4 v = acc[j][i][n];
        uint2 pk;
        pk.x = pack2(v[0] * args.alpha + b4[0], v[1] * args.alpha + b4[1]);
        pk.y = pack2(v[2] * args.alpha + b4[2], v[3] * args.alpha + b4[3]);
        *reinterpret_cast<uint2*>(smem + ml * CPITCH + nl * 2) = pk;
      }
    }
  }
  __syncthreads();
  if constexpr (DBG == 5) rt[3] = __builtin_amdgcn_s_memrealtime();
  epi_rows<512>(args, smem, m0, n0);
  if constexpr (DBG == 5) {
    rt[4] = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    rt[5] = __builtin_amdgcn_s_memrealtime();
    if (args.dbg && wave == 0 && lane < 6) {
      const uint64_t v = lane == 0 ? rt[0] : lane == 1 ? rt[1] : lane == 2 ? rt[2] : lane == 3 ? rt[3] : lane == 4 ? rt[4] : rt[5];
      reinterpret_cast<uint64_t*>(args.dbg)[(long)blockIdx.x * 8 + lane] = v;
    }
  }
}

// sum the split partials of each tail tile, apply alpha / bias / residual, write bf16
// The split partials of 8 columns (row r of a tile), summed in split order: every load issued before the first
// add (a split-long load->add chain cost ~2 us per partial), non-temporal (each partial is read once).  Loads are
// unconditional (index clamped: no branch, one counted wait), W = 4 or 8 at a time.
template <int W>
__device__ __forceinline__ void fixup_sum_w(const float* p, int split, f32x4& lo, f32x4& hi) {
  for (int z0 = 0; z0 < split; z0 += W) {
    f32x4 pl[W], ph[W];
#pragma unroll
    for (int u = 0; u < W; ++u) {
      const long zz = min(z0 + u, split - 1);
      pl[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + zz * 65536));
      ph[u] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + zz * 65536 + 4));
    }
#pragma unroll
    for (int u = 0; u < W; ++u)
      if (z0 + u < split) {
        lo += pl[u];
        hi += ph[u];
      }
  }
}
__device__ __forceinline__ void fixup_sum(const float* p, int split, f32x4& lo, f32x4& hi) {
  if (split <= 4) fixup_sum_w<4>(p, split, lo, hi);
  else fixup_sum_w<8>(p, split, lo, hi);
}

__global__ __launch_bounds__(256) void splitk_fixup_kernel(const GemmArgs args, int tiles_m, int tiles_n, int dp,
                                                           int split, const float* __restrict__ ws, int GM) {
  const int tile = blockIdx.x >> 5, rblk = blockIdx.x & 31;
  int m0, n0;
  v5_tile(dp + tile, tiles_m, tiles_n, m0, n0, GM);
  const int r = rblk * 8 + (threadIdx.x >> 5), c = (threadIdx.x & 31) * 8;
  const int m = m0 + r;
  if (m >= args.M) return;
  f32x4 lo = f32x4{0.f, 0.f, 0.f, 0.f}, hi = lo;
  fixup_sum(ws + (long)tile * split * 65536 + r * 256 + c, split, lo, hi);
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  if (args.alpha != 1.f || args.bias) {  // the main epilogues' expression, v * alpha + b in one (contracted) step
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float bq = args.bias ? bf2f(args.bias[n0 + c + q]) : 0.f;
      v[q] = v[q] * args.alpha + bq;
    }
  }
  u32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) o[q] = pack2(v[2 * q], v[2 * q + 1]);
  if (n0 + c < args.rope_cols) {
    // RoPE as the main epilogue does it: on the bf16-rounded products, partner column +-64 of the head
    // (the tile holds whole heads, so the partner's partials are in the same partial tiles)
    const int d = c & 127;
    const bool lo_half = d < 64;
    const int pc = lo_half ? c + 64 : c - 64, dd = lo_half ? d : d - 64;
    f32x4 plo = f32x4{0.f, 0.f, 0.f, 0.f}, phi = plo;
    fixup_sum(ws + (long)tile * split * 65536 + r * 256 + pc, split, plo, phi);
    const float pv[8] = {plo[0], plo[1], plo[2], plo[3], phi[0], phi[1], phi[2], phi[3]};
    const int t = m % args.rope_T;
    const u32x4 cw = *reinterpret_cast<const u32x4*>(args.rope_cs + (long)t * 64 + dd);
    const u32x4 sw = *reinterpret_cast<const u32x4*>(args.rope_sn + (long)t * 64 + dd);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float rr[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int sh = 16 * hh;
        const float x = round_bf(v[2 * q + hh]), pr = round_bf(pv[2 * q + hh] * args.alpha);
        const float cf = bits2f((cw[q] >> sh) & 0xffff), sf = bits2f((sw[q] >> sh) & 0xffff);
        rr[hh] = lo_half ? round_bf(x * cf) + round_bf(-pr * sf) : round_bf(x * cf) + round_bf(pr * sf);
      }
      o[q] = pack2(rr[0], rr[1]);
    }
  }
  if (args.res) {  // residual added after the bf16 rounding of the product, as the main epilogue does
    const u32x4 rv = *reinterpret_cast<const u32x4*>(args.res + (long)m * args.ldr + n0 + c);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = pack2(bits2f(o[q] & 0xffff) + bits2f(rv[q] & 0xffff), bits2f(o[q] >> 16) + bits2f(rv[q] >> 16));
  }
  if (args.swg_gu) {
    swiglu_bwd_store8(args, m, n0 + c, o);
    return;
  }
  gemm_out_store(reinterpret_cast<u32x4*>(reinterpret_cast<bf16*>(args.C) + (long)m * args.ldc + n0 + c), o);
}

// The device's CU count: an immutable property, read once per device (std::call_once), so the
// library holds no mutable state -- the split-K workspace comes with every call (SplitOpts).
constexpr int kMaxDevices = 64;
int device_cus() {
  static std::once_flag once[kMaxDevices];
  static int cus[kMaxDevices];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
  std::call_once(once[dev], [dev] {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  });
  return cus[dev];
}

// Per call: the caller's split-K workspace and an optional pinned split of the tail round.
struct SplitOpts {
  int split = 0;              // 0: the cost model's choice; 1: no split; 2..8: that split (bounded below)
  float* ws = nullptr;        // fp32 partial tiles (256 KiB each); NULL: no split
  size_t ws_bytes = 0;
};

struct SplitPlan {
  int dp, split, tail;
};

// The tail round (tiles % CUs leftover tiles) as pieces of 1/s of a tile: ceil(tail s / cus) waves of T / s,
// plus the fp32 partials (256 KiB per piece, written here and read by the fixup: ~0.13 us each at ~4 TB/s).
// T = one tile's K loop, ~1.9 us per bf16 K-tile (2.3 per MX K-tile) at the measured rate.  At most one
// round of pieces (tail s <= CUs) and as many as ws_bytes holds.
// w4 (the 4-wave bf16 kernel): T = 1.3 us per K-tile and at most ~0.78 x CUs pieces.  Fitted on
// the step shapes' pinned-split sweep (tools/w4_split_sweep.py, profiles/r04/w4_split_sweep.log): a tail round
// that leaves CUs idle runs them at a higher clock (the chip is power-limited under this load), so few large
// pieces beat a full round of small ones (304-tile shapes: 4 pieces per tail tile, not 5; 1152 tiles: no split).
SplitPlan plan_split(int M, int N, int ntot, int K2, bool mx, bool drop, int cus, int pinned, size_t ws_bytes,
                     bool w4 = false) {
  const int tiles = ((M + 255) / 256) * (N / 256);
  SplitPlan pl{tiles, 1, 0};
  if (tiles <= cus || pinned == 1) return pl;
  const int tail = tiles % cus;
  if (!tail) return pl;
  const long ws_pieces = (long)(ws_bytes / (65536 * sizeof(float)));
  const int piece_cap = w4 ? cus * 25 / 32 : cus;
  const int sp_max = (int)std::min<long>(std::min(std::min(8, ntot / 4), piece_cap / tail), ws_pieces / tail);
  int split = 1;
  if (pinned > 1) {
    split = std::max(1, std::min(pinned, sp_max));
  } else {
    const double T = ntot * (w4 ? 1.3 : (mx ? 2.3 : 1.9));
    double best = T;
    for (int sp = 2; sp <= sp_max; ++sp) {
      const double cost = (double)((tail * sp + cus - 1) / cus) / sp * T + 0.13 * tail * sp;
      if (cost < best - 1e-9) {
        best = cost;
        split = sp;
      }
    }
  }
  // (with dropout every extension tile must sit in K-range 0, which applies the mask)
  const bool drop_ok = !drop || (long)(K2 / BK) * split <= ntot;
  if (split >= 2 && ntot >= 16 && drop_ok) pl = SplitPlan{tiles - tail, split, tail};
  return pl;
}

[[maybe_unused]] constexpr size_t W4_CNT_BYTES = OSPO_WS_GEMM_TAIL_CNT_BYTES;  // the w4 tail's arrival counters at the END of the split-K workspace
#include "gemm_w4.h"

// The 4-wave hand-scheduled kernel (gemm_w4.h) when the shape fits it: bf16, <= 2 LoRA extension tiles,
// 32-bit buffer offsets, and every work unit with enough main K-tiles for its program (plain: 4; the
// dropout unit that carries the extension tiles: 3).  Returns OSPO_ERR_UNSUPPORTED otherwise (the caller
// then runs the v5 kernel).  DBG 1 (ablation): no loads after the prologue.
template <bool DROP, int DBG = 0, int V = 0, bool MX = false>
int launch_w4(const GemmArgs& a_in, hipStream_t s, const SplitOpts& so) {
#ifdef OSPO_ABLATION
  GemmArgs a = a_in;
  if (const char* e = getenv("OSPO_GEMM_EPI")) a.epi_var = atoi(e);  // A/B: plain-epilogue store variants
#else
  const GemmArgs& a = a_in;
#endif
  constexpr int EB = MX ? 1 : 2;
  if (a.N % 256 || a.K % (MX ? 128 : 64) || a.K2 % 64 || a.K2 > 128) return OSPO_ERR_UNSUPPORTED;
  if ((long)a.M * a.lda * EB >= (1L << 31) || (long)a.N * a.ldb * EB >= (1L << 31)) return OSPO_ERR_UNSUPPORTED;
  if (a.K2 > 0 && ((long)a.M * a.lda2 * 2 >= (1L << 31) || (long)a.N * a.ldb2 * 2 >= (1L << 31)))
    return OSPO_ERR_UNSUPPORTED;
  if (MX && (!a.sa || !a.sb)) return OSPO_ERR_UNSUPPORTED;
  const int tm = (a.M + 255) / 256, tn = a.N / 256;
  const int nt1 = MX ? a.K / 128 : a.K / 64, nt2 = a.K2 / 64, ntot = nt1 + nt2;
  const SplitPlan pl = plan_split(a.M, a.N, ntot, a.K2, MX, DROP, device_cus(), so.split, so.ws ? so.ws_bytes : 0,
                                  true);
  for (int z = 0; z < (pl.tail ? pl.split : 1); ++z) {  // every unit's program must fit (z = 0: the whole range)
    const int tb = pl.tail ? (int)((long)ntot * z / pl.split) : 0;
    const int tc = pl.tail ? (int)((long)ntot * (z + 1) / pl.split) - tb : ntot;
    const W4Range r = w4_range(DROP, nt1, nt2, tb, tc);
    const bool drop_unit = DROP && r.ne > 0;
    if (r.ne > 2 || r.nm < (drop_unit ? 3 : 4) || (!DROP && r.ne > 0 && tb + r.nm != nt1)) return OSPO_ERR_UNSUPPORTED;
  }
  if (pl.tail && ntot < 4) return OSPO_ERR_UNSUPPORTED;
  const int grid = pl.dp + pl.tail * pl.split;
  // ablation build, OSPO_GEMM_INL=1: the tail's split-K combine inside the launch (round 5, measured and rejected:
  // 33.40 / 33.44 pairs/s against 34.55 / 34.62 with the fixup launch on one box, GEMM 403 vs 386 us per launch,
  // profiles/r05/gemm_inlaunch_ab.txt -- the last arriver reads (split - 1) x 256 KiB of partials at one CU's rate
  // and every piece's write-through stores are slower than the fixup's streaming), when the workspace carries
  // the arrival counters past its whole partial tiles (ws_bytes = n x 256 KiB + W4_CNT_BYTES, zero at allocation,
  // left zero by every call; ops.gemm_workspace allocates them)
  unsigned* cnt = nullptr;
#ifdef OSPO_ABLATION
  static const bool want_inl = getenv("OSPO_GEMM_INL") && atoi(getenv("OSPO_GEMM_INL")) == 1;
  if (want_inl && pl.tail && so.ws && so.ws_bytes % (65536 * sizeof(float)) == W4_CNT_BYTES &&
      pl.tail <= (int)(W4_CNT_BYTES / sizeof(unsigned)))
    cnt = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(so.ws) + so.ws_bytes - W4_CNT_BYTES);
#endif
  hipLaunchKernelGGL((gemm_nt_w4_kernel<DROP, DBG, V, MX>), dim3(grid), dim3(256), 0, s, a, tm, tn, pl.dp, pl.split,
                     so.ws, g_v5_gm, cnt);
  OSPO_CHECK_LAUNCH();
  if (pl.tail && !cnt) {
    hipLaunchKernelGGL(splitk_fixup_kernel, dim3(pl.tail * 32), dim3(256), 0, s, a, tm, tn, pl.dp, pl.split,
                       (const float*)so.ws, g_v5_gm);
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}

template <int DBG = 0, bool DROP = false, bool MX = false, int SP = 0>
int launch_v5(const GemmArgs& a, hipStream_t s, const SplitOpts& so, bool allow_split = true) {
  if (a.N % 256) return OSPO_ERR_SHAPE;
  if constexpr (SP == 5 || SP >= 7) {  // 32-bit buffer offsets: operands beyond 2 GiB take the generic staging
    if ((long)a.M * a.lda * 2 >= (1L << 31) || (long)a.N * a.ldb * 2 >= (1L << 31))
      return launch_v5<DBG, DROP, MX, (SP == 5 ? 6 : 1)>(a, s, so, allow_split);
  }
  const int tm = (a.M + 255) / 256, tn = a.N / 256;
  const int ntot = (MX ? a.K / 128 : a.K / BK) + a.K2 / BK;
  const SplitPlan pl = plan_split(a.M, a.N, ntot, a.K2, MX, DROP, device_cus(), allow_split ? so.split : 1,
                                  so.ws ? so.ws_bytes : 0);
  const int grid = pl.dp + pl.tail * pl.split;
  hipLaunchKernelGGL((gemm_nt_v5_kernel<DBG, DROP, MX, SP>), dim3(grid), dim3(512), 0, s, a, tm, tn, pl.dp, pl.split,
                     so.ws, g_v5_gm);
  OSPO_CHECK_LAUNCH();
  if (pl.tail) {
    hipLaunchKernelGGL(splitk_fixup_kernel, dim3(pl.tail * 32), dim3(256), 0, s, a, tm, tn, pl.dp, pl.split,
                       (const float*)so.ws, g_v5_gm);
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}

#ifdef OSPO_ABLATION
// ----------------------------------------------------------------------------
// v6 (ablation build only, variant 32; rejected): the SP8 schedule as a PERSISTENT kernel with the epilogue
// inside the ping-pong.  Bit-identical to v5 on every epilogue, but 0.2-4 % slower on the step shapes and
// 20-30 % on single-round ones (profiles/r03/rejected/gemm_v6_persistent_ab.jsonl).
//
// v5 runs one work unit (a 256 x 256 tile, or a split-K piece of a tail tile) per workgroup: each
// unit pays a prologue (the first K-tiles' DMA, ~1.8 us) and an LDS-staged epilogue (accumulators ->
// LDS ~2 us, 16-B row stores ~2.2 us, ~10 us with a residual) during which no MFMA runs -- ~15 % of a
// 4096-deep unit.  Here gridDim.x <= CUs workgroups walk the same unit list (virtual id v = blockIdx.x
// + k * gridDim.x, mapped to tiles exactly as v5 maps blockIdx, so the XCD placement is unchanged):
//  * the LDS ring runs on across units: the last two K-tiles of a unit stage the next unit's first
//    two (the v5 prologue pattern), so a unit starts with its operands landed;
//  * the epilogue stores straight from the accumulators (8-B bf16 / 16-B fp32 stores per lane, no
//    LDS, no barrier), each wave group in its own R section right after its last M section, so it
//    overlaps the other group's MFMAs;
//  * the B fragments of a wave are columns {n * 64 + wn * 16 + 0..15} of each B half (v5: wn * 32 +
//    n * 16): a head's RoPE partner columns d and d + 64 sit in the same lane, so the RoPE epilogue
//    needs no exchange.
// Every output element gets the same MFMA operands in the same K order as v5: results are
// bit-identical (the split-K partial tiles and their fixup are v5's).
// The first wait after an epilogue keeps the standard count (vmcnt counts loads, stores and LDS-DMA together
// in issue order; the epilogue's stores sit between the next unit's B(1) and A(1) pieces, so the count is
// stricter there -- it also waits for the older stores -- never looser).

typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));  // the buffer-intrinsic 8-B operand

// byte offset of the 16-B piece (h, i) of a lane in a main K-tile-0 half (rows clamped, chunks XOR-swizzled);
// a device function: the same code as a lambda called from another lambda loses the kernel's host stub
__device__ __forceinline__ uint32_t v6_voff(const GemmArgs& args, int um0, int un0, int h, int i, int wave, int rr8,
                                            int c8) {
  const bool isA = h < 2;
  const int row = (h & 1) * 128 + (wave * 2 + i) * 8 + rr8;
  const int g = min((isA ? um0 : un0) + row, isA ? args.M - 1 : args.N - 1);
  return (uint32_t)g * (uint32_t)(isA ? args.lda : args.ldb) * 2u + ((c8 ^ rr8) << 4);
}

// RES: the residual-add epilogue (o / down projections); else the plain / RoPE one (one instance each keeps
// the register allocation of the other's epilogue out of the loop).
template <bool DROP, bool RES>
__global__ __launch_bounds__(512) void gemm_nt_v6_kernel(const GemmArgs args, int tiles_m, int tiles_n, int dp,
                                                         int split, float* __restrict__ ws, int GM, int n_units) {
  constexpr int HALF = 16384, SLOT = 4 * HALF;  // half order in a slot: A0 A1 B0 B1
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool g1 = wave >= 4;
  const int wm = wave >> 2, wn = wave & 3;
  const int rr8 = lane >> 3, c8 = lane & 7;
  const int frow = lane & 15, fcol = lane >> 4;
  const int nt1 = args.K / BK, nt2 = args.K2 / BK, ntot = nt1 + nt2;
  const int Mlast = args.M - 1, Nlast = args.N - 1;
  const int G = gridDim.x;

  // ---- the unit list (v5's blockIdx mapping)
  int v = blockIdx.x;
  if (v >= n_units) return;
  int m0, n0, tb, nt, part;
  auto unit_of = [&](int vv, int& um0, int& un0, int& utb, int& unt, int& upart) {
    upart = -1;
    if (vv < dp) {
      const int xcd = vv & 7, slot = vv >> 3, q = dp >> 3, r = dp & 7;
      const int L = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
      v5_tile(L, tiles_m, tiles_n, um0, un0, GM);
      utb = 0;
      unt = ntot;
    } else {
      const int u = vv - dp, z = u % split;
      upart = u;
      v5_tile(dp + u / split, tiles_m, tiles_n, um0, un0, GM);
      utb = (int)((long)ntot * z / split);
      unt = (int)((long)ntot * (z + 1) / split) - utb;
    }
  };
  unit_of(v, m0, n0, tb, nt, part);

  // ---- staging: buffer_load ... lds from per-lane offsets (main tiles), global_load_lds (extension tiles)
  const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
      (void*)args.A, 0, (int)(((long)Mlast * args.lda + args.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
      (void*)args.B, 0, (int)(((long)Nlast * args.ldb + args.K) * 2), 0x00020000);
  // lane-derived values re-derived from an opaque copy of the lane id where used, so the compiler
  // cannot hoist per-lane 64-bit addresses out of the unit loop (they would be spilled)
  auto opaque_lane = [&]() __attribute__((always_inline)) {
    int l = lane;
    asm volatile("" : "+v"(l));
    return l;
  };
  uint32_t voff[4][2];  // the current unit's main-tile offsets (the next unit's are computed where used)
  auto make_voff = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) voff[h][i] = v6_voff(args, m0, n0, h, i, wave, rr8, c8);
  };
  make_voff();
  auto abs_t = [&](int utb, int tl) {
    const int q = utb + tl;
    return DROP ? (q < nt2 ? nt1 + q : q - nt2) : q;
  };
  // one half-tile (2 pieces per wave) of local tile tl of a unit into slot parity par; CUR: the current
  // unit (precomputed offsets), else the unit at (um0, un0)
  // (CUR is a plain bool, constant after inlining: a generic lambda here loses the kernel's host stub)
  auto stage_piece = [&](bool CUR, int um0, int un0, int utb, int tl, int h, int par)
      __attribute__((always_inline)) {
    char* dst = smem + par * SLOT + h * HALF;
    const int t = abs_t(utb, tl);
    if (t < nt1) {
      int ol = 0;
      if (!CUR) ol = opaque_lane();
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(h < 2 ? rsA : rsB, (LDS_AS void*)(dst + (wave * 2 + i) * 1024), 16,
                                                 CUR ? voff[h][i] : v6_voff(args, um0, un0, h, i, wave, (ol >> 3) & 7, ol & 7),
                                                 t * 128, 0, 0);
    } else {
      const int ol = opaque_lane(), rr8 = (ol >> 3) & 7, c8 = ol & 7;
      const bool isA = h < 2;
      const bf16* base = isA ? args.A2 : args.B2;
      const int ld = isA ? args.lda2 : args.ldb2;
      const int k0 = (t - nt1) * BK;
      const int row0 = (isA ? um0 : un0) + (h & 1) * 128;
      const int last = isA ? Mlast : Nlast;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = wave * 2 + i;
        const int g = min(row0 + p * 8 + rr8, last);
        glds16(base + (long)g * ld + k0 + ((c8 ^ rr8) << 3), dst + p * 1024);
      }
    }
  };

  f32x4 acc[4][4][2];
  bf16x8 af[4][2];
  bf16x8 bsp[2][2][2];  // [B half][n][k-substep]: the whole K-tile's B fragments
  auto zero_acc = [&]() {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[q][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- prologue of the first unit: tile 0 complete, B0 B1 of tile 1 in flight (v5 BAL)
  int gb = 0;  // global index of the current unit's tile 0 (slot parity of its tile t = (gb + t) & 1)
  stage_piece(true, m0, n0, tb, 0, 2, 0);
  stage_piece(true, m0, n0, tb, 0, 3, 0);
  stage_piece(true, m0, n0, tb, 0, 0, 0);
  stage_piece(true, m0, n0, tb, 0, 1, 0);
  if (nt > 1) {
    stage_piece(true, m0, n0, tb, 1, 2, 1);
    stage_piece(true, m0, n0, tb, 1, 3, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (g1) {  // the ping-pong offset
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  for (;;) {
    const int vn = v + G;
    const bool has_next = vn < n_units;
    int m0n = 0, n0n = 0, tbn = 0, ntn = 0, partn = -1;
    if (has_next) {
      unit_of(vn, m0n, n0n, tbn, ntn, partn);
    }
    zero_acc();

    // one K-tile = 2 phases of 32 MFMAs per wave (v5 run_tile_sp5).  ST: t+1, t+2 are main tiles of this
    // unit (constant waits, fast staging, no branch); PAR: slot parity of tile t when known (else -1).
    auto run_tile = [&](int t, auto steady, auto parity) __attribute__((always_inline)) {
      constexpr bool ST = decltype(steady)::value;
      constexpr int PAR = decltype(parity)::value;
      const int par = PAR >= 0 ? PAR : ((gb + t) & 1);
      const char* slot = smem + par * SLOT;
      // tiles t+1 / t+2 in the concatenated sequence: this unit's, else the next unit's first two
      const bool n1 = ST || t + 1 < nt || has_next;
      const bool n2 = ST || t + 2 < nt || (has_next && t + 2 - nt < ntn);
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const char* la = slot + p * HALF;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int s = 0; s < 2; ++s)
            af[i][s] = *reinterpret_cast<const bf16x8*>(la + mmaj_off(wm * 64 + i * 16 + frow, 4 * s + fcol));
        if (p == 0) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                bsp[h][n][s] = *reinterpret_cast<const bf16x8*>(slot + (2 + h) * HALF +
                                                                 mmaj_off(n * 64 + wn * 16 + frow, 4 * s + fcol));
        }
        // refills: A0 A1 of tile t+1 in R(t,0), B0 B1 of tile t+2 in R(t,1)
        if (ST) {
          if (p == 0) {
            stage_piece(true, m0, n0, tb, t + 1, 0, PAR >= 0 ? 1 - PAR : 1 - par);
            stage_piece(true, m0, n0, tb, t + 1, 1, PAR >= 0 ? 1 - PAR : 1 - par);
          } else {
            stage_piece(true, m0, n0, tb, t + 2, 2, par);
            stage_piece(true, m0, n0, tb, t + 2, 3, par);
          }
        } else {
          if (p == 0 && n1) {
            if (t + 1 < nt) {
              stage_piece(true, m0, n0, tb, t + 1, 0, 1 - par);
              stage_piece(true, m0, n0, tb, t + 1, 1, 1 - par);
            } else {
              stage_piece(false, m0n, n0n, tbn, t + 1 - nt, 0, 1 - par);
              stage_piece(false, m0n, n0n, tbn, t + 1 - nt, 1, 1 - par);
            }
          }
          if (p == 1 && n2) {
            if (t + 2 < nt) {
              stage_piece(true, m0, n0, tb, t + 2, 2, par);
              stage_piece(true, m0, n0, tb, t + 2, 3, par);
            } else {
              stage_piece(false, m0n, n0n, tbn, t + 2 - nt, 2, par);
              stage_piece(false, m0n, n0n, tbn, t + 2 - nt, 3, par);
            }
          }
        }
        // counted waits: p 0 -> A1(t) (8 newer: B(t+1), A(t+1)); 
        // p 1 -> A0 B of t+1 (6 newer: A1(t+1), B(t+2))
        auto waits = [&]() __attribute__((always_inline)) {
          if (ST) {
            if (p == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
          } else {
            if (p == 0) {
              // tile 0 after an epilogue: its EPI_STORES stores sit between B(1) and A(1)
              if (n1 && t == 0 && gb > 0) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");  // 8 + EPI_STORES
              else wait_vmcnt_exact(n1 ? 8 : 0);
            }
            if (p == 1 && n1) wait_vmcnt_exact(n2 ? 6 : 2);
          }
        };
        if (g1) waits();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int j = 2 * p + q;  // p 0: quadrants j 0 (ia 0, ib 0), 1 (0, 1); p 1: j 2 (1, 1), 3 (1, 0)
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int s = 0; s < 2; ++s)
                acc[j][i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bsp[ib][n][s], af[i][s], acc[j][i][n], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        if (!g1) waits();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
    };
    using PRT = std::integral_constant<int, -1>;
    using STT = std::integral_constant<bool, true>;
    using STF = std::integral_constant<bool, false>;
    // with dropout the extension tiles come first (tb == 0); their masked sum is scaled between the loops
    const int pre = (DROP && tb == 0) ? (nt2 < nt ? nt2 : nt) : 0;
    int t = 0;
    for (; t < pre; ++t) run_tile(t, STF{}, PRT{});
    if (t == 0) run_tile(t++, STF{}, PRT{});  // tile 0 waits with the previous epilogue's stores counted
    if (DROP && pre > 0) {
      const int ol = opaque_lane(), gq = ol >> 4, lq = ol & 15;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ia = (j >= 2) ? 1 : 0;
        const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int n = 0; n < 2; ++n) {
            const uint32_t m = (uint32_t)(m0 + ia * 128 + wm * 64 + i * 16 + lq);
            const uint32_t c = (uint32_t)(n0 + ib * 128 + n * 64 + wn * 16 + 4 * gq);
            bool keep[4];
            drop_keep_pairs<2>(m * (uint32_t)args.drop_ld + c, args.drop_seed, args.drop_thresh, keep);  // c % 4 == 0
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[j][i][n][e] *= keep[e] ? args.drop_scale : 0.f;
          }
      }
    }
    // steady tiles: t+1 and t+2 are main tiles of this unit (non-dropout: the extension tiles come last)
    const int main_lim = DROP ? nt : min(nt, max(0, nt1 - tb));
    if (((gb + t) & 1) && t < main_lim - 2) run_tile(t++, STT{}, PRT{});
    for (; t + 1 < main_lim - 2; t += 2) {
      run_tile(t, STT{}, std::integral_constant<int, 0>{});
      run_tile(t + 1, STT{}, std::integral_constant<int, 1>{});
    }
    for (; t < main_lim - 2; ++t) run_tile(t, STT{}, PRT{});
    for (; t < nt; ++t) run_tile(t, STF{}, PRT{});

    // ---- epilogue: straight from the accumulators (lane: row m0 + ia*128 + wm*64 + i*16 + l16, columns
    // n0 + ib*128 + n*64 + wn*16 + 4g .. +3), no LDS, no barrier.  Every wave issues exactly EPI_STORES (32)
    // stores, unconditionally (bf16 rows >= M: buffer stores past num_records, dropped), and waits for all of its
    // epilogue loads before its last store: the next unit's first wait counts them (run_tile).
    {
      const int ol = opaque_lane(), g = ol >> 4, l16 = ol & 15;
      if (part >= 0) {  // split-K piece: the raw fp32 partial tile [256][256] (v5's layout)
        float* wt = ws + (long)part * 65536;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ia = (j >= 2) ? 1 : 0;
          const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int ml = ia * 128 + wm * 64 + i * 16 + l16;
              const int nl = ib * 128 + n * 64 + wn * 16 + 4 * g;
              *reinterpret_cast<f32x4*>(wt + ml * 256 + nl) = acc[j][i][n];
            }
        }
      } else {
        const __amdgpu_buffer_rsrc_t rsC =
            __builtin_amdgcn_make_buffer_rsrc(args.C, 0, (int)((long)args.M * args.ldc * 2), 0x00020000);
        auto st8 = [&](int m, int c, uint2 v) __attribute__((always_inline)) {
          u32x2v w;
          w.x = v.x;
          w.y = v.y;
          __builtin_amdgcn_raw_buffer_store_b64(w, rsC, (uint32_t)m * (uint32_t)args.ldc * 2u + (uint32_t)c * 2u, 0, 0);
        };
        if (!RES && n0 < args.rope_cols) {
          // RoPE on the bf16-rounded products (HF rotate-half, per-op bf16 rounding as v5's epilogue): the
          // partner of head column d < 64 (n = 0) is d + 64 (n = 1), same lane.  cos / sin tables [T][64].
          uint2 cw[2][4], sw[2][4];
#pragma unroll
          for (int ia = 0; ia < 2; ++ia)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int m = min(m0 + ia * 128 + wm * 64 + i * 16 + l16, Mlast);
              const int tt = m % args.rope_T;
              cw[ia][i] = *reinterpret_cast<const uint2*>(args.rope_cs + (long)tt * 64 + wn * 16 + 4 * g);
              sw[ia][i] = *reinterpret_cast<const uint2*>(args.rope_sn + (long)tt * 64 + wn * 16 + 4 * g);
            }
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ia = (j >= 2) ? 1 : 0;
            const int ib = (j == 1 || j == 2) ? 1 : 0;
            const bool rope_half = n0 + ib * 128 < args.rope_cols;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int m = m0 + ia * 128 + wm * 64 + i * 16 + l16;
              const int c = n0 + ib * 128 + wn * 16 + 4 * g;
              uint2 o1, o2;
              o1.x = pack2(acc[j][i][0][0], acc[j][i][0][1]);
              o1.y = pack2(acc[j][i][0][2], acc[j][i][0][3]);
              o2.x = pack2(acc[j][i][1][0], acc[j][i][1][1]);
              o2.y = pack2(acc[j][i][1][2], acc[j][i][1][3]);
              if (rope_half) {
                const uint32_t x1w[2] = {o1.x, o1.y}, x2w[2] = {o2.x, o2.y};
                const uint32_t cww[2] = {cw[ia][i].x, cw[ia][i].y}, sww[2] = {sw[ia][i].x, sw[ia][i].y};
                uint32_t r1w[2], r2w[2];
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                  float r1[2], r2[2];
#pragma unroll
                  for (int hh = 0; hh < 2; ++hh) {
                    const int sh = 16 * hh;
                    const float x1 = bits2f((x1w[qq] >> sh) & 0xffff), x2 = bits2f((x2w[qq] >> sh) & 0xffff);
                    const float cf = bits2f((cww[qq] >> sh) & 0xffff), sf = bits2f((sww[qq] >> sh) & 0xffff);
                    r1[hh] = round_bf(x1 * cf) + round_bf(-x2 * sf);
                    r2[hh] = round_bf(x2 * cf) + round_bf(x1 * sf);
                  }
                  r1w[qq] = pack2(r1[0], r1[1]);
                  r2w[qq] = pack2(r2[0], r2[1]);
                }
                o1 = uint2{r1w[0], r1w[1]};
                o2 = uint2{r2w[0], r2w[1]};
              }
              st8(m, c, o1);
              st8(m, c + 64, o2);
            }
          }
        } else {
          // bias (per column) and alpha before the bf16 rounding; the bf16 residual after it (v5's order)
          float b4[2][2][4];
#pragma unroll
          for (int ib = 0; ib < 2; ++ib)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int e = 0; e < 4; ++e)
                b4[ib][n][e] = args.bias ? bf2f(args.bias[n0 + ib * 128 + n * 64 + wn * 16 + 4 * g + e]) : 0.f;
          // residual: quadrant j + 1's 8 loads in flight while quadrant j is stored (rows >= M read as 0)
          u32x2v rv[2][4][2];
          __amdgpu_buffer_rsrc_t rsR;
          auto load_res = [&](int j, u32x2v (&r)[4][2]) __attribute__((always_inline)) {
            const int ia = (j >= 2) ? 1 : 0;
            const int ib = (j == 1 || j == 2) ? 1 : 0;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int n = 0; n < 2; ++n) {
                const int m = m0 + ia * 128 + wm * 64 + i * 16 + l16;
                const int c = n0 + ib * 128 + n * 64 + wn * 16 + 4 * g;
                r[i][n] = __builtin_amdgcn_raw_buffer_load_b64(
                    rsR, (uint32_t)m * (uint32_t)args.ldr * 2u + (uint32_t)c * 2u, 0, 0);
              }
          };
          if (RES) {
            rsR = __builtin_amdgcn_make_buffer_rsrc((void*)args.res, 0, (int)((long)args.M * args.ldr * 2),
                                                    0x00020000);
            load_res(0, rv[0]);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int ia = (j >= 2) ? 1 : 0;
            const int ib = (j == 1 || j == 2) ? 1 : 0;
            if (RES) {
              if (j < 3) load_res(j + 1, rv[(j + 1) & 1]);
              // quadrant j's loads done: newer are (j > 0) quadrant j-1's 8 stores and (j < 3) quadrant j+1's loads
              if (j == 0 || j == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
              else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
              for (int n = 0; n < 2; ++n) {
                const int m = m0 + ia * 128 + wm * 64 + i * 16 + l16;
                const int c = n0 + ib * 128 + n * 64 + wn * 16 + 4 * g;
                const f32x4 a4 = acc[j][i][n];
                uint2 pk;
                pk.x = pack2(a4[0] * args.alpha + b4[ib][n][0], a4[1] * args.alpha + b4[ib][n][1]);
                pk.y = pack2(a4[2] * args.alpha + b4[ib][n][2], a4[3] * args.alpha + b4[ib][n][3]);
                if (RES) {
                  const u32x2v r = rv[j & 1][i][n];
                  pk.x = pack2(bits2f(pk.x & 0xffff) + bits2f(r.x & 0xffff), bits2f(pk.x >> 16) + bits2f(r.x >> 16));
                  pk.y = pack2(bits2f(pk.y & 0xffff) + bits2f(r.y & 0xffff), bits2f(pk.y >> 16) + bits2f(r.y >> 16));
                }
                st8(m, c, pk);
              }
          }
        }
      }
    }
    if (!has_next) break;
    gb += nt;
    v = vn;
    m0 = m0n; n0 = n0n; tb = tbn; nt = ntn; part = partn;
    make_voff();
  }
  if (!g1) {  // re-align the barrier count
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
}


template <bool DROP>
int launch_v6(const GemmArgs& a, hipStream_t s, const SplitOpts& so) {
  if (a.N % 256) return OSPO_ERR_SHAPE;
  const int ntot = a.K / BK + a.K2 / BK;
  // v6 needs 32-bit buffer offsets and >= 2 K-tiles per unit, and has no fused SwiGLU-backward epilogue
  if (a.swg_gu || ntot < 2 || (long)a.M * a.lda * 2 >= (1L << 31) || (long)a.N * a.ldb * 2 >= (1L << 31) ||
      ((long)a.M + 256) * a.ldc * 2 >= (1L << 31) || (a.res && ((long)a.M + 256) * a.ldr * 2 >= (1L << 31)))
    return launch_v5<0, DROP, false, 8>(a, s, so);
  const int tm = (a.M + 255) / 256, tn = a.N / 256;
  const int cus = device_cus();
  const SplitPlan pl = plan_split(a.M, a.N, ntot, a.K2, false, DROP, cus, so.split, so.ws ? so.ws_bytes : 0);
  const int units = pl.dp + pl.tail * pl.split;
  const int grid = units > cus ? std::max(8, cus / 8 * 8) : units;  // a multiple of 8: v & 7 = blockIdx.x & 7
  if (!DROP && a.res)  // (the dropout entry point takes no residual)
    hipLaunchKernelGGL((gemm_nt_v6_kernel<DROP, !DROP>), dim3(grid), dim3(512), 0, s, a, tm, tn, pl.dp, pl.split,
                       so.ws, g_v5_gm, units);
  else
    hipLaunchKernelGGL((gemm_nt_v6_kernel<DROP, false>), dim3(grid), dim3(512), 0, s, a, tm, tn, pl.dp, pl.split,
                       so.ws, g_v5_gm, units);
  OSPO_CHECK_LAUNCH();
  if (pl.tail) {
    hipLaunchKernelGGL(splitk_fixup_kernel, dim3(pl.tail * 32), dim3(256), 0, s, a, tm, tn, pl.dp, pl.split,
                       (const float*)so.ws, g_v5_gm);
    OSPO_CHECK_LAUNCH();
  }
  return OSPO_OK;
}
#endif  // OSPO_ABLATION

template <int FM, int STAGES, bool REMAP, bool PRIO, int WM = 2, int WN = 4, int FN = 4, int DBG = 0>
int launch_v3(const GemmArgs& a, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  if (a.N % BN) return OSPO_ERR_SHAPE;
  const int tm = (a.M + BM - 1) / BM, tn = a.N / BN;
  hipLaunchKernelGGL((gemm_nt_v3_kernel<FM, STAGES, REMAP, PRIO, WM, WN, FN, DBG>), dim3(tm * tn), dim3(64 * WM * WN), 0,
                     s, a, tm, tn);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

#ifdef OSPO_ABLATION
uint32_t* g_dbg_buf = nullptr;  // variant 29: s_memtime stamps, 16 words per wave
int g_gemm_variant = 0;  // 0 = SP schedule + split-K tail (default); 17 = the 8-phase schedule; others: A/B, see dispatch
#else
[[maybe_unused]] constexpr int g_gemm_variant = 0;  // the product library runs the default schedule only
#endif

// the bf16 256 x 256 schedule every entry point runs (the ablation build can switch it for A/B)
template <bool DROP>
int launch_default(const GemmArgs& a, hipStream_t s, const SplitOpts& so) {
#ifdef OSPO_ABLATION
  if (g_gemm_variant == 17) return launch_v5<0, DROP>(a, s, so);
  if (g_gemm_variant == 14) return launch_v5<0, DROP, false, 1>(a, s, so);
  if (g_gemm_variant == 24) return launch_v5<0, DROP, false, 5>(a, s, so);
  if (g_gemm_variant == 25) return launch_v5<0, DROP, false, 6>(a, s, so);
  if (g_gemm_variant == 26) return launch_v5<0, DROP, false, 7>(a, s, so);
  if (g_gemm_variant == 27) return launch_v5<0, DROP, false, 8>(a, s, so);
  if (g_gemm_variant == 28) return launch_v5<0, DROP, false, 9>(a, s, so);
  if (g_gemm_variant == 32) return launch_v6<DROP>(a, s, so);  // persistent SP8 (rejected)
  if (g_gemm_variant == 41) {
    const int r = launch_w4<DROP, 1>(a, s, so);
    if (r != OSPO_ERR_UNSUPPORTED) return r;
  }
  if (g_gemm_variant == 42) {  // w4 with workgroup stamps (tools/w4_stamps.py)
    GemmArgs d = a;
    d.dbg = g_dbg_buf;
    const int r = launch_w4<DROP, 2>(d, s, so);
    if (r != OSPO_ERR_UNSUPPORTED) return r;
  }
  if constexpr (!DROP) {  // schedule variants 43.. = gen_gemm_w4.py ABL_VARIANTS 1..
    int r = OSPO_ERR_UNSUPPORTED;
    if (g_gemm_variant == 43) r = launch_w4<false, 0, 1>(a, s, so);
    if (g_gemm_variant == 44) r = launch_w4<false, 0, 2>(a, s, so);
    if (g_gemm_variant == 45) r = launch_w4<false, 0, 3>(a, s, so);
    if (g_gemm_variant == 46) r = launch_w4<false, 0, 4>(a, s, so);
    if (g_gemm_variant == 47) r = launch_w4<false, 0, 5>(a, s, so);
    if (g_gemm_variant == 48) r = launch_w4<false, 0, 6>(a, s, so);
    if (g_gemm_variant == 49) r = launch_w4<false, 0, 7>(a, s, so);
    if (g_gemm_variant == 50) r = launch_w4<false, 0, 8>(a, s, so);
    if (g_gemm_variant == 51) r = launch_w4<false, 0, 9>(a, s, so);
    if (r != OSPO_ERR_UNSUPPORTED) return r;
  }
  if (g_gemm_variant == 27) return launch_v5<0, DROP, false, 8>(a, s, so);  // the round-3 default (SP8)
#endif
  // the 4-wave hand-scheduled kernel where it applies (gemm_w4.h), else SP8
  const int r = launch_w4<DROP>(a, s, so);
  if (r != OSPO_ERR_UNSUPPORTED) return r;
  return launch_v5<0, DROP, false, 8>(a, s, so);
}

// the MXFP8 256 x 256 schedule (the ablation build can switch it: 17 = 8-phase, 14 = SP1)
template <bool DROP>
int launch_mx(const GemmArgs& a, hipStream_t s, const SplitOpts& so) {
#ifdef OSPO_ABLATION
  if (g_gemm_variant == 17) return launch_v5<0, DROP, true>(a, s, so);
  if (g_gemm_variant == 14) return launch_v5<0, DROP, true, 1>(a, s, so);
  if constexpr (!DROP) {
    // variant 52: the 4-wave hand-scheduled loop (w4_mx programs).  Bit-identical to SP8 under the same split
    // (tools/w4mx_check.py) and within 1 % per shape alone, but the config-5 step ran 1.1 % slower with it
    // (profiles/r04/w4mx_check.log, step_mx8_w4_ab.txt): not the default.
    if (g_gemm_variant == 52) {
      const int r = launch_w4<false, 0, 0, true>(a, s, so);
      if (r != OSPO_ERR_UNSUPPORTED) return r;
    }
  }
#endif
  return launch_v5<0, DROP, true, 8>(a, s, so);
}

// NT tile: 256 x 256 (8-phase, split-K tail) whenever N % 256 == 0, else the 64 x 64 simple kernel.
int pick_nt_tile(int M, int N) {
  (void)M;
  return (N % 256) ? 64 : 256;
}

}  // namespace

extern "C" int ospo_gemm_nt_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                                 const void* A2, int lda2, const void* B2, int ldb2, int K2, float alpha,
                                 const void* bias, const void* residual, int ldr, void* C, int ldc, int tail_split,
                                 void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!A || !B || !C) return OSPO_ERR_ARG;
  if (tail_split < 0 || tail_split > 8 || (ws && !aligned16(ws))) return OSPO_ERR_ARG;
  const SplitOpts so{tail_split, (float*)ws, ws ? ws_bytes : 0};
  if (M <= 0 || N <= 0 || K <= 0 || K % BK || K2 < 0 || K2 % BK || N % 64) return OSPO_ERR_SHAPE;
  if (K2 > 0 && (!A2 || !B2)) return OSPO_ERR_ARG;
  if (lda < K || ldb < K || ldc < N || (lda % 8) || (ldb % 8) || (ldc % 8)) return OSPO_ERR_SHAPE;
  if (K2 > 0 && (lda2 < K2 || ldb2 < K2 || lda2 % 8 || ldb2 % 8)) return OSPO_ERR_SHAPE;
  if (residual && (ldr < N || ldr % 8)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B) || !aligned16(C) || (residual && !aligned16(residual)) ||
      (K2 > 0 && (!aligned16(A2) || !aligned16(B2))))
    return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, (const bf16*)A2, (const bf16*)B2, lda, ldb, lda2, ldb2,
             M, N, K, K2, alpha, (const bf16*)bias, (const bf16*)residual, ldr, C, ldc, 1, 0, 0};
  const int tile = pick_nt_tile(M, N);
  if (tile == 64) return launch<2, 2, 2, 2, false, false, EPI_BF16>(a, stream);
#ifndef OSPO_ABLATION
  return launch_default<false>(a, stream, so);  // w4 (gemm_w4.h), else SP8; + split-K tail
#else
  switch (g_gemm_variant) {
    // A/B alternatives (tools/gemm_bench.py); results identical, schedules differ
    case 1: return launch<2, 4, 8, 4, false, false, EPI_BF16>(a, stream);            // simple double-buffered
    case 2: return launch<2, 4, 5, 4, false, false, EPI_BF16>(a, stream);            // simple, 160 x 256
    case 3: return launch_v3<8, 2, true, true>(a, stream);                           // v3 register-prefetch
    case 4: return launch_v4<8, 3>(a, stream);                                       // v4 BK=32 ring
    case 5: return launch_v5<0>(a, stream, so, false);                                   // 8-phase, no split tail
    // decompositions (results invalid): 10 no loads / 11 no MFMA (simple); 12 no loads / 13 no MFMA (8-phase)
    case 10: return launch<2, 4, 8, 4, false, false, EPI_BF16, 1>(a, stream);
    case 11: return launch<2, 4, 8, 4, false, false, EPI_BF16, 2>(a, stream);
    case 12: return launch_v5<1>(a, stream, so, false);
    case 13: return launch_v5<2>(a, stream, so, false);
    // SP schedule (2 phases of 32 MFMAs per K-tile): 14 + split tail, 15 no loads, 16 no MFMA
    case 14: return launch_v5<0, false, false, 1>(a, stream, so, true);  // SP1 (2 + 6 refills, generic staging)
    case 15: return launch_v5<1, false, false, 1>(a, stream, so, false);
    case 16: return launch_v5<2, false, false, 1>(a, stream, so, false);
    case 18: return launch_v5<0, false, false, 2>(a, stream, so, true);  // SP without s_setprio
    case 19: return launch_v5<0, false, false, 3>(a, stream, so, true);  // SP, refills ahead of the reads
    case 24: return launch_v5<0, false, false, 5>(a, stream, so, true);  // SP5: 4 + 4 refills, buffer-offset staging
    case 25: return launch_v5<0, false, false, 6>(a, stream, so, true);  // SP, 4 + 4 refills, generic staging
    case 26: return launch_v5<0, false, false, 7>(a, stream, so, true);  // SP, 2 + 6 refills, buffer-offset staging
    case 27: return launch_v5<0, false, false, 8>(a, stream, so, true);  // SP8 (SP5 unrolled by 2): the round-3 default
    case 28: return launch_v5<0, false, false, 9>(a, stream, so, true);  // SP8 + B0 of the next tile read early
    case 29: { GemmArgs d = a; d.dbg = g_dbg_buf; return launch_v5<4, false, false, 8>(d, stream, so, false); }  // SP8 + stamps
    case 30: { GemmArgs d = a; d.dbg = g_dbg_buf; return launch_v5<5, false, false, 8>(d, stream, so, false); }  // SP8 + phase stamps
    case 17: return launch_v5<0>(a, stream, so, true);                                   // 8-phase + split-K tail
    case 32: return launch_v6<false>(a, stream, so);                                  // persistent SP8 (v6, rejected)
    case 40: case 41: case 42: case 43: case 44: case 45: case 46: case 47: case 48: case 49: case 50: case 51: case 52:
      return launch_default<false>(a, stream, so);                                   // 4-wave hand-scheduled (w4)
    default: return launch_default<false>(a, stream, so);                            // w4 / SP8 + split-K tail
  }
#endif
}

extern "C" int ospo_gemm_nt_rope_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                                      const void* A2, int lda2, const void* B2, int ldb2, int K2, void* C, int ldc,
                                      const void* rope_cos, const void* rope_sin, int T, int rope_cols, int tail_split,
                                      void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!A || !B || !C || !rope_cos || !rope_sin) return OSPO_ERR_ARG;
  if (tail_split < 0 || tail_split > 8 || (ws && !aligned16(ws))) return OSPO_ERR_ARG;
  const SplitOpts so{tail_split, (float*)ws, ws ? ws_bytes : 0};
  if (M <= 0 || N <= 0 || K <= 0 || K % BK || K2 < 0 || K2 % BK || N % 256 || T <= 0) return OSPO_ERR_SHAPE;
  if (rope_cols < 0 || rope_cols % 128 || rope_cols > N) return OSPO_ERR_SHAPE;
  if (K2 > 0 && (!A2 || !B2)) return OSPO_ERR_ARG;
  if (lda < K || ldb < K || ldc < N || (lda % 8) || (ldb % 8) || (ldc % 8)) return OSPO_ERR_SHAPE;
  if (K2 > 0 && (lda2 < K2 || ldb2 < K2 || lda2 % 8 || ldb2 % 8)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B) || !aligned16(C) || !aligned16(rope_cos) || !aligned16(rope_sin) ||
      (K2 > 0 && (!aligned16(A2) || !aligned16(B2))))
    return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, (const bf16*)A2, (const bf16*)B2, lda, ldb, lda2, ldb2,
             M, N, K, K2, 1.f, nullptr, nullptr, 0, C, ldc, 1, 0, 0};
  a.rope_cs = (const bf16*)rope_cos;
  a.rope_sn = (const bf16*)rope_sin;
  a.rope_T = T;
  a.rope_cols = rope_cols;
  // split-K tail fixups apply the RoPE epilogue too
  return launch_default<false>(a, stream, so);
}

extern "C" int ospo_gemm_nt_dropout_bf16(const void* A, int lda, const void* B, int ldb, int M, int N, int K,
                                         const void* A2, int lda2, const void* B2, int ldb2, int K2, void* C, int ldc,
                                         unsigned drop_seed, float drop_p, const void* keep_bits, int tail_split,
                                         void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!A || !B || !C || !A2 || !B2) return OSPO_ERR_ARG;
  if (tail_split < 0 || tail_split > 8 || (ws && !aligned16(ws))) return OSPO_ERR_ARG;
  const SplitOpts so{tail_split, (float*)ws, ws ? ws_bytes : 0};
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || K % BK || K2 <= 0 || K2 % BK) return OSPO_ERR_SHAPE;
  if (N % 256) return OSPO_ERR_UNSUPPORTED;
  if ((long)M * N > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
  if (lda < K || ldb < K || ldc < N || (lda % 8) || (ldb % 8) || (ldc % 8)) return OSPO_ERR_SHAPE;
  if (lda2 < K2 || ldb2 < K2 || lda2 % 8 || ldb2 % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B) || !aligned16(C) || !aligned16(A2) || !aligned16(B2)) return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, (const bf16*)A2, (const bf16*)B2, lda, ldb, lda2, ldb2,
             M, N, K, K2, 1.f, nullptr, nullptr, 0, C, ldc, 1, 0, 0};
  if (drop_p == 0.f)
    return launch_default<false>(a, stream, so);
  if (N & 1) return OSPO_ERR_SHAPE;  // mask pairs (drop_keep) start at even indices
  a.drop_seed = drop_seed;
  a.drop_thresh = drop_threshold(drop_p);
  a.drop_scale = 1.f / (1.f - drop_p);
  a.drop_ld = N;
  if (keep_bits) {
    if (!aligned16(keep_bits) || N % 128) return OSPO_ERR_ALIGN;  // 16-B rows of the bit block
    a.drop_bits = (const uint8_t*)keep_bits;
  }
  return launch_default<true>(a, stream, so);
}

extern "C" int ospo_gemm_nt_swiglu_bwd_bf16(const void* A, int lda, const void* B, int ldb, int M, int F, int K,
                                            const void* A2, int lda2, const void* B2, int ldb2, int K2,
                                            const void* gu, int ld_gu, void* dgu, int ld_dgu, unsigned drop_seed,
                                            float drop_p, int tail_split, void* ws, size_t ws_bytes,
                                            hipStream_t stream) {
  if (!A || !B || !gu || !dgu || (K2 > 0 && (!A2 || !B2))) return OSPO_ERR_ARG;
  if (tail_split < 0 || tail_split > 8 || (ws && !aligned16(ws))) return OSPO_ERR_ARG;
  const SplitOpts so{tail_split, (float*)ws, ws ? ws_bytes : 0};
  if (drop_p < 0.f || drop_p >= 1.f || (drop_p > 0.f && K2 <= 0)) return OSPO_ERR_ARG;
  if (M <= 0 || F <= 0 || K <= 0 || K % BK || K2 < 0 || K2 % BK) return OSPO_ERR_SHAPE;
  if (F % 256) return OSPO_ERR_UNSUPPORTED;
  if ((long)M * F > 0xFFFFFFFFL) return OSPO_ERR_SHAPE;  // 32-bit mask index
  if (lda < K || ldb < K || (lda % 8) || (ldb % 8) || ld_gu < 2 * F || ld_dgu < 2 * F || ld_gu % 8 || ld_dgu % 8)
    return OSPO_ERR_SHAPE;
  if (K2 > 0 && (lda2 < K2 || ldb2 < K2 || lda2 % 8 || ldb2 % 8)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B) || !aligned16(gu) || !aligned16(dgu) ||
      (K2 > 0 && (!aligned16(A2) || !aligned16(B2))))
    return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, (const bf16*)A2, (const bf16*)B2, lda, ldb, lda2, ldb2,
             M, F, K, K2, 1.f, nullptr, nullptr, 0, nullptr, 0, 1, 0, 0};
  a.swg_gu = (const bf16*)gu;
  a.swg_dgu = (bf16*)dgu;
  a.ld_gu = ld_gu;
  a.ld_dgu = ld_dgu;
  if (drop_p == 0.f)
    return launch_default<false>(a, stream, so);
  a.drop_seed = drop_seed;
  a.drop_thresh = drop_threshold(drop_p);
  a.drop_scale = 1.f / (1.f - drop_p);
  a.drop_ld = F;
  return launch_default<true>(a, stream, so);
}

extern "C" int ospo_gemm_nt_mx8(const void* A8, int lda, const void* Asc, const void* B8, int ldb, const void* Bsc,
                                int M, int N, int K, const void* A2, int lda2, const void* B2, int ldb2, int K2,
                                float alpha, const void* bias, const void* residual, int ldr, void* C, int ldc,
                                const void* rope_cos, const void* rope_sin, int rope_T, int rope_cols,
                                unsigned drop_seed, float drop_p, int tail_split, void* ws, size_t ws_bytes,
                                hipStream_t stream) {
  if (!A8 || !Asc || !B8 || !Bsc || !C) return OSPO_ERR_ARG;
  if (tail_split < 0 || tail_split > 8 || (ws && !aligned16(ws))) return OSPO_ERR_ARG;
  const SplitOpts so{tail_split, (float*)ws, ws ? ws_bytes : 0};
  if (M <= 0 || N <= 0 || K <= 0 || K % 128 || K2 < 0 || K2 % BK) return OSPO_ERR_SHAPE;
  if (N % 256) return OSPO_ERR_UNSUPPORTED;
  if (K2 > 0 && (!A2 || !B2)) return OSPO_ERR_ARG;
  if (lda < K || ldb < K || ldc < N || (lda % 16) || (ldb % 16) || (ldc % 8)) return OSPO_ERR_SHAPE;
  if (K2 > 0 && (lda2 < K2 || ldb2 < K2 || lda2 % 8 || ldb2 % 8)) return OSPO_ERR_SHAPE;
  if (residual && (ldr < N || ldr % 8)) return OSPO_ERR_SHAPE;
  if (!aligned16(A8) || !aligned16(B8) || !aligned16(C) || !aligned16(Asc) || !aligned16(Bsc) ||
      (residual && !aligned16(residual)) || (K2 > 0 && (!aligned16(A2) || !aligned16(B2))))
    return OSPO_ERR_ALIGN;
  const bool rope = rope_cols > 0, drop = drop_p > 0.f;
  if (drop_p < 0.f || drop_p >= 1.f) return OSPO_ERR_ARG;
  if (rope && (!rope_cos || !rope_sin || rope_T <= 0 || rope_cols % 128 || rope_cols > N || bias || residual ||
               alpha != 1.f || drop))
    return OSPO_ERR_ARG;
  if (drop && (K2 <= 0 || bias || residual || alpha != 1.f || (long)M * N > 0xFFFFFFFFL)) return OSPO_ERR_ARG;
  GemmArgs a{(const bf16*)A8, (const bf16*)B8, (const bf16*)A2, (const bf16*)B2, lda, ldb, lda2, ldb2,
             M, N, K, K2, alpha, (const bf16*)bias, (const bf16*)residual, ldr, C, ldc, 1, 0, 0};
  a.sa = (const uint32_t*)Asc;
  a.sb = (const uint32_t*)Bsc;
  if (rope) {
    a.rope_cs = (const bf16*)rope_cos;
    a.rope_sn = (const bf16*)rope_sin;
    a.rope_T = rope_T;
    a.rope_cols = rope_cols;
    return launch_mx<false>(a, stream, so);
  }
  if (drop) {
    a.drop_seed = drop_seed;
    a.drop_thresh = drop_threshold(drop_p);
    a.drop_scale = 1.f / (1.f - drop_p);
    a.drop_ld = N;
    return launch_mx<true>(a, stream, so);
  }
  return launch_mx<false>(a, stream, so);
}

// Box probe (bench.py box_probe, outside the timed region): the product's plain w4 program on A [M][K] . B [N][K]^T,
// never split, with s_memtime / s_memrealtime stamps per workgroup (gemm_w4.h DBG 2) -- the same K loop as every
// bf16 GEMM of the step, so its rate and in-kernel clock on fixed random data say how fast this box's GEMM runs.
extern "C" int ospo_gemm_clock_probe_bf16(const void* A, const void* B, void* C, int M, int N, int K, void* stamps,
                                          size_t stamps_bytes, hipStream_t stream) {
  if (!A || !B || !C || !stamps) return OSPO_ERR_ARG;
  if (M <= 0 || M % 256 || N <= 0 || N % 256 || K < 4 * BK || K % BK) return OSPO_ERR_SHAPE;
  if ((long)M * K * 2 >= (1L << 31) || (long)N * K * 2 >= (1L << 31)) return OSPO_ERR_SHAPE;
  if (stamps_bytes < (size_t)(M / 256) * (N / 256) * 8 * sizeof(uint64_t)) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B) || !aligned16(C) || !aligned16(stamps)) return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, nullptr, nullptr, K, K, 0, 0, M, N, K, 0, 1.f, nullptr, nullptr, 0, C, N,
             1, 0, 0};
  a.dbg = (uint32_t*)stamps;
  const SplitOpts so{1, nullptr, 0};
  return launch_w4<false, 2>(a, stream, so);
}

extern "C" size_t ospo_gemm_nt_ws_bytes(int M, int N, int K, int K2, int mx, int tail_split) {
  if (M <= 0 || N <= 0 || N % 256 || K <= 0 || K2 < 0 || tail_split < 0 || tail_split > 8) return 0;
  const int ntot = (mx ? K / 128 : K / BK) + K2 / BK;
  // with dropout the plan can only shrink (drop_ok), so the plan without it bounds the bytes
  const SplitPlan pl = plan_split(M, N, ntot, K2, mx != 0, false, device_cus(), tail_split, SIZE_MAX);
  const SplitPlan p4 = plan_split(M, N, ntot, K2, false, false, device_cus(), tail_split, SIZE_MAX, true);  // w4
  const size_t pieces = std::max((size_t)pl.tail * pl.split, mx ? (size_t)0 : (size_t)p4.tail * p4.split);
  return pieces * 65536 * sizeof(float);
}

#ifdef OSPO_ABLATION
extern "C" int ospo_gemm_set_debug_buffer(void* p) {
  g_dbg_buf = (uint32_t*)p;
  return OSPO_OK;
}

extern "C" int ospo_set_gemm_variant(int v) {
  if (v >= 20 && v <= 23) {  // L2 row-group size of the default schedule: 2, 8, 16, 4
    const int gms[4] = {2, 8, 16, 4};
    g_v5_gm = gms[v - 20];
    g_gemm_variant = 0;
    return OSPO_OK;
  }
  if (v < 0 || (v > 32 && (v < 40 || v > 52)) || (v > 5 && v < 10) || v == 20 || v == 21 || v == 22 || v == 23)
    return OSPO_ERR_ARG;
  g_v5_gm = 4;
  g_gemm_variant = v;
  return OSPO_OK;
}
#endif

extern "C" int ospo_gemm_nt_tile(int M, int N) { return pick_nt_tile(M, N); }

static int gemm_f32acc_impl(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor, int M, int N,
                            int K, int k_splits, float alpha, float* C, int ldc, int diag_nblk, int diag_r,
                            uint32_t drop_seed, float drop_p, hipStream_t stream,
                            const uint8_t* keep_bits = nullptr);

extern "C" int ospo_gemm_f32acc(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor,
                                int M, int N, int K, int k_splits, float alpha, float* C, int ldc,
                                int diag_nblk, int diag_r, hipStream_t stream) {
  return gemm_f32acc_impl(A, lda, a_kmajor, B, ldb, b_kmajor, M, N, K, k_splits, alpha, C, ldc, diag_nblk, diag_r, 0u,
                          0.f, stream);
}

extern "C" int ospo_gemm_f32acc_bdrop(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor,
                                      int M, int N, int K, int k_splits, float alpha, float* C, int ldc, int diag_nblk,
                                      int diag_r, uint32_t drop_seed, float drop_p, const void* keep_bits,
                                      hipStream_t stream) {
  if (!b_kmajor || !(drop_p > 0.f && drop_p < 1.f)) return OSPO_ERR_ARG;
  if (keep_bits && N % 8) return OSPO_ERR_SHAPE;  // whole bytes per 8 columns
  return gemm_f32acc_impl(A, lda, a_kmajor, B, ldb, b_kmajor, M, N, K, k_splits, alpha, C, ldc, diag_nblk, diag_r,
                          drop_seed, drop_p, stream, (const uint8_t*)keep_bits);
}

static int gemm_f32acc_impl(const void* A, int lda, int a_kmajor, const void* B, int ldb, int b_kmajor, int M, int N,
                            int K, int k_splits, float alpha, float* C, int ldc, int diag_nblk, int diag_r,
                            uint32_t drop_seed, float drop_p, hipStream_t stream, const uint8_t* keep_bits) {
  if (!A || !B || !C) return OSPO_ERR_ARG;
  if (M <= 0 || N <= 0 || K <= 0 || K % BK || N % 64) return OSPO_ERR_SHAPE;
  if (k_splits < 1) k_splits = 1;
  if (k_splits > K / BK) k_splits = K / BK;
  if (a_kmajor ? (lda < ((M + 63) / 64) * 64) : (lda < K)) return OSPO_ERR_SHAPE;
  if (b_kmajor ? (ldb < N) : (ldb < K)) return OSPO_ERR_SHAPE;
  if ((lda % 8) || (ldb % 8)) return OSPO_ERR_SHAPE;
  if (diag_nblk > 0 && diag_r <= 0) return OSPO_ERR_ARG;
  if (diag_nblk <= 0 && ldc < N) return OSPO_ERR_SHAPE;
  if (!aligned16(A) || !aligned16(B)) return OSPO_ERR_ALIGN;
  GemmArgs a{(const bf16*)A, (const bf16*)B, nullptr, nullptr, lda, ldb, 0, 0, M, N, K, 0, alpha,
             nullptr, nullptr, 0, C, ldc, k_splits, diag_nblk, diag_r};
  if (drop_p > 0.f) {  // mask on B [K, N] (K-major), index m * N + n
    if (N & 1) return OSPO_ERR_SHAPE;  // mask pairs (drop_keep) start at even indices
    a.drop_seed = drop_seed;
    a.drop_thresh = drop_threshold(drop_p);
    a.drop_scale = 1.f / (1.f - drop_p);
    a.drop_ld = N;
    a.drop_bits = keep_bits;
  }
  const bool wideN = (N % 256 == 0);
  const bool tallM = a_kmajor ? (M % 256 == 0 && lda >= M) : (M >= 1024);
  if (!a_kmajor && !b_kmajor) return launch<2, 2, 2, 2, false, false, EPI_F32_ATOMIC>(a, stream);
  if (!a_kmajor && b_kmajor) return launch<2, 2, 2, 2, false, true, EPI_F32_ATOMIC>(a, stream);
  if (a_kmajor && !b_kmajor) return OSPO_ERR_UNSUPPORTED;
  // both K-major (LoRA weight gradients): big tiles only when they alone fill the chip,
  // otherwise 64 x 64 tiles (parallelism from tiles, not from more fp32-atomic K splits)
  const long ks = a.k_splits > 1 ? a.k_splits : 1;
#ifdef OSPO_ABLATION
  static const bool legacy = getenv("OSPO_F32ACC_LEGACY") != nullptr;  // A/B of the tile rule only
#else
  constexpr bool legacy = false;
#endif
  if (legacy) {
    if (wideN && !tallM) return launch<2, 4, 2, 4, true, true, EPI_F32_ATOMIC>(a, stream);
    if (tallM && !wideN) return launch<4, 2, 4, 2, true, true, EPI_F32_ATOMIC>(a, stream);
    return launch<2, 2, 2, 2, true, true, EPI_F32_ATOMIC>(a, stream);
  }
  if (wideN && !tallM && (long)(N / 256) * ((M + 63) / 64) * ks >= 384)
    return launch<2, 4, 2, 4, true, true, EPI_F32_ATOMIC>(a, stream);   // 64 x 256
  if (tallM && !wideN && (long)(M / 256) * ((N + 63) / 64) * ks >= 384)
    return launch<4, 2, 4, 2, true, true, EPI_F32_ATOMIC>(a, stream);   // 256 x 64
  return launch<2, 2, 2, 2, true, true, EPI_F32_ATOMIC>(a, stream);
}
