// Step-3 autoregressive text-to-image sampling on gfx950 (BASELINE config 4):
// the decode loop of ospo/wrapper/image_generation.py:132-171 (= ospo/inference.py:122-163) --
// Janus-Pro LLM over a KV cache for 2B rows (B prompts x {cond, uncond}), gen_head on the last
// position, classifier-free guidance, softmax(logits / T) and one sampled VQ token per image per
// step, fed back through prepare_gen_img_embeds.
//
// MI355X-first shape of the step (R = 2B <= 64 rows):
//  * every Linear is a weight stream (R rows against [N, K] weights): decode_gemv runs the
//    register-direct skinny MFMA loop of skinny.h with the WEIGHT as the 16-row operand and the
//    R activation rows as <= 4 small tiles, so each weight byte is loaded once, 16 B per lane,
//    with 2 x 4 batches of loads in flight per wave; split-K partials only when the weight has
//    too few 16-row blocks to fill 256 CUs;
//  * attention reads the KV cache [R][H][Tmax][128] row-contiguous per (row, head): one
//    workgroup per (query, head), keys range [pad_start[r], pos] (the reference's left padding
//    is an attention mask, positions run 0..T-1 through it);
//  * all step-dependent state (position, step index) lives in a device counter, so the whole
//    step is captured once in a hipGraph and replayed (ospo_amd/generate.py);
//  * sampling is inverse-CDF on the bf16 probabilities with a uniform per image and step,
//    summed in a fixed order (64-element chunks, then the 256 chunk sums) that
//    oracle/generate_ref.py restates, so a token is a deterministic function of (logits, u).
#include "common.h"
#include "skinny.h"

#include <algorithm>

namespace {

constexpr int HD = 128;  // head_dim (Janus-Pro)

// -------------------------------------------------------------------- GEMV
// out[r][n] = act(x[r] . W[n] + bias[n]) (+ res[r][n]);  act = GELU(erf) of the bf16-rounded
// pre-activation when gelu (vision_head's first Linear).
__device__ __forceinline__ void gemv_store(float v, int r, int n, const bf16* bias, int gelu, const bf16* res,
                                           int ldr, bf16* out, int ldo) {
  float y = v + (bias ? bf2f(bias[n]) : 0.f);
  if (gelu) y = gelu_erf(round_bf(y));
  if (res) y = round_bf(y) + bf2f(res[(long)r * ldr + n]);
  out[(long)r * ldo + n] = f2bf(y);
}

template <int NT>
__global__ __launch_bounds__(64 * SK_WAVES) void gemv_kernel(const bf16* __restrict__ W, int ldw,
                                                             const bf16* __restrict__ X, int ldx, int R, int K,
                                                             const bf16* __restrict__ bias, int gelu,
                                                             const bf16* __restrict__ res, int ldr,
                                                             bf16* __restrict__ out, int ldo,
                                                             f32x4* __restrict__ ws) {
  __shared__ f32x4 red[SK_WAVES][NT][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int nb = blockIdx.x, z = blockIdx.y, splits = gridDim.y;
  const int n = nb * 16 + l16;
  const int nsteps = K >> 5;
  const int s_begin = (int)((long)nsteps * z / splits), s_end = (int)((long)nsteps * (z + 1) / splits);
  const int n_i = (s_end - s_begin - wave + SK_WAVES - 1) / SK_WAVES;
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16* wrow = W + (long)n * ldw + 8 * g + 32 * s_begin;
  const bf16* bp[NT];
  bool bok[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int r = 16 * j + l16;
    bok[j] = r < R;
    bp[j] = X + (long)(bok[j] ? r : 0) * ldx + 8 * g + 32 * s_begin;
  }
  sk_loop<NT>(wrow, bp, bok, wave, n_i, acc);  // acc[j][q] = sum_k W[n][k] x[16j + 4g + q][k]
#pragma unroll
  for (int j = 0; j < NT; ++j) red[wave][j][lane] = acc[j];
  __syncthreads();
  if (wave >= NT) return;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 0; w < SK_WAVES; ++w) v += red[w][wave][lane];
  if (splits > 1) {
    ws[((long)(z * gridDim.x + nb) * NT + wave) * 64 + lane] = v;
    return;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 16 * wave + 4 * g + q;
    if (r < R) gemv_store(v[q], r, n, bias, gelu, res, ldr, out, ldo);
  }
}

template <int NT>
__global__ __launch_bounds__(64 * NT) void gemv_reduce_kernel(const f32x4* __restrict__ ws, int splits, int NB, int R,
                                                            const bf16* __restrict__ bias, int gelu,
                                                            const bf16* __restrict__ res, int ldr,
                                                            bf16* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63, j = threadIdx.x >> 6, nb = blockIdx.x;
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z = 0; z < splits; ++z) v += ws[((long)(z * NB + nb) * NT + j) * 64 + lane];
  const int n = nb * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 16 * j + 4 * g + q;
    if (r < R) gemv_store(v[q], r, n, bias, gelu, res, ldr, out, ldo);
  }
}

// GEMV v2: a workgroup owns 64 weight rows (wave w: rows 16w..16w+15) x a K range; the R <= 32
// activation rows of each 512-k chunk are staged once in LDS (one 1-KiB LDS-DMA per row, pitch
// 1040 B so the 16 fragment rows of a ds_read_b128 land in distinct banks) and shared by the four
// waves, while each wave streams its 16 weight rows with all of the chunk's loads (16 x 1 KiB) in
// flight at once.  v1 above re-read x from L2 for every 16 weight rows (2x the weight traffic).
constexpr int G2_ROWS = 64, G2_KC = 512, G2_PITCH = G2_KC * 2 + 16;
constexpr int G2_MAX_SPLITS = 16;  // gemv2/3_kper cap the split count (K / 512 <= 16 up to K = 8192)
template <int NT>
__global__ __launch_bounds__(256) void gemv2_kernel(const bf16* __restrict__ W, int ldw, const bf16* __restrict__ X,
                                                    int ldx, int R, int K, int kper, const bf16* __restrict__ bias,
                                                    int gelu, const bf16* __restrict__ res, int ldr,
                                                    bf16* __restrict__ out, int ldo, f32x4* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) char xs[16 * NT * G2_PITCH];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * G2_ROWS + wave * 16 + l16;
  const int z = blockIdx.y, splits = gridDim.y;
  const int k_begin = z * kper, k_end = min(K, k_begin + kper);
  const bf16* wrow = W + (long)n * ldw;
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = k_begin; kc < k_end; kc += G2_KC) {
    const int nsteps = min(G2_KC, k_end - kc) >> 5;
    // stage x rows [0, 16 NT) x [kc, kc + 512): wave w takes rows w, w+4, ...
    for (int r = wave; r < 16 * NT; r += 4) {
      const int rr = r < R ? r : R - 1;  // rows >= R are masked at the fragment
      const int col = min(kc + 8 * lane, K - 8);
      __builtin_amdgcn_global_load_lds(X + (long)rr * ldx + col, (LDS_AS void*)(xs + r * G2_PITCH), 16, 0, 0);
    }
    asm volatile("" ::: "memory");  // the x DMA is issued before the weight loads (the vmcnt below counts on it)
    bf16x8 wv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int k = kc + 32 * min(s, nsteps - 1) + 8 * g;
      wv[s] = *reinterpret_cast<const bf16x8*>(wrow + k);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // the x DMA (issued first) has landed
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < nsteps) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 xf = *reinterpret_cast<const bf16x8*>(xs + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
          if (16 * j + l16 >= R) xf = bf16x8{};
          acc[j] = MFMA(xf, wv[s], acc[j]);  // D[x row 4g+q][w row l16]
        }
      }
    }
    __syncthreads();  // every wave done with the chunk before it is restaged
  }
  const int nb = n >> 4;
  if (splits > 1) {
#pragma unroll
    for (int j = 0; j < NT; ++j) ws[((long)(z * (gridDim.x * 4) + nb) * NT + j) * 64 + lane] = acc[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * j + 4 * g + q;
      if (r < R) gemv_store(acc[j][q], r, n, bias, gelu, res, ldr, out, ldo);
    }
}

template <int NT>
__global__ __launch_bounds__(256) void gemv2_reduce_kernel(const f32x4* __restrict__ ws, int splits, int NB, int R,
                                                           const bf16* __restrict__ bias, int gelu,
                                                           const bf16* __restrict__ res, int ldr,
                                                           bf16* __restrict__ out, int ldo) {
  const int lane = threadIdx.x & 63, nb = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (nb >= NB) return;
  const int n = nb * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    // every split's partial in flight at once, then summed in split order
    f32x4 p[G2_MAX_SPLITS];
#pragma unroll
    for (int z = 0; z < G2_MAX_SPLITS; ++z)
      if (z < splits) p[z] = ws[((long)(z * NB + nb) * NT + j) * 64 + lane];
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int z = 0; z < G2_MAX_SPLITS; ++z)
      if (z < splits) v += p[z];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * j + 4 * g + q;
      if (r < R) gemv_store(v[q], r, n, bias, gelu, res, ldr, out, ldo);
    }
  }
}

// GEMV v3: v2's schedule with 8 waves = 128 weight rows per workgroup: half the x staging per
// weight byte.  Split partials as v2 (summed by gemv2_reduce_kernel).
//
// TL (round 2): W in the MFMA-tiled decode layout (ospo_decode_gemv with ldw = 0): tile (nb, ks) =
// rows 16 nb .. +15 x k 32 ks .. +31 is 1 KiB at ((nb * K/32 + ks) * 512) elements, lane-ordered
// (element 8 * (16 g + l16) + e = W[16 nb + l16][32 ks + 8 g + e]), so each 16-B fragment load of a
// wave reads one contiguous KiB (8 whole 128-B lines) instead of 16 rows x 64 B (half lines) of the
// row-major weight.  Same fragments, same MFMA order: bit-identical to the row-major form.
constexpr int G3_WAVES = 8, G3_ROWS = 16 * G3_WAVES;
template <int NT, bool TL = false>
__global__ __launch_bounds__(64 * G3_WAVES) void gemv3_kernel(const bf16* __restrict__ W, int ldw,
                                                              const bf16* __restrict__ X, int ldx, int R, int K,
                                                              int kper, const bf16* __restrict__ bias, int gelu,
                                                              const bf16* __restrict__ res, int ldr,
                                                              bf16* __restrict__ out, int ldo, f32x4* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) char xs[16 * NT * G2_PITCH];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * G3_ROWS + wave * 16 + l16;
  const int z = blockIdx.y, splits = gridDim.y;
  const int k_begin = z * kper, k_end = min(K, k_begin + kper);
  const bf16* wrow = TL ? W + ((long)(n >> 4) * (K >> 5) * 64 + lane) * 8 : W + (long)n * ldw;
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = k_begin; kc < k_end; kc += G2_KC) {
    const int nsteps = min(G2_KC, k_end - kc) >> 5;
    for (int r = wave; r < 16 * NT; r += G3_WAVES) {
      const int rr = r < R ? r : R - 1;
      const int col = min(kc + 8 * lane, K - 8);
      __builtin_amdgcn_global_load_lds(X + (long)rr * ldx + col, (LDS_AS void*)(xs + r * G2_PITCH), 16, 0, 0);
    }
    asm volatile("" ::: "memory");
    bf16x8 wv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (TL) {
        wv[s] = *reinterpret_cast<const bf16x8*>(wrow + (long)((kc >> 5) + min(s, nsteps - 1)) * 512);
      } else {
        const int k = kc + 32 * min(s, nsteps - 1) + 8 * g;
        wv[s] = *reinterpret_cast<const bf16x8*>(wrow + k);
      }
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // this wave's x DMA (issued first) has landed
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < nsteps) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 xf = *reinterpret_cast<const bf16x8*>(xs + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
          if (16 * j + l16 >= R) xf = bf16x8{};
          acc[j] = MFMA(xf, wv[s], acc[j]);
        }
      }
    }
    __syncthreads();
  }
  const int nb = n >> 4, NB = gridDim.x * G3_WAVES;
  if (splits > 1) {
#pragma unroll
    for (int j = 0; j < NT; ++j) ws[((long)(z * NB + nb) * NT + j) * 64 + lane] = acc[j];
    return;
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * j + 4 * g + q;
      if (r < R) gemv_store(acc[j][q], r, n, bias, gelu, res, ldr, out, ldo);
    }
}

// Split-sum + consumer fusions of the decode step (v3 partial layout [split][N/16][NT][64] f32x4,
// lane (g, l16) = rows 16 j + 4 g + q, column 16 nb + l16).  Each sums the splits in split order and
// rounds exactly as gemv_store (bf16 product), then applies its consumer with that consumer's own
// rounding, so the outputs are bit-identical to gemv + ospo_kv_store / ospo_swiglu_fwd.
template <int NT>
__device__ __forceinline__ f32x4 split_sum(const f32x4* __restrict__ ws, int splits, int NB, int nb, int j, int lane) {
  f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int z0 = 0; z0 < splits; z0 += 8) {
    f32x4 p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (z0 + u < splits) p[u] = ws[((long)((z0 + u) * NB + nb) * NT + j) * 64 + lane];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (z0 + u < splits) v += p[u];
  }
  return v;
}

// q|k|v = x . W_qkv^T: grid (3H head slices, NT), 256 threads; thread (pr = t >> 6, lane) owns columns
// d = 16 pr + l16 and d + 64 of its head (the RoPE pair) for 4 rows.
template <int NT>
__global__ __launch_bounds__(256) void gemv_reduce_kv_kernel(const f32x4* __restrict__ ws, int splits, int R,
                                                             const int* __restrict__ pos_dev,
                                                             const bf16* __restrict__ cs, const bf16* __restrict__ sn,
                                                             bf16* __restrict__ kc, bf16* __restrict__ vc, int H,
                                                             int Tmax, bf16* __restrict__ q_out, int ldq) {
  const int lane = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int hs = blockIdx.x, j = blockIdx.y;
  const int which = hs / H, h = hs % H;
  const int NB = 3 * H * 8;
  const int nb = hs * 8 + pr;
  const int g = lane >> 4, d = pr * 16 + (lane & 15);
  const int p = *pos_dev;
  if (p >= Tmax) return;
  const f32x4 v1 = split_sum<NT>(ws, splits, NB, nb, j, lane);
  const f32x4 v2 = split_sum<NT>(ws, splits, NB, nb + 4, j, lane);
  const float c = which < 2 ? bf2f(cs[(long)p * 64 + d]) : 0.f;
  const float sv = which < 2 ? bf2f(sn[(long)p * 64 + d]) : 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 16 * j + 4 * g + q;
    if (r >= R) continue;
    const float x1 = round_bf(v1[q]), x2 = round_bf(v2[q]);
    float o1 = x1, o2 = x2;
    if (which < 2) {  // rotate-half RoPE, rounded per op as kv_store_kernel
      o1 = round_bf(x1 * c) + round_bf(-x2 * sv);
      o2 = round_bf(x2 * c) + round_bf(x1 * sv);
    }
    if (which == 0) {
      bf16* qo = q_out + (long)r * ldq + h * HD;
      qo[d] = f2bf(o1);
      qo[d + 64] = f2bf(o2);
    } else {
      bf16* cache = (which == 1 ? kc : vc) + (((long)r * H + h) * Tmax + p) * HD;
      cache[d] = f2bf(o1);
      cache[d + 64] = f2bf(o2);
    }
  }
}

// gate|up = x . W_gu^T, h = bf16(bf16(silu(gate)) * up): grid (F / 64, NT), 256 threads; thread
// (pr, lane) owns gate column 16 (4 bx + pr) + l16 and its up column F + that.
template <int NT>
__global__ __launch_bounds__(256) void gemv_reduce_swiglu_kernel(const f32x4* __restrict__ ws, int splits, int R, int F,
                                                                 bf16* __restrict__ hout, int ldh) {
  const int lane = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int j = blockIdx.y;
  const int NB = 2 * F / 16;
  const int nb = blockIdx.x * 4 + pr;
  const int g = lane >> 4, col = nb * 16 + (lane & 15);
  const f32x4 vg = split_sum<NT>(ws, splits, NB, nb, j, lane);
  const f32x4 vu = split_sum<NT>(ws, splits, NB, nb + F / 16, j, lane);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 16 * j + 4 * g + q;
    if (r >= R) continue;
    const float gt = round_bf(vg[q]), up = round_bf(vu[q]);
    hout[(long)r * ldh + col] = f2bf(round_bf(silu(gt)) * up);
  }
}

// ------------------------------------------------------- KV cache write
// rows [R][nq] of qkv (q|k|v, H heads of 128 each): position p = pos0 + i (pos0 = *pos_dev, or 0).
// rope: HF rotate-half on q and k at position p, rounded per op like the eager bf16 path
// (ops.hip rope_kernel); q is written to q_out (else left in place), k / v to the caches.
__global__ void kv_store_kernel(bf16* __restrict__ qkv, int ld, int R, int nq, const int* __restrict__ pos_dev,
                                int rope, const bf16* __restrict__ cs, const bf16* __restrict__ sn,
                                bf16* __restrict__ kc, bf16* __restrict__ vc, int H, int Tmax,
                                bf16* __restrict__ q_out, int ldq) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)R * nq * H * 8;  // 8 chunks of 8 rotation pairs per head
  if (tid >= total) return;
  const int ch = tid & 7;
  const int h = (int)((tid >> 3) % H);
  const long ri = (tid >> 3) / H;
  const int r = (int)(ri / nq), i = (int)(ri % nq);
  const int p = (pos_dev ? *pos_dev : 0) + i;
  if (p >= Tmax) return;
  bf16* row = qkv + ri * ld;
  const int D = H * HD;
  float c[8], s[8];
  if (rope) {
    unpack8(*reinterpret_cast<const u32x4*>(cs + (long)p * 64 + ch * 8), c);
    unpack8(*reinterpret_cast<const u32x4*>(sn + (long)p * 64 + ch * 8), s);
  }
  const long cbase = (((long)r * H + h) * Tmax + p) * HD + ch * 8;
#pragma unroll
  for (int which = 0; which < 2; ++which) {  // 0 = q, 1 = k
    bf16* base = row + which * D + h * HD + ch * 8;
    u32x4 v1 = *reinterpret_cast<const u32x4*>(base), v2 = *reinterpret_cast<const u32x4*>(base + 64);
    if (rope) {
      float a[8], b[8], o1[8], o2[8];
      unpack8(v1, a);
      unpack8(v2, b);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        o1[q] = round_bf(a[q] * c[q]) + round_bf(-b[q] * s[q]);
        o2[q] = round_bf(b[q] * c[q]) + round_bf(a[q] * s[q]);
      }
      v1 = pack8(o1);
      v2 = pack8(o2);
    }
    if (which == 0) {
      if (q_out) {
        bf16* qo = q_out + ri * ldq + h * HD + ch * 8;
        *reinterpret_cast<u32x4*>(qo) = v1;
        *reinterpret_cast<u32x4*>(qo + 64) = v2;
      } else if (rope) {
        *reinterpret_cast<u32x4*>(base) = v1;
        *reinterpret_cast<u32x4*>(base + 64) = v2;
      }
    } else {
      *reinterpret_cast<u32x4*>(kc + cbase) = v1;
      *reinterpret_cast<u32x4*>(kc + cbase + 64) = v2;
    }
  }
  const bf16* vsrc = row + 2 * D + h * HD + ch * 8;
  *reinterpret_cast<u32x4*>(vc + cbase) = *reinterpret_cast<const u32x4*>(vsrc);
  *reinterpret_cast<u32x4*>(vc + cbase + 64) = *reinterpret_cast<const u32x4*>(vsrc + 64);
}

// ------------------------------------------------------------ attention
// one workgroup (256 threads) per (query row, head): keys [start[r], p], p = pos0 + i.
// HF eager bf16: s = bf16(bf16(q.k) * scale); fp32 softmax over the unmasked keys (masked keys
// get finfo.min and contribute exactly 0); P rounded to bf16; o = bf16(sum P v) with fp32 sums.
constexpr int ATT_MAXT = 2048;
__global__ __launch_bounds__(256) void attn_cache_kernel(const bf16* __restrict__ q, int ldq,
                                                         const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                         int H, int Tmax, const int* __restrict__ start,
                                                         const int* __restrict__ pos_dev, int nq, float scale,
                                                         bf16* __restrict__ out, int ldo) {
  __shared__ float sc[ATT_MAXT];
  __shared__ float red[8];
  __shared__ float2 part[4][64];
  const int ri = blockIdx.x, h = blockIdx.y;
  const int r = ri / nq, i = ri % nq;
  const int p = (pos_dev ? *pos_dev : 0) + i;
  const int s0 = start[r];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  bf16* orow = out + (long)ri * ldo + h * HD;
  if (p < s0 || p >= Tmax) {  // a padded query position: never consumed (its key is masked for everyone)
    if (wave == 0) reinterpret_cast<uint32_t*>(orow)[lane] = 0u;
    return;
  }
  const int L = p - s0 + 1;
  const uint32_t qv = reinterpret_cast<const uint32_t*>(q + (long)ri * ldq + h * HD)[lane];
  const float q0 = bits2f(qv & 0xffff), q1 = bits2f(qv >> 16);
  const long hb = ((long)r * H + h) * Tmax;
  const uint32_t* kb = reinterpret_cast<const uint32_t*>(kc + (hb + s0) * HD) + lane;
  // scores: wave w takes keys w, w+4, ...; 8 keys' loads in flight before the reductions
  for (int k0 = wave * 8; k0 < L; k0 += 32) {
    uint32_t kv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = min(k0 + u, L - 1);
      kv[u] = kb[(long)k * (HD / 2)];
    }
    float d[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) d[u] = wave_sum(q0 * bits2f(kv[u] & 0xffff) + q1 * bits2f(kv[u] >> 16));
    if (lane < 8 && k0 + lane < L) {
      float dv = d[0];
#pragma unroll
      for (int u = 1; u < 8; ++u) dv = (lane == u) ? d[u] : dv;
      sc[k0 + lane] = round_bf(round_bf(dv) * scale);
    }
  }
  __syncthreads();
  float m = -INFINITY;
  for (int k = threadIdx.x; k < L; k += 256) m = fmaxf(m, sc[k]);
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int k = threadIdx.x; k < L; k += 256) {
    const float e = __expf(sc[k] - m);
    sc[k] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (lane == 0) red[4 + wave] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  // o[2d..2d+1] = sum_k bf16(e_k / sum) v[k][2d..]: thread (kg = wave, d = lane), keys kg, kg+4, ...
  const uint32_t* vb = reinterpret_cast<const uint32_t*>(vc + (hb + s0) * HD) + lane;
  float a0 = 0.f, a1 = 0.f;
#pragma unroll 8
  for (int k = wave; k < L; k += 4) {
    const float pk = round_bf(sc[k] * inv);
    const uint32_t vv = vb[(long)k * (HD / 2)];
    a0 += pk * bits2f(vv & 0xffff);
    a1 += pk * bits2f(vv >> 16);
  }
  part[wave][lane] = make_float2(a0, a1);
  __syncthreads();
  if (wave == 0) {
    float o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      o0 += part[w][lane].x;
      o1 += part[w][lane].y;
    }
    reinterpret_cast<uint32_t*>(orow)[lane] = pack2(o0, o1);
  }
}

// v2 of the cached attention: 16-B loads.  Lane (key group kg = 4 w + (lane >> 4), chunk
// c = lane & 15) holds 8 head dims; a wave reads 4 whole K (V) rows per load instruction (1 KiB),
// 4 instructions in flight.  The q.k dot is 8 FMAs + a 16-lane DPP reduction (no LDS round
// trip); P.V accumulates 8 dims per lane over keys kg, kg + 16, ..., then the 16 key groups are
// summed in a fixed order.  Rounding points as attn_cache_kernel.
__device__ __forceinline__ float dpp_sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xf, 0xf, false));  // row_ror:8
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x124, 0xf, 0xf, false));  // row_ror:4
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4e, 0xf, 0xf, false));   // quad xor 2
  x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xb1, 0xf, 0xf, false));   // quad xor 1
  return x;
}

// non-temporal weight / KV-cache loads (decode streams read once per step); -DOSPO_DLIN_NTW=0 for the A/B
#ifndef OSPO_DLIN_NTW
#define OSPO_DLIN_NTW 1
#endif
// KV-cache rows: each workgroup reads its own row's cache once per step (5 GB over 30 layers late in an image,
// far past the 256 MB MALL): non-temporal, like the weight streams (OSPO_DLIN_NTW)
__device__ __forceinline__ u32x4 kv_load(const bf16* p) {
#if OSPO_DLIN_NTW
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
  return *reinterpret_cast<const u32x4*>(p);
#endif
}

__global__ __launch_bounds__(256) void attn_cache2_kernel(const bf16* __restrict__ q, int ldq,
                                                          const bf16* __restrict__ kc, const bf16* __restrict__ vc,
                                                          int H, int Tmax, const int* __restrict__ start,
                                                          const int* __restrict__ pos_dev, int nq, float scale,
                                                          bf16* __restrict__ out, int ldo) {
  __shared__ float sc[ATT_MAXT];
  __shared__ float red[8];
  __shared__ f32x4 part[16][16][2];
  const int ri = blockIdx.x, h = blockIdx.y;
  const int r = ri / nq, i = ri % nq;
  const int p = (pos_dev ? *pos_dev : 0) + i;
  const int s0 = start[r];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = lane & 15, kg = wave * 4 + (lane >> 4);
  bf16* orow = out + (long)ri * ldo + h * HD;
  if (p < s0 || p >= Tmax) {  // a padded query position: never consumed
    if (threadIdx.x < 16) *reinterpret_cast<u32x4*>(orow + 8 * threadIdx.x) = u32x4{0u, 0u, 0u, 0u};
    return;
  }
  const int L = p - s0 + 1;
  float qf[8];
  unpack8(*reinterpret_cast<const u32x4*>(q + (long)ri * ldq + h * HD + 8 * c), qf);
  const long hb = ((long)r * H + h) * Tmax;
  const bf16* kb = kc + (hb + s0) * HD + 8 * c;
  for (int k0 = kg; k0 < L; k0 += 64) {
    u32x4 kv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) kv[u] = kv_load(kb + (long)min(k0 + 16 * u, L - 1) * HD);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float kf[8];
      unpack8(kv[u], kf);
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qf[e], kf[e], d);
      d = dpp_sum16(d);
      if (c == 0 && k0 + 16 * u < L) sc[k0 + 16 * u] = round_bf(round_bf(d) * scale);
    }
  }
  __syncthreads();
  float m = -INFINITY;
  for (int k = threadIdx.x; k < L; k += 256) m = fmaxf(m, sc[k]);
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int k = threadIdx.x; k < L; k += 256) {
    const float e = __expf(sc[k] - m);
    sc[k] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (lane == 0) red[4 + wave] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  const bf16* vb = vc + (hb + s0) * HD + 8 * c;
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  for (int k0 = kg; k0 < L; k0 += 64) {
    u32x4 vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) vv[u] = kv_load(vb + (long)min(k0 + 16 * u, L - 1) * HD);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float pk = (k0 + 16 * u < L) ? round_bf(sc[min(k0 + 16 * u, L - 1)] * inv) : 0.f;
      float vf[8];
      unpack8(vv[u], vf);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = fmaf(pk, vf[e], a[e]);
    }
  }
  part[kg][c][0] = f32x4{a[0], a[1], a[2], a[3]};
  part[kg][c][1] = f32x4{a[4], a[5], a[6], a[7]};
  __syncthreads();
  if (threadIdx.x < 16) {
    const int cc = threadIdx.x;
    f32x4 o0 = part[0][cc][0], o1 = part[0][cc][1];
#pragma unroll
    for (int g2 = 1; g2 < 16; ++g2) {
      o0 += part[g2][cc][0];
      o1 += part[g2][cc][1];
    }
    const float o[8] = {o0[0], o0[1], o0[2], o0[3], o1[0], o1[1], o1[2], o1[3]};
    *reinterpret_cast<u32x4*>(orow + 8 * cc) = pack8(o);
  }
}

// ------------------------------------------------ fused decode Linear (round 3)
// ospo_decode_linear: one launch per Linear of the decode step (the round-2 step ran each as a GEMV, a
// split-sum launch and, before q|k|v and gate|up, an RMSNorm launch: ~10 launches of 5-13 us per layer,
// most of them ramp).  gemv3's weight stream (tiled layout, 128 rows per workgroup, K split over
// gridDim.y), plus:
//  * NORM: the RMSNorm of the input folded into the x staging.  X is the PRE-norm residual stream; its
//    row sums of squares come from the producer's epilogue (ss_in [ss_groups][32]: one partial per
//    128-column group), summed here in group order; xn = bf16(w * bf16(x * rsqrt(ss / K + eps))) is
//    formed in LDS once per 512-k chunk, rounded as rmsnorm_fwd rounds it.
//  * the split sum in the launch: every workgroup stores its fp32 partial write-through (sc1) and takes a
//    ticket on its row group's counter (workspace head, zero at allocation); the last arriver sums the
//    partials in split order (gemv2_reduce_kernel's order) and runs the consumer:
//      DL_PLAIN   out = act(v + bias) (+ residual) as gemv_store, and, with ss_out, the row sums of
//                 squares of out over the group's 128 columns (ss_out [N/128][32]) for the next RMSNorm;
//      DL_KV      RoPE + KV-cache store of one head slice (row group = head slice; as gemv_reduce_kv);
//      DL_SWIGLU  h = bf16(bf16(silu(gate)) * up) from a gate|up weight whose row group g holds gate rows
//                 64g .. 64g+63 then up rows F + 64g .. (ops.interleave_gate_up); out cols 64g .. +63.
//    The last arriver zeroes its counter again.  No fence: sc1 stores are visible device-wide once
//    acknowledged (vmcnt(0) before the ticket) and sc1 loads do not hit a stale line.
enum { DL_PLAIN = 0, DL_KV = 1, DL_SWIGLU = 2 };
constexpr int DL_CNT_BYTES = OSPO_WS_DECODE_LINEAR_CNT_BYTES;  // workspace head: one counter per 128-row group (N <= 131072)
struct DlArgs {
  const bf16* W;
  const bf16* X;
  int ldx, R, K, kper;
  const float* ss_in;
  int ss_groups;
  const bf16* ln_w;
  float eps;
  const bf16* bias;
  int gelu;
  const bf16* res;
  int ldr;
  bf16* out;
  int ldo;
  float* ss_out;
  const int* pos;
  const bf16* cs;
  const bf16* sn;
  bf16* kc;
  bf16* vc;
  int H, Tmax;
  float* part;
  unsigned* cnt;
  int part_bytes;
  // dmlp_kernel (round 5): h publish / consume flags, one per gate|up row group, tagged with the epoch
  // (*epoch_step) * 64 + epoch_layer + 1 of this call; tmo: set when a consumer gives up waiting
  unsigned* hflag = nullptr;
  const int* epoch_step = nullptr;
  int epoch_layer = 0;
  unsigned* tmo = nullptr;
  int kv_hm = 0;  // DL_KV: head-major row groups (round 5, ospo_decode_qkv_heads)
};

// Round 5, decode MLP in one launch (dmlp_kernel): the gate|up workgroups PUBLISH their group's h columns
// (write-through stores, then the group's flag = epoch); the down workgroups CONSUME them: their first chunk's
// weights are issued before they wait for the flags of the gate|up groups their K range reads.
enum { DL_ROLE_PLAIN = 0, DL_ROLE_PUB = 1, DL_ROLE_CONS = 2 };
constexpr unsigned DL_SPIN_LIMIT = 1u << 22;  // bounded wait (~1 s): a give-up sets the error word, never hangs

__device__ __forceinline__ unsigned dl_epoch(const DlArgs& a) {
  return (unsigned)(*a.epoch_step) * 64u + (unsigned)a.epoch_layer + 1u;  // never 0 (the flags' reset value)
}

// The end of a decode-Linear workgroup (dlin_kernel, dlin_pipe_kernel): the split sum, then the consumer.
// The workgroup holds the partials accs[u] of the nz consecutive splits z0 .. z0 + nz - 1 of row group grp.
// nz < splits: each is stored write-through (sc1) at its split's slot, the workgroup takes nz tickets on the
// group's counter, and the last arriver sums all splits' partials in split order; nz == splits: the same sum
// in registers.  Either way every output is summed as ((0 + p_0) + p_1) + ..., the reduce kernels' order.
template <int NT, int EPI, int U>
__device__ __forceinline__ void dlin_finish(const DlArgs& a, const f32x4 (&accs)[U][NT], int nz, int grp, int z0,
                                            int splits, int ngroups, char* xs, float (*ssr)[32], unsigned* flag) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = grp * G3_ROWS + wave * 16 + l16;
  const int R = a.R;
  const int nb = n >> 4, NB = ngroups * G3_WAVES;
  const bool ticket = splits > 1 && nz < splits;
  f32x4 acc[NT];
  if (ticket) {
    const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc((void*)a.part, 0, a.part_bytes, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < nz) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, accs[u][j]), rsP,
                                                 (uint32_t)(((((z0 + u) * NB + nb) * NT + j) * 64 + lane) * 16), 0, 16);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(a.cnt + grp, (unsigned)nz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = (t + (unsigned)nz == (unsigned)splits) ? 1u : 0u;
    }
    __syncthreads();
    if (*flag == 0u) return;
    // no instruction: keeps the sc1 partial loads below the ticket (sc1 stores drained before it, sc1 loads
    // after it: the hand-off Valid form of cdna_hip_programming.md, where this replaces the agent-scope acquire)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int zs = 0; zs < splits; zs += 8) {  // 8 partials in flight, summed in split order
        u32x4 pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (zs + u < splits)
            pv[u] = __builtin_amdgcn_raw_buffer_load_b128(rsP, (uint32_t)(((((zs + u) * NB + nb) * NT + j) * 64 + lane) * 16),
                                                          0, 16);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (zs + u < splits) v += __builtin_bit_cast(f32x4, pv[u]);
      }
      acc[j] = v;
    }
  } else if (splits > 1) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (u < nz) v += accs[u][j];
      acc[j] = v;
    }
  } else {
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = accs[0][j];
  }
  if constexpr (EPI == DL_PLAIN) {
    float ssq[NT][4];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * j + 4 * g + q;
        float y = acc[j][q] + (a.bias ? bf2f(a.bias[n]) : 0.f);
        if (a.gelu) y = gelu_erf(round_bf(y));
        if (a.res) y = round_bf(y) + bf2f(a.res[(long)(r < R ? r : 0) * a.ldr + n]);
        y = round_bf(y);
        if (r < R) a.out[(long)r * a.ldo + n] = f2bf(y);
        ssq[j][q] = dpp_sum16(y * y);  // over the wave's 16 columns
      }
    if (a.ss_out) {
      if (l16 == 0) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) ssr[wave][16 * j + 4 * g + q] = ssq[j][q];
      }
      __syncthreads();
      if (threadIdx.x < 16 * NT) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < G3_WAVES; ++w) s += ssr[w][threadIdx.x];
        a.ss_out[grp * 32 + threadIdx.x] = s;
      }
    }
  } else {
    // the group's 128 columns x 16 NT rows, bf16-rounded sums, through LDS (the x staging is free)
    float* ep = reinterpret_cast<float*>(xs);
    __syncthreads();  // (dlin_pipe_kernel: every wave is past its last chunk's LDS reads)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) ep[(16 * j + 4 * g + q) * 129 + wave * 16 + l16] = round_bf(acc[j][q]);
    __syncthreads();
    if constexpr (EPI == DL_KV) {
      // row groups q_0 .. q_H-1, k_0 .., v_0 .. (nn.Linear order), or head-major q_h, k_h, v_h (kv_hm: the
      // head-range launches of ospo_decode_qkv_heads, whose out / cache pointers start at their first head)
      const int hs = grp, which = a.kv_hm ? hs % 3 : hs / a.H, h = a.kv_hm ? hs / 3 : hs % a.H;
      const int p = *a.pos;
      if (p < a.Tmax) {
        for (int it = threadIdx.x; it < R * 64; it += 64 * G3_WAVES) {
          const int r = it >> 6, d = it & 63;
          const float x1 = ep[r * 129 + d], x2 = ep[r * 129 + d + 64];
          float o1 = x1, o2 = x2;
          if (which < 2) {  // rotate-half RoPE, rounded per op as kv_store_kernel
            const float c = bf2f(a.cs[(long)p * 64 + d]), sv = bf2f(a.sn[(long)p * 64 + d]);
            o1 = round_bf(x1 * c) + round_bf(-x2 * sv);
            o2 = round_bf(x2 * c) + round_bf(x1 * sv);
          }
          bf16* dst = which == 0 ? a.out + (long)r * a.ldo + h * HD
                                 : (which == 1 ? a.kc : a.vc) + (((long)r * a.H + h) * a.Tmax + p) * HD;
          dst[d] = f2bf(o1);
          dst[d + 64] = f2bf(o2);
        }
      }
    } else if (a.hflag) {
      // dmlp_kernel's producer: 8 columns per thread as one 16-B write-through store (the same rounding as the
      // scalar path below), every storing wave drained, the barrier, then this group's flag = epoch (R1 publish)
      const __amdgpu_buffer_rsrc_t rsH =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.out, 0, (int)((long)R * a.ldo * 2), 0x00020000);
      for (int it = threadIdx.x; it < R * 8; it += 64 * G3_WAVES) {
        const int r = it >> 3, c8 = (it & 7) * 8;
        float hv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) hv[e] = round_bf(silu(ep[r * 129 + c8 + e])) * ep[r * 129 + 64 + c8 + e];
        __builtin_amdgcn_raw_buffer_store_b128(pack8(hv), rsH, (uint32_t)(((long)r * a.ldo + 64 * grp + c8) * 2), 0, 16);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(a.hflag + grp, dl_epoch(a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      for (int it = threadIdx.x; it < R * 64; it += 64 * G3_WAVES) {
        const int r = it >> 6, c = it & 63;
        const float gt = ep[r * 129 + c], up = ep[r * 129 + 64 + c];
        a.out[(long)r * a.ldo + 64 * grp + c] = f2bf(round_bf(silu(gt)) * up);
      }
    }
  }
  if (ticket && threadIdx.x == 0) __hip_atomic_store(a.cnt + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT, int EPI, bool NORM>
__global__ __launch_bounds__(64 * G3_WAVES) void dlin_kernel(const DlArgs a) {
  static_assert(16 * NT * G2_PITCH >= 16 * NT * 129 * 4, "epilogue tile fits the x staging");
  __shared__ __attribute__((aligned(16))) char xs[16 * NT * G2_PITCH];
  __shared__ float rs[32];
  __shared__ float sst[NORM ? 1024 : 1];
  __shared__ float ssr[G3_WAVES][32];
  __shared__ unsigned flag;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = blockIdx.x * G3_ROWS + wave * 16 + l16;
  const int z = blockIdx.y, splits = gridDim.y;
  const int K = a.K, R = a.R;
  const int k_begin = z * a.kper, k_end = min(K, k_begin + a.kper);
  const bf16* wrow = a.W + ((long)(n >> 4) * (K >> 5) * 64 + lane) * 8;
  // NORM: the producer's ss partials (<= 32 groups x 32 rows) are loaded here, two per thread, and only
  // used after the first chunk's wait: a serial per-group load chain in one wave cost ~20 us per launch
  float ssv[2] = {0.f, 0.f};
  if constexpr (NORM) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = threadIdx.x + 512 * u;
      if (i < a.ss_groups * 32) ssv[u] = a.ss_in[i];
    }
  }
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;  // NORM: 8 columns x rows tr, tr + 8, ...
  for (int kc = k_begin; kc < k_end; kc += G2_KC) {
    const int nsteps = min(G2_KC, k_end - kc) >> 5;
    for (int r = wave; r < 16 * NT; r += G3_WAVES) {
      const int rr = r < R ? r : R - 1;
      const int col = min(kc + 8 * lane, K - 8);
      __builtin_amdgcn_global_load_lds(a.X + (long)rr * a.ldx + col, (LDS_AS void*)(xs + r * G2_PITCH), 16, 0, 0);
    }
    u32x4 lw = u32x4{0u, 0u, 0u, 0u};
    if constexpr (NORM) lw = *reinterpret_cast<const u32x4*>(a.ln_w + min(kc + 8 * tc, K - 8));
    asm volatile("" ::: "memory");  // x DMA (+ the norm weights) before the weight loads: vmcnt(16) covers them
    bf16x8 wv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bf16x8* wp = reinterpret_cast<const bf16x8*>(wrow + (long)((kc >> 5) + min(s, nsteps - 1)) * 512);
#if OSPO_DLIN_NTW
      wv[s] = __builtin_nontemporal_load(wp);  // the weight stream is read once per step: no cache allocation
#else
      wv[s] = *wp;
#endif
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    __syncthreads();
    if constexpr (NORM) {
      if (kc == k_begin) {  // rstd of the 32 rows: the partials summed in group order
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (threadIdx.x + 512 * u < 1024) sst[threadIdx.x + 512 * u] = ssv[u];
        __syncthreads();
        if (threadIdx.x < 32) {
          float s = 0.f;
          for (int q = 0; q < a.ss_groups; ++q) s += sst[q * 32 + threadIdx.x];
          rs[threadIdx.x] = rsqrtf(s / (float)K + a.eps);
        }
        __syncthreads();
      }
      float wf[8];
      unpack8(lw, wf);
#pragma unroll
      for (int i = 0; i < 2 * NT; ++i) {
        const int r = tr + 8 * i;
        u32x4* p = reinterpret_cast<u32x4*>(xs + r * G2_PITCH + tc * 16);
        float f[8];
        unpack8(*p, f);
        const float rr = rs[r < R ? r : R - 1];
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = wf[q] * round_bf(f[q] * rr);
        *p = pack8(f);
      }
      __syncthreads();
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < nsteps) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 xf = *reinterpret_cast<const bf16x8*>(xs + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
          if (16 * j + l16 >= R) xf = bf16x8{};
          acc[j] = MFMA(xf, wv[s], acc[j]);  // D[x row 4g+q][w row l16]
        }
      }
    }
    __syncthreads();
  }
  f32x4 accs[1][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) accs[0][j] = acc[j];
  dlin_finish<NT, EPI, 1>(a, accs, 1, blockIdx.x, z, splits, gridDim.x, xs, ssr, &flag);
}

// Pipelined decode Linear (round 5, verdict r4 item 8).  dlin_kernel's workgroup loads a 512-k chunk, waits,
// computes, and only then loads the next: every chunk pays a full memory round trip, and a launch is one or
// two such rounds of one-shot workgroups (q|k|v 26.6 us for 100 MB, gate|up 41.0 us for 180 MB, down 23.3 us
// for 90 MB, cold weights; warm in the Infinity Cache only 5-10 % faster: tools/dlin_warm_ab.py,
// profiles/r05/dlin_warm_ab.log).  Here a workgroup (grid ngroups x splits / U, at most one per CU: two
// register sets) owns the U consecutive splits z0 = U blockIdx.y .. of its row group and streams their chunks
// with the NEXT chunk's x rows (a second LDS image) and weight fragments (a second register set, 16 per wave)
// in flight under the current chunk's MFMAs.  Per split the MFMA order is dlin_kernel's; the splits' partials
// stay in registers and are summed in split order (dlin_finish): outputs bit-identical to dlin_kernel's.
// Needs K % kper == 0 and splits % U == 0 (host).  All LDS in one array (a second __shared__ object can make
// hipcc drain the LDS-DMA before every LDS read: cdna_hip_programming.md section 5, trap (a)).
// LDS of dlin_pipe_body: two x images, then rstd, the ss partials (NORM), the ss_out rows, the ticket flag
template <int NT>
constexpr int dl_pipe_lds(bool norm) {
  return 2 * 16 * NT * G2_PITCH + (32 + (norm ? 1024 : 4) + G3_WAVES * 32 + 4) * 4;
}

// the gate|up groups g0 .. g1 - 1 published with this call's epoch: wave 0 polls (one flag per lane), then
// the agent-scope acquire, then the workgroup's barrier (cdna_hip_programming.md Guideline 16, R1 consume)
__device__ __forceinline__ void dl_wait_flags(const DlArgs& a, int g0, int g1) {
  if (threadIdx.x < 64) {
    const unsigned ep = dl_epoch(a);
    const int lane = threadIdx.x;
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      for (int g = g0 + lane; g < g1; g += 64)
        ok &= __hip_atomic_load(a.hflag + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep;
      if (__all(ok)) break;
      if (++spins > DL_SPIN_LIMIT) {
        if (lane == 0) __hip_atomic_store(a.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the invalidate done before the barrier releases the readers
  }
  __syncthreads();
}

template <int NT, int EPI, bool NORM, int U, int ROLE = DL_ROLE_PLAIN>
__device__ __forceinline__ void dlin_pipe_body(const DlArgs& a, int gx, int gy, int ngroups, int splits,
                                               char* smem) {
  constexpr int XB = 16 * NT * G2_PITCH;  // one x image: 16 NT rows x 512 k (padded pitch)
  constexpr int SST = NORM ? 1024 : 4;
  float* rs = reinterpret_cast<float*>(smem + 2 * XB);
  float* sst = rs + 32;
  float(*ssr)[32] = reinterpret_cast<float(*)[32]>(sst + SST);
  unsigned* flag = reinterpret_cast<unsigned*>(sst + SST + G3_WAVES * 32);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = gx * G3_ROWS + wave * 16 + l16;
  const int z0 = gy * U;
  const int K = a.K, R = a.R, kper = a.kper;
  const int cpu = (kper + G2_KC - 1) / G2_KC;  // chunks per split (every split kper long: K % kper == 0)
  const int C = U * cpu;                        // this workgroup's chunks
  const bf16* wrow = a.W + ((long)(n >> 4) * (K >> 5) * 64 + lane) * 8;
  float ssv[2] = {0.f, 0.f};
  if constexpr (NORM) {  // issued first: the first chunk's vmcnt(16) covers them (as dlin_kernel)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = threadIdx.x + 512 * u;
      if (i < a.ss_groups * 32) ssv[u] = a.ss_in[i];
    }
  }
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;  // NORM: 8 columns x rows tr, tr + 8, ...
  bf16x8 wv[2][16];
  u32x4 lw[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
  auto chunk_k = [&](int c, int& kc, int& nsteps) __attribute__((always_inline)) {
    const int u = c / cpu, i = c - u * cpu;
    const int kb = (z0 + u) * kper;
    kc = kb + i * G2_KC;
    nsteps = min(G2_KC, kb + kper - kc) >> 5;
  };
  // chunk c's x rows -> image B, its norm weights, its 16 weight fragments per wave -> wv[B] (dlin_kernel's
  // order: x DMA and norm weights first, so a vmcnt(16) after them leaves exactly the weights in flight)
  auto issue_x = [&](auto b_c, int c) __attribute__((always_inline)) {
    constexpr int B = decltype(b_c)::value;
    int kc, nsteps;
    chunk_k(c, kc, nsteps);
    for (int r = wave; r < 16 * NT; r += G3_WAVES) {
      const int rr = r < R ? r : R - 1;
      const int col = min(kc + 8 * lane, K - 8);
      __builtin_amdgcn_global_load_lds(a.X + (long)rr * a.ldx + col, (LDS_AS void*)(smem + B * XB + r * G2_PITCH), 16,
                                       0, 0);
    }
    if constexpr (NORM) lw[B] = *reinterpret_cast<const u32x4*>(a.ln_w + min(kc + 8 * tc, K - 8));
    asm volatile("" ::: "memory");
  };
  auto issue_w = [&](auto b_c, int c) __attribute__((always_inline)) {
    constexpr int B = decltype(b_c)::value;
    int kc, nsteps;
    chunk_k(c, kc, nsteps);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bf16x8* wp = reinterpret_cast<const bf16x8*>(wrow + (long)((kc >> 5) + min(s, nsteps - 1)) * 512);
#if OSPO_DLIN_NTW
      wv[B][s] = __builtin_nontemporal_load(wp);
#else
      wv[B][s] = *wp;
#endif
    }
  };
  auto issue = [&](auto b_c, int c) __attribute__((always_inline)) {
    issue_x(b_c, c);
    issue_w(b_c, c);
  };
  f32x4 accs[U][NT], acc[NT];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < NT; ++j) accs[u][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  // chunk c from image / register set B; the next chunk goes to B ^ 1 before the MFMAs.  At the barrier only
  // chunk c's loads are in flight, so __syncthreads()'s drain costs nothing here.  (A third stage, two chunks
  // in flight, needs 3 x 64 weight registers and spilled at 256 VGPRs.)
  auto body = [&](auto b_c, int c) __attribute__((always_inline)) {
    constexpr int B = decltype(b_c)::value;
    char* xs = smem + B * XB;
    if (ROLE == DL_ROLE_CONS && c == 0)  // the consumer issued chunk 0's x rows after its weights
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk c's x rows (+ norm weights) landed
    __syncthreads();
    if constexpr (NORM) {
      if (c == 0) {  // rstd of the 32 rows: the partials summed in group order
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (threadIdx.x + 512 * u < 1024) sst[threadIdx.x + 512 * u] = ssv[u];
        __syncthreads();
        if (threadIdx.x < 32) {
          float s = 0.f;
          for (int q = 0; q < a.ss_groups; ++q) s += sst[q * 32 + threadIdx.x];
          rs[threadIdx.x] = rsqrtf(s / (float)K + a.eps);
        }
        __syncthreads();
      }
      float wf[8];
      unpack8(lw[B], wf);
#pragma unroll
      for (int i = 0; i < 2 * NT; ++i) {
        const int r = tr + 8 * i;
        u32x4* p = reinterpret_cast<u32x4*>(xs + r * G2_PITCH + tc * 16);
        float f[8];
        unpack8(*p, f);
        const float rr = rs[r < R ? r : R - 1];
#pragma unroll
        for (int q = 0; q < 8; ++q) f[q] = wf[q] * round_bf(f[q] * rr);
        *p = pack8(f);
      }
      __syncthreads();
    }
    // the other image and register set were last read by chunk c - 1's MFMAs, before the barrier above
    if (c + 1 < C) {
      if constexpr (B == 0) issue(I1{}, c + 1);
      else issue(I0{}, c + 1);
    }
    int kc, nsteps;
    chunk_k(c, kc, nsteps);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < nsteps) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 xf = *reinterpret_cast<const bf16x8*>(xs + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
          if (16 * j + l16 >= R) xf = bf16x8{};
          acc[j] = MFMA(xf, wv[B][s], acc[j]);  // D[x row 4g+q][w row l16]
        }
      }
    }
    if (c - (c / cpu) * cpu == cpu - 1) {  // the split's last chunk: its partial enters a shift register
#pragma unroll                               // (constant indices: a runtime index put accs in scratch)
      for (int uu = U - 1; uu > 0; --uu)
#pragma unroll
        for (int j = 0; j < NT; ++j) accs[uu][j] = accs[uu - 1][j];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        accs[0][j] = acc[j];
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  if constexpr (ROLE == DL_ROLE_CONS) {  // chunk 0's weights in flight while the producers finish
    issue_w(I0{}, 0);
    const int k0 = z0 * kper, k1 = min(K, (z0 + U) * kper);
    dl_wait_flags(a, k0 / 64, (k1 + 63) / 64);
    issue_x(I0{}, 0);
  } else {
    issue(I0{}, 0);
  }
  for (int c = 0; c < C; c += 2) {
    body(I0{}, c);
    if (c + 1 < C) body(I1{}, c + 1);
  }
  f32x4 part[U][NT];  // split z0 + u's partial sits at accs[U - 1 - u]
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int j = 0; j < NT; ++j) part[u][j] = accs[U - 1 - u][j];
  dlin_finish<NT, EPI, U>(a, part, U, gx, z0, splits, ngroups, smem, ssr, flag);
}

template <int NT, int EPI, bool NORM, int U>
__global__ __launch_bounds__(64 * G3_WAVES) void dlin_pipe_kernel(const DlArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[dl_pipe_lds<NT>(NORM)];
  dlin_pipe_body<NT, EPI, NORM, U>(a, blockIdx.x, blockIdx.y, gridDim.x, gridDim.y * U, smem);
}

// The decode MLP in one launch (round 5): workgroups 0 .. ngu - 1 are gate|up (+ the folded RMSNorm, SwiGLU;
// one workgroup per row group, all UG splits in registers) publishing h; the rest are down (+ residual, ss_out;
// U = 1, split-K summed by ticket) consuming it.  Blocks dispatch in order, so every producer is resident or
// done before a consumer occupies a CU, and the consumers' waits are bounded either way (tmo).
template <int NT, int UG>
__global__ __launch_bounds__(64 * G3_WAVES) void dmlp_kernel(const DlArgs gu, const DlArgs dn, int ngu, int ndn,
                                                             int dn_splits) {
  __shared__ __attribute__((aligned(16))) char smem[dl_pipe_lds<NT>(true)];
  if ((int)blockIdx.x < ngu) {
    dlin_pipe_body<NT, DL_SWIGLU, true, UG, DL_ROLE_PUB>(gu, blockIdx.x, 0, ngu, UG, smem);
  } else {
    const int u = blockIdx.x - ngu;
    dlin_pipe_body<NT, DL_PLAIN, false, 1, DL_ROLE_CONS>(dn, u % ndn, u / ndn, ndn, dn_splits, smem);
  }
}

// Round 5: the cached attention and the o projection in ONE launch (dattn_o_kernel, ospo_decode_attn_o).
// Attention workgroups (8 waves = two 4-wave halves, one (row, head) each: attn_cache2_kernel's arithmetic, so
// the same bits) store their output rows write-through and take a ticket on their head; the head's last one
// publishes the head's flag = epoch.  The o workgroups (dlin_kernel's one-chunk form: kper = 512, four heads)
// issue their weights first, wait for their four heads' flags, then stage x and run dlin_finish (split sum by
// ticket, residual, ss_out) -- decode_linear's bits.  <= 80 VGPRs (6 waves per SIMD) and ~34 KB of LDS: three
// workgroups per CU, so at R = 32 the 512 attention and 256 o workgroups are resident together.
struct AttnArgs {
  const bf16* q;
  int ldq;
  const bf16* kc;
  const bf16* vc;
  int H, Tmax;
  const int* start;
  const int* pos;
  float scale;
  bf16* out;
  int ldo, R;
};
constexpr int ATT_HALF_LDS = ATT_MAXT * 4 + 16 * 16 * 2 * 16 + 8 * 4;  // sc, part, red of one half

// one (row ri, head h) on the 256 threads tid of a half; no early return (the halves share the barriers): a padded
// query position (or ri >= R) runs with L = 0 -- no loads, a zero output as attn_cache2_kernel writes -- and a row
// ri >= R stores nothing.  Ends with this thread's write-through stores acknowledged.
__device__ __forceinline__ void attn_row_pub(const AttnArgs& at, int ri, int h, int tid, char* hs) {
  float* sc = reinterpret_cast<float*>(hs);
  f32x4(*part)[16][2] = reinterpret_cast<f32x4(*)[16][2]>(hs + ATT_MAXT * 4);
  float* red = reinterpret_cast<float*>(hs + ATT_MAXT * 4 + 16 * 16 * 2 * 16);
  const bool inr = ri < at.R;
  const int rc = inr ? ri : at.R - 1;
  const int p = *at.pos;
  const int s0 = at.start[rc];
  const int L = (inr && p >= s0 && p < at.Tmax) ? p - s0 + 1 : 0;
  const int lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, kg = wave * 4 + (lane >> 4);
  float qf[8];
  unpack8(*reinterpret_cast<const u32x4*>(at.q + (long)rc * at.ldq + h * HD + 8 * c), qf);
  const long hb = ((long)rc * at.H + h) * at.Tmax;
  const bf16* kb = at.kc + (hb + s0) * HD + 8 * c;
  for (int k0 = kg; k0 < L; k0 += 64) {
    u32x4 kv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) kv[u] = kv_load(kb + (long)min(k0 + 16 * u, L - 1) * HD);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float kf[8];
      unpack8(kv[u], kf);
      float d = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) d = fmaf(qf[e], kf[e], d);
      d = dpp_sum16(d);
      if (c == 0 && k0 + 16 * u < L) sc[k0 + 16 * u] = round_bf(round_bf(d) * at.scale);
    }
  }
  __syncthreads();
  float m = -INFINITY;
  for (int k = tid; k < L; k += 256) m = fmaxf(m, sc[k]);
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float sum = 0.f;
  for (int k = tid; k < L; k += 256) {
    const float e = __expf(sc[k] - m);
    sc[k] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  __syncthreads();
  if (lane == 0) red[4 + wave] = sum;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  const bf16* vb = at.vc + (hb + s0) * HD + 8 * c;
  float a[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) a[e] = 0.f;
  for (int k0 = kg; k0 < L; k0 += 64) {
    u32x4 vv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) vv[u] = kv_load(vb + (long)min(k0 + 16 * u, L - 1) * HD);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float pk = (k0 + 16 * u < L) ? round_bf(sc[min(k0 + 16 * u, L - 1)] * inv) : 0.f;
      float vf[8];
      unpack8(vv[u], vf);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] = fmaf(pk, vf[e], a[e]);
    }
  }
  part[kg][c][0] = f32x4{a[0], a[1], a[2], a[3]};
  part[kg][c][1] = f32x4{a[4], a[5], a[6], a[7]};
  __syncthreads();
  if (tid < 16 && inr) {
    const int cc = tid;
    f32x4 o0 = part[0][cc][0], o1 = part[0][cc][1];
#pragma unroll
    for (int g2 = 1; g2 < 16; ++g2) {
      o0 += part[g2][cc][0];
      o1 += part[g2][cc][1];
    }
    const float o[8] = {o0[0], o0[1], o0[2], o0[3], o1[0], o1[1], o1[2], o1[3]};
    // write-through (sc1): visible device-wide once acknowledged, before the flag
    const __amdgpu_buffer_rsrc_t rsO =
        __builtin_amdgcn_make_buffer_rsrc((void*)at.out, 0, (int)((long)at.R * at.ldo * 2), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(L > 0 ? pack8(o) : u32x4{0u, 0u, 0u, 0u}, rsO,
                                           (uint32_t)(((long)ri * at.ldo + h * HD + 8 * cc) * 2), 0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// o workgroup (row group grp, split z of kper = G2_KC = 4 heads): dlin_kernel's one-chunk body with the weights
// issued before the wait on the attention flags of heads [k_begin / 128, + 4) over rows 0 .. R - 1
template <int NT, bool LATE_W = false>  // LATE_W (ablation A/B): the weights issued after the wait
__device__ __forceinline__ void dlin_cons_heads(const DlArgs& a, int grp, int z, int ngroups, int splits, char* smem) {
  char* xs = smem;
  float(*ssr)[32] = reinterpret_cast<float(*)[32]>(smem + 16 * NT * G2_PITCH);
  unsigned* flag = reinterpret_cast<unsigned*>(smem + 16 * NT * G2_PITCH + G3_WAVES * 32 * 4);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int n = grp * G3_ROWS + wave * 16 + l16;
  const int K = a.K, R = a.R;
  const int kc = z * G2_KC;
  const bf16* wrow = a.W + ((long)(n >> 4) * (K >> 5) * 64 + lane) * 8;
  bf16x8 wv[16];
  auto issue_w = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const bf16x8* wp = reinterpret_cast<const bf16x8*>(wrow + (long)((kc >> 5) + s) * 512);
#if OSPO_DLIN_NTW
      wv[s] = __builtin_nontemporal_load(wp);
#else
      wv[s] = *wp;
#endif
    }
  };
  if constexpr (!LATE_W) issue_w();
  if (threadIdx.x < 64) {  // wave 0 polls its four heads' flags (one lane each), then the agent-scope acquire
    const unsigned ep = dl_epoch(a);
    const int h0 = kc / HD, nh = G2_KC / HD;
    unsigned spins = 0;
    for (;;) {
      const bool ok = lane >= nh || __hip_atomic_load(a.hflag + h0 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ep;
      if (__all(ok)) break;
      if (++spins > DL_SPIN_LIMIT) {
        if (lane == 0) __hip_atomic_store(a.tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if constexpr (LATE_W) issue_w();
  for (int r = wave; r < 16 * NT; r += G3_WAVES) {
    const int rr = r < R ? r : R - 1;
    __builtin_amdgcn_global_load_lds(a.X + (long)rr * a.ldx + kc + 8 * lane, (LDS_AS void*)(xs + r * G2_PITCH), 16, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bf16x8 xf = *reinterpret_cast<const bf16x8*>(xs + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
      if (16 * j + l16 >= R) xf = bf16x8{};
      acc[j] = MFMA(xf, wv[s], acc[j]);
    }
  }
  __syncthreads();
  f32x4 accs[1][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) accs[0][j] = acc[j];
  dlin_finish<NT, DL_PLAIN, 1>(a, accs, 1, grp, z, splits, ngroups, xs, ssr, flag);
}

template <int NT>
constexpr int dattn_o_lds() {
  return std::max(2 * ATT_HALF_LDS, 16 * NT * G2_PITCH + G3_WAVES * 32 * 4 + 16);
}

// blocks 0 .. n_attn - 1: attention, head-major (h = b / nrp, rows 2 (b % nrp), + 1), so the heads of the first
// o splits finish first; then the o workgroups split-major (z = u / ngroups).  Blocks dispatch in order: every
// producer is resident or done before a consumer takes a slot, and the waits are bounded either way (tmo).
template <int NT, bool LATE_W = false>
__device__ __forceinline__ void dattn_o_body(const AttnArgs& at, const DlArgs& o, int n_attn, int nrp, int ngroups,
                                             int splits, char* smem) {
  if ((int)blockIdx.x < n_attn) {
    const int h = blockIdx.x / nrp, rp = blockIdx.x - h * nrp;
    const int half = threadIdx.x >> 8;
    attn_row_pub(at, 2 * rp + half, h, threadIdx.x & 255, smem + half * ATT_HALF_LDS);
    __syncthreads();
    // both rows' stores acknowledged: a ticket on the head's counter (flags[H + h]); the head's last workgroup
    // zeroes it and publishes the head's flag = epoch (flags[h])
    if (threadIdx.x == 0) {
      unsigned* tk = o.hflag + at.H + h;
      if (__hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)nrp - 1u) {
        __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(o.hflag + h, dl_epoch(o), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    const int u = blockIdx.x - n_attn;
    dlin_cons_heads<NT, LATE_W>(o, u % ngroups, u / ngroups, ngroups, splits, smem);
  }
}

template <int NT, bool LATE_W = false>
__global__ __launch_bounds__(64 * G3_WAVES) __attribute__((amdgpu_waves_per_eu(6))) void dattn_o_kernel(
    const AttnArgs at, const DlArgs o, int n_attn, int nrp, int ngroups, int splits) {
  __shared__ __attribute__((aligned(16))) char smem[dattn_o_lds<NT>()];
  dattn_o_body<NT, LATE_W>(at, o, n_attn, nrp, ngroups, splits, smem);
}
#ifdef OSPO_ABLATION
// A/B (ablation build, OSPO_ATTN_O_VAR=2): the compiler's register budget (~86 VGPRs: two workgroups per CU, the o
// workgroups dispatched only as attention workgroups retire)
template <int NT>
__global__ __launch_bounds__(64 * G3_WAVES) void dattn_o2_kernel(const AttnArgs at, const DlArgs o, int n_attn, int nrp,
                                                                 int ngroups, int splits) {
  __shared__ __attribute__((aligned(16))) char smem[dattn_o_lds<NT>()];
  dattn_o_body<NT>(at, o, n_attn, nrp, ngroups, splits, smem);
}
#endif

#ifdef OSPO_ABLATION
// ABLATION BUILD ONLY (measured and rejected): ospo_decode_linear v2 (round 3): the same units, partials, summation order and consumers as dlin_kernel
// (bit-identical outputs), but ~256 long-lived workgroups instead of one workgroup per (row group, split).
// dlin_kernel's workgroups each load one 128-KiB unit and end after one round trip for the weights and one
// for the partial store + ticket, at 2-3 resident per CU, so its launches ran at 2.8-4.0 TB/s (T2I profile,
// profiles/r03/t2i_step_breakdown_v1_decode_linear.txt).  Here workgroup w owns split z = w % splits and the
// row groups g0 .. g0 + G - 1 of set w / splits:
//  * the x rows of ALL its chunks (<= DL2_MAXC x 512 k) are staged (and RMSNorm-folded) once;
//  * it streams units (group, chunk) in group order with the next unit's 16 weight fragments per wave in
//    flight under the current unit's MFMAs (registers double-buffered by a 2x-unrolled loop);
//  * a finished group's partial is stored write-through at once; its ticket is taken one unit later, after
//    the vmcnt(0) that the next unit's weights need anyway and a barrier (every wave's stores acknowledged;
//    a ticket right after the store would drain the prefetched weights: vmcnt retires in issue order), and
//    the last arriver sums + runs the consumer there, in an LDS tile of its own (xs still holds the x).
constexpr int DL2_MAXC = 4;   // 512-k chunks per split: kper <= 2048
constexpr int DL2_WGS = 256;  // workgroups to aim for: one per CU of an MI355X

template <int NT, int EPI, bool NORM>
__global__ __launch_bounds__(64 * G3_WAVES) void dlin2_kernel(const DlArgs a, int splits, int G, int ngroups) {
  __shared__ __attribute__((aligned(16))) char xs[DL2_MAXC * 16 * NT * G2_PITCH];
  __shared__ __attribute__((aligned(16))) float ep[16 * NT * 129];
  __shared__ float rs[32];
  __shared__ float sst[NORM ? 1024 : 1];
  __shared__ float ssr[G3_WAVES][32];
  __shared__ unsigned flag;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, g = lane >> 4;
  const int z = blockIdx.x % splits, set = blockIdx.x / splits;
  const int g0 = set * G, ng = min(G, ngroups - g0);
  const int K = a.K, R = a.R;
  const int k_begin = z * a.kper, k_end = min(K, k_begin + a.kper);
  const int nch = (k_end - k_begin + G2_KC - 1) / G2_KC;  // <= DL2_MAXC (host check)
  const int U = ng * nch;
  const int NB = ngroups * G3_WAVES;
  const __amdgpu_buffer_rsrc_t rsP = __builtin_amdgcn_make_buffer_rsrc((void*)a.part, 0, a.part_bytes, 0x00020000);

  float ssv[2] = {0.f, 0.f};
  if constexpr (NORM) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = threadIdx.x + 512 * u;
      if (i < a.ss_groups * 32) ssv[u] = a.ss_in[i];
    }
  }
  // x rows of every chunk of the split, once
  for (int c = 0; c < nch; ++c) {
    const int kc = k_begin + c * G2_KC;
    for (int r = wave; r < 16 * NT; r += G3_WAVES) {
      const int rr = r < R ? r : R - 1;
      const int col = min(kc + 8 * lane, K - 8);
      __builtin_amdgcn_global_load_lds(a.X + (long)rr * a.ldx + col,
                                       (LDS_AS void*)(xs + (c * 16 * NT + r) * G2_PITCH), 16, 0, 0);
    }
  }
  const int tc = threadIdx.x & 63, tr = threadIdx.x >> 6;  // NORM: 8 columns x rows tr, tr + 8, ...
  u32x4 lw[DL2_MAXC];
#pragma unroll
  for (int c = 0; c < DL2_MAXC; ++c) {
    lw[c] = u32x4{0u, 0u, 0u, 0u};
    if (NORM && c < nch) lw[c] = *reinterpret_cast<const u32x4*>(a.ln_w + min(k_begin + c * G2_KC + 8 * tc, K - 8));
  }
  asm volatile("" ::: "memory");  // x DMA + norm weights before the first unit's weights: vmcnt(16) covers them

  auto load_unit = [&](int u, bf16x8 (&wv)[16]) __attribute__((always_inline)) {
    const int q = u / nch;
    const int c = u - q * nch;
    const int kc = k_begin + c * G2_KC;
    const int nsteps = min(G2_KC, k_end - kc) >> 5;
    const bf16* wr = a.W + ((long)((g0 + q) * G3_WAVES + wave) * (K >> 5) * 64 + lane) * 8;
#pragma unroll
    for (int s = 0; s < 16; ++s) wv[s] = *reinterpret_cast<const bf16x8*>(wr + (long)((kc >> 5) + min(s, nsteps - 1)) * 512);
  };
  bf16x8 wa[16];
  load_unit(0, wa);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __syncthreads();
  if constexpr (NORM) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (threadIdx.x + 512 * u < 1024) sst[threadIdx.x + 512 * u] = ssv[u];
    __syncthreads();
    if (threadIdx.x < 32) {
      float s = 0.f;
      for (int q = 0; q < a.ss_groups; ++q) s += sst[q * 32 + threadIdx.x];
      rs[threadIdx.x] = rsqrtf(s / (float)K + a.eps);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < DL2_MAXC; ++c) {
      if (c < nch) {
        float wf[8];
        unpack8(lw[c], wf);
#pragma unroll
        for (int i = 0; i < 2 * NT; ++i) {
          const int r = tr + 8 * i;
          u32x4* p = reinterpret_cast<u32x4*>(xs + (c * 16 * NT + r) * G2_PITCH + tc * 16);
          float f[8];
          unpack8(*p, f);
          const float rr = rs[r < R ? r : R - 1];
#pragma unroll
          for (int q = 0; q < 8; ++q) f[q] = wf[q] * round_bf(f[q] * rr);
          *p = pack8(f);
        }
      }
    }
    __syncthreads();
  }

  // the last arriver of row group gp: the splits' partials in split order, then the consumer
  auto finish = [&](int gp, const f32x4 (&own)[NT], bool load) __attribute__((always_inline)) {
    const int n = gp * G3_ROWS + wave * 16 + l16, nb = gp * G3_WAVES + wave;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[j] = own[j];
      if (!load) continue;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int z0 = 0; z0 < splits; z0 += 8) {  // 8 partials in flight, summed in split order
        u32x4 pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (z0 + u < splits)
            pv[u] = __builtin_amdgcn_raw_buffer_load_b128(rsP, (uint32_t)(((((z0 + u) * NB + nb) * NT + j) * 64 + lane) * 16),
                                                          0, 16);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (z0 + u < splits) v += __builtin_bit_cast(f32x4, pv[u]);
      }
      acc[j] = v;
    }
    if constexpr (EPI == DL_PLAIN) {
      float ssq[NT][4];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 16 * j + 4 * g + q;
          float y = acc[j][q] + (a.bias ? bf2f(a.bias[n]) : 0.f);
          if (a.gelu) y = gelu_erf(round_bf(y));
          if (a.res) y = round_bf(y) + bf2f(a.res[(long)(r < R ? r : 0) * a.ldr + n]);
          y = round_bf(y);
          if (r < R) a.out[(long)r * a.ldo + n] = f2bf(y);
          ssq[j][q] = dpp_sum16(y * y);  // over the wave's 16 columns
        }
      if (a.ss_out) {
        if (l16 == 0) {
#pragma unroll
          for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) ssr[wave][16 * j + 4 * g + q] = ssq[j][q];
        }
        __syncthreads();
        if (threadIdx.x < 16 * NT) {
          float s = 0.f;
#pragma unroll
          for (int w = 0; w < G3_WAVES; ++w) s += ssr[w][threadIdx.x];
          a.ss_out[gp * 32 + threadIdx.x] = s;
        }
      }
    } else {
      // the group's 128 columns x 16 NT rows, bf16-rounded sums, through LDS
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) ep[(16 * j + 4 * g + q) * 129 + wave * 16 + l16] = round_bf(acc[j][q]);
      __syncthreads();
      if constexpr (EPI == DL_KV) {
        const int which = gp / a.H, h = gp % a.H;
        const int p = *a.pos;
        if (p < a.Tmax) {
          for (int it = threadIdx.x; it < R * 64; it += 64 * G3_WAVES) {
            const int r = it >> 6, d = it & 63;
            const float x1 = ep[r * 129 + d], x2 = ep[r * 129 + d + 64];
            float o1 = x1, o2 = x2;
            if (which < 2) {  // rotate-half RoPE, rounded per op as kv_store_kernel
              const float cv = bf2f(a.cs[(long)p * 64 + d]), sv = bf2f(a.sn[(long)p * 64 + d]);
              o1 = round_bf(x1 * cv) + round_bf(-x2 * sv);
              o2 = round_bf(x2 * cv) + round_bf(x1 * sv);
            }
            bf16* dst = which == 0 ? a.out + (long)r * a.ldo + h * HD
                                   : (which == 1 ? a.kc : a.vc) + (((long)r * a.H + h) * a.Tmax + p) * HD;
            dst[d] = f2bf(o1);
            dst[d + 64] = f2bf(o2);
          }
        }
      } else {
        for (int it = threadIdx.x; it < R * 64; it += 64 * G3_WAVES) {
          const int r = it >> 6, cc = it & 63;
          const float gt = ep[r * 129 + cc], up = ep[r * 129 + 64 + cc];
          a.out[(long)r * a.ldo + 64 * gp + cc] = f2bf(round_bf(silu(gt)) * up);
        }
      }
      __syncthreads();  // ep is reused by the next finished group
    }
    if (splits > 1 && threadIdx.x == 0) __hip_atomic_store(a.cnt + gp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  f32x4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int pend = -1;  // a group whose partial is stored and not yet ticketed
  // (no lambda calls another lambda here: hipcc's host pass then dropped the kernel's launch stub)
  for (int u = 0; u < U; ++u) {
    const int q = u / nch;
    const int c = u - q * nch;
    const int kc = k_begin + c * G2_KC;
    const int nsteps = min(G2_KC, k_end - kc) >> 5;
    if (pend >= 0) {  // its stores (every wave's) and this unit's weights (issued before them) have landed
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // all waves' partial stores acknowledged before the ticket
      if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(a.cnt + pend, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag = (t == (unsigned)splits - 1u) ? 1u : 0u;
      }
    }
    bf16x8 cur[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) cur[s] = wa[s];  // waits for this unit's weights, then frees wa for the next
    if (u + 1 < U) load_unit(u + 1, wa);
    const char* xc = xs + c * 16 * NT * G2_PITCH;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < nsteps) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          bf16x8 xf = *reinterpret_cast<const bf16x8*>(xc + (16 * j + l16) * G2_PITCH + (32 * s + 8 * g) * 2);
          if (16 * j + l16 >= R) xf = bf16x8{};
          acc[j] = MFMA(xf, cur[s], acc[j]);  // D[x row 4g+q][w row l16]
        }
      }
    }
    if (pend >= 0) {
      __syncthreads();  // flag
      const bool last = flag != 0u;
      __syncthreads();  // every wave has read it before the next ticket overwrites it
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (as in dlin_kernel's last arriver)
        finish(pend, acc, true);
      }
      pend = -1;
    }
    if (c == nch - 1) {  // group g0 + q complete
      const int gi = g0 + q;
      if (splits > 1) {  // its partial, write-through; the ticket comes one unit later
        const int nb = gi * G3_WAVES + wave;
#pragma unroll
        for (int j = 0; j < NT; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j]), rsP,
                                                 (uint32_t)((((z * NB + nb) * NT + j) * 64 + lane) * 16), 0, 16);
        pend = gi;
      } else {
        finish(gi, acc, false);  // unsplit: one workgroup per group, the consumer on the registers
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (pend >= 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(a.cnt + pend, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag = (t == (unsigned)splits - 1u) ? 1u : 0u;
    }
    __syncthreads();
    if (flag != 0u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (as above)
      finish(pend, acc, true);
    }
  }
}
#endif  // OSPO_ABLATION

// --------------------------------------------------------- CFG + sampling
// one workgroup per image b: logits rows 2b (cond) and 2b+1 (uncond) [V] bf16 (train.py-style
// interleaving of image_generation.py:132-141, 156-157).  l = bf16(lu + bf16(w * bf16(lc - lu))),
// l = bf16(l / T); p = bf16(softmax(l)) (fp32 inside, like torch's bf16 softmax); token = first j
// with cumsum(p)_j > u * sum(p), sums in 64-element chunks (thread t owns chunk t) then the
// chunk sums in order (a rounding overshoot takes the last token with mass).  V <= 256 * 64.
// torch.multinomial draws from the same distribution with its own generator; the uniform here
// comes from a seeded device buffer, so a run is reproducible and checkable token by token.
constexpr int SMP_CHUNK = 64;
__global__ __launch_bounds__(256) void cfg_sample_kernel(const bf16* __restrict__ logits, int ldl, int V, float cfg_w,
                                                         float temp, const float* __restrict__ u,
                                                         int B, const int* __restrict__ step_dev, int n_steps,
                                                         int* __restrict__ tokens, int* __restrict__ next_ids,
                                                         float* __restrict__ probs_out) {
  __shared__ float csum[256];
  __shared__ float red[8];
  __shared__ int pick[2];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int step = step_dev ? *step_dev : 0;
  if (step >= n_steps) return;
  const bf16* lc = logits + (long)(2 * b) * ldl;
  const bf16* lu = logits + (long)(2 * b + 1) * ldl;
  const int j0 = t * SMP_CHUNK;
  const int nj = max(0, min(SMP_CHUNK, V - j0));
  float l[SMP_CHUNK];
  float m = -INFINITY;
  const bool vec = nj == SMP_CHUNK && ((ldl | V) & 7) == 0 && ((uintptr_t)logits & 15) == 0;  // 16-B loads: 8 per row, not 64
#pragma unroll
  for (int q8 = 0; q8 < SMP_CHUNK; q8 += 8) {
    float c8[8], u8[8];
    if (vec) {
      unpack8(*reinterpret_cast<const u32x4*>(lc + j0 + q8), c8);
      unpack8(*reinterpret_cast<const u32x4*>(lu + j0 + q8), u8);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        c8[e] = q8 + e < nj ? bf2f(lc[j0 + q8 + e]) : 0.f;
        u8[e] = q8 + e < nj ? bf2f(lu[j0 + q8 + e]) : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int q = q8 + e;
      float v = -INFINITY;
      if (q < nj) {
        const float c = c8[e], un = u8[e];
        v = round_bf(un + round_bf(cfg_w * round_bf(c - un)));
        if (temp != 1.f) v = round_bf(v / temp);
      }
      l[q] = v;
      m = fmaxf(m, v);
    }
  }
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
#pragma unroll  // every loop over l[] fully unrolled: a runtime index put l[] in scratch (round 5: 64 -> 47 us was
  for (int q = 0; q < SMP_CHUNK; ++q) {  // the chunk-sum chain; the rest was these scratch round trips)
    const float e = q < nj ? expf(l[q] - m) : 0.f;
    l[q] = e;
    s += e;
  }
  s = wave_sum(s);
  __syncthreads();
  if (lane == 0) red[4 + wave] = s;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  float cs = 0.f;
#pragma unroll
  for (int q = 0; q < SMP_CHUNK; ++q) {
    const float pq = q < nj ? round_bf(l[q] * inv) : 0.f;
    l[q] = pq;
    cs += pq;
    if (probs_out && q < nj) probs_out[(long)b * V + j0 + q] = pq;
  }
  csum[t] = cs;
  __syncthreads();
  if (wave == 0) {
    // The chunk sums in order: the running sum before every chunk (pre) and the total, as ONE serial chain of
    // fp32 adds in chunk order -- the values of a sequential loop over chunks 0..255, bit for bit -- but with
    // each sum broadcast from its lane by v_readlane into the add (one wave, register operands) instead of a
    // dependent LDS load per chunk in one thread (round 5: that loop, twice over 256 chunks, was most of the
    // kernel's 64 us).  Lane l holds chunks 4 l .. 4 l + 3.
    float cv[4], pre[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) cv[i] = csum[4 * lane + i];
    float run = 0.f;
#pragma unroll
    for (int L = 0; L < 64; ++L) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ci = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cv[i]), L));
        if (lane == L) pre[i] = run;
        run += ci;
      }
    }
    const float tot = run;
    const float target = u[(long)step * B + b] * tot;
    // the first chunk c with pre[c] + csum[c] > target (the loop's break), else the last chunk with mass
    int fi = -1, li = -1;
#pragma unroll
    for (int i = 3; i >= 0; --i)
      if (pre[i] + cv[i] > target) fi = i;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (cv[i] > 0.f) li = i;
    const unsigned long long hit = __ballot(fi >= 0), mass = __ballot(li >= 0);
    int src, idx;
    if (hit) {
      src = __builtin_ctzll(hit);
      idx = __shfl(fi, src);
    } else if (mass) {  // target at the very top (rounding): the last chunk with mass
      src = 63 - __builtin_clzll(mass);
      idx = __shfl(li, src);
    } else {
      src = 0;
      idx = 0;
    }
    const float pv = idx == 0 ? pre[0] : (idx == 1 ? pre[1] : (idx == 2 ? pre[2] : pre[3]));
    const float run_at = __shfl(pv, src);
    if (lane == 0) {
      pick[0] = 4 * src + idx;
      red[0] = run_at;
      red[1] = target;
    }
  }
  __syncthreads();
  if (t == pick[0]) {
    float run = red[0];
    const float target = red[1];
    int tok = -1, last = j0;
    bool done = false;
#pragma unroll
    for (int q = 0; q < SMP_CHUNK; ++q) {  // the scan with its break as a predicate (constant indices)
      if (q < nj && !done) {
        if (l[q] > 0.f) last = j0 + q;
        run += l[q];
        if (run > target) {
          tok = j0 + q;
          done = true;
        }
      }
    }
    if (tok < 0) tok = last;  // u * total at the very top of the chunk (rounding): its last nonzero
    tokens[(long)b * n_steps + step] = tok;
    next_ids[2 * b] = tok;
    next_ids[2 * b + 1] = tok;
  }
}

__global__ void embed_rows_kernel(const int* __restrict__ ids, long n, const bf16* __restrict__ table, int V, int D,
                                  bf16* __restrict__ out) {
  const int cpr = D / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= n * cpr) return;
  const long r = tid / cpr;
  const int c = tid % cpr;
  const int id = min(max(ids[r], 0), V - 1);  // the host validates ids; clamped so they cannot fault
  reinterpret_cast<u32x4*>(out + r * D)[c] = reinterpret_cast<const u32x4*>(table + (long)id * D)[c];
}

__global__ void advance_kernel(int* pos, int* step) {
  if (threadIdx.x == 0) {
    *pos += 1;
    *step += 1;
  }
}

int gemv_splits(int nblocks, int K) {
  int s = 1;
  while (nblocks * s < 1024 && (K >> 5) / (2 * s) >= 8 * SK_WAVES) s *= 2;
  return s;
}
#ifdef OSPO_ABLATION
int g_gemv_splits = 0;   // A/B knob: > 0 forces the v2 / v3 split count (clamped to K / 512 and 16)
int g_gemv_variant = 3;  // 1 = skinny-loop GEMV, 2 = LDS-shared x, 3 = v2 with 128 rows per workgroup (default)
#else
constexpr int g_gemv_splits = 0;
constexpr int g_gemv_variant = 3;  // the product library runs the v3 GEMV
#endif
// v2 K split: ~1024 workgroups, at least one 512-k chunk each; returns k per split (multiple of 32)
int gemv2_kper(int N, int K) {
  const int groups = N / G2_ROWS;
  int splits = (1024 + groups - 1) / groups;
  splits = std::max(1, std::min(std::min(splits, K / G2_KC), G2_MAX_SPLITS));
  if (g_gemv_splits > 0) splits = std::max(1, std::min(std::min(g_gemv_splits, K / G2_KC), G2_MAX_SPLITS));
  int kper = (K + splits - 1) / splits;
  return (kper + 31) / 32 * 32;
}

// v3 K split: the largest power of two <= min(8, K / 512) that keeps the grid within 1024
// workgroups (4 per CU).  Power-of-two splits of K = 4096 give whole 512-k chunks; splits of 3 or
// 6 leave a short tail chunk per workgroup and measured up to 30 % slower (tools/gemv_sweep.py).
int gemv3_kper(int N, int K) {
  const int groups = N / G3_ROWS;
  int splits = 1;
  while (splits * 2 <= std::min(8, K / G2_KC) && groups * splits * 2 <= 1024) splits *= 2;
  // A/B knob: down to 256-k splits (half a staged chunk)
  if (g_gemv_splits > 0) splits = std::max(1, std::min(std::min(g_gemv_splits, K / 256), G2_MAX_SPLITS));
  int kper = (K + splits - 1) / splits;
  return (kper + 31) / 32 * 32;
}

// dlin_pipe_kernel's splits per workgroup: the smallest U in {1, 2, 4} dividing splits that keeps the grid
// within one workgroup per CU (its two register sets leave room for one 8-wave workgroup per CU); 0 = the
// one-shot dlin_kernel.  The pipelined form is taken only where a split spans >= 2 chunks (gate|up: 4 splits
// of 1024 k, down: 8 of 1376): with one chunk per split (q|k|v, o) it holds one chunk in flight per CU where
// dlin_kernel's two resident workgroups hold two, and measured slower (q|k|v 26.8 -> 30.1 us, o equal;
// gate|up 40.9 -> 38.3, down 23.2 -> 21.2: profiles/r05/dlin_pipe_ab.log).  all: every shape it fits (A/B).
int dlin_pipe_units(int ngroups, int splits, int K, int kper, bool all = false) {
  static int ncu[16] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return 0;
  if (ncu[dev] == 0 && hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  if (K % kper != 0 || (!all && kper < 2 * G2_KC)) return 0;
  for (int u = 1; u <= 4 && u <= splits; u *= 2)
    if (splits % u == 0 && (long)ngroups * (splits / u) <= ncu[dev]) return u;
  return 0;
}

}  // namespace

extern "C" size_t ospo_decode_gemv_ws_bytes(int R, int N, int K) {
  if (R <= 0 || R > 64 || N <= 0 || N % 16 || K <= 0) return 0;
  const int nt = (R + 15) / 16, nb = N / 16;
  const size_t v1 = (size_t)gemv_splits(nb, K) * nb * nt * 64 * sizeof(f32x4);
  if (N % G2_ROWS || K % 32) return v1;
  const int kper = gemv2_kper(N, K);
  const size_t v2 = (size_t)((K + kper - 1) / kper) * nb * nt * 64 * sizeof(f32x4);
  size_t v3 = 0;
  if (N % G3_ROWS == 0) {
    const int kp = gemv3_kper(N, K);
    v3 = (size_t)((K + kp - 1) / kp) * nb * nt * 64 * sizeof(f32x4);
  }
  return std::max(std::max(v1, v2), v3);
}

#ifdef OSPO_ABLATION
extern "C" int ospo_set_gemv_splits(int s) {
  if (s < 0 || s > G2_MAX_SPLITS) return OSPO_ERR_ARG;
  g_gemv_splits = s;
  return OSPO_OK;
}

extern "C" int ospo_set_gemv_variant(int v) {
  if (v < 1 || v > 3) return OSPO_ERR_ARG;
  g_gemv_variant = v;
  return OSPO_OK;
}
#endif

// the fused split-sum consumers need the v3 schedule with a K split (else: gemv + the consumer)
extern "C" int ospo_decode_gemv_fusable(int R, int N, int K) {
  if (g_gemv_variant != 3 || R <= 0 || R > 32 || N % G3_ROWS || K < 8 || K % 32) return 0;
  const int kper = gemv3_kper(N, K);
  return (K + kper - 1) / kper > 1 ? 1 : 0;
}

static int gemv3_partials(const bf16* w, int ldw, const bf16* x, int ldx, int R, int N, int K, f32x4* ws,
                          size_t ws_bytes, hipStream_t stream, int& splits) {
  const int kper = gemv3_kper(N, K);
  splits = (K + kper - 1) / kper;
  if (!ws || ws_bytes < ospo_decode_gemv_ws_bytes(R, N, K) || !aligned16(ws)) return OSPO_ERR_ARG;
  const dim3 grid(N / G3_ROWS, splits);
  auto kfn = R <= 16 ? (ldw == 0 ? gemv3_kernel<1, true> : gemv3_kernel<1, false>)
                     : (ldw == 0 ? gemv3_kernel<2, true> : gemv3_kernel<2, false>);
  hipLaunchKernelGGL(kfn, grid, dim3(64 * G3_WAVES), 0, stream, w, ldw, x, ldx, R, K, kper, nullptr, 0, nullptr, 0,
                     nullptr, 0, ws);
  return OSPO_OK;
}

extern "C" int ospo_decode_gemv_kv(const void* W, int ldw, const void* X, int ldx, int R, int n_heads, int head_dim,
                                   int K, void* ws, size_t ws_bytes, const int* pos_dev, const void* rope_cos,
                                   const void* rope_sin, void* k_cache, void* v_cache, int Tmax, void* q_out, int ldq,
                                   hipStream_t stream) {
  if (!W || !X || !pos_dev || !rope_cos || !rope_sin || !k_cache || !v_cache || !q_out) return OSPO_ERR_ARG;
  if (head_dim != HD) return OSPO_ERR_UNSUPPORTED;
  const int N = 3 * n_heads * HD;
  if (!ospo_decode_gemv_fusable(R, N, K)) return OSPO_ERR_UNSUPPORTED;
  if ((ldw != 0 && ldw < K) || ldx < K || ldw % 8 || ldx % 8 || ldq < n_heads * HD || Tmax <= 0) return OSPO_ERR_SHAPE;
  if (!aligned16(W) || !aligned16(X)) return OSPO_ERR_ALIGN;
  int splits = 0;
  const int rc = gemv3_partials((const bf16*)W, ldw, (const bf16*)X, ldx, R, N, K, (f32x4*)ws, ws_bytes, stream, splits);
  if (rc != OSPO_OK) return rc;
  const dim3 grid(3 * n_heads, (R + 15) / 16);
  if (R <= 16)
    hipLaunchKernelGGL((gemv_reduce_kv_kernel<1>), grid, dim3(256), 0, stream, (const f32x4*)ws, splits, R, pos_dev,
                       (const bf16*)rope_cos, (const bf16*)rope_sin, (bf16*)k_cache, (bf16*)v_cache, n_heads, Tmax,
                       (bf16*)q_out, ldq);
  else
    hipLaunchKernelGGL((gemv_reduce_kv_kernel<2>), grid, dim3(256), 0, stream, (const f32x4*)ws, splits, R, pos_dev,
                       (const bf16*)rope_cos, (const bf16*)rope_sin, (bf16*)k_cache, (bf16*)v_cache, n_heads, Tmax,
                       (bf16*)q_out, ldq);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_decode_gemv_swiglu(const void* W, int ldw, const void* X, int ldx, int R, int F, int K, void* ws,
                                       size_t ws_bytes, void* h, int ldh, hipStream_t stream) {
  if (!W || !X || !h) return OSPO_ERR_ARG;
  const int N = 2 * F;
  if (F % 64 || !ospo_decode_gemv_fusable(R, N, K)) return OSPO_ERR_UNSUPPORTED;
  if ((ldw != 0 && ldw < K) || ldx < K || ldw % 8 || ldx % 8 || ldh < F) return OSPO_ERR_SHAPE;
  if (!aligned16(W) || !aligned16(X)) return OSPO_ERR_ALIGN;
  int splits = 0;
  const int rc = gemv3_partials((const bf16*)W, ldw, (const bf16*)X, ldx, R, N, K, (f32x4*)ws, ws_bytes, stream, splits);
  if (rc != OSPO_OK) return rc;
  const dim3 grid(F / 64, (R + 15) / 16);
  if (R <= 16)
    hipLaunchKernelGGL((gemv_reduce_swiglu_kernel<1>), grid, dim3(256), 0, stream, (const f32x4*)ws, splits, R, F,
                       (bf16*)h, ldh);
  else
    hipLaunchKernelGGL((gemv_reduce_swiglu_kernel<2>), grid, dim3(256), 0, stream, (const f32x4*)ws, splits, R, F,
                       (bf16*)h, ldh);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" size_t ospo_decode_linear_ws_bytes(int R, int N, int K) {
  if (R <= 0 || R > 32 || N <= 0 || N % G3_ROWS || N / G3_ROWS > DL_CNT_BYTES / 4 || K < 32 || K % 32) return 0;
  const int kp = gemv3_kper(N, K), splits = (K + kp - 1) / kp;
  return DL_CNT_BYTES + (size_t)splits * (N / 16) * ((R + 15) / 16) * 64 * sizeof(f32x4);
}

extern "C" int ospo_decode_linear(const void* W, const void* X, int ldx, int R, int N, int K, const float* ss_in,
                                  int ss_groups, const void* ln_w, float eps, int epi, const void* bias, int gelu,
                                  const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* pos_dev,
                                  const void* rope_cos, const void* rope_sin, void* k_cache, void* v_cache, int n_heads,
                                  int Tmax, void* ws, size_t ws_bytes, hipStream_t stream);
static int decode_linear_impl(const void* W, const void* X, int ldx, int R, int N, int K, const float* ss_in,
                              int ss_groups, const void* ln_w, float eps, int epi, const void* bias, int gelu,
                              const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* pos_dev,
                              const void* rope_cos, const void* rope_sin, void* k_cache, void* v_cache, int n_heads,
                              int Tmax, void* ws, size_t ws_bytes, hipStream_t stream, int kv_hm, int nh);

extern "C" int ospo_decode_qkv_heads(const void* W_hm, const void* X, int ldx, int R, int D, const float* ss_in,
                                     int ss_groups, const void* ln_w, float eps, void* q_out, int ldo,
                                     const int* pos_dev, const void* rope_cos, const void* rope_sin, void* k_cache,
                                     void* v_cache, int n_heads, int h0, int nh, int Tmax, void* ws, size_t ws_bytes,
                                     hipStream_t stream) {
  if (!W_hm || !q_out || !k_cache || !v_cache) return OSPO_ERR_ARG;
  if (n_heads <= 0 || h0 < 0 || nh <= 0 || h0 + nh > n_heads || D != n_heads * HD) return OSPO_ERR_SHAPE;
  // head-major tiled rows: head h's q, k, v groups are rows 384 h .. 384 h + 383 (16-row tiles of K / 32 x 512)
  const bf16* W = (const bf16*)W_hm + (long)h0 * 3 * HD * D;
  return decode_linear_impl(W, X, ldx, R, 3 * nh * HD, D, ss_in, ss_groups, ln_w, eps, DL_KV, nullptr, 0, nullptr, 0,
                            (bf16*)q_out + h0 * HD, ldo, nullptr, pos_dev, rope_cos, rope_sin,
                            (bf16*)k_cache + (long)h0 * Tmax * HD, (bf16*)v_cache + (long)h0 * Tmax * HD, n_heads, Tmax,
                            ws, ws_bytes, stream, 1, nh);
}

extern "C" int ospo_decode_mlp(const void* W_gu, const void* W_down, const void* xmid, int ldx, int R, int D, int F,
                               const float* ss_in, int ss_groups, const void* ln_w, float eps, void* h, int ldh,
                               void* out, int ldo, float* ss_out, const int* step_dev, int layer, unsigned* flags,
                               unsigned* tmo, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!W_gu || !W_down || !xmid || !ss_in || !ln_w || !h || !out || !step_dev || !flags || !tmo || !ws)
    return OSPO_ERR_ARG;
  if (R <= 0 || R > 32 || D <= 0 || F <= 0 || D % G3_ROWS || (2 * F) % G3_ROWS || F % 64 || D % 32) return OSPO_ERR_SHAPE;
  if (ldx < D || ldx % 8 || ldh < F || ldh % 8 || ldo < D || layer < 0 || layer >= 63) return OSPO_ERR_SHAPE;
  if (ss_groups <= 0 || ss_groups > 32 || !(eps >= 0.f)) return OSPO_ERR_ARG;
  const size_t need = ospo_decode_linear_ws_bytes(R, D, F);
  if (need == 0 || ws_bytes < need) return OSPO_ERR_ARG;
  if (!aligned16(W_gu) || !aligned16(W_down) || !aligned16(xmid) || !aligned16(h) || !aligned16(ws) ||
      !aligned16(ln_w))
    return OSPO_ERR_ALIGN;
  // the one-launch form needs exactly the plans of the two launches: gate|up one workgroup per row group with
  // all its splits (U = splits = 4), down the pipelined form with one split per workgroup
  const int kg = gemv3_kper(2 * F, D), sg = (D + kg - 1) / kg, ng = 2 * F / G3_ROWS;
  const int kd = gemv3_kper(D, F), sd = (F + kd - 1) / kd, nd = D / G3_ROWS;
  if (dlin_pipe_units(ng, sg, D, kg) != 4 || sg != 4 || dlin_pipe_units(nd, sd, F, kd) != 1) return OSPO_ERR_UNSUPPORTED;
  if ((long)R * ldh * 2 >= (1L << 31)) return OSPO_ERR_UNSUPPORTED;  // the h stores' buffer range
  DlArgs g;
  g.W = (const bf16*)W_gu; g.X = (const bf16*)xmid; g.ldx = ldx; g.R = R; g.K = D; g.kper = kg;
  g.ss_in = ss_in; g.ss_groups = ss_groups; g.ln_w = (const bf16*)ln_w; g.eps = eps;
  g.bias = nullptr; g.gelu = 0; g.res = nullptr; g.ldr = 0; g.out = (bf16*)h; g.ldo = ldh; g.ss_out = nullptr;
  g.pos = nullptr; g.cs = g.sn = nullptr; g.kc = g.vc = nullptr; g.H = 0; g.Tmax = 0;
  g.cnt = nullptr; g.part = nullptr; g.part_bytes = 0;  // (all splits in registers: no partials, no tickets)
  g.hflag = flags; g.epoch_step = step_dev; g.epoch_layer = layer; g.tmo = tmo;
  DlArgs d = g;
  d.W = (const bf16*)W_down; d.X = (const bf16*)h; d.ldx = ldh; d.K = F; d.kper = kd;
  d.ss_in = nullptr; d.ss_groups = 0; d.ln_w = nullptr; d.eps = 0.f;
  d.res = (const bf16*)xmid; d.ldr = ldx; d.out = (bf16*)out; d.ldo = ldo; d.ss_out = ss_out;
  d.cnt = (unsigned*)ws; d.part = (float*)((char*)ws + DL_CNT_BYTES); d.part_bytes = (int)(need - DL_CNT_BYTES);
  const dim3 grid(ng + nd * sd);
  if (R <= 16)
    hipLaunchKernelGGL((dmlp_kernel<1, 4>), grid, dim3(64 * G3_WAVES), 0, stream, g, d, ng, nd, sd);
  else
    hipLaunchKernelGGL((dmlp_kernel<2, 4>), grid, dim3(64 * G3_WAVES), 0, stream, g, d, ng, nd, sd);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_decode_attn_o(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int n_heads,
                                  int Tmax, const int* start, const int* pos_dev, float scale, void* attn_out,
                                  int ld_attn, const void* W_o, const void* residual, int ldr, void* out, int ldo,
                                  float* ss_out, const int* step_dev, int layer, unsigned* flags, unsigned* tmo,
                                  void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!q || !k_cache || !v_cache || !start || !pos_dev || !attn_out || !W_o || !residual || !out || !step_dev ||
      !flags || !tmo || !ws)
    return OSPO_ERR_ARG;
  const int D = n_heads * HD;
  if (R <= 0 || R > 32 || n_heads <= 0 || Tmax <= 0 || Tmax > ATT_MAXT || layer < 0 || layer >= 63) return OSPO_ERR_SHAPE;
  if (ldq < D || ldq % 8 || ld_attn < D || ld_attn % 8 || ldr < D || ldo < D) return OSPO_ERR_SHAPE;
  const size_t need = ospo_decode_linear_ws_bytes(R, D, D);
  if (need == 0 || ws_bytes < need) return OSPO_ERR_ARG;
  if (!aligned16(q) || !aligned16(k_cache) || !aligned16(v_cache) || !aligned16(attn_out) || !aligned16(W_o) ||
      !aligned16(ws))
    return OSPO_ERR_ALIGN;
  // the o workgroups take one 512-k chunk = four heads each, with decode_linear's split plan
  const int kper = gemv3_kper(D, D), splits = (D + kper - 1) / kper, ngroups = D / G3_ROWS;
  if (kper != G2_KC || D % G2_KC || (long)R * ld_attn * 2 >= (1L << 31)) return OSPO_ERR_UNSUPPORTED;
  AttnArgs at;
  at.q = (const bf16*)q; at.ldq = ldq; at.kc = (const bf16*)k_cache; at.vc = (const bf16*)v_cache;
  at.H = n_heads; at.Tmax = Tmax; at.start = start; at.pos = pos_dev; at.scale = scale;
  at.out = (bf16*)attn_out; at.ldo = ld_attn; at.R = R;
  DlArgs o;
  o.W = (const bf16*)W_o; o.X = (const bf16*)attn_out; o.ldx = ld_attn; o.R = R; o.K = D; o.kper = kper;
  o.ss_in = nullptr; o.ss_groups = 0; o.ln_w = nullptr; o.eps = 0.f;
  o.bias = nullptr; o.gelu = 0; o.res = (const bf16*)residual; o.ldr = ldr;
  o.out = (bf16*)out; o.ldo = ldo; o.ss_out = ss_out;
  o.pos = nullptr; o.cs = o.sn = nullptr; o.kc = o.vc = nullptr; o.H = n_heads; o.Tmax = 0;
  o.cnt = (unsigned*)ws; o.part = (float*)((char*)ws + DL_CNT_BYTES); o.part_bytes = (int)(need - DL_CNT_BYTES);
  o.hflag = flags; o.epoch_step = step_dev; o.epoch_layer = layer; o.tmo = tmo;
  const int nrp = (R + 1) / 2, n_attn = nrp * n_heads;
  const dim3 grid(n_attn + ngroups * splits);
  auto kfn = R <= 16 ? dattn_o_kernel<1> : dattn_o_kernel<2>;
#ifdef OSPO_ABLATION
  static const int var = getenv("OSPO_ATTN_O_VAR") ? atoi(getenv("OSPO_ATTN_O_VAR")) : 0;
  if (var == 1) kfn = R <= 16 ? dattn_o_kernel<1, true> : dattn_o_kernel<2, true>;
  if (var == 2) kfn = R <= 16 ? dattn_o2_kernel<1> : dattn_o2_kernel<2>;
#endif
  hipLaunchKernelGGL(kfn, grid, dim3(64 * G3_WAVES), 0, stream, at, o, n_attn, nrp, ngroups, splits);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_decode_linear(const void* W, const void* X, int ldx, int R, int N, int K, const float* ss_in,
                                  int ss_groups, const void* ln_w, float eps, int epi, const void* bias, int gelu,
                                  const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* pos_dev,
                                  const void* rope_cos, const void* rope_sin, void* k_cache, void* v_cache, int n_heads,
                                  int Tmax, void* ws, size_t ws_bytes, hipStream_t stream) {
  return decode_linear_impl(W, X, ldx, R, N, K, ss_in, ss_groups, ln_w, eps, epi, bias, gelu, residual, ldr, out, ldo,
                            ss_out, pos_dev, rope_cos, rope_sin, k_cache, v_cache, n_heads, Tmax, ws, ws_bytes, stream, 0,
                            n_heads);
}

// kv_hm / nh: ospo_decode_qkv_heads' head-range launch (head-major row groups, nh heads of the n_heads the cache
// strides use); ospo_decode_linear: 0 / n_heads
static int decode_linear_impl(const void* W, const void* X, int ldx, int R, int N, int K, const float* ss_in,
                              int ss_groups, const void* ln_w, float eps, int epi, const void* bias, int gelu,
                              const void* residual, int ldr, void* out, int ldo, float* ss_out, const int* pos_dev,
                              const void* rope_cos, const void* rope_sin, void* k_cache, void* v_cache, int n_heads,
                              int Tmax, void* ws, size_t ws_bytes, hipStream_t stream, int kv_hm, int nh) {
  if (!W || !X || !out || !ws) return OSPO_ERR_ARG;
  const size_t need = ospo_decode_linear_ws_bytes(R, N, K);
  if (need == 0 || ldx < K || ldx % 8) return OSPO_ERR_SHAPE;
  if (ws_bytes < need) return OSPO_ERR_ARG;
  if (!aligned16(W) || !aligned16(X) || !aligned16(ws)) return OSPO_ERR_ALIGN;
  if (ss_in && (ss_groups <= 0 || !ln_w || !aligned16(ln_w) || !(eps >= 0.f))) return OSPO_ERR_ARG;
  if (ss_in && ss_groups > 32) return OSPO_ERR_UNSUPPORTED;  // rows of <= 4096 columns (32 groups of 128)
  if (epi == DL_PLAIN) {
    if (ldo < N || (residual && ldr < N)) return OSPO_ERR_SHAPE;
  } else if (epi == DL_KV) {
    if (bias || gelu || residual || ss_out) return OSPO_ERR_UNSUPPORTED;
    if (!pos_dev || !rope_cos || !rope_sin || !k_cache || !v_cache) return OSPO_ERR_ARG;
    if (n_heads <= 0 || nh <= 0 || N != 3 * nh * HD || ldo < nh * HD || Tmax <= 0) return OSPO_ERR_SHAPE;
  } else if (epi == DL_SWIGLU) {
    if (bias || gelu || residual || ss_out) return OSPO_ERR_UNSUPPORTED;
    if (ldo < N / 2) return OSPO_ERR_SHAPE;
  } else {
    return OSPO_ERR_ARG;
  }
  const int kper = gemv3_kper(N, K), splits = (K + kper - 1) / kper;
  DlArgs a;
  a.W = (const bf16*)W; a.X = (const bf16*)X; a.ldx = ldx; a.R = R; a.K = K; a.kper = kper;
  a.ss_in = ss_in; a.ss_groups = ss_groups; a.ln_w = (const bf16*)ln_w; a.eps = eps;
  a.bias = (const bf16*)bias; a.gelu = gelu; a.res = (const bf16*)residual; a.ldr = ldr;
  a.out = (bf16*)out; a.ldo = ldo; a.ss_out = ss_out;
  a.pos = pos_dev; a.cs = (const bf16*)rope_cos; a.sn = (const bf16*)rope_sin; a.kc = (bf16*)k_cache;
  a.vc = (bf16*)v_cache; a.H = n_heads; a.Tmax = Tmax; a.kv_hm = kv_hm;
  a.cnt = (unsigned*)ws; a.part = (float*)((char*)ws + DL_CNT_BYTES); a.part_bytes = (int)(need - DL_CNT_BYTES);
  const bool norm = ss_in != nullptr;
  // the pipelined form (dlin_pipe_kernel, U splits per workgroup, at most one workgroup per CU) where the shape
  // allows it, else one workgroup per (row group, split).  Ablation build: OSPO_DLIN_PIPE=0 runs dlin_kernel
  // (the A/B), OSPO_DLIN_V2 the rejected streaming form (~256 long-lived workgroups)
  const int ngroups = N / G3_ROWS;
  int U = dlin_pipe_units(ngroups, splits, K, kper);
  bool v2 = false;
#ifdef OSPO_ABLATION
  static const bool want_v2 = getenv("OSPO_DLIN_V2") != nullptr;
  static const int pipe_env = getenv("OSPO_DLIN_PIPE") ? atoi(getenv("OSPO_DLIN_PIPE")) : -1;
  if (pipe_env == 1) U = dlin_pipe_units(ngroups, splits, K, kper, true);  // A/B: every shape it fits
  if (pipe_env == 0 || want_v2) U = 0;
  v2 = want_v2 && (kper + G2_KC - 1) / G2_KC <= DL2_MAXC;
  const int G = std::max(1, (ngroups * splits + DL2_WGS - 1) / DL2_WGS), nsets = (ngroups + G - 1) / G;
#define DLIN_V2(NT_, EPI_)                                                                                           \
  if (v2) {                                                                                                          \
    hipLaunchKernelGGL((norm ? dlin2_kernel<NT_, EPI_, true> : dlin2_kernel<NT_, EPI_, false>), dim3(splits * nsets), \
                       dim3(64 * G3_WAVES), 0, stream, a, splits, G, ngroups);                                       \
  } else
#else
#define DLIN_V2(NT_, EPI_)
#endif
#define DLIN_PIPE(NT_, EPI_, U_)                                                                                     \
  hipLaunchKernelGGL((norm ? dlin_pipe_kernel<NT_, EPI_, true, U_> : dlin_pipe_kernel<NT_, EPI_, false, U_>),         \
                     dim3(ngroups, splits / U_), dim3(64 * G3_WAVES), 0, stream, a)
#define DLIN(NT_, EPI_)                                                                                              \
  DLIN_V2(NT_, EPI_)                                                                                                 \
  if (U == 1) {                                                                                                      \
    DLIN_PIPE(NT_, EPI_, 1);                                                                                         \
  } else if (U == 2) {                                                                                               \
    DLIN_PIPE(NT_, EPI_, 2);                                                                                         \
  } else if (U == 4) {                                                                                               \
    DLIN_PIPE(NT_, EPI_, 4);                                                                                         \
  } else {                                                                                                           \
    hipLaunchKernelGGL((norm ? dlin_kernel<NT_, EPI_, true> : dlin_kernel<NT_, EPI_, false>), dim3(ngroups, splits),  \
                       dim3(64 * G3_WAVES), 0, stream, a);                                                           \
  }
#define DLIN_NT(EPI_) \
  if (R <= 16) { DLIN(1, EPI_); } else { DLIN(2, EPI_); }
  if (epi == DL_PLAIN) {
    DLIN_NT(DL_PLAIN)
  } else if (epi == DL_KV) {
    DLIN_NT(DL_KV)
  } else {
    DLIN_NT(DL_SWIGLU)
  }
#undef DLIN_NT
#undef DLIN
#undef DLIN_PIPE
#undef DLIN_V2
  (void)v2;
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_decode_gemv(const void* W, int ldw, const void* X, int ldx, int R, int N, int K, const void* bias,
                                int gelu, const void* residual, int ldr, void* out, int ldo, void* ws, size_t ws_bytes,
                                hipStream_t stream) {
  if (!W || !X || !out) return OSPO_ERR_ARG;
  if (R <= 0 || R > 64 || N <= 0 || N % 16 || K <= 0 || K % 32) return OSPO_ERR_SHAPE;
  if (ldw == 0 && (g_gemv_variant != 3 || R > 32 || N % G3_ROWS)) return OSPO_ERR_UNSUPPORTED;  // tiled: v3 only
  if ((ldw != 0 && ldw < K) || ldx < K || ldo < N || ldw % 8 || ldx % 8 || (residual && (ldr < N))) return OSPO_ERR_SHAPE;
  if (!aligned16(W) || !aligned16(X)) return OSPO_ERR_ALIGN;
  const int nt = (R + 15) / 16, nb = N / 16;
  const bf16 *w = (const bf16*)W, *x = (const bf16*)X, *bs = (const bf16*)bias, *rs = (const bf16*)residual;
  bf16* o = (bf16*)out;
  f32x4* wsp = (f32x4*)ws;
  if (g_gemv_variant == 3 && R <= 32 && N % G3_ROWS == 0 && K >= 8) {
    const int kper = gemv3_kper(N, K);
    const int splits = (K + kper - 1) / kper;
    if (splits > 1 && (!ws || ws_bytes < ospo_decode_gemv_ws_bytes(R, N, K) || !aligned16(ws))) return OSPO_ERR_ARG;
    const dim3 grid(N / G3_ROWS, splits);
#define GEMV3(NT_)                                                                                                \
  {                                                                                                               \
    auto kfn = ldw == 0 ? gemv3_kernel<NT_, true> : gemv3_kernel<NT_, false>;                                     \
    hipLaunchKernelGGL(kfn, grid, dim3(64 * G3_WAVES), 0, stream, w, ldw, x, ldx, R, K, kper, bs, gelu, rs, ldr, o,  \
                       ldo, wsp);                                                                                 \
  }                                                                                                               \
  if (splits > 1)                                                                                                 \
    hipLaunchKernelGGL((gemv2_reduce_kernel<NT_>), dim3((nb + 3) / 4), dim3(256), 0, stream, wsp, splits, nb, R, bs,    \
                       gelu, rs, ldr, o, ldo);
    if (nt == 1) {
      GEMV3(1)
    } else {
      GEMV3(2)
    }
#undef GEMV3
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  if (g_gemv_variant >= 2 && R <= 32 && N % G2_ROWS == 0 && K >= 8) {
    const int kper = gemv2_kper(N, K);
    const int splits = (K + kper - 1) / kper;
    if (splits > 1 && (!ws || ws_bytes < ospo_decode_gemv_ws_bytes(R, N, K) || !aligned16(ws))) return OSPO_ERR_ARG;
    const dim3 grid(N / G2_ROWS, splits);
#define GEMV2(NT_)                                                                                              \
  hipLaunchKernelGGL((gemv2_kernel<NT_>), grid, dim3(256), 0, stream, w, ldw, x, ldx, R, K, kper, bs, gelu, rs, ldr, \
                     o, ldo, wsp);                                                                              \
  if (splits > 1)                                                                                               \
    hipLaunchKernelGGL((gemv2_reduce_kernel<NT_>), dim3((nb + 3) / 4), dim3(256), 0, stream, wsp, splits, nb, R, bs,  \
                       gelu, rs, ldr, o, ldo);
    if (nt == 1) {
      GEMV2(1)
    } else {
      GEMV2(2)
    }
#undef GEMV2
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  const int splits = gemv_splits(nb, K);
  if (splits > 1 && (!ws || ws_bytes < ospo_decode_gemv_ws_bytes(R, N, K) || !aligned16(ws))) return OSPO_ERR_ARG;
  const dim3 grid(nb, splits);
#define GEMV(NT_)                                                                                                   \
  hipLaunchKernelGGL((gemv_kernel<NT_>), grid, dim3(64 * SK_WAVES), 0, stream, w, ldw, x, ldx, R, K, bs, gelu, rs, ldr, \
                     o, ldo, wsp);                                                                                  \
  if (splits > 1)                                                                                                   \
    hipLaunchKernelGGL((gemv_reduce_kernel<NT_>), dim3(nb), dim3(64 * NT_), 0, stream, wsp, splits, nb, R, bs, gelu,   \
                       rs, ldr, o, ldo);
  switch (nt) {
    case 1: GEMV(1) break;
    case 2: GEMV(2) break;
    case 3: GEMV(3) break;
    default: GEMV(4) break;
  }
#undef GEMV
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_kv_store(void* qkv, int ld, int R, int nq, const int* pos_dev, int rope, const void* rope_cos,
                             const void* rope_sin, void* k_cache, void* v_cache, int n_heads, int head_dim, int Tmax,
                             void* q_out, int ld_q, hipStream_t stream) {
  if (!qkv || !k_cache || !v_cache) return OSPO_ERR_ARG;
  if (head_dim != HD) return OSPO_ERR_UNSUPPORTED;
  if (R <= 0 || nq <= 0 || n_heads <= 0 || Tmax <= 0 || ld < 3 * n_heads * HD || ld % 8) return OSPO_ERR_SHAPE;
  if (rope && (!rope_cos || !rope_sin)) return OSPO_ERR_ARG;
  if (q_out && (ld_q < n_heads * HD || ld_q % 8)) return OSPO_ERR_SHAPE;
  if (!aligned16(qkv) || !aligned16(k_cache) || !aligned16(v_cache) || (q_out && !aligned16(q_out)))
    return OSPO_ERR_ALIGN;
  const long total = (long)R * nq * n_heads * 8;
  hipLaunchKernelGGL(kv_store_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, (bf16*)qkv, ld, R,
                     nq, pos_dev, rope, (const bf16*)rope_cos, (const bf16*)rope_sin, (bf16*)k_cache, (bf16*)v_cache,
                     n_heads, Tmax, (bf16*)q_out, ld_q);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_attn_cache(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int nq,
                               int n_heads, int head_dim, int Tmax, const int* start, const int* pos_dev, float scale,
                               void* out, int ldo, hipStream_t stream) {
  if (!q || !k_cache || !v_cache || !start || !out) return OSPO_ERR_ARG;
  if (head_dim != HD) return OSPO_ERR_UNSUPPORTED;
  if (R <= 0 || nq <= 0 || n_heads <= 0 || Tmax <= 0 || Tmax > ATT_MAXT) return OSPO_ERR_SHAPE;
  if (ldq < n_heads * HD || ldo < n_heads * HD || ldq % 2 || ldo % 2) return OSPO_ERR_SHAPE;
  // v2 (16-B loads) needs 16-B aligned q / out rows and caches; else the 4-B form
  const bool v2 = ldq % 8 == 0 && ldo % 8 == 0 && aligned16(q) && aligned16(out) && aligned16(k_cache) &&
                  aligned16(v_cache);
  hipLaunchKernelGGL(v2 ? attn_cache2_kernel : attn_cache_kernel, dim3(R * nq, n_heads), dim3(256), 0, stream,
                     (const bf16*)q, ldq, (const bf16*)k_cache, (const bf16*)v_cache, n_heads, Tmax, start, pos_dev, nq,
                     scale, (bf16*)out, ldo);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_attn_cache_heads(const void* q, int ldq, const void* k_cache, const void* v_cache, int R, int nq,
                                     int n_heads, int h0, int nh, int Tmax, const int* start, const int* pos_dev,
                                     float scale, void* out, int ldo, hipStream_t stream) {
  if (!q || !k_cache || !v_cache || !start || !out) return OSPO_ERR_ARG;
  if (R <= 0 || nq <= 0 || n_heads <= 0 || h0 < 0 || nh <= 0 || h0 + nh > n_heads || Tmax <= 0 || Tmax > ATT_MAXT)
    return OSPO_ERR_SHAPE;
  if (ldq < n_heads * HD || ldo < n_heads * HD || ldq % 8 || ldo % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(q) || !aligned16(out) || !aligned16(k_cache) || !aligned16(v_cache)) return OSPO_ERR_ALIGN;
  // heads h0 .. h0 + nh - 1: the same kernel with its pointers at head h0 (the cache strides keep n_heads)
  hipLaunchKernelGGL(attn_cache2_kernel, dim3(R * nq, nh), dim3(256), 0, stream, (const bf16*)q + h0 * HD, ldq,
                     (const bf16*)k_cache + (long)h0 * Tmax * HD, (const bf16*)v_cache + (long)h0 * Tmax * HD, n_heads,
                     Tmax, start, pos_dev, nq, scale, (bf16*)out + h0 * HD, ldo);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_cfg_sample(const void* logits, int ldl, int V, int B, float cfg_weight, float temperature,
                               const float* u, const int* step_dev, int n_steps, int* tokens, int* next_ids,
                               float* probs_out, hipStream_t stream) {
  if (!logits || !u || !tokens || !next_ids) return OSPO_ERR_ARG;
  if (V <= 0 || V > 256 * SMP_CHUNK || B <= 0 || ldl < V || n_steps <= 0) return OSPO_ERR_SHAPE;
  if (!(temperature > 0.f)) return OSPO_ERR_ARG;
  hipLaunchKernelGGL(cfg_sample_kernel, dim3(B), dim3(256), 0, stream, (const bf16*)logits, ldl, V, cfg_weight,
                     temperature, u, B, step_dev, n_steps, tokens, next_ids, probs_out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_decode_advance(int* pos_dev, int* step_dev, hipStream_t stream) {
  if (!pos_dev || !step_dev) return OSPO_ERR_ARG;
  hipLaunchKernelGGL(advance_kernel, dim3(1), dim3(64), 0, stream, pos_dev, step_dev);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_embed_rows(const int* ids, long n, const void* table, int vocab, int D, void* out,
                               hipStream_t stream) {
  if (!ids || !table || !out) return OSPO_ERR_ARG;
  if (n <= 0 || vocab <= 0 || D <= 0 || D % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(table) || !aligned16(out)) return OSPO_ERR_ALIGN;
  const long total = n * (D / 8);
  hipLaunchKernelGGL(embed_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, ids, n,
                     (const bf16*)table, vocab, D, (bf16*)out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
