// Memory-bound kernels of the SimPO step on gfx950: RMSNorm, RoPE, SwiGLU,
// GELU, input assembly, row gather/scatter, the gen_head log-prob, the SimPO
// loss, LoRA operand packing and the fused clip + AdamW.  All bf16 traffic is
// 16 B per lane (8 bf16); reductions are wave shuffles (64 lanes) + LDS.
#include "common.h"
#include "mx8.h"

#include <math.h>

#include <algorithm>

namespace {

// block-wide sum for 256-thread blocks
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}
__device__ __forceinline__ float block_max256(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}


constexpr int RMS_MAXIT = 8;  // D <= 256 threads * 8 it * 8 = 16384

// ------------------------------------------------------------------ RMSNorm
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                          bf16* __restrict__ y, float* __restrict__ rstd, int D,
                                                          float eps) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int nch = D / 8;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * D);
  u32x4 v[RMS_MAXIT];
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < RMS_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      v[it] = xr[c];
      float f[8];
      unpack8(v[it], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += f[q] * f[q];
    }
  }
  const float tot = block_sum256(ss, red);
  const float r = rsqrtf(tot / (float)D + eps);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4* yr = reinterpret_cast<u32x4*>(y + row * D);
#pragma unroll
  for (int it = 0; it < RMS_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      float f[8], g[8];
      unpack8(v[it], f);
      unpack8(wr[c], g);
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = g[q] * round_bf(f[q] * r);
      yr[c] = pack8(f);
    }
  }
  if (threadIdx.x == 0) rstd[row] = r;
}

__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                          const bf16* __restrict__ w, const float* __restrict__ rstd,
                                                          const bf16* __restrict__ dres, bf16* __restrict__ dx,
                                                          int D) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const int nch = D / 8;
  const float r = rstd[row];
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * D);
  const u32x4* dr = reinterpret_cast<const u32x4*>(dy + row * D);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4 xv[RMS_MAXIT], gv[RMS_MAXIT];
  float dot = 0.f;
#pragma unroll
  for (int it = 0; it < RMS_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      xv[it] = xr[c];
      float f[8], d[8], ww[8];
      unpack8(xv[it], f);
      unpack8(dr[c], d);
      unpack8(wr[c], ww);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        d[q] *= ww[q];
        dot += d[q] * f[q] * r;
      }
      gv[it] = pack8(d);  // dy*w rounded is not reused for math below; recompute in fp32
    }
  }
  const float mdot = block_sum256(dot, red) / (float)D;
  u32x4* outr = reinterpret_cast<u32x4*>(dx + row * D);
  const u32x4* rr = dres ? reinterpret_cast<const u32x4*>(dres + row * D) : nullptr;
#pragma unroll
  for (int it = 0; it < RMS_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      float f[8], d[8], ww[8], o[8];
      unpack8(xv[it], f);
      unpack8(dr[c], d);
      unpack8(wr[c], ww);
      float res[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (rr) unpack8(rr[c], res);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = res[q] + r * (d[q] * ww[q] - f[q] * r * mdot);
      outr[c] = pack8(o);
    }
  }
  (void)gv;
}

// Wave-per-row forms (D <= 64 lanes x 16 chunks x 8 = 8192): every load of the row is
// issued before the first use (IT x 16 B in flight per lane), the reduction is a
// wave shuffle, 4 rows per workgroup -- ~3x the bytes in flight of the block form.
template <int IT, bool FULL>
__global__ __launch_bounds__(256) void rmsnorm_fwd_w_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                            bf16* __restrict__ y, float* __restrict__ rstd, long M,
                                                            int D, float eps, const Mx8Out mo) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = D >> 3;
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * D);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  u32x4 v[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) v[it] = xr[c];
  }
  float ss = 0.f;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) {
      float f[8];
      unpack8(v[it], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) ss += f[q] * f[q];
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
  // re-unpack in the second pass instead of keeping IT x 8 floats alive (occupancy)
#pragma unroll
  for (int it = 0; it < IT; ++it) asm volatile("" : "+v"(v[it]));
  asm volatile("" ::: "memory");  // keep the w loads in this pass
  u32x4* yr = reinterpret_cast<u32x4*>(y + row * D);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) {
      float f[8], g[8];
      unpack8(v[it], f);
      unpack8(wr[c], g);
#pragma unroll
      for (int q = 0; q < 8; ++q) f[q] = g[q] * round_bf(f[q] * r);
      const u32x4 pk = pack8(f);
      yr[c] = pk;
      if (mo.q) {  // the fp8 variant's GEMM operand, from the bf16 values just stored
        unpack8(pk, f);
        mx8_store8(mo, row, c, f);
      }
    }
  }
  if (lane == 0) rstd[row] = r;
}

// EARLY (ablation build, OSPO_RMS_EARLY=1): the residual-grad loads issued with x and dy, before the dot (one
// memory round trip per row instead of two; 154 against 150 VGPRs, both 3 waves per SIMD): bit-identical and
// slower, 31.2 / 32.7 against 30.1 / 30.4 us at M 4800 x D 4096 (profiles/r06/rmsnorm_bwd_early_ab.log)
template <int IT, bool FULL, bool EARLY = false>
__global__ __launch_bounds__(256) void rmsnorm_bwd_w_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                            const bf16* __restrict__ w, const float* __restrict__ rstd,
                                                            const bf16* __restrict__ dres, bf16* __restrict__ dx,
                                                            long M, int D, const Mx8Out mo) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = D >> 3;
  const float r = rstd[row];
  const u32x4* xr = reinterpret_cast<const u32x4*>(x + row * D);
  const u32x4* dr = reinterpret_cast<const u32x4*>(dy + row * D);
  const u32x4* wr = reinterpret_cast<const u32x4*>(w);
  const u32x4* rr = dres ? reinterpret_cast<const u32x4*>(dres + row * D) : nullptr;
  // x and dy (the dot's operands) first; the residual grad is loaded after the dot, so it does not
  // hold IT more registers across it (round 2: 160 -> ~110 VGPRs; 150 on the round-6 compiler, 3 waves per SIMD)
  u32x4 xv[IT], dv[IT], rv[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) {
      xv[it] = __builtin_nontemporal_load(xr + c);  // (read once: non-temporal)
      dv[it] = __builtin_nontemporal_load(dr + c);
      if (EARLY && rr) rv[it] = __builtin_nontemporal_load(rr + c);
    }
  }
  float dot = 0.f;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) {
      float f[8], d[8], ww[8];
      unpack8(xv[it], f);
      unpack8(dv[it], d);
      unpack8(wr[c], ww);
#pragma unroll
      for (int q = 0; q < 8; ++q) dot += d[q] * ww[q] * f[q] * r;
    }
  }
  const float mdot = wave_sum(dot) / (float)D;
  asm volatile("" ::: "memory");  // the residual loads stay below the dot
  if (!EARLY && rr) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int c = it * 64 + lane;
      if (FULL || c < nch) rv[it] = __builtin_nontemporal_load(rr + c);
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) asm volatile("" : "+v"(xv[it]), "+v"(dv[it]));
  asm volatile("" ::: "memory");
  u32x4* outr = reinterpret_cast<u32x4*>(dx + row * D);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int c = it * 64 + lane;
    if (FULL || c < nch) {
      float f[8], d[8], ww[8], o[8];
      unpack8(xv[it], f);
      unpack8(dv[it], d);
      unpack8(wr[c], ww);
      float res[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (rr) unpack8(rv[it], res);
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = res[q] + r * (d[q] * ww[q] - f[q] * r * mdot);
      const u32x4 pk = pack8(o);
      outr[c] = pk;
      if (mo.q) {
        unpack8(pk, o);
        mx8_store8(mo, row, c, o);
      }
    }
  }
}

// --------------------------------------------------------------------- RoPE
// one thread = 8 rotation pairs (i..i+7, i+h..i+h+7) of one (row, head, q|k)
template <bool BWD>
__global__ void rope_kernel(bf16* __restrict__ x, int ld, int q_col, int k_col, long rows, int T, int H, int hd,
                            const bf16* __restrict__ cs, const bf16* __restrict__ sn) {
  const int half = hd / 2;
  const int per_head = half / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = rows * H * 2 * per_head;
  if (tid >= total) return;
  const int ch = tid % per_head;
  long rest = tid / per_head;
  const int which = rest % 2;
  rest /= 2;
  const int h = rest % H;
  const long row = rest / H;
  const int t = row % T;
  bf16* base = x + row * ld + (which ? k_col : q_col) + h * hd + ch * 8;
  u32x4* p1 = reinterpret_cast<u32x4*>(base);
  u32x4* p2 = reinterpret_cast<u32x4*>(base + half);
  float a[8], b[8], c[8], s[8], o1[8], o2[8];
  unpack8(*p1, a);
  unpack8(*p2, b);
  unpack8(*reinterpret_cast<const u32x4*>(cs + (long)t * half + ch * 8), c);
  unpack8(*reinterpret_cast<const u32x4*>(sn + (long)t * half + ch * 8), s);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (!BWD) {
      // x*cos + rotate_half(x)*sin, rotate_half = [-x2, x1]; bf16 rounding per op
      o1[q] = round_bf(a[q] * c[q]) + round_bf(-b[q] * s[q]);
      o2[q] = round_bf(b[q] * c[q]) + round_bf(a[q] * s[q]);
    } else {
      o1[q] = a[q] * c[q] + b[q] * s[q];
      o2[q] = b[q] * c[q] - a[q] * s[q];
    }
  }
  *p1 = pack8(o1);
  *p2 = pack8(o2);
}

// ------------------------------------------------------------------- SwiGLU
// Grid (column blocks of 128 chunks, rows): no 64-bit division of a flat index (it was ~50 of the
// kernels' ~350 instructions per thread); consecutive threads still take consecutive 8-column chunks
// of one row (the MXFP8 stores need 4 of them per 32-block).
__global__ void swiglu_fwd_kernel(const bf16* __restrict__ gu, int ldg, bf16* __restrict__ h, int ldh, long M, int F,
                                  const Mx8Out mo) {
  const int cpr = F / 8;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cpr) return;
  const long m = blockIdx.y;
  float g[8], u[8], o[8];
  unpack8(*reinterpret_cast<const u32x4*>(gu + m * ldg + c * 8), g);
  unpack8(*reinterpret_cast<const u32x4*>(gu + m * ldg + F + c * 8), u);
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = round_bf(silu(g[q])) * u[q];
  const u32x4 pk = pack8(o);
  *reinterpret_cast<u32x4*>(h + m * ldh + c * 8) = pk;
  if (mo.q) {  // 4 consecutive threads = one 32-block of the row (F % 32 == 0)
    unpack8(pk, o);
    mx8_store8(mo, m, c, o);
  }
}

__global__ void swiglu_bwd_kernel(const bf16* __restrict__ dh, int lddh, const bf16* __restrict__ gu, int ldg,
                                  bf16* __restrict__ dgu, int lddg, long M, int F, const Mx8Out mo) {
  const int cpr = F / 8;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cpr) return;
  const long m = blockIdx.y;
  float d[8], g[8], u[8], dg[8], du[8];
  unpack8(*reinterpret_cast<const u32x4*>(dh + m * lddh + c * 8), d);
  unpack8(*reinterpret_cast<const u32x4*>(gu + m * ldg + c * 8), g);
  unpack8(*reinterpret_cast<const u32x4*>(gu + m * ldg + F + c * 8), u);
  swiglu_bwd8(d, g, u, dg, du);
  const u32x4 pg = pack8(dg), pu = pack8(du);
  *reinterpret_cast<u32x4*>(dgu + m * lddg + c * 8) = pg;
  *reinterpret_cast<u32x4*>(dgu + m * lddg + F + c * 8) = pu;
  if (mo.q) {  // [dgate | dup] as one row of 2F columns (F % 32 == 0: blocks never straddle the halves)
    unpack8(pg, dg);
    unpack8(pu, du);
    mx8_store8(mo, m, c, dg);
    mx8_store8(mo, m, F / 8 + c, du);
  }
}

// --------------------------------------------------------------------- GELU
__global__ void gelu_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long n8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float f[8];
  unpack8(reinterpret_cast<const u32x4*>(x)[i], f);
#pragma unroll
  for (int q = 0; q < 8; ++q) f[q] = gelu_erf(f[q]);
  reinterpret_cast<u32x4*>(y)[i] = pack8(f);
}
__global__ void gelu_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ xp, bf16* __restrict__ dx,
                                long n8) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float d[8], f[8];
  unpack8(reinterpret_cast<const u32x4*>(dy)[i], d);
  unpack8(reinterpret_cast<const u32x4*>(xp)[i], f);
#pragma unroll
  for (int q = 0; q < 8; ++q) d[q] *= gelu_erf_grad(f[q]);
  reinterpret_cast<u32x4*>(dx)[i] = pack8(d);
}

// ------------------------------------------------------------ input assembly
__global__ void assemble_kernel(const int* __restrict__ ids, int B, int Lt, const bf16* __restrict__ table, int V,
                                const bf16* __restrict__ img, int N, int D, bf16* __restrict__ x0, long rows) {
  const int cpr = D / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= rows * cpr) return;
  const long r = tid / cpr;
  const int c = tid % cpr;
  const int T = Lt + N;
  const int s = r / T, t = r % T;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (t < Lt) {
    const int id = ids[(s % B) * Lt + t];
    // id < 0: right padding (zero row); ids >= V are rejected by the host, clamped here so they cannot fault
    if (id >= 0) v = reinterpret_cast<const u32x4*>(table + (long)min(id, V - 1) * D)[c];
  } else {
    v = reinterpret_cast<const u32x4*>(img + ((long)s * N + (t - Lt)) * D)[c];
  }
  reinterpret_cast<u32x4*>(x0 + r * D)[c] = v;
}

__global__ void gen_aligner_in_kernel(const int* __restrict__ ids, int R, const bf16* __restrict__ emb, int V, int E,
                                      const bf16* __restrict__ w1, const bf16* __restrict__ b1, int D,
                                      bf16* __restrict__ out) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= (long)R * D) return;
  const long r = tid / D;
  const int d = tid % D;
  const bf16* e = emb + (long)min(max(ids[r], 0), V - 1) * E;
  const bf16* wr = w1 + (long)d * E;
  float acc = 0.f;
  for (int j = 0; j < E; ++j) acc += bf2f(e[j]) * bf2f(wr[j]);
  const float pre = round_bf(acc + bf2f(b1[d]));
  out[tid] = f2bf(gelu_erf(pre));
}

// E == 8, D % 8 == 0: a thread owns 8 consecutive outputs of a row -- one 16-B load of the embedding row,
// 8 x 16 B of w1 rows, one 16-B store (the scalar kernel above did 2-B accesses per output).  Same
// per-output arithmetic as gen_aligner_in_kernel (sequential fp32 dot over j, bf16 pre-activation).
__global__ void gen_aligner_in8_kernel(const int* __restrict__ ids, int R, const bf16* __restrict__ emb, int V,
                                       const bf16* __restrict__ w1, const bf16* __restrict__ b1, int D,
                                       bf16* __restrict__ out) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int cpr = D / 8;
  if (tid >= (long)R * cpr) return;
  const long r = tid / cpr;
  const int d0 = (int)(tid % cpr) * 8;
  float e[8], bb[8], o[8];
  unpack8(*reinterpret_cast<const u32x4*>(emb + (long)min(max(ids[r], 0), V - 1) * 8), e);
  unpack8(*reinterpret_cast<const u32x4*>(b1 + d0), bb);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float w[8];
    unpack8(*reinterpret_cast<const u32x4*>(w1 + (long)(d0 + q) * 8), w);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += e[j] * w[j];
    o[q] = gelu_erf(round_bf(acc + bb[q]));
  }
  *reinterpret_cast<u32x4*>(out + r * D + d0) = pack8(o);
}

__global__ void gather_rows_kernel(const bf16* __restrict__ src, int lds, int T, int t0, int N, int D,
                                   bf16* __restrict__ dst, long rows_out) {
  const int cpr = D / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= rows_out * cpr) return;
  const long r = tid / cpr;
  const int c = tid % cpr;
  const long s = r / N, i = r % N;
  reinterpret_cast<u32x4*>(dst + r * D)[c] = reinterpret_cast<const u32x4*>(src + (s * T + t0 + i) * lds)[c];
}

__global__ void scatter_rows_kernel(const bf16* __restrict__ src, int S, int T, int t0, int N, int D,
                                    bf16* __restrict__ dst, int ldd, long total_rows) {
  const int cpr = D / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= total_rows * cpr) return;
  const long r = tid / cpr;
  const int c = tid % cpr;
  const long s = r / T;
  const int t = r % T;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (s < S && t >= t0 && t < t0 + N) v = reinterpret_cast<const u32x4*>(src + (s * N + (t - t0)) * D)[c];
  reinterpret_cast<u32x4*>(dst + r * ldd)[c] = v;
}

// ------------------------------------------------------------------ logprob
constexpr int LP_MAXIT = 8;  // V <= 256 * 8 * 8 = 16384

__global__ __launch_bounds__(256) void logprob_fwd_kernel(const bf16* __restrict__ logits, int V,
                                                          const int* __restrict__ labels, float* __restrict__ lse,
                                                          float* __restrict__ tok) {
  __shared__ float red[4];
  const long r = blockIdx.x;
  const int nch = V / 8;
  const u32x4* lr = reinterpret_cast<const u32x4*>(logits + r * V);
  u32x4 v[LP_MAXIT];
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < LP_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      v[it] = lr[c];
      float f[8];
      unpack8(v[it], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) mx = fmaxf(mx, f[q]);
    }
  }
  mx = block_max256(mx, red);
  float se = 0.f;
#pragma unroll
  for (int it = 0; it < LP_MAXIT; ++it) {
    const int c = it * 256 + threadIdx.x;
    if (c < nch) {
      float f[8];
      unpack8(v[it], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) se += __expf(f[q] - mx);
    }
  }
  se = block_sum256(se, red);
  if (threadIdx.x == 0) {
    const float l = mx + __logf(se);
    lse[r] = l;
    tok[r] = bf2f(logits[r * V + min(max(labels[r], 0), V - 1)]) - l;
  }
}

__global__ __launch_bounds__(256) void seq_mean_kernel(const float* __restrict__ tok, int N, float* __restrict__ out) {
  __shared__ float red[4];
  const long s = blockIdx.x;
  float a = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) a += tok[s * N + i];
  a = block_sum256(a, red);
  if (threadIdx.x == 0) out[s] = a / (float)N;
}

__global__ void logprob_bwd_kernel(const bf16* __restrict__ logits, int V, const int* __restrict__ labels,
                                   const float* __restrict__ lse, int N, const float* __restrict__ gseq,
                                   bf16* __restrict__ dl, long R) {
  const int nch = V / 8;
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= R * nch) return;
  const long r = tid / nch;
  const int c = tid % nch;
  const float gs = gseq[r / N] / (float)N;
  const float l = lse[r];
  const int lab = labels[r];
  float f[8];
  unpack8(reinterpret_cast<const u32x4*>(logits + r * V)[c], f);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int vi = c * 8 + q;
    f[q] = gs * (((vi == lab) ? 1.f : 0.f) - __expf(f[q] - l));
  }
  reinterpret_cast<u32x4*>(dl + r * V)[c] = pack8(f);
}

// -------------------------------------------------------------------- SimPO
__device__ __forceinline__ float logsigmoid(float x) { return x >= 0.f ? -log1pf(__expf(-x)) : x - log1pf(__expf(x)); }
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(256) void simpo_fwd_kernel(const float* __restrict__ lp, int B, float beta, float gbr,
                                                        float ls, int type, float* __restrict__ losses,
                                                        float* __restrict__ mean, float* __restrict__ rewards) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    const float z = (lp[i] - lp[B + i]) - gbr;
    float l;
    if (type == 0)
      l = -logsigmoid(beta * z) * (1.f - ls) - logsigmoid(-beta * z) * ls;
    else
      l = fmaxf(1.f - beta * z, 0.f);
    losses[i] = l;
    acc += l;
    rewards[i] = beta * lp[i];
    rewards[B + i] = beta * lp[B + i];
  }
  acc = block_sum256(acc, red);
  if (threadIdx.x == 0) mean[0] = acc / (float)B;
}

__global__ void simpo_bwd_kernel(const float* __restrict__ lp, int B, float beta, float gbr, float ls, int type,
                                 const float* __restrict__ gl, float* __restrict__ glp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const float z = (lp[i] - lp[B + i]) - gbr;
  float dz;
  if (type == 0)
    dz = -beta * (1.f - ls) * sigmoidf(-beta * z) + beta * ls * sigmoidf(beta * z);
  else
    dz = (1.f - beta * z > 0.f) ? -beta : 0.f;
  dz *= gl[0] / (float)B;
  glp[i] = dz;
  glp[B + i] = -dz;
}

// ---------------------------------------------------------------- LoRA pack
// blockIdx.y = layer: sources advance by layer_stride elements of the flat LoRA
// buffer, destinations are [n_layers][...] contiguous
__global__ void lora_pack_kernel(const bf16* __restrict__ Af, const bf16* __restrict__ Bf, int nmods, int r, int Kin,
                                 int Nmod, int Rp, bf16* __restrict__ Acat, bf16* __restrict__ AcatT,
                                 bf16* __restrict__ Bcat, bf16* __restrict__ BT, long layer_stride) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long na = (long)Rp * Kin;
  const long nb = (long)nmods * Nmod * Rp;
  const int used = nmods * r;
  const long l = blockIdx.y;
  Af += l * layer_stride;
  Bf += l * layer_stride;
  Acat += l * na;
  AcatT += l * na;
  Bcat += l * nb;
  if (BT) BT += l * (long)used * Nmod;
  if (tid < na) {
    const int j = tid / Kin, k = tid % Kin;
    const bf16 v = j < used ? Af[(long)j * Kin + k] : f2bf(0.f);
    Acat[tid] = v;
    AcatT[(long)k * Rp + j] = v;
  }
  if (tid < nb) {
    const long n = tid / Rp;
    const int j = tid % Rp;
    bf16 v = f2bf(0.f);
    if (j < used && j / r == n / Nmod) v = Bf[n * r + (j % r)];
    Bcat[tid] = v;
  }
  if (BT && tid < (long)used * Nmod) {  // per-module B^T, [nmods*r, Nmod]
    const int jr = tid / Nmod, n = tid % Nmod;
    BT[tid] = Bf[((long)(jr / r) * Nmod + n) * r + (jr % r)];
  }
}

// The same repack, 8 elements (16 B) per thread in every destination: the element-wise kernel above
// wrote AcatT with 2-B stores at a 2*Rp-B stride and every region 2 B at a time (~105 us per call
// for 30 layers, ~1.3 TB/s).  Regions of the flattened chunk index: Acat [Rp][Kin], AcatT [Kin][Rp],
// Bcat [nmods*Nmod][Rp], BT [used][Nmod].  Needs r, Rp, Kin, Nmod multiples of 8 (a chunk of 8 rank
// columns then lies inside one module's block).  Bit-identical to lora_pack_kernel (pure copies).
__global__ __launch_bounds__(256) void lora_pack8_kernel(const bf16* __restrict__ Af, const bf16* __restrict__ Bf,
                                                         int nmods, int r, int Kin, int Nmod, int Rp,
                                                         bf16* __restrict__ Acat, bf16* __restrict__ AcatT,
                                                         bf16* __restrict__ Bcat, bf16* __restrict__ BT,
                                                         long layer_stride) {
  const long l = blockIdx.y;
  const int used = nmods * r;
  const long na = (long)Rp * Kin / 8, nb = (long)nmods * Nmod * Rp / 8, nbt = BT ? (long)used * Nmod / 8 : 0;
  long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  Af += l * layer_stride;
  Bf += l * layer_stride;
  const uint4 z = {0u, 0u, 0u, 0u};
  if (c < na) {  // Acat rows: row j < used copies A row j
    const int j = (int)(c / (Kin / 8));
    const int k = (int)(c % (Kin / 8)) * 8;
    const uint4 v = j < used ? *reinterpret_cast<const uint4*>(Af + (long)j * Kin + k) : z;
    *reinterpret_cast<uint4*>(Acat + l * Rp * (long)Kin + (long)j * Kin + k) = v;
    return;
  }
  c -= na;
  if (c < na) {  // AcatT row k: A[j0..j0+7][k]
    const int k = (int)(c / (Rp / 8));
    const int j0 = (int)(c % (Rp / 8)) * 8;
    unsigned short e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = j0 + q;
      e[q] = j < used ? reinterpret_cast<const unsigned short*>(Af)[(long)j * Kin + k] : (unsigned short)0;
    }
    uint4 v;
    v.x = e[0] | ((unsigned)e[1] << 16); v.y = e[2] | ((unsigned)e[3] << 16);
    v.z = e[4] | ((unsigned)e[5] << 16); v.w = e[6] | ((unsigned)e[7] << 16);
    *reinterpret_cast<uint4*>(AcatT + l * Rp * (long)Kin + (long)k * Rp + j0) = v;
    return;
  }
  c -= na;
  if (c < nb) {  // Bcat row n: B_mod(n)[n] in rank columns [r mod, r mod + r), zeros elsewhere
    const long n = c / (Rp / 8);
    const int j0 = (int)(c % (Rp / 8)) * 8;
    uint4 v = z;
    if (j0 < used && j0 / r == n / Nmod) v = *reinterpret_cast<const uint4*>(Bf + n * r + (j0 % r));
    *reinterpret_cast<uint4*>(Bcat + l * (long)nmods * Nmod * Rp + n * Rp + j0) = v;
    return;
  }
  c -= nb;
  if (c < nbt) {  // BT row jr: B_mod[n0..n0+7][jr % r]
    const int jr = (int)(c / (Nmod / 8));
    const int n0 = (int)(c % (Nmod / 8)) * 8;
    const unsigned short* src = reinterpret_cast<const unsigned short*>(Bf) + ((long)(jr / r) * Nmod + n0) * r + (jr % r);
    unsigned short e[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) e[q] = src[(long)q * r];
    uint4 v;
    v.x = e[0] | ((unsigned)e[1] << 16); v.y = e[2] | ((unsigned)e[3] << 16);
    v.z = e[4] | ((unsigned)e[5] << 16); v.w = e[6] | ((unsigned)e[7] << 16);
    *reinterpret_cast<uint4*>(BT + l * (long)used * Nmod + (long)jr * Nmod + n0) = v;
  }
}

// ---------------------------------------------------------------- optimizer
// sum(g^2) in a fixed order: per-block partials over a grid that depends on n only, then one block sums them in
// block order (fp32 atomics made the clip coefficient, and with it the bf16 AdamW update, differ between DP
// ranks that hold bit-identical all-reduced grads)
constexpr int SUMSQ_BLOCKS = 2048;
__global__ __launch_bounds__(256) void sumsq_part_kernel(const float* __restrict__ g, long n, float* __restrict__ part) {
  __shared__ float red[4];
  float a = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) a += g[i] * g[i];
  a = block_sum256(a, red);
  if (threadIdx.x == 0) part[blockIdx.x] = a;
}
__global__ __launch_bounds__(256) void sumsq_final_kernel(const float* __restrict__ part, int nb,
                                                          float* __restrict__ out) {
  __shared__ float red[4];
  float a = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) a += part[i];
  a = block_sum256(a, red);
  if (threadIdx.x == 0) out[0] += a;
}

__global__ void adamw_kernel(bf16* __restrict__ p, const float* __restrict__ g, bf16* __restrict__ m,
                             bf16* __restrict__ v, long n, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2_sqrt, const float* __restrict__ sumsq, float max_norm) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float clip = 1.f;
  if (max_norm > 0.f) {
    const float tot = sqrtf(sumsq[0]);
    clip = fminf(max_norm / (tot + 1e-6f), 1.f);
  }
  // reference: bf16 grads (param dtype), clip_grad_norm_ scales them in place
  float gi = round_bf(g[i]);
  if (clip < 1.f) gi = round_bf(gi * clip);
  float pi = bf2f(p[i]);
  if (wd != 0.f) pi = round_bf(pi * (1.f - lr * wd));
  float mi = bf2f(m[i]), vi = bf2f(v[i]);
  mi = round_bf(mi + (1.f - b1) * (gi - mi));            // exp_avg.lerp_(grad, 1-beta1)
  vi = round_bf(round_bf(vi * b2) + (1.f - b2) * gi * gi);  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  const float denom = round_bf(round_bf(round_bf(sqrtf(vi)) / bc2_sqrt) + eps);
  pi = pi - (lr / bc1) * (mi / denom);                     // param.addcdiv_(exp_avg, denom, -step_size)
  p[i] = f2bf(pi);
  m[i] = f2bf(mi);
  v[i] = f2bf(vi);
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ s, bf16* __restrict__ d, long n, float scale) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = f2bf(s[i] * scale);
}

inline unsigned blocks(long n, int per = 256) { return (unsigned)((n + per - 1) / per); }

// ---------------------------------------------------- grouped row . vector sums
// partial[g][c] = sum over rows [c*rpc, min((c+1)*rpc, rpg)) of group g of x[row] . w (fp32, fixed order:
// each thread its 16-B column chunks of every row, then the block tree); the finish kernel adds a group's
// partials in chunk order, so the result is deterministic.
__global__ __launch_bounds__(256) void row_dot_partial_kernel(const bf16* __restrict__ x, long ldx, int rpg, int rpc,
                                                              int D, const float* __restrict__ w,
                                                              float* __restrict__ partial) {
  __shared__ float red[4];
  const int g = blockIdx.y, c = blockIdx.x;
  const int r0 = c * rpc, r1 = min(rpg, r0 + rpc);
  const int nch = D / 8;
  float acc = 0.f;
  for (int r = r0; r < r1; ++r) {
    const u32x4* xr = reinterpret_cast<const u32x4*>(x + ((long)g * rpg + r) * ldx);
    for (int ch = threadIdx.x; ch < nch; ch += 256) {
      float f[8];
      unpack8(xr[ch], f);
      const f32x4 w0 = *reinterpret_cast<const f32x4*>(w + ch * 8);
      const f32x4 w1 = *reinterpret_cast<const f32x4*>(w + ch * 8 + 4);
      acc += f[0] * w0[0] + f[1] * w0[1] + f[2] * w0[2] + f[3] * w0[3] + f[4] * w1[0] + f[5] * w1[1] +
             f[6] * w1[2] + f[7] * w1[3];
    }
  }
  const float tot = block_sum256(acc, red);
  if (threadIdx.x == 0) partial[(long)g * gridDim.x + c] = tot;
}

__global__ void row_dot_finish_kernel(const float* __restrict__ partial, int nc, int G, const float* __restrict__ add,
                                      float add_scale, int accumulate, float* __restrict__ out) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  float s = accumulate ? out[g] : 0.f;
  float p = 0.f;
  for (int c = 0; c < nc; ++c) p += partial[(long)g * nc + c];
  s += p;
  if (add) s += add_scale * add[0];
  out[g] = s;
}

int row_dot_chunks(int rpg, int D, int* rpc) {
  const int r = std::max(1, std::min(rpg, 65536 / std::max(D, 1)));  // ~64K elements per workgroup
  *rpc = r;
  return (rpg + r - 1) / r;
}

}  // namespace

extern "C" size_t ospo_row_dot_sum_ws_bytes(int n_groups, int rows_per_group, int D) {
  if (n_groups <= 0 || rows_per_group <= 0 || D <= 0) return 0;
  int rpc = 0;
  const int nc = row_dot_chunks(rows_per_group, D, &rpc);
  return (size_t)n_groups * nc * sizeof(float);
}

extern "C" int ospo_row_dot_sum(const void* x, long ldx, int n_groups, int rows_per_group, int D, const float* w,
                                const float* add, float add_scale, int accumulate, float* out, void* ws,
                                size_t ws_bytes, hipStream_t st) {
  if (!x || !w || !out || !ws) return OSPO_ERR_ARG;
  if (n_groups <= 0 || rows_per_group <= 0 || D <= 0 || D % 8 || ldx < D || ldx % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(x) || !aligned16(w) || !aligned16(ws)) return OSPO_ERR_ALIGN;
  if (ws_bytes < ospo_row_dot_sum_ws_bytes(n_groups, rows_per_group, D)) return OSPO_ERR_ARG;
  if (n_groups > 65535) return OSPO_ERR_SHAPE;
  int rpc = 0;
  const int nc = row_dot_chunks(rows_per_group, D, &rpc);
  hipLaunchKernelGGL(row_dot_partial_kernel, dim3(nc, n_groups), dim3(256), 0, st, (const bf16*)x, ldx,
                     rows_per_group, rpc, D, w, (float*)ws);
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(row_dot_finish_kernel, dim3(blocks(n_groups)), dim3(256), 0, st, (const float*)ws, nc, n_groups,
                     add, add_scale, accumulate, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

// =================================================================== C ABI
extern "C" const char* ospo_strerror(int s) {
  switch (s) {
    case OSPO_OK: return "ok";
    case OSPO_ERR_SHAPE: return "shape / leading-dimension violation";
    case OSPO_ERR_ALIGN: return "pointer not 16-byte aligned";
    case OSPO_ERR_HIP: return "HIP launch error";
    case OSPO_ERR_UNSUPPORTED: return "unsupported configuration";
    case OSPO_ERR_ARG: return "bad argument";
    default: return "unknown ospo status";
  }
}
extern "C" int ospo_abi_version(void) { return OSPO_ABI_VERSION; }

extern "C" size_t ospo_ws_counter_bytes(int kind) {
  switch (kind) {
    case OSPO_WS_GEMM_TAIL: return OSPO_WS_GEMM_TAIL_CNT_BYTES;
    case OSPO_WS_SKINNY: return OSPO_WS_SKINNY_CNT_BYTES;
    case OSPO_WS_LORA_GDB: return OSPO_WS_LORA_GDB_CNT_BYTES;
    case OSPO_WS_DECODE_LINEAR: return OSPO_WS_DECODE_LINEAR_CNT_BYTES;
    default: return 0;
  }
}

// host restatement of the device dropout hash (tests pin ospo_amd/dropout.py against it)
extern "C" unsigned ospo_dropout_hash(unsigned idx, unsigned seed) { return drop_hash(idx, seed); }

static int rmsnorm_fwd_impl(const void* x, const void* w, void* y, float* rstd, int M, int D, float eps,
                            const Mx8Out& mo, hipStream_t st) {
  if (!x || !w || !y || !rstd) return OSPO_ERR_ARG;
  if (M <= 0 || D % 8 || D > 256 * 8 * RMS_MAXIT) return OSPO_ERR_SHAPE;
  if (!aligned16(x) || !aligned16(w) || !aligned16(y)) return OSPO_ERR_ALIGN;
  const int it = (D / 8 + 63) / 64;
  const dim3 gw((M + 3) / 4);
  const bf16 *xb = (const bf16*)x, *wb = (const bf16*)w;
  const long Ml = M;
  if (D == 4096) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<8, true>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (D == 2048) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<4, true>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (it <= 1) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<1, false>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (it <= 2) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<2, false>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (it <= 4) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<4, false>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (it <= 8) hipLaunchKernelGGL((rmsnorm_fwd_w_kernel<8, false>), gw, dim3(256), 0, st, xb, wb, (bf16*)y, rstd, Ml, D, eps, mo);
  else if (mo.q) return OSPO_ERR_UNSUPPORTED;
  else hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3(M), dim3(256), 0, st, xb, wb, (bf16*)y, rstd, D, eps);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

static int rmsnorm_bwd_impl(const void* dy, const void* x, const void* w, const float* rstd, const void* dres,
                            void* dx, int M, int D, const Mx8Out& mo, hipStream_t st) {
  if (!dy || !x || !w || !rstd || !dx) return OSPO_ERR_ARG;
  if (M <= 0 || D % 8 || D > 256 * 8 * RMS_MAXIT) return OSPO_ERR_SHAPE;
  if (!aligned16(dy) || !aligned16(x) || !aligned16(w) || !aligned16(dx) || (dres && !aligned16(dres)))
    return OSPO_ERR_ALIGN;
  const int it = (D / 8 + 63) / 64;
  const dim3 gw((M + 3) / 4);
  const bf16 *dyb = (const bf16*)dy, *xb = (const bf16*)x, *wb = (const bf16*)w, *rb = (const bf16*)dres;
  const long Ml = M;
#ifdef OSPO_ABLATION
  static const bool early = getenv("OSPO_RMS_EARLY") != nullptr;
  if (D == 4096 && early) {
    hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<8, true, true>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
#endif
  if (D == 4096) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<8, true>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (D == 2048) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<4, true>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (it <= 1) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<1, false>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (it <= 2) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<2, false>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (it <= 4) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<4, false>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (it <= 8) hipLaunchKernelGGL((rmsnorm_bwd_w_kernel<8, false>), gw, dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, Ml, D, mo);
  else if (mo.q) return OSPO_ERR_UNSUPPORTED;
  else hipLaunchKernelGGL(rmsnorm_bwd_kernel, dim3(M), dim3(256), 0, st, dyb, xb, wb, rstd, rb, (bf16*)dx, D);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

static bool mx8_out_ok(const void* q, int ldq, const void* s, int M, int K) {
  return q && s && K % 128 == 0 && ldq >= K && ldq % 16 == 0 && M > 0 && aligned16(q) && aligned16(s);
}

extern "C" int ospo_rmsnorm_fwd(const void* x, const void* w, void* y, float* rstd, int M, int D, float eps,
                                hipStream_t st) {
  return rmsnorm_fwd_impl(x, w, y, rstd, M, D, eps, Mx8Out{nullptr, 0, nullptr, 0}, st);
}
extern "C" int ospo_rmsnorm_fwd_mx8(const void* x, const void* w, void* y, float* rstd, int M, int D, float eps,
                                    void* q, int ldq, void* s, hipStream_t st) {
  if (!mx8_out_ok(q, ldq, s, M, D)) return OSPO_ERR_ARG;
  return rmsnorm_fwd_impl(x, w, y, rstd, M, D, eps, Mx8Out{(uint8_t*)q, ldq, (uint8_t*)s, D}, st);
}
extern "C" int ospo_rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd, const void* dres,
                                void* dx, int M, int D, hipStream_t st) {
  return rmsnorm_bwd_impl(dy, x, w, rstd, dres, dx, M, D, Mx8Out{nullptr, 0, nullptr, 0}, st);
}
extern "C" int ospo_rmsnorm_bwd_mx8(const void* dy, const void* x, const void* w, const float* rstd, const void* dres,
                                    void* dx, int M, int D, void* q, int ldq, void* s, hipStream_t st) {
  if (!mx8_out_ok(q, ldq, s, M, D)) return OSPO_ERR_ARG;
  return rmsnorm_bwd_impl(dy, x, w, rstd, dres, dx, M, D, Mx8Out{(uint8_t*)q, ldq, (uint8_t*)s, D}, st);
}

static int rope_common(bool bwd, void* x, int ld, int q_col, int k_col, int S, int T, int H, int hd, const void* c,
                       const void* s, hipStream_t st) {
  if (!x || !c || !s) return OSPO_ERR_ARG;
  if (S <= 0 || T <= 0 || H <= 0 || hd % 16 || ld % 8 || q_col % 8 || k_col % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(x) || !aligned16(c) || !aligned16(s)) return OSPO_ERR_ALIGN;
  const long rows = (long)S * T;
  const long total = rows * H * 2 * (hd / 16);
  if (bwd)
    hipLaunchKernelGGL(rope_kernel<true>, dim3(blocks(total)), dim3(256), 0, st, (bf16*)x, ld, q_col, k_col, rows, T,
                       H, hd, (const bf16*)c, (const bf16*)s);
  else
    hipLaunchKernelGGL(rope_kernel<false>, dim3(blocks(total)), dim3(256), 0, st, (bf16*)x, ld, q_col, k_col, rows,
                       T, H, hd, (const bf16*)c, (const bf16*)s);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
extern "C" int ospo_rope_fwd(void* qkv, int ld, int q_col, int k_col, int S, int T, int n_heads, int head_dim,
                             const void* cos_tab, const void* sin_tab, hipStream_t st) {
  return rope_common(false, qkv, ld, q_col, k_col, S, T, n_heads, head_dim, cos_tab, sin_tab, st);
}
extern "C" int ospo_rope_bwd(void* dqkv, int ld, int q_col, int k_col, int S, int T, int n_heads, int head_dim,
                             const void* cos_tab, const void* sin_tab, hipStream_t st) {
  return rope_common(true, dqkv, ld, q_col, k_col, S, T, n_heads, head_dim, cos_tab, sin_tab, st);
}

static int swiglu_fwd_impl(const void* gu, int ld_gu, void* h, int ld_h, int M, int F, const Mx8Out& mo,
                           hipStream_t st) {
  if (!gu || !h) return OSPO_ERR_ARG;
  if (M <= 0 || F % 8 || ld_gu < 2 * F || ld_h < F || ld_gu % 8 || ld_h % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(gu) || !aligned16(h)) return OSPO_ERR_ALIGN;
  if (M > 65535) return OSPO_ERR_SHAPE;  // rows on grid.y
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(blocks(F / 8, 128), M), dim3(128), 0, st, (const bf16*)gu, ld_gu,
                     (bf16*)h, ld_h, (long)M, F, mo);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
static int swiglu_bwd_impl(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, int M, int F,
                           const Mx8Out& mo, hipStream_t st) {
  if (!dh || !gu || !dgu) return OSPO_ERR_ARG;
  if (M <= 0 || F % 8 || ld_gu < 2 * F || ld_dgu < 2 * F || ld_dh < F || ld_dh % 8 || ld_gu % 8 || ld_dgu % 8)
    return OSPO_ERR_SHAPE;
  if (!aligned16(dh) || !aligned16(gu) || !aligned16(dgu)) return OSPO_ERR_ALIGN;
  if (M > 65535) return OSPO_ERR_SHAPE;  // rows on grid.y
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(blocks(F / 8, 128), M), dim3(128), 0, st, (const bf16*)dh, ld_dh,
                     (const bf16*)gu, ld_gu, (bf16*)dgu, ld_dgu, (long)M, F, mo);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
extern "C" int ospo_swiglu_fwd(const void* gu, int ld_gu, void* h, int ld_h, int M, int F, hipStream_t st) {
  return swiglu_fwd_impl(gu, ld_gu, h, ld_h, M, F, Mx8Out{nullptr, 0, nullptr, 0}, st);
}
extern "C" int ospo_swiglu_fwd_mx8(const void* gu, int ld_gu, void* h, int ld_h, int M, int F, void* q, int ldq,
                                   void* s, hipStream_t st) {
  if (!mx8_out_ok(q, ldq, s, M, F)) return OSPO_ERR_ARG;
  return swiglu_fwd_impl(gu, ld_gu, h, ld_h, M, F, Mx8Out{(uint8_t*)q, ldq, (uint8_t*)s, F}, st);
}
extern "C" int ospo_swiglu_bwd(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, int M,
                               int F, hipStream_t st) {
  return swiglu_bwd_impl(dh, ld_dh, gu, ld_gu, dgu, ld_dgu, M, F, Mx8Out{nullptr, 0, nullptr, 0}, st);
}
extern "C" int ospo_swiglu_bwd_mx8(const void* dh, int ld_dh, const void* gu, int ld_gu, void* dgu, int ld_dgu, int M,
                                   int F, void* q, int ldq, void* s, hipStream_t st) {
  if (F % 64 || !mx8_out_ok(q, ldq, s, M, 2 * F)) return OSPO_ERR_ARG;
  return swiglu_bwd_impl(dh, ld_dh, gu, ld_gu, dgu, ld_dgu, M, F, Mx8Out{(uint8_t*)q, ldq, (uint8_t*)s, 2 * F}, st);
}

extern "C" int ospo_gelu_fwd(const void* x, void* y, long n, hipStream_t st) {
  if (!x || !y) return OSPO_ERR_ARG;
  if (n <= 0 || n % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(x) || !aligned16(y)) return OSPO_ERR_ALIGN;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(blocks(n / 8)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, n / 8);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
extern "C" int ospo_gelu_bwd(const void* dy, const void* x_pre, void* dx, long n, hipStream_t st) {
  if (!dy || !x_pre || !dx) return OSPO_ERR_ARG;
  if (n <= 0 || n % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(dy) || !aligned16(x_pre) || !aligned16(dx)) return OSPO_ERR_ALIGN;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(blocks(n / 8)), dim3(256), 0, st, (const bf16*)dy, (const bf16*)x_pre,
                     (bf16*)dx, n / 8);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_assemble_inputs(const int* text_ids, int B, int Lt, const void* text_table, int vocab,
                                    const void* img_emb, int N, int D, void* x0, hipStream_t st) {
  if (!text_table || !img_emb || !x0 || (Lt > 0 && !text_ids)) return OSPO_ERR_ARG;
  if (B <= 0 || Lt < 0 || N <= 0 || D % 8 || vocab <= 0) return OSPO_ERR_SHAPE;
  if (!aligned16(text_table) || !aligned16(img_emb) || !aligned16(x0)) return OSPO_ERR_ALIGN;
  const long rows = 2L * B * (Lt + N);
  const long n = rows * (D / 8);
  hipLaunchKernelGGL(assemble_kernel, dim3(blocks(n)), dim3(256), 0, st, text_ids, B, Lt, (const bf16*)text_table,
                     vocab, (const bf16*)img_emb, N, D, (bf16*)x0, rows);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_gen_aligner_in(const int* ids, int R, const void* gen_embed, int img_vocab, int E,
                                   const void* w1, const void* b1, int D, void* out, hipStream_t st) {
  if (!ids || !gen_embed || !w1 || !b1 || !out) return OSPO_ERR_ARG;
  if (R <= 0 || E <= 0 || D <= 0 || img_vocab <= 0) return OSPO_ERR_SHAPE;
  if (E == 8 && D % 8 == 0 && aligned16(gen_embed) && aligned16(w1) && aligned16(b1) && aligned16(out)) {
    const long n8 = (long)R * (D / 8);
    hipLaunchKernelGGL(gen_aligner_in8_kernel, dim3(blocks(n8)), dim3(256), 0, st, ids, R, (const bf16*)gen_embed,
                       img_vocab, (const bf16*)w1, (const bf16*)b1, D, (bf16*)out);
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  const long n = (long)R * D;
  hipLaunchKernelGGL(gen_aligner_in_kernel, dim3(blocks(n)), dim3(256), 0, st, ids, R, (const bf16*)gen_embed,
                     img_vocab, E,
                     (const bf16*)w1, (const bf16*)b1, D, (bf16*)out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_gather_rows(const void* src, int ld_src, int S, int T, int t0, int N, int D, void* dst,
                                hipStream_t st) {
  if (!src || !dst) return OSPO_ERR_ARG;
  if (S <= 0 || N <= 0 || t0 < 0 || t0 + N > T || D % 8 || ld_src % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(src) || !aligned16(dst)) return OSPO_ERR_ALIGN;
  const long rows = (long)S * N;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks(rows * (D / 8))), dim3(256), 0, st, (const bf16*)src, ld_src, T,
                     t0, N, D, (bf16*)dst, rows);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_scatter_rows(const void* src, int S, int T, int t0, int N, int D, void* dst, int ld_dst,
                                 int total_rows, hipStream_t st) {
  if (!src || !dst) return OSPO_ERR_ARG;
  if (S <= 0 || N <= 0 || t0 < 0 || t0 + N > T || D % 8 || ld_dst % 8 || total_rows < (long)S * T)
    return OSPO_ERR_SHAPE;
  if (!aligned16(src) || !aligned16(dst)) return OSPO_ERR_ALIGN;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(blocks((long)total_rows * (D / 8))), dim3(256), 0, st,
                     (const bf16*)src, S, T, t0, N, D, (bf16*)dst, ld_dst, (long)total_rows);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_logprob_fwd(const void* logits, int V, const int* labels, int R, int N, float* lse,
                                float* token_logp, float* seq_logps, hipStream_t st) {
  if (!logits || !labels || !lse || !token_logp || !seq_logps) return OSPO_ERR_ARG;
  if (R <= 0 || N <= 0 || R % N || V % 8 || V > 256 * 8 * LP_MAXIT) return OSPO_ERR_SHAPE;
  if (!aligned16(logits)) return OSPO_ERR_ALIGN;
  hipLaunchKernelGGL(logprob_fwd_kernel, dim3(R), dim3(256), 0, st, (const bf16*)logits, V, labels, lse, token_logp);
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(seq_mean_kernel, dim3(R / N), dim3(256), 0, st, token_logp, N, seq_logps);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_logprob_bwd(const void* logits, int V, const int* labels, const float* lse, int R, int N,
                                const float* g_seq, void* dlogits, hipStream_t st) {
  if (!logits || !labels || !lse || !g_seq || !dlogits) return OSPO_ERR_ARG;
  if (R <= 0 || N <= 0 || R % N || V % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(logits) || !aligned16(dlogits)) return OSPO_ERR_ALIGN;
  const long n = (long)R * (V / 8);
  hipLaunchKernelGGL(logprob_bwd_kernel, dim3(blocks(n)), dim3(256), 0, st, (const bf16*)logits, V, labels, lse, N,
                     g_seq, (bf16*)dlogits, (long)R);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_simpo_fwd(const float* logps, int B, float beta, float gbr, float ls, int loss_type,
                              float* losses, float* loss_mean, float* rewards, hipStream_t st) {
  if (!logps || !losses || !loss_mean || !rewards) return OSPO_ERR_ARG;
  if (loss_type != 0 && loss_type != 1) return OSPO_ERR_ARG;
  if (B <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(simpo_fwd_kernel, dim3(1), dim3(256), 0, st, logps, B, beta, gbr, ls, loss_type, losses,
                     loss_mean, rewards);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
extern "C" int ospo_simpo_bwd(const float* logps, int B, float beta, float gbr, float ls, int loss_type,
                              const float* g_loss, float* glogps, hipStream_t st) {
  if (!logps || !g_loss || !glogps) return OSPO_ERR_ARG;
  if (loss_type != 0 && loss_type != 1) return OSPO_ERR_ARG;
  if (B <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(simpo_bwd_kernel, dim3(blocks(B)), dim3(256), 0, st, logps, B, beta, gbr, ls, loss_type, g_loss,
                     glogps);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_lora_pack(const void* A_flat, const void* B_flat, int nmods, int r, int Kin, int Nmod, int Rp,
                              void* Acat, void* AcatT, void* Bcat, void* BT, int n_layers, long layer_stride,
                              hipStream_t st) {
  if (!A_flat || !B_flat || !Acat || !AcatT || !Bcat) return OSPO_ERR_ARG;
  if (nmods <= 0 || r <= 0 || Kin <= 0 || Nmod <= 0 || Rp < nmods * r || n_layers < 1 || n_layers > 65535 ||
      (n_layers > 1 && layer_stride <= 0))
    return OSPO_ERR_SHAPE;
  const bool v8 = r % 8 == 0 && Rp % 8 == 0 && Kin % 8 == 0 && Nmod % 8 == 0 && layer_stride % 8 == 0 &&
                  aligned16(A_flat) && aligned16(B_flat) && aligned16(Acat) && aligned16(AcatT) &&
                  aligned16(Bcat) && (!BT || aligned16(BT));
  if (v8) {
    const long chunks = 2 * ((long)Rp * Kin / 8) + (long)nmods * Nmod * Rp / 8 + (BT ? (long)nmods * r * Nmod / 8 : 0);
    hipLaunchKernelGGL(lora_pack8_kernel, dim3(blocks(chunks), n_layers), dim3(256), 0, st, (const bf16*)A_flat,
                       (const bf16*)B_flat, nmods, r, Kin, Nmod, Rp, (bf16*)Acat, (bf16*)AcatT, (bf16*)Bcat,
                       (bf16*)BT, layer_stride);
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  const long n = std::max((long)Rp * Kin, (long)nmods * Nmod * Rp);
  hipLaunchKernelGGL(lora_pack_kernel, dim3(blocks(n), n_layers), dim3(256), 0, st, (const bf16*)A_flat,
                     (const bf16*)B_flat, nmods, r, Kin, Nmod, Rp, (bf16*)Acat, (bf16*)AcatT, (bf16*)Bcat, (bf16*)BT,
                     layer_stride);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_sumsq(const float* g, long n, float* out, float* ws, hipStream_t st) {
  if (!g || !out || !ws) return OSPO_ERR_ARG;
  if (n <= 0) return OSPO_ERR_SHAPE;
  long nb = (n + 255) / 256;
  if (nb > SUMSQ_BLOCKS) nb = SUMSQ_BLOCKS;
  hipLaunchKernelGGL(sumsq_part_kernel, dim3((unsigned)nb), dim3(256), 0, st, g, n, ws);
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(sumsq_final_kernel, dim3(1), dim3(256), 0, st, (const float*)ws, (int)nb, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_adamw_clip(void* params, const float* grads, void* exp_avg, void* exp_avg_sq, long n, float lr,
                               float beta1, float beta2, float eps, float weight_decay, int step, const float* sumsq,
                               float max_norm, hipStream_t st) {
  if (!params || !grads || !exp_avg || !exp_avg_sq || (max_norm > 0.f && !sumsq)) return OSPO_ERR_ARG;
  if (n <= 0 || step < 1) return OSPO_ERR_SHAPE;
  const float bc1 = 1.f - powf(beta1, (float)step);
  const float bc2 = 1.f - powf(beta2, (float)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(blocks(n)), dim3(256), 0, st, (bf16*)params, grads, (bf16*)exp_avg,
                     (bf16*)exp_avg_sq, n, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), sumsq, max_norm);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_f32_to_bf16(const float* src, void* dst, long n, float scale, hipStream_t st) {
  if (!src || !dst) return OSPO_ERR_ARG;
  if (n <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(blocks(n)), dim3(256), 0, st, src, (bf16*)dst, n, scale);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
