// Causal flash attention (forward + backward) for the Janus-Pro decoder on gfx950.
// Replaces HF 4.38.2 LlamaAttention eager path (QK^T/sqrt(d), causal mask, fp32
// softmax, PV) reached from ospo/wrapper/train.py:352 -- no [T,T] matrix is
// ever materialised.
//
// Forward: workgroup = 4 waves = 64 query rows of one (sequence, head); each
// wave owns 16 query rows.  S^T = K.Q^T is computed with the KEY on the MFMA
// row and the QUERY on the lane, so the online softmax of one query row is
// lane-local (+2 shuffles across the 4 lane groups), and the P^T accumulator
// feeds P.V directly as the B operand (k order permuted identically on both
// sides).  V^T fragments come from ds_read_b64_tr_b16 (hardware transpose).
//
// Backward: two atomic-free kernels.  dK/dV: workgroup = 64 keys, each wave
// owns 16 keys (dK^T, dV^T in registers) and sweeps the query tiles at/after
// its block.  dQ: workgroup = 64 query rows sweeping key tiles 0..qb, the
// forward's shape, dQ^T in registers.  (S, dP are recomputed by both: 7 MFMA
// products instead of 5, but no fp32 atomics -- at T=600 the atomic dQ
// traffic alone was ~460 MB/call.)
//
// LDS images are [row][128 x bf16] (256-B rows) with 16-B chunk swizzle
// chunk ^ 2*(row & 7): conflict-free for both the ds_read_b128 row reads and
// the ds_read_b64_tr_b16 column reads (CDNA4 LDS banking, 64 x 4 B banks).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int HD = 128;     // head dim
constexpr int QB = 64;      // query rows per workgroup (fwd) / per tile (bwd)
constexpr int KB = 64;      // keys per tile (fwd) / per workgroup (bwd)
constexpr int ROWB = HD * 2;
constexpr int TILE_BYTES = 64 * ROWB;  // 16 KiB

__device__ __forceinline__ int aswz(int row) { return (row & 7) << 1; }
__device__ __forceinline__ int aoff(int row, int chunk) { return row * ROWB + ((chunk ^ aswz(row)) << 4); }

__device__ __forceinline__ void glds16(const void* gsrc, char* lds_dst_uniform) {
  __builtin_amdgcn_global_load_lds(gsrc, (LDS_AS void*)lds_dst_uniform, 16, 0, 0);
}

// Stage 64 rows x 128 bf16 (rows row0.., clamped to [0, row_lim)) of a strided
// buffer into an LDS image: 16 pieces of 1 KiB (4 rows each) over the NW waves.
template <int NW>
__device__ __forceinline__ void stage64(const bf16* base, int ld, int row0, int row_lim, int col0, char* lds,
                                        int wave, int lane) {
#pragma unroll
  for (int p = wave; p < 16; p += NW) {
    const int row = p * 4 + (lane >> 4);
    const int ch = (lane & 15) ^ aswz(row);
    int gr = row0 + row;
    gr = gr < row_lim ? gr : row_lim - 1;
    glds16(base + (long)gr * ld + col0 + ch * 8, lds + p * 1024);
  }
}

// 16x32 fragment, row read: rows r0+(lane&15), k = 32*s + 8*(lane>>4) .. +7
__device__ __forceinline__ bf16x8 frag_row(const char* lds, int r0, int s, int lane) {
  const int r = r0 + (lane & 15);
  return *reinterpret_cast<const bf16x8*>(lds + aoff(r, 4 * s + (lane >> 4)));
}

// 16x32 fragment, transposed read for an operand whose k runs along the image
// ROWS in the permuted accumulator order: element j<4 <- row kbase+4g+j,
// j>=4 <- row kbase+16+4g+(j-4); the 16 fragment rows are image columns c0..c0+15.
__device__ __forceinline__ bf16x8 frag_tr_perm(const char* lds, int kbase, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r1 = kbase + 4 * g + q;
  const int r2 = r1 + 16;
  const int x = (c0 >> 3) + (p >> 1);
  const int h = (p & 1) << 3;
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + r1 * ROWB + ((x ^ aswz(r1)) << 4) + h));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + r2 * ROWB + ((x ^ aswz(r2)) << 4) + h));
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Inline-asm form of frag_tr_perm: the two ds_read_b64_tr_b16 are invisible to the
// compiler's waitcnt pass, which otherwise (a) drains vmcnt(0) before every transposed
// read -- it cannot tell them from the in-flight LDS-DMA of the next tile -- and (b)
// issues one read pair per MFMA behind lgkmcnt(0).  Callers issue a batch, then
// trp_wait() the whole batch once (registers tied, then a sched_barrier).
__device__ __forceinline__ uint32_t lds_u32(const char* p) {
  return (uint32_t)(uintptr_t)((LDS_AS const char*)p);
}
__device__ __forceinline__ void trp_issue(const char* lds, int kbase, int c0, int lane, i16x4& lo, i16x4& hi) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r1 = kbase + 4 * g + q;
  const int r2 = r1 + 16;
  const int x = (c0 >> 3) + (p >> 1);
  const int h = (p & 1) << 3;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_u32(lds + r1 * ROWB + ((x ^ aswz(r1)) << 4) + h)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_u32(lds + r2 * ROWB + ((x ^ aswz(r2)) << 4) + h)));
}
__device__ __forceinline__ bf16x8 trp_join(const i16x4& lo, const i16x4& hi) {
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// wait for 4 transposed fragments (8 reads): all registers tied to the wait
__device__ __forceinline__ void trp_wait4(i16x4 (&lo)[4], i16x4 (&hi)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]),
                 "+v"(hi[3])::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
// wait for 8 transposed fragments (16 reads): all registers tied to the wait
__device__ __forceinline__ void trp_wait8(i16x4 (&lo)[8], i16x4 (&hi)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(lo[0]), "+v"(lo[1]), "+v"(lo[2]), "+v"(lo[3]), "+v"(lo[4]), "+v"(lo[5]), "+v"(lo[6]),
                 "+v"(lo[7]), "+v"(hi[0]), "+v"(hi[1]), "+v"(hi[2]), "+v"(hi[3]), "+v"(hi[4]), "+v"(hi[5]),
                 "+v"(hi[6]), "+v"(hi[7])::"memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Same, natural k order (element j <- row kbase + 8g + j): for the dQ = dS.K product.
__device__ __forceinline__ bf16x8 frag_tr_nat(const char* lds, int kbase, int c0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r1 = kbase + 8 * g + q;
  const int r2 = r1 + 4;
  const int x = (c0 >> 3) + (p >> 1);
  const int h = (p & 1) << 3;
  i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + r1 * ROWB + ((x ^ aswz(r1)) << 4) + h));
  i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS i16x4*)(lds + r2 * ROWB + ((x ^ aswz(r2)) << 4) + h));
  i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 pack_perm(const f32x4& a, const f32x4& b) {
  bf16x8 v;
  v[0] = f2bf(a[0]); v[1] = f2bf(a[1]); v[2] = f2bf(a[2]); v[3] = f2bf(a[3]);
  v[4] = f2bf(b[0]); v[5] = f2bf(b[1]); v[6] = f2bf(b[2]); v[7] = f2bf(b[3]);
  return v;
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

constexpr float L2E = 1.4426950408889634f;  // exp(x) = exp2(x * log2 e): v_exp_f32 is a base-2 exponential

// Two f32 -> bf16 (RNE) in one v_cvt_pk_bf16_f32, back to f32.
__device__ __forceinline__ void bf_round2(float& a, float& b) {
  const bf16x2 r = __builtin_convertvector((f32x2){a, b}, bf16x2);
  const unsigned u = __builtin_bit_cast(unsigned, r);
  a = __uint_as_float(u << 16);
  b = __uint_as_float(u & 0xffff0000u);
}
// HF eager bf16 scores (modeling_llama.py: matmul output, then * 1/sqrt(d), each rounded to bf16)
__device__ __forceinline__ void hf_scores2(float& a, float& b, float scale) {
  bf_round2(a, b);
  a *= scale;
  b *= scale;
  bf_round2(a, b);
}
// Reductions over the 4 lane groups (lanes l, l^16, l^32, l^48) with the CDNA4 half-row swaps
// (VALU, no LDS round trip like ds_bpermute); every lane gets the same bits (a+b == b+a).
__device__ __forceinline__ float grp_max(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const unsigned w = __float_as_uint(x);
  const auto q = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float grp_sum(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const unsigned w = __float_as_uint(x);
  const auto q = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// RoPE backward (transpose of the rotate-half rotation) on fp32 accumulators whose lane
// holds d = 16dt + 4g + j, dt = 0..7: d < 64 pairs with d + 64 (dt + 4) in the same lane.
// cs / sn: bf16 [T][64] tables, t = the row's position in its sequence.
__device__ __forceinline__ void rope_bwd_acc(f32x4 (&v)[8], const bf16* cs, const bf16* sn, int t, int g) {
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    const uint2 cw = *reinterpret_cast<const uint2*>(cs + (long)t * 64 + 16 * dt + 4 * g);
    const uint2 sw = *reinterpret_cast<const uint2*>(sn + (long)t * 64 + 16 * dt + 4 * g);
    const float c[4] = {bits2f(cw.x & 0xffff), bits2f(cw.x >> 16), bits2f(cw.y & 0xffff), bits2f(cw.y >> 16)};
    const float sv[4] = {bits2f(sw.x & 0xffff), bits2f(sw.x >> 16), bits2f(sw.y & 0xffff), bits2f(sw.y >> 16)};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float a = v[dt][j], b = v[dt + 4][j];
      v[dt][j] = a * c[j] + b * sv[j];
      v[dt + 4][j] = b * c[j] - a * sv[j];
    }
  }
}

// ============================================================== forward ====
template <int NW, int DBG = 0>  // DBG 1: no K/V loads after the first tile (ablation, results invalid)
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(const bf16* __restrict__ qkv, int ldq, int qc, int kc, int vc,
                                                       bf16* __restrict__ out, int ldo, float* __restrict__ lse,
                                                       int T, int H, float scale) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // K0 V0 K1 V1
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // grid (H, S, blocks): workgroups dispatch in linear order, so every head's longest key sweep
  // (the last query block) goes first across the whole chip, then the next longest (LPT order)
  const int qb = gridDim.z - 1 - blockIdx.z;
  const int h = blockIdx.x, s = blockIdx.y;
  const int g = lane >> 4, l16 = lane & 15;
  const long rowbase = (long)s * T;
  const int rows_lim_seq = T;  // clamp inside the sequence

  // this lane's query row
  constexpr int RB = 16 * NW;  // query rows per workgroup
  const int qrow = qb * RB + wave * 16 + l16;
  const int qr_c = qrow < T ? qrow : T - 1;
  bf16x8 qf[4];
  {
    const bf16* qp = qkv + (rowbase + qr_c) * ldq + qc + h * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d) qf[d] = *reinterpret_cast<const bf16x8*>(qp + 32 * d + 8 * g);
  }

  f32x4 o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -1e30f, l_run = 0.f;

  const int last = (qb * RB + RB - 1 < T ? qb * RB + RB - 1 : T - 1);
  const int n_kv = last / KB + 1;  // causal: key tiles up to the block's last row
  const bf16* kbase = qkv + rowbase * ldq + kc + h * HD;
  const bf16* vbase = qkv + rowbase * ldq + vc + h * HD;

  stage64<NW>(kbase, ldq, 0, rows_lim_seq, 0, smem, wave, lane);
  stage64<NW>(vbase, ldq, 0, rows_lim_seq, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lim = qrow < T ? qrow : T - 1;  // last key this row attends to (padding rows: T - 1)
  // One K/V tile.  DIAG (the tiles that may hold a key after some row of the block, or past T):
  // masked scores become -inf, which v_exp_f32 maps to 0 -- no per-element branch or compare
  // outside those tiles.
  for (int kt = 0; kt < n_kv; ++kt) {
    const bool diag = (kt * KB + KB - 1 > qb * RB) || ((kt + 1) * KB > T);
    const int buf = kt & 1;
    if (DBG == 0 && kt + 1 < n_kv) {
      char* nb = smem + (buf ^ 1) * 2 * TILE_BYTES;
      stage64<NW>(kbase, ldq, (kt + 1) * KB, rows_lim_seq, 0, nb, wave, lane);
      stage64<NW>(vbase, ldq, (kt + 1) * KB, rows_lim_seq, 0, nb + TILE_BYTES, wave, lane);
    }
    const char* Ks = smem + buf * 2 * TILE_BYTES;
    const char* Vs = Ks + TILE_BYTES;

    // S^T[key][q] for 4 key sub-tiles of 16
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < 4; ++d) st[t] = MFMA(frag_row(Ks, 16 * t, d, lane), qf[d], st[t]);
    }
    // element (t, j) is key kt*KB + 4g + 16t + j; off the diagonal no element is masked
    const int rel = diag ? lim - (kt * KB + 4 * g) : 64;
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float a = st[t][j], b = st[t][j + 1];
        hf_scores2(a, b, scale);
        a = (16 * t + j > rel) ? -INFINITY : a;
        b = (16 * t + j + 1 > rel) ? -INFINITY : b;
        st[t][j] = a;
        st[t][j + 1] = b;
        tmax = fmaxf(tmax, fmaxf(a, b));
      }
    tmax = grp_max(tmax);
    const float m_new = fmaxf(m_run, tmax);  // finite: m_run starts at -1e30
    const float alpha = __builtin_amdgcn_exp2f((m_run - m_new) * L2E);
    const float mb = m_new * L2E;
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(st[t][j], L2E, -mb));
        st[t][j] = p;
        psum += p;
      }
    psum = grp_sum(psum);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] *= alpha;

    // O^T[d][q] += V^T[d][key] . P^T[key][q]: V^T fragments in batches of 4 (asm reads: no
    // vmcnt drain of the in-flight next tile, 4 LDS waits per tile instead of 16)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 pb = pack_perm(st[2 * u], st[2 * u + 1]);
#pragma unroll
      for (int d0 = 0; d0 < 8; d0 += 4) {
        i16x4 vlo[4], vhi[4];
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) trp_issue(Vs, 32 * u, 16 * (d0 + dd), lane, vlo[dd], vhi[dd]);
        trp_wait4(vlo, vhi);
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) o[d0 + dd] = MFMA(trp_join(vlo[dd], vhi[dd]), pb, o[d0 + dd]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  if (qrow < T) {
    const float inv = 1.f / l_run;
    bf16* op = out + (rowbase + qrow) * ldo + h * HD;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      uint2 pk;
      pk.x = pack2(o[dt][0] * inv, o[dt][1] * inv);
      pk.y = pack2(o[dt][2] * inv, o[dt][3] * inv);
      *reinterpret_cast<uint2*>(op + 16 * dt + 4 * g) = pk;
    }
    if (g == 0) lse[((long)s * H + h) * T + qrow] = m_run + __logf(l_run);
  }
}

// ============================================================ backward =====
// dK / dV: workgroup = 4 waves = 64 keys of one (sequence, head); each wave
// owns 16 keys (K, V fragments in registers, dK^T dV^T accumulators) and
// sweeps the query tiles at/after its block.  Q / dO tiles (+ lse, delta) are
// double-buffered in LDS through global_load_lds; no atomics.
// DBG (A/B decomposition only, results invalid): 1 = no softmax VALU (P = S, dS = dP),
// 2 = no dV/dK products, 3 = no S/dP products, 4 = no Q/dO loads after the first tile, 5 = no dS^T stores
template <int NW, int DBG = 0>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dkdv_kernel(const bf16* __restrict__ qkv, int ldq, int qc, int kc,
                                                            int vc, const bf16* __restrict__ dout, int ldd,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                            int ldg, int T, int H, float scale,
                                                            const bf16* __restrict__ rcs, const bf16* __restrict__ rsn,
                                                            bf16* __restrict__ dsT, int ds_ld) {
  // LDS: [Q | dO] x 2 buffers, then lse[2][64], delta[2][64]
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES + 4 * 64 * 4];
  float* Lsb = reinterpret_cast<float*>(smem + 4 * TILE_BYTES);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int kb = blockIdx.z, h = blockIdx.x, s = blockIdx.y;  // kb = 0 (longest sweeps) dispatched first, chip-wide
  const int g = lane >> 4, l16 = lane & 15;
  const long rowbase = (long)s * T;
  const int nq = (T + QB - 1) / QB;
  constexpr int KBW = 16 * NW;  // keys per workgroup
  const int key_l = kb * KBW + wave * 16 + l16;
  const int key_c = key_l < T ? key_l : T - 1;
  bf16x8 kf[4], vf[4];
  {
    const bf16* kp = qkv + (rowbase + key_c) * ldq + kc + h * HD;
    const bf16* vp = qkv + (rowbase + key_c) * ldq + vc + h * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      kf[d] = *reinterpret_cast<const bf16x8*>(kp + 32 * d + 8 * g);
      vf[d] = *reinterpret_cast<const bf16x8*>(vp + 32 * d + 8 * g);
    }
  }
  f32x4 dk[8], dv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { dk[i] = f32x4{0.f, 0.f, 0.f, 0.f}; dv[i] = f32x4{0.f, 0.f, 0.f, 0.f}; }

  const bf16* qbase = qkv + rowbase * ldq + qc + h * HD;
  const bf16* obase = dout + rowbase * ldd + h * HD;
  const float* lse_sh = lse + ((long)s * H + h) * T;
  const float* del_sh = delta + ((long)s * H + h) * T;
  // dS^T of this (sequence, head): [keys][queries], ds_ld columns per key row (dsT == nullptr: not kept)
  bf16* dsrow = dsT ? dsT + ((long)s * H + h) * ds_ld * (long)ds_ld + (long)key_l * ds_ld : nullptr;

  auto stage = [&](int qt, int b) {
    char* Qs = smem + b * 2 * TILE_BYTES;
    stage64<NW>(qbase, ldq, qt * QB, T, 0, Qs, wave, lane);
    stage64<NW>(obase, ldd, qt * QB, T, 0, Qs + TILE_BYTES, wave, lane);
    if (wave < 2) {  // 64 lanes x 4 B: lse (wave 0) / delta (wave 1) of the tile's 64 queries
      int q = qt * QB + lane;
      q = q < T ? q : T - 1;
      const float* src = (wave == 0 ? lse_sh : del_sh) + q;
      __builtin_amdgcn_global_load_lds(src, (LDS_AS void*)(Lsb + (wave * 2 + b) * 64), 4, 0, 0);
    }
  };

  const int qt0 = (kb * KBW) / QB;  // first query tile with a row >= the block's first key
  stage(qt0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto tile = [&](const int qt, auto diag_c) {
    constexpr bool DIAG = decltype(diag_c)::value;
    const int b = (qt - qt0) & 1;
    if (qt + 1 < nq && DBG != 4) stage(qt + 1, b ^ 1);
    const char* Qs = smem + b * 2 * TILE_BYTES;
    const char* Os = Qs + TILE_BYTES;
    const float* Ls = Lsb + b * 64;
    const float* Dl = Lsb + (2 + b) * 64;

    // S[q][key], dP[q][key] for 4 q sub-tiles; lane: key = l16, q = 16a + 4g + j
    f32x4 sv[4], dp[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      sv[a] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[a] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if constexpr (DBG == 3) {
          asm volatile("" ::"v"(frag_row(Qs, 16 * a, d, lane)), "v"(frag_row(Os, 16 * a, d, lane)));
        } else {
          sv[a] = MFMA(frag_row(Qs, 16 * a, d, lane), kf[d], sv[a]);
          dp[a] = MFMA(frag_row(Os, 16 * a, d, lane), vf[d], dp[a]);
        }
      }
    }
    // element (a, j) is query qt*QB + 4g + 16a + j: masked below the key (causal) or at / past T
    const int lo = key_l - (qt * QB + 4 * g), hi = T - (qt * QB + 4 * g);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      if constexpr (DBG == 1) break;
      // this lane's 4 queries of sub-tile a are consecutive: one 16-B LDS read each for lse, delta
      const f32x4 lq = *reinterpret_cast<const f32x4*>(Ls + 16 * a + 4 * g);
      const f32x4 dq4 = *reinterpret_cast<const f32x4*>(Dl + 16 * a + 4 * g);
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float x = sv[a][j], y = sv[a][j + 1];
        hf_scores2(x, y, scale);
        if (DIAG) {
          const int e = 16 * a + j;
          x = (e < lo || e >= hi) ? -INFINITY : x;
          y = (e + 1 < lo || e + 1 >= hi) ? -INFINITY : y;
        }
        const float px = __builtin_amdgcn_exp2f((x - lq[j]) * L2E);
        const float py = __builtin_amdgcn_exp2f((y - lq[j + 1]) * L2E);
        sv[a][j] = px;
        sv[a][j + 1] = py;
        dp[a][j] = px * (dp[a][j] - dq4[j]) * scale;
        dp[a][j + 1] = py * (dp[a][j + 1] - dq4[j + 1]) * scale;
      }
      if (dsrow && DBG != 5) {  // dS^T[key][q .. q+3] in bf16, the values the dK product below rounds to (8 B per lane)
        uint2 pk;
        pk.x = pack2(dp[a][0], dp[a][1]);
        pk.y = pack2(dp[a][2], dp[a][3]);
        *reinterpret_cast<uint2*>(dsrow + qt * QB + 16 * a + 4 * g) = pk;
      }
    }
    // dV^T[d][key] += dO^T[d][q] . P[q][key];  dK^T[d][key] += Q^T[d][q] . (scale dS)[q][key]
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 pb = pack_perm(sv[2 * u], sv[2 * u + 1]);
      const bf16x8 sb = pack_perm(dp[2 * u], dp[2 * u + 1]);
      // transposed fragments through the asm reads in batches of 2 + 2: the builtin form makes the
      // compiler drain vmcnt(0) (the next tile's DMA) before the first of them
#pragma unroll
      for (int d0 = 0; d0 < 8; d0 += 2) {
        i16x4 lo[4], hi[4];
        trp_issue(Os, 32 * u, 16 * d0, lane, lo[0], hi[0]);
        trp_issue(Os, 32 * u, 16 * (d0 + 1), lane, lo[1], hi[1]);
        trp_issue(Qs, 32 * u, 16 * d0, lane, lo[2], hi[2]);
        trp_issue(Qs, 32 * u, 16 * (d0 + 1), lane, lo[3], hi[3]);
        trp_wait4(lo, hi);
        if constexpr (DBG != 2) {
          dv[d0] = MFMA(trp_join(lo[0], hi[0]), pb, dv[d0]);
          dv[d0 + 1] = MFMA(trp_join(lo[1], hi[1]), pb, dv[d0 + 1]);
          dk[d0] = MFMA(trp_join(lo[2], hi[2]), sb, dk[d0]);
          dk[d0 + 1] = MFMA(trp_join(lo[3], hi[3]), sb, dk[d0 + 1]);
        } else {
          asm volatile("" ::"v"(pb), "v"(sb));
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  // keys >= T (clamped copies of key T-1) are never stored, so only causality and the T edge mask
  for (int qt = qt0; qt < nq; ++qt) {
    if (qt * QB < kb * KBW + KBW || (qt + 1) * QB > T)
      tile(qt, std::true_type{});
    else
      tile(qt, std::false_type{});
  }

  // lane holds [d = 16dt + 4g + j][key = l16]
  if (key_l < T) {
    if (rcs) rope_bwd_acc(dk, rcs, rsn, key_l, g);
    bf16* kp = dqkv + (rowbase + key_l) * ldg + kc + h * HD;
    bf16* vp = dqkv + (rowbase + key_l) * ldg + vc + h * HD;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      uint2 a, b;
      a.x = pack2(dk[dt][0], dk[dt][1]); a.y = pack2(dk[dt][2], dk[dt][3]);
      b.x = pack2(dv[dt][0], dv[dt][1]); b.y = pack2(dv[dt][2], dv[dt][3]);
      *reinterpret_cast<uint2*>(kp + 16 * dt + 4 * g) = a;
      *reinterpret_cast<uint2*>(vp + 16 * dt + 4 * g) = b;
    }
  }
}

// dQ: the forward's shape -- workgroup = 64 query rows, each wave 16 rows on
// the lanes; sweeps key tiles 0..qb with K / V double-buffered in LDS.
// dS^T[key][q] = P^T (dP^T - delta), dP^T = V . dO^T; dQ^T[d][q] += K^T[d][key] . dS^T.
// dQ lives in registers for the whole sweep: no atomics, no workspace.
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dq_kernel(const bf16* __restrict__ qkv, int ldq, int qc, int kc,
                                                          int vc, const bf16* __restrict__ dout, int ldd,
                                                          const bf16* __restrict__ o, int ldo,
                                                          const float* __restrict__ lse,
                                                          float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                          int ldg, int T, int H, float scale,
                                                          const bf16* __restrict__ rcs, const bf16* __restrict__ rsn) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // K0 V0 K1 V1
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int qb = gridDim.z - 1 - blockIdx.z;  // longest sweeps first, chip-wide (see the forward)
  const int h = blockIdx.x, s = blockIdx.y;
  const int g = lane >> 4, l16 = lane & 15;
  const long rowbase = (long)s * T;

  constexpr int RB = 16 * NW;
  const int qrow = qb * RB + wave * 16 + l16;
  const int qr_c = qrow < T ? qrow : T - 1;
  bf16x8 qf[4], of[4];
  float dpart = 0.f;  // delta = rowsum(dO * O), this lane's 32 of the head's 128 columns
  {
    const bf16* qp = qkv + (rowbase + qr_c) * ldq + qc + h * HD;
    const bf16* op = dout + (rowbase + qr_c) * ldd + h * HD;
    const bf16* oo = o + (rowbase + qr_c) * ldo + h * HD;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      qf[d] = *reinterpret_cast<const bf16x8*>(qp + 32 * d + 8 * g);
      of[d] = *reinterpret_cast<const bf16x8*>(op + 32 * d + 8 * g);
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(oo + 32 * d + 8 * g);
#pragma unroll
      for (int i = 0; i < 8; ++i) dpart += bf2f(of[d][i]) * bf2f(ov[i]);
    }
  }
  const float del_q = grp_sum(dpart);
  const float lse_q = lse[((long)s * H + h) * T + qr_c];
  if (g == 0 && qrow < T) delta[((long)s * H + h) * T + qrow] = del_q;  // for the dK/dV kernel (launched next)

  f32x4 dq[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int last = (qb * RB + RB - 1 < T ? qb * RB + RB - 1 : T - 1);
  const int n_kv = last / KB + 1;
  const bf16* kbase = qkv + rowbase * ldq + kc + h * HD;
  const bf16* vbase = qkv + rowbase * ldq + vc + h * HD;
  stage64<NW>(kbase, ldq, 0, T, 0, smem, wave, lane);
  stage64<NW>(vbase, ldq, 0, T, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lim = qrow < T ? qrow : T - 1;
  const float lse_b = lse_q * L2E;
  auto tile = [&](const int kt, auto diag_c) {
    constexpr bool DIAG = decltype(diag_c)::value;
    const int buf = kt & 1;
    if (kt + 1 < n_kv) {
      char* nb = smem + (buf ^ 1) * 2 * TILE_BYTES;
      stage64<NW>(kbase, ldq, (kt + 1) * KB, T, 0, nb, wave, lane);
      stage64<NW>(vbase, ldq, (kt + 1) * KB, T, 0, nb + TILE_BYTES, wave, lane);
    }
    const char* Ks = smem + buf * 2 * TILE_BYTES;
    const char* Vs = Ks + TILE_BYTES;

    f32x4 st[4], dpt[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dpt[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        st[t] = MFMA(frag_row(Ks, 16 * t, d, lane), qf[d], st[t]);
        dpt[t] = MFMA(frag_row(Vs, 16 * t, d, lane), of[d], dpt[t]);
      }
    }
    const int rel = lim - (kt * KB + 4 * g);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        float a = st[t][j], b = st[t][j + 1];
        hf_scores2(a, b, scale);
        if (DIAG) {
          a = (16 * t + j > rel) ? -INFINITY : a;
          b = (16 * t + j + 1 > rel) ? -INFINITY : b;
        }
        const float pa = __builtin_amdgcn_exp2f(fmaf(a, L2E, -lse_b));
        const float pb = __builtin_amdgcn_exp2f(fmaf(b, L2E, -lse_b));
        st[t][j] = pa * (dpt[t][j] - del_q) * scale;
        st[t][j + 1] = pb * (dpt[t][j + 1] - del_q) * scale;
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16x8 sb = pack_perm(st[2 * u], st[2 * u + 1]);
#pragma unroll
      for (int d0 = 0; d0 < 8; d0 += 4) {  // asm transposed reads: no vmcnt drain of the next tile's DMA
        i16x4 lo[4], hi[4];
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) trp_issue(Ks, 32 * u, 16 * (d0 + dd), lane, lo[dd], hi[dd]);
        trp_wait4(lo, hi);
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) dq[d0 + dd] = MFMA(trp_join(lo[dd], hi[dd]), sb, dq[d0 + dd]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  for (int kt = 0; kt < n_kv; ++kt) {
    if ((kt * KB + KB - 1 > qb * RB) || ((kt + 1) * KB > T))
      tile(kt, std::true_type{});
    else
      tile(kt, std::false_type{});
  }

  if (qrow < T) {
    if (rcs) rope_bwd_acc(dq, rcs, rsn, qrow, g);
    bf16* dp = dqkv + (rowbase + qrow) * ldg + qc + h * HD;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt) {
      uint2 pk;
      pk.x = pack2(dq[dt][0], dq[dt][1]);
      pk.y = pack2(dq[dt][2], dq[dt][3]);
      *reinterpret_cast<uint2*>(dp + 16 * dt + 4 * g) = pk;
    }
  }
}


// delta[s, h, t] = rowsum(dO * O) over the head's 128 columns (fp32): the softmax-backward term the
// dK/dV kernel reads.  One workgroup per row s*T + t; 16 lanes per head, 8 columns (16 B) per lane.
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(const bf16* __restrict__ dout, int ldd,
                                                             const bf16* __restrict__ o, int ldo,
                                                             float* __restrict__ delta, int T, int H) {
  const long row = blockIdx.x;
  const int s = (int)(row / T), t = (int)(row % T);
  for (int c = threadIdx.x; c < H * 16; c += 256) {
    const int h = c >> 4;
    const u32x4 a = *reinterpret_cast<const u32x4*>(dout + row * ldd + c * 8);
    const u32x4 b = *reinterpret_cast<const u32x4*>(o + row * ldo + c * 8);
    float fa[8], fb[8];
    unpack8(a, fa);
    unpack8(b, fb);
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += fa[i] * fb[i];
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) v += __shfl_xor(v, m, 16);
    if ((c & 15) == 0) delta[((long)s * H + h) * T + t] = v;
  }
}

// wait for 2 transposed fragments (4 reads): registers tied to the wait
__device__ __forceinline__ void trp_wait2(i16x4 (&lo)[2], i16x4 (&hi)[2]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(lo[0]), "+v"(lo[1]), "+v"(hi[0]), "+v"(hi[1])::"memory");
  __builtin_amdgcn_sched_barrier(0);
}
// transposed fragment, natural k order (element j <- row kbase + 8g + j), asm form (see trp_issue)
__device__ __forceinline__ void trn_issue(const char* lds, int kbase, int c0, int lane, i16x4& lo, i16x4& hi) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int r1 = kbase + 8 * g + q;
  const int r2 = r1 + 4;
  const int x = (c0 >> 3) + (p >> 1);
  const int hh = (p & 1) << 3;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_u32(lds + r1 * ROWB + ((x ^ aswz(r1)) << 4) + hh)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_u32(lds + r2 * ROWB + ((x ^ aswz(r2)) << 4) + hh)));
}

// dQ = dS . K from the dS^T the dK/dV kernel stored: workgroup = NW waves x 32 query rows of one
// (sequence, head); per 64-key tile the K tile [key][d] and the dS^T tile [key][128 queries] are
// staged in LDS (LDS-DMA, double-buffered) and both MFMA operands come from transposed reads:
// dQ^T[d][q] += K^T[d][key] . dS^T[key][q], each K^T fragment feeding the wave's two query
// sub-tiles.  One product instead of the three (S, dP, dQ) of attn_bwd_dq_kernel.  Causal masking
// is already in dS (zeros).  RoPE backward fused into the store.
template <int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dq_ds_kernel(const bf16* __restrict__ qkv, int ldq, int qc,
                                                             int kc, const bf16* __restrict__ dsT, int ds_ld,
                                                             bf16* __restrict__ dqkv, int ldg, int T, int H,
                                                             const bf16* __restrict__ rcs,
                                                             const bf16* __restrict__ rsn) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // [K | dS^T] x 2 buffers
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int RB = 32 * NW;  // query rows per workgroup
  const int qb = gridDim.z - 1 - blockIdx.z;  // longest sweeps first, chip-wide
  const int h = blockIdx.x, s = blockIdx.y;
  const int g = lane >> 4, l16 = lane & 15;
  const long rowbase = (long)s * T;
  const bf16* kbase = qkv + rowbase * ldq + kc + h * HD;
  const bf16* dbase = dsT + ((long)s * H + h) * ds_ld * (long)ds_ld;

  f32x4 dq[2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 8; ++i) dq[a][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int last = (qb * RB + RB - 1 < T ? qb * RB + RB - 1 : T - 1);
  const int n_kv = last / KB + 1;
  auto stage = [&](int kt, int b) {
    char* Ks = smem + b * 2 * TILE_BYTES;
    stage64<NW>(kbase, ldq, kt * KB, T, 0, Ks, wave, lane);
    stage64<NW>(dbase, ds_ld, kt * KB, ds_ld, qb * RB, Ks + TILE_BYTES, wave, lane);
  };
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < n_kv; ++kt) {
    const int b = kt & 1;
    if (kt + 1 < n_kv) stage(kt + 1, b ^ 1);
    const char* Ks = smem + b * 2 * TILE_BYTES;
    const char* Ds = Ks + TILE_BYTES;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      i16x4 blo[2], bhi[2];
      trn_issue(Ds, 32 * ks, wave * 32, lane, blo[0], bhi[0]);
      trn_issue(Ds, 32 * ks, wave * 32 + 16, lane, blo[1], bhi[1]);
      trp_wait2(blo, bhi);
      const bf16x8 b0 = trp_join(blo[0], bhi[0]), b1 = trp_join(blo[1], bhi[1]);
#pragma unroll
      for (int d0 = 0; d0 < 8; d0 += 4) {
        i16x4 lo[4], hi[4];
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) trn_issue(Ks, 32 * ks, 16 * (d0 + dd), lane, lo[dd], hi[dd]);
        trp_wait4(lo, hi);
#pragma unroll
        for (int dd = 0; dd < 4; ++dd) {
          const bf16x8 a = trp_join(lo[dd], hi[dd]);
          dq[0][d0 + dd] = MFMA(a, b0, dq[0][d0 + dd]);
          dq[1][d0 + dd] = MFMA(a, b1, dq[1][d0 + dd]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // lane holds [d = 16dt + 4g + j][q = l16] of query sub-tile a
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int qrow = qb * RB + wave * 32 + 16 * a + l16;
    if (qrow < T) {
      if (rcs) rope_bwd_acc(dq[a], rcs, rsn, qrow, g);
      bf16* dp = dqkv + (rowbase + qrow) * ldg + qc + h * HD;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt) {
        uint2 pk;
        pk.x = pack2(dq[a][dt][0], dq[a][dt][1]);
        pk.y = pack2(dq[a][dt][2], dq[a][dt][3]);
        *reinterpret_cast<uint2*>(dp + 16 * dt + 4 * g) = pk;
      }
    }
  }
}

// dS^T rows / columns per (sequence, head): T rounded up to the dQ kernel's 128-query blocks
int ds_pitch(int T) { return (T + 127) / 128 * 128; }

// waves per workgroup (16 query rows / keys each): 8 shares every staged K/V (Q/dO)
// tile between twice the rows; the ablation build's OSPO_ATTN_WAVES=4 selects the 64-row form (A/B)
int attn_waves() {
#ifdef OSPO_ABLATION
  static const int nw = [] {
    const char* e = getenv("OSPO_ATTN_WAVES");
    return (e && atoi(e) == 4) ? 4 : 8;
  }();
  return nw;
#else
  return 8;
#endif
}

}  // namespace

extern "C" int ospo_flash_attn_fwd(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col, void* o,
                                   int ld_o, float* lse, int S, int T, int n_heads, int head_dim, float scale,
                                   hipStream_t stream) {
  if (!qkv || !o || !lse) return OSPO_ERR_ARG;
  if (head_dim != HD) return OSPO_ERR_UNSUPPORTED;
  if (S <= 0 || T <= 0 || n_heads <= 0 || ld_qkv % 8 || ld_o % 8 || q_col % 8 || k_col % 8 || v_col % 8)
    return OSPO_ERR_SHAPE;
  if (!aligned16(qkv) || !aligned16(o)) return OSPO_ERR_ALIGN;
  const int nw = attn_waves();
  dim3 grid(n_heads, S, (T + 16 * nw - 1) / (16 * nw));
#ifdef OSPO_ABLATION
  static const bool dbg = getenv("OSPO_ATTN_DBG") != nullptr;  // ablation only (results invalid)
  auto kfn = dbg ? attn_fwd_kernel<8, 1> : (nw == 8 ? attn_fwd_kernel<8, 0> : attn_fwd_kernel<4, 0>);
#else
  auto kfn = attn_fwd_kernel<8, 0>;
#endif
  hipLaunchKernelGGL(kfn, grid, dim3(64 * nw), 0, stream, (const bf16*)qkv, ld_qkv, q_col, k_col, v_col,
                     (bf16*)o, ld_o, lse, T, n_heads, scale);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" size_t ospo_flash_attn_bwd_ws_bytes(int S, int T, int n_heads) {
  if (S <= 0 || T <= 0 || n_heads <= 0) return 0;
  const long p = ds_pitch(T);
  return (size_t)S * n_heads * p * p * sizeof(bf16);
}

extern "C" int ospo_flash_attn_bwd(const void* qkv, int ld_qkv, int q_col, int k_col, int v_col, const void* o,
                                   int ld_o, const void* dout, int ld_do, const float* lse, float* delta_ws,
                                   void* ds_ws, void* dqkv, int ld_dqkv, int S, int T, int n_heads,
                                   int head_dim, float scale, const void* rope_cos, const void* rope_sin,
                                   hipStream_t stream) {
  if (!qkv || !o || !dout || !lse || !delta_ws || !dqkv) return OSPO_ERR_ARG;
  if (head_dim != HD) return OSPO_ERR_UNSUPPORTED;
  if (S <= 0 || T <= 0 || n_heads <= 0 || ld_qkv % 8 || ld_o % 8 || ld_do % 8 || ld_dqkv % 8) return OSPO_ERR_SHAPE;
  if (q_col % 8 || k_col % 8 || v_col % 8) return OSPO_ERR_SHAPE;
  if (!aligned16(qkv) || !aligned16(o) || !aligned16(dout) || !aligned16(dqkv)) return OSPO_ERR_ALIGN;
  if (ds_ws && !aligned16(ds_ws)) return OSPO_ERR_ALIGN;
  if ((rope_cos == nullptr) != (rope_sin == nullptr)) return OSPO_ERR_ARG;
  if (rope_cos && (((uintptr_t)rope_cos & 7) || ((uintptr_t)rope_sin & 7))) return OSPO_ERR_ALIGN;
  const bf16* rc = (const bf16*)rope_cos;
  const bf16* rs = (const bf16*)rope_sin;
  const int nw = attn_waves();
  dim3 grid(n_heads, S, (T + 16 * nw - 1) / (16 * nw));
#ifdef OSPO_ABLATION
  static const int dkdv_dbg = [] {  // ablation only (results invalid): tools/attn_bench.py
    const char* e = getenv("OSPO_ATTN_DKDV_DBG");
    return e ? atoi(e) : 0;
  }();
  auto dkdv = nw == 4 ? attn_bwd_dkdv_kernel<4> : attn_bwd_dkdv_kernel<8>;
  if (nw == 8 && dkdv_dbg == 1) dkdv = attn_bwd_dkdv_kernel<8, 1>;
  if (nw == 8 && dkdv_dbg == 2) dkdv = attn_bwd_dkdv_kernel<8, 2>;
  if (nw == 8 && dkdv_dbg == 3) dkdv = attn_bwd_dkdv_kernel<8, 3>;
  if (nw == 8 && dkdv_dbg == 4) dkdv = attn_bwd_dkdv_kernel<8, 4>;
  if (nw == 8 && dkdv_dbg == 5) dkdv = attn_bwd_dkdv_kernel<8, 5>;  // no dS^T stores
#else
  auto dkdv = attn_bwd_dkdv_kernel<8>;
#endif
  if (ds_ws && nw == 8) {
    // delta, then dK/dV (which also stores dS^T), then dQ = dS . K: 5 MFMA products instead of 7
    const int p = ds_pitch(T);
    hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3(S * T), dim3(256), 0, stream, (const bf16*)dout, ld_do,
                       (const bf16*)o, ld_o, delta_ws, T, n_heads);
    OSPO_CHECK_LAUNCH();
    hipLaunchKernelGGL(dkdv, grid, dim3(64 * nw), 0, stream, (const bf16*)qkv, ld_qkv, q_col, k_col, v_col,
                       (const bf16*)dout, ld_do, lse, delta_ws, (bf16*)dqkv, ld_dqkv, T, n_heads, scale, rc, rs,
                       (bf16*)ds_ws, p);
    OSPO_CHECK_LAUNCH();
    dim3 gq(n_heads, S, (T + 127) / 128);
    hipLaunchKernelGGL(attn_bwd_dq_ds_kernel<4>, gq, dim3(256), 0, stream, (const bf16*)qkv, ld_qkv, q_col, k_col,
                       (const bf16*)ds_ws, p, (bf16*)dqkv, ld_dqkv, T, n_heads, rc, rs);
    OSPO_CHECK_LAUNCH();
    return OSPO_OK;
  }
  // no dS workspace: dQ first (it also produces delta = rowsum(dO * O)), recomputing S and dP
  dim3 gq(n_heads, S, (T + 16 * nw - 1) / (16 * nw));
  hipLaunchKernelGGL(nw == 8 ? attn_bwd_dq_kernel<8> : attn_bwd_dq_kernel<4>, gq, dim3(64 * nw), 0, stream,
                     (const bf16*)qkv, ld_qkv, q_col, k_col, v_col, (const bf16*)dout, ld_do, (const bf16*)o, ld_o,
                     lse, delta_ws, (bf16*)dqkv, ld_dqkv, T, n_heads, scale, rc, rs);
  OSPO_CHECK_LAUNCH();
  hipLaunchKernelGGL(dkdv, grid, dim3(64 * nw), 0, stream, (const bf16*)qkv, ld_qkv, q_col, k_col,
                     v_col, (const bf16*)dout, ld_do, lse, delta_ws, (bf16*)dqkv, ld_dqkv, T, n_heads, scale, rc, rs,
                     (bf16*)nullptr, 0);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
