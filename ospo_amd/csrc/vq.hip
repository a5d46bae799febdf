// VQ image tokenizer (encoder + quantizer) of Janus-Pro's gen_vision_model on gfx950 (SURVEY §8f
// rank 3): janus/models/vq_model.py Encoder (:46-124) -> quant_conv -> VectorQuantizer (:236-282),
// the step before the SimPO path (ospo/wrapper/train.py:246-264 encodes every image of a batch);
// and its pixel decoder (decode_code :505-508: codebook rows -> post_quant_conv -> Decoder :127-214,
// the Upsample's nearest 2x read on the fly by the convolution) for step-3 sampling.
//
// fp32 end to end: the ids must be bit-exact, and bf16 moves ~10 % of them.
//  * Convolutions are implicit GEMMs on v_mfma_f32_32x32x2_f32 (f32 in / f32 accumulate, exact
//    products -- a k-ordered fmaf chain): NHWC activations (channels contiguous), weights
//    [Cout][KH][KW][Cin]; a workgroup computes 128 output pixels x 64 output channels, K walks
//    (ky, kx, 32-channel chunk) with the shifted pixel rows gathered into LDS (zero outside the
//    image, which also gives Downsample's asymmetric (0,1,0,1) padding), double buffered.
//    Bias and the ResnetBlock / AttnBlock residual are fused into the epilogue.  The AttnBlock's
//    q.k^T and p.v^T products are the same kernel as 1x1 "convolutions" over the 576 tokens.
//  * GroupNorm(32, eps 1e-6) (+ swish): fp64 per-channel sums over pixel slices (coalesced rows),
//    folded per group, finalised to (mean, rstd), then one vectorised normalise pass.
//  * Quantizer: l2-normalised z against the l2-normalised codebook, d = |z|^2 + |e|^2 - 2 z.e in
//    fp32, first index of the minimum (torch.argmin).
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int CV_BM = 128, CV_BN = 64, CV_BK = 32;

struct ConvArgs {
  const float* x;  // [B][H][W][Cin]
  const float* w;  // [Cout][KH][KW][Cin]
  const float* bias;
  const float* res;  // [B][Ho][Wo][Cout] or null
  float* out;        // [B][Ho][Wo][Cout]
  int B, H, W, Cin, Cout, KH, KW, stride, pad_t, pad_l, Ho, Wo;
  long x_bstride, w_bstride, o_bstride;  // per-image strides of x / w / out when w is per image (attention)
  int up;  // 1: the input is read as its nearest-neighbour 2x upsampling (2H x 2W), Decoder's Upsample
};

// grid: (ceil(npix / 128), ceil(Cout / 64), nz); 256 threads; wave w: pixels 32w..32w+31 x 64 channels.
// conv mode (nz = 1): the B images are folded into the pixel index.  per-image-weight mode (nz = B, the
// attention products): block z works on image z only, with w + z * w_bstride as its weights.
__global__ __launch_bounds__(256) void conv_f32_kernel(const ConvArgs a, int per_image_w) {
  __shared__ float As[2][CV_BK][CV_BM];  // [k][pixel]
  __shared__ float Bs[2][CV_BK][CV_BN];  // [k][cout]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int zimg = blockIdx.z;
  const long npix = per_image_w ? (long)a.Ho * a.Wo : (long)a.B * a.Ho * a.Wo;
  const long p0 = (long)blockIdx.x * CV_BM;
  const int c0 = blockIdx.y * CV_BN;
  const float* xbase = a.x + (per_image_w ? (long)zimg * a.x_bstride : 0);
  const float* wbase = a.w + (per_image_w ? (long)zimg * a.w_bstride : 0);
  float* obase = a.out + (per_image_w ? (long)zimg * a.o_bstride : 0);
  const float* rbase = a.res ? a.res + (per_image_w ? (long)zimg * a.o_bstride : 0) : nullptr;
  // A loader: thread t -> pixel t >> 1, channels (t & 1) * 16 .. +16 of the chunk
  const int lp = t >> 1, lc = (t & 1) * 16;
  const long gp = p0 + lp;
  int ib = 0, oy = 0, ox = 0;
  const bool pvalid = gp < npix;
  if (pvalid) {
    ib = (int)(gp / ((long)a.Ho * a.Wo));
    const int r = (int)(gp % ((long)a.Ho * a.Wo));
    oy = r / a.Wo;
    ox = r % a.Wo;
  }
  // B loader: thread t -> cout t >> 2, channels (t & 3) * 8 .. +8
  const int bc = t >> 2, bk = (t & 3) * 8;
  const int cchunks = (a.Cin + CV_BK - 1) / CV_BK;
  const int nk = a.KH * a.KW * cchunks;
  const bool vec = (a.Cin % 4) == 0;
  float ra[16], rb[8];
  auto gload = [&](int kt) {
    const int cc = kt % cchunks, kk = kt / cchunks;
    const int ky = kk / a.KW, kx = kk % a.KW;
    const int ci0 = cc * CV_BK;
    const int iy = oy * a.stride - a.pad_t + ky, ix = ox * a.stride - a.pad_l + kx;
    const bool in = pvalid && iy >= 0 && iy < (a.H << a.up) && ix >= 0 && ix < (a.W << a.up);
    const float* src = xbase + (((long)ib * a.H + (in ? iy >> a.up : 0)) * a.W + (in ? ix >> a.up : 0)) * a.Cin +
                       ci0 + lc;
    if (in && vec && ci0 + lc + 16 <= a.Cin) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(src + 4 * q);
        ra[4 * q] = v[0]; ra[4 * q + 1] = v[1]; ra[4 * q + 2] = v[2]; ra[4 * q + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) ra[q] = (in && ci0 + lc + q < a.Cin) ? src[q] : 0.f;
    }
    const int co = c0 + bc;
    const float* wsrc = wbase + (((long)(co < a.Cout ? co : 0) * a.KH + ky) * a.KW + kx) * a.Cin + ci0 + bk;
    if (co < a.Cout && vec && ci0 + bk + 8 <= a.Cin) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(wsrc + 4 * q);
        rb[4 * q] = v[0]; rb[4 * q + 1] = v[1]; rb[4 * q + 2] = v[2]; rb[4 * q + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) rb[q] = (co < a.Cout && ci0 + bk + q < a.Cin) ? wsrc[q] : 0.f;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 16; ++q) As[buf][lc + q][lp] = ra[q];
#pragma unroll
    for (int q = 0; q < 8; ++q) Bs[buf][bk + q][bc] = rb[q];
  };
  f32x16 acc[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < CV_BK; ks += 2) {
      const int k = ks + (lane >> 5);
      const float av = As[buf][k][wave * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float bv = Bs[buf][k][j * 32 + (lane & 31)];
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }
  // epilogue: lane holds D[row][col], col = lane & 31 (cout), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (pixel)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int co = c0 + j * 32 + (lane & 31);
    if (co >= a.Cout) continue;
    const float bsv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long p = p0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (p >= npix) continue;
      float v = acc[j][r] + bsv;
      const long o = p * a.Cout + co;
      if (rbase) v += rbase[o];
      obase[o] = v;
    }
  }
}

// ------------------------------------------------------------------ GroupNorm
// stats: grid (B, S): workgroup (b, s) walks pixels [HW s / S, HW (s+1) / S) of image b with thread t
// on channels t, t + 256, ... (coalesced rows); fp64 per-channel sums are folded into per-group
// partials [b][s][g][2] through LDS.
constexpr int GN_S = 64;
__global__ __launch_bounds__(256) void gn_stats_kernel(const float* __restrict__ x, int HW, int C, int G,
                                                       double* __restrict__ part) {
  __shared__ double red[2][1024];
  const int b = blockIdx.x, s = blockIdx.y;
  const long lo = (long)HW * s / GN_S, hi = (long)HW * (s + 1) / GN_S;
  const float* xb = x + (long)b * HW * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    double s1 = 0.0, s2 = 0.0;
    for (long p = lo; p < hi; ++p) {
      const double v = xb[p * C + c];
      s1 += v;
      s2 += v * v;
    }
    red[0][c] = s1;
    red[1][c] = s2;
  }
  __syncthreads();
  const int cpg = C / G;
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      s1 += red[0][c];
      s2 += red[1][c];
    }
    double* o = part + (((long)b * GN_S + s) * G + g) * 2;
    o[0] = s1;
    o[1] = s2;
  }
}

// per (b, g): mean and rstd (biased variance, eps inside the sqrt) from the partials
__global__ void gn_finalize_kernel(const double* __restrict__ part, int B, int HW, int C, int G, float eps,
                                   float* __restrict__ stats) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * G) return;
  const int b = i / G, g = i % G;
  double s1 = 0.0, s2 = 0.0;
  for (int s = 0; s < GN_S; ++s) {
    s1 += part[(((long)b * GN_S + s) * G + g) * 2];
    s2 += part[(((long)b * GN_S + s) * G + g) * 2 + 1];
  }
  const double n = (double)HW * (C / G);
  const double mean = s1 / n;
  const double var = fmax(s2 / n - mean * mean, 0.0);
  stats[2 * i] = (float)mean;
  stats[2 * i + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// y = (x - mean) * rstd * gamma + beta; swish: y * sigmoid(y).  4 channels per thread (C % 4 == 0).
__global__ void gn_apply_kernel(const float* __restrict__ x, long total4, int HW, int C, int G,
                                const float* __restrict__ stats, const float* __restrict__ gamma,
                                const float* __restrict__ beta, int swish, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total4) return;
  const long e = i * 4;
  const int c = (int)(e % C);
  const int b = (int)(e / ((long)HW * C));
  const int g = c / (C / G);  // C / G is a multiple of 4 here, so the 4 channels share a group
  const float mean = stats[2 * (b * G + g)], rstd = stats[2 * (b * G + g) + 1];
  const f32x4 v = *reinterpret_cast<const f32x4*>(x + e);
  f32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float t = (v[q] - mean) * rstd * gamma[c + q] + beta[c + q];
    if (swish) t = t * (1.f / (1.f + expf(-t)));
    o[q] = t;
  }
  *reinterpret_cast<f32x4*>(y + e) = o;
}

// ------------------------------------------------------------ attention helpers
// rows of [n][cols]: y = softmax(x * scale) (fp32, max-subtracted)
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* __restrict__ x, int cols, float scale) {
  __shared__ float red[8];
  float* row = x + (long)blockIdx.x * cols;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < cols; c += 256) m = fmaxf(m, row[c] * scale);
  m = wave_max(m);
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
  for (int c = threadIdx.x; c < cols; c += 256) {
    const float e = expf(row[c] * scale - m);
    row[c] = e;
    s += e;
  }
  s = wave_sum(s);
  __syncthreads();
  if (lane == 0) red[4 + wave] = s;
  __syncthreads();
  const float inv = 1.f / (red[4] + red[5] + red[6] + red[7]);
  for (int c = threadIdx.x; c < cols; c += 256) row[c] *= inv;
}

// [B][R][C] -> [B][C][R]
__global__ void transpose_kernel(const float* __restrict__ x, int R, int C, float* __restrict__ y) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z;
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const float* xb = x + (long)b * R * C;
  float* yb = y + (long)b * R * C;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    if (r < R && c < C) tile[i][threadIdx.x] = xb[(long)r * C + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (r < R && c < C) yb[(long)c * R + r] = tile[threadIdx.x][i];
  }
}

// ---------------------------------------------------------------- quantizer
// one workgroup per 16 vectors; 256 threads scan the codebook (thread t: codes t, t+256, ...) for
// each vector, then an (distance, index) min-reduction with the lower index winning ties.
constexpr int VQ_E = 8;
__global__ __launch_bounds__(256) void vq_quantize_kernel(const float* __restrict__ z, long n,
                                                          const float* __restrict__ cb, int ncodes,
                                                          int* __restrict__ ids, float* __restrict__ dmin) {
  __shared__ float zs[16][VQ_E];
  __shared__ float zsq[16];
  __shared__ float bd[16][256];
  __shared__ int bi[16][256];
  const long v0 = (long)blockIdx.x * 16;
  const int t = threadIdx.x;
  if (t < 16) {
    const long v = v0 + t;
    float e[VQ_E], ss = 0.f;
#pragma unroll
    for (int q = 0; q < VQ_E; ++q) {
      e[q] = v < n ? z[v * VQ_E + q] : 0.f;
      ss += e[q] * e[q];
    }
    const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);  // F.normalize: x / max(||x||, eps)
    float s2 = 0.f;
#pragma unroll
    for (int q = 0; q < VQ_E; ++q) {
      zs[t][q] = e[q] * inv;
      s2 += zs[t][q] * zs[t][q];
    }
    zsq[t] = s2;
  }
  __syncthreads();
  float best[16];
  int bidx[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    best[k] = INFINITY;
    bidx[k] = 0;
  }
  for (int c = t; c < ncodes; c += 256) {
    float e[VQ_E];
#pragma unroll
    for (int q = 0; q < VQ_E; ++q) e[q] = cb[(long)c * VQ_E + q];
    float ee = 0.f;
#pragma unroll
    for (int q = 0; q < VQ_E; ++q) ee += e[q] * e[q];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < VQ_E; ++q) dot += zs[k][q] * e[q];
      const float d = (zsq[k] + ee) - 2.f * dot;
      if (d < best[k]) {  // strictly less: the first (lowest) index of this thread's codes wins ties
        best[k] = d;
        bidx[k] = c;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    bd[k][t] = best[k];
    bi[k][t] = bidx[k];
  }
  __syncthreads();
  if (t < 16) {
    float b = INFINITY;
    int idx = 0x7fffffff;
    for (int i = 0; i < 256; ++i) {
      const float d = bd[t][i];
      const int j = bi[t][i];
      if (d < b || (d == b && j < idx)) {
        b = d;
        idx = j;
      }
    }
    const long v = v0 + t;
    if (v < n) {
      ids[v] = idx;
      if (dmin) dmin[v] = b;
    }
  }
}

// codebook rows l2-normalised (F.normalize over the embedding dim)
__global__ void l2norm_rows_kernel(const float* __restrict__ x, long n, int d, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float ss = 0.f;
  for (int q = 0; q < d; ++q) ss += x[i * d + q] * x[i * d + q];
  const float inv = 1.f / fmaxf(sqrtf(ss), 1e-12f);
  for (int q = 0; q < d; ++q) y[i * d + q] = x[i * d + q] * inv;
}

// decode_code's get_codebook_entry (vq_model.py:284-298): rows of the l2-normalised codebook, NHWC
__global__ void vq_embed_codes_kernel(const int* __restrict__ ids, long n, const float* __restrict__ cb,
                                      int n_codes, int e, float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * e) return;
  int id = ids[i / e];
  id = id < 0 ? 0 : (id >= n_codes ? n_codes - 1 : id);
  out[i] = cb[(long)id * e + i % e];
}

// image_generation.py:175-181: clip((x + 1) / 2 * 255, 0, 255) in fp32, stored as uint8 (truncation)
__global__ void vq_to_uint8_kernel(const float* __restrict__ x, long n, unsigned char* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = fminf(fmaxf((x[i] + 1.f) / 2.f * 255.f, 0.f), 255.f);
  out[i] = (unsigned char)v;
}

}  // namespace

extern "C" int ospo_vq_conv2d(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH, int KW,
                              int stride, int pad_t, int pad_l, int Ho, int Wo, const float* bias,
                              const float* residual, float* out, hipStream_t stream) {
  if (!x || !w || !out) return OSPO_ERR_ARG;
  if (B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || stride <= 0 || Ho <= 0 ||
      Wo <= 0 || pad_t < 0 || pad_l < 0)
    return OSPO_ERR_SHAPE;
  if ((long)(Ho - 1) * stride - pad_t + KH > H + KH || (long)(Wo - 1) * stride - pad_l + KW > W + KW)
    return OSPO_ERR_SHAPE;
  ConvArgs a{x, w, bias, residual, out, B, H, W, Cin, Cout, KH, KW, stride, pad_t, pad_l, Ho, Wo, 0, 0, 0};
  const long npix = (long)B * Ho * Wo;
  hipLaunchKernelGGL(conv_f32_kernel, dim3((unsigned)((npix + CV_BM - 1) / CV_BM), (Cout + CV_BN - 1) / CV_BN),
                     dim3(256), 0, stream, a, 0);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

// out[b][i][j] = sum_c x[b][i][c] * w[b][j][c] (+ residual): a per-image "1x1 convolution" whose weight is
// another activation (AttnBlock's q.k^T and p.v^T); grid z = image.
extern "C" int ospo_vq_conv2d_up2(const float* x, int B, int H, int W, int Cin, const float* w, int Cout, int KH,
                                  int KW, int pad, const float* bias, const float* residual, float* out,
                                  hipStream_t stream) {
  if (!x || !w || !out) return OSPO_ERR_ARG;
  if (B <= 0 || H <= 0 || W <= 0 || Cin <= 0 || Cout <= 0 || KH <= 0 || KW <= 0 || pad < 0) return OSPO_ERR_SHAPE;
  const int Ho = 2 * H + 2 * pad - KH + 1, Wo = 2 * W + 2 * pad - KW + 1;
  if (Ho <= 0 || Wo <= 0) return OSPO_ERR_SHAPE;
  ConvArgs a{x, w, bias, residual, out, B, H, W, Cin, Cout, KH, KW, 1, pad, pad, Ho, Wo, 0, 0, 0, 1};
  const long npix = (long)B * Ho * Wo;
  hipLaunchKernelGGL(conv_f32_kernel, dim3((unsigned)((npix + CV_BM - 1) / CV_BM), (Cout + CV_BN - 1) / CV_BN),
                     dim3(256), 0, stream, a, 0);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_embed_codes(const int* ids, long n, const float* codebook_l2, int n_codes, int e_dim,
                                   float* out, hipStream_t stream) {
  if (!ids || !codebook_l2 || !out) return OSPO_ERR_ARG;
  if (n <= 0 || n_codes <= 0 || e_dim <= 0) return OSPO_ERR_SHAPE;
  const long tot = n * e_dim;
  hipLaunchKernelGGL(vq_embed_codes_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, ids, n,
                     codebook_l2, n_codes, e_dim, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_to_uint8(const float* x, long n, unsigned char* out, hipStream_t stream) {
  if (!x || !out) return OSPO_ERR_ARG;
  if (n <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(vq_to_uint8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, n, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_bmm_nt(const float* x, const float* w, int B, int n_rows, int n_cols, int K, float* out,
                              hipStream_t stream) {
  if (!x || !w || !out) return OSPO_ERR_ARG;
  if (B <= 0 || n_rows <= 0 || n_cols <= 0 || K <= 0) return OSPO_ERR_SHAPE;
  ConvArgs a{x, w, nullptr, nullptr, out, 1, n_rows, 1, K, n_cols, 1, 1, 1, 0, 0, n_rows, 1,
             (long)n_rows * K, (long)n_cols * K, (long)n_rows * n_cols};
  hipLaunchKernelGGL(conv_f32_kernel, dim3((n_rows + CV_BM - 1) / CV_BM, (n_cols + CV_BN - 1) / CV_BN, B),
                     dim3(256), 0, stream, a, 1);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" size_t ospo_vq_groupnorm_ws_bytes(int B, int G) {
  return (size_t)B * GN_S * G * 2 * sizeof(double) + (size_t)B * G * 2 * sizeof(float) + 16;
}

extern "C" int ospo_vq_groupnorm(const float* x, int B, int HW, int C, int G, const float* gamma, const float* beta,
                                 float eps, int swish, float* out, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (!x || !gamma || !beta || !out || !ws) return OSPO_ERR_ARG;
  if (B <= 0 || HW <= 0 || C <= 0 || G <= 0 || C % G || (C / G) % 4 || C > 1024) return OSPO_ERR_SHAPE;
  if (ws_bytes < ospo_vq_groupnorm_ws_bytes(B, G)) return OSPO_ERR_SHAPE;
  if (!aligned16(x) || !aligned16(out)) return OSPO_ERR_ALIGN;
  double* part = (double*)ws;
  float* stats = (float*)(part + (size_t)B * GN_S * G * 2);
  hipLaunchKernelGGL(gn_stats_kernel, dim3(B, GN_S), dim3(256), 0, stream, x, HW, C, G, part);
  hipLaunchKernelGGL(gn_finalize_kernel, dim3((B * G + 255) / 256), dim3(256), 0, stream, part, B, HW, C, G, eps,
                     stats);
  const long total4 = (long)B * HW * C / 4;
  hipLaunchKernelGGL(gn_apply_kernel, dim3((unsigned)((total4 + 255) / 256)), dim3(256), 0, stream, x, total4, HW, C,
                     G, stats, gamma, beta, swish, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_softmax_rows(float* x, int rows, int cols, float scale, hipStream_t stream) {
  if (!x) return OSPO_ERR_ARG;
  if (rows <= 0 || cols <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3(rows), dim3(256), 0, stream, x, cols, scale);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_transpose(const float* x, int B, int R, int C, float* out, hipStream_t stream) {
  if (!x || !out || x == out) return OSPO_ERR_ARG;
  if (B <= 0 || R <= 0 || C <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(transpose_kernel, dim3((C + 31) / 32, (R + 31) / 32, B), dim3(32, 8), 0, stream, x, R, C, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_l2norm_rows(const float* x, long n, int d, float* out, hipStream_t stream) {
  if (!x || !out) return OSPO_ERR_ARG;
  if (n <= 0 || d <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, x, n, d, out);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}

extern "C" int ospo_vq_quantize(const float* z, long n, int e_dim, const float* codebook_l2, int n_codes, int* ids,
                                float* dmin, hipStream_t stream) {
  if (!z || !codebook_l2 || !ids) return OSPO_ERR_ARG;
  if (e_dim != VQ_E) return OSPO_ERR_UNSUPPORTED;
  if (n <= 0 || n_codes <= 0) return OSPO_ERR_SHAPE;
  hipLaunchKernelGGL(vq_quantize_kernel, dim3((unsigned)((n + 15) / 16)), dim3(256), 0, stream, z, n, codebook_l2,
                     n_codes, ids, dmin);
  OSPO_CHECK_LAUNCH();
  return OSPO_OK;
}
