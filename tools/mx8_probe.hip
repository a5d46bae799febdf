// Probe of the gfx950 block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4) operand and
// scale layout, and of the hardware f32 -> OCP e4m3 conversion, against host references.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mx8_probe.hip -o tools/mx8_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// host: exact decode of an e4m3fn byte
static float dec_e4m3(uint8_t b) {
  const int s = b >> 7, e = (b >> 3) & 15, m = b & 7;
  if (e == 15 && m == 7) return NAN;
  float v = e ? std::ldexp(1.f + m / 8.f, e - 7) : std::ldexp(m / 8.f, -6);
  return s ? -v : v;
}
// host: RNE encode with saturation to +-448
static uint8_t enc_e4m3(float x) {
  uint8_t best = 0;
  float bd = INFINITY;
  for (int b = 0; b < 256; ++b) {
    const float v = dec_e4m3((uint8_t)b);
    if (std::isnan(v)) continue;
    if ((b >> 7) != (std::signbit(x) ? 1 : 0)) continue;
    const float d = std::fabs(v - x);
    if (d < bd || (d == bd && ((b & 1) == 0))) { bd = d; best = (uint8_t)b; }
  }
  return best;
}

// lane l supplies A bytes a[l*32 .. +32), B bytes b[l*32 .. +32), scales sa[l], sb[l]
template <int OPA, int OPB>
__global__ void mfma_probe(const int* a, const int* b, const int* sa, const int* sb, float* d) {
  const int l = threadIdx.x;
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) { av[i] = a[l * 8 + i]; bv[i] = b[l * 8 + i]; }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, OPA, sa[l], OPB, sb[l]);
  for (int i = 0; i < 4; ++i) d[l * 4 + i] = c[i];
}

__global__ void cvt_probe(const float* x, uint8_t* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const int r = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
  y[2 * i] = (uint8_t)(r & 0xff);
  y[2 * i + 1] = (uint8_t)((r >> 8) & 0xff);
}

int main() {
  srand(1);
  // ---------------- MFMA layout: A[16][128], B[128][16] (B given as Bt[16][128])
  const uint8_t small[9] = {0xC8, 0xC4, 0xC0, 0xB8, 0x00, 0x38, 0x40, 0x44, 0x48};  // -4..4
  std::vector<uint8_t> A(16 * 128), Bt(16 * 128);
  for (auto& v : A) v = small[rand() % 9];
  for (auto& v : Bt) v = small[rand() % 9];
  // scales: per (row, kblock) for A and per (col, kblock) for B, E8M0 in {126,127,128}
  uint8_t SA[16][4], SB[16][4];
  for (int r = 0; r < 16; ++r)
    for (int q = 0; q < 4; ++q) { SA[r][q] = 126 + rand() % 3; SB[r][q] = 126 + rand() % 3; }
  // lane l: row l&15; scale of lane l = (row l&15, k-block l>>4)
  std::vector<uint8_t> la(64 * 32), lb(64 * 32);
  std::vector<int> sa(64), sb(64), sa_op(64), sb_op(64);
  for (int l = 0; l < 64; ++l) {
    for (int j = 0; j < 32; ++j) {
      // measured: bytes 0..15 hold k = 16g + j, bytes 16..31 hold k = 64 + 16g + (j - 16), g = l >> 4
      const int k = (j < 16) ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16);
      la[l * 32 + j] = A[(l & 15) * 128 + k];
      lb[l * 32 + j] = Bt[(l & 15) * 128 + k];
    }
    sa[l] = SA[l & 15][l >> 4];
    sb[l] = SB[l & 15][l >> 4];
    // opsel test: the scale byte in byte 2 (A) / byte 1 (B), garbage elsewhere
    sa_op[l] = (0xEE << 24) | (sa[l] << 16) | (0xEE << 8) | 0xEE;
    sb_op[l] = (0xEE << 24) | (0xEE << 16) | (sb[l] << 8) | 0xEE;
  }
  double ref[16][16];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double s = 0;
      for (int k = 0; k < 128; ++k)
        s += (double)dec_e4m3(A[i * 128 + k]) * std::ldexp(1.0, SA[i][k / 32] - 127) * dec_e4m3(Bt[j * 128 + k]) *
             std::ldexp(1.0, SB[j][k / 32] - 127);
      ref[i][j] = s;
    }
  int *da, *db, *dsa, *dsb;
  float* dd;
  CK(hipMalloc(&da, 64 * 32));
  CK(hipMalloc(&db, 64 * 32));
  CK(hipMalloc(&dsa, 256));
  CK(hipMalloc(&dsb, 256));
  CK(hipMalloc(&dd, 64 * 4 * 4));
  CK(hipMemcpy(da, la.data(), 64 * 32, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, lb.data(), 64 * 32, hipMemcpyHostToDevice));
  auto check = [&](const char* name) {
    float h[256];
    CK(hipMemcpy(h, dd, sizeof(h), hipMemcpyDeviceToHost));
    int bad = 0;
    double maxe = 0;
    for (int l = 0; l < 64; ++l)
      for (int q = 0; q < 4; ++q) {
        const int col = l & 15, row = (l >> 4) * 4 + q;  // C/D map of the 16x16 family
        const double e = std::fabs(h[l * 4 + q] - ref[row][col]);
        maxe = e > maxe ? e : maxe;
        if (e > 1e-3) ++bad;
      }
    printf("%-48s %s (bad %d / 256, max err %.3g)\n", name, bad ? "FAIL" : "PASS", bad, maxe);
  };
  {
    uint8_t SA1[16][4], SB1[16][4];
    memcpy(SA1, SA, sizeof(SA)); memcpy(SB1, SB, sizeof(SB));
    for (int r = 0; r < 16; ++r) for (int q = 0; q < 4; ++q) { SA[r][q] = 127; SB[r][q] = 127; }
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0;
        for (int k = 0; k < 128; ++k) s += (double)dec_e4m3(A[i * 128 + k]) * dec_e4m3(Bt[j * 128 + k]);
        ref[i][j] = s;
      }
    std::vector<int> one(64, 127);
    CK(hipMemcpy(dsa, one.data(), 256, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsb, one.data(), 256, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    CK(hipDeviceSynchronize());
    check("unit scales: layout row=l&15 k=32*(l>>4)+j");
    // pairing discovery: A row 0 one-hot at slot sa = g*32+j (lane 16g, byte j); B col 0 bit patterns
    int pairs[128];
    for (int sa_ = 0; sa_ < 128; ++sa_) {
      std::vector<uint8_t> pa(64 * 32, 0), pb(64 * 32, 0);
      pa[(16 * (sa_ >> 5)) * 32 + (sa_ & 31)] = 0x38;
      CK(hipMemcpy(da, pa.data(), 64 * 32, hipMemcpyHostToDevice));
      int code = 0;
      for (int bit = 0; bit < 7; ++bit) {
        for (int sb_ = 0; sb_ < 128; ++sb_) pb[(16 * (sb_ >> 5)) * 32 + (sb_ & 31)] = ((sb_ >> bit) & 1) ? 0x38 : 0;
        CK(hipMemcpy(db, pb.data(), 64 * 32, hipMemcpyHostToDevice));
        hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
        float h[256];
        CK(hipMemcpy(h, dd, sizeof(h), hipMemcpyDeviceToHost));
        if (h[0] > 0.5f) code |= 1 << bit;  // lane 0 reg 0 = D[0][0]
      }
      pairs[sa_] = code;
    }
    int ident = 1;
    for (int i = 0; i < 128; ++i) ident &= pairs[i] == i;
    printf("A-slot -> B-slot pairing identity: %s\n", ident ? "yes" : "no");
    if (!ident) { for (int i = 0; i < 128; ++i) printf("%d ", pairs[i]); printf("\n"); }
    // scale discovery: unit data (all ones in A row 0 / B col 0 slots), one lane's scale = 128 (x2)
    {
      std::vector<uint8_t> pa(64 * 32, 0), pb(64 * 32, 0);
      for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) { pa[l * 32 + j] = 0x38; pb[l * 32 + j] = 0x38; }
      CK(hipMemcpy(da, pa.data(), 64 * 32, hipMemcpyHostToDevice));
      CK(hipMemcpy(db, pb.data(), 64 * 32, hipMemcpyHostToDevice));
      CK(hipMemcpy(dsb, one.data(), 256, hipMemcpyHostToDevice));
      for (int L = 0; L < 64; L += 5) {
        std::vector<int> sc(64, 127);
        sc[L] = 128;
        CK(hipMemcpy(dsa, sc.data(), 256, hipMemcpyHostToDevice));
        hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
        float h[256];
        CK(hipMemcpy(h, dd, sizeof(h), hipMemcpyDeviceToHost));
        printf("A scale lane %2d x2 -> D rows sum:", L);
        for (int row = 0; row < 16; ++row) {
          const int l = (row >> 2) * 16, q = row & 3;  // D[row][0] = lane (row>>2)*16 + 0, reg row&3
          printf(" %g", h[l * 4 + q]);
        }
        printf("\n");
      }
    }
    // k-block of each scale lane: A one-hot at (row 0, slot g*32), B ones; lane 16q scale x2
    {
      std::vector<uint8_t> pb(64 * 32, 0x38);
      CK(hipMemcpy(db, pb.data(), 64 * 32, hipMemcpyHostToDevice));
      for (int side = 0; side < 2; ++side)
        for (int q = 0; q < 4; ++q) {
          printf("%s scale lane %2d x2 -> D[0][0] per data block g:", side ? "B" : "A", 16 * q);
          for (int g = 0; g < 4; ++g) {
            std::vector<uint8_t> pa(64 * 32, 0);
            pa[(16 * g) * 32] = 0x38;
            CK(hipMemcpy(side ? db : da, pa.data(), 64 * 32, hipMemcpyHostToDevice));
            CK(hipMemcpy(side ? da : db, pb.data(), 64 * 32, hipMemcpyHostToDevice));
            std::vector<int> sc(64, 127);
            sc[16 * q] = 128;
            CK(hipMemcpy(side ? dsb : dsa, sc.data(), 256, hipMemcpyHostToDevice));
            CK(hipMemcpy(side ? dsa : dsb, one.data(), 256, hipMemcpyHostToDevice));
            hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
            float h[256];
            CK(hipMemcpy(h, dd, sizeof(h), hipMemcpyDeviceToHost));
            printf(" %g", h[0]);
          }
          printf("\n");
        }
    }
    CK(hipMemcpy(da, la.data(), 64 * 32, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, lb.data(), 64 * 32, hipMemcpyHostToDevice));
    memcpy(SA, SA1, sizeof(SA)); memcpy(SB, SB1, sizeof(SB));
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        double s = 0;
        for (int k = 0; k < 128; ++k)
          s += (double)dec_e4m3(A[i * 128 + k]) * std::ldexp(1.0, SA[i][k / 32] - 127) * dec_e4m3(Bt[j * 128 + k]) *
               std::ldexp(1.0, SB[j][k / 32] - 127);
        ref[i][j] = s;
      }
  }
  CK(hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  CK(hipDeviceSynchronize());
  check("layout k=16g+j | 64+16g+j-16, scale lane = (row, k/32)");
  CK(hipMemcpy(dsa, sa_op.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb_op.data(), 256, hipMemcpyHostToDevice));
  hipLaunchKernelGGL((mfma_probe<2, 1>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  CK(hipDeviceSynchronize());
  check("opsel: A scale byte 2, B scale byte 1");

  // ---------------- numerics of one scaled MFMA on random e4m3 data: error vs exact, / sum|a b|
  {
    double worst = 0, worst_abs_rel = 0;
    for (int trial = 0; trial < 200; ++trial) {
      std::vector<uint8_t> ra(64 * 32), rb(64 * 32);
      for (auto& v : ra) { do { v = rand() & 0xff; } while ((v & 0x7f) == 0x7f); }
      for (auto& v : rb) { do { v = rand() & 0xff; } while ((v & 0x7f) == 0x7f); }
      std::vector<int> s1(64), s2(64);
      for (int l = 0; l < 64; ++l) { s1[l] = 120 + rand() % 10; s2[l] = 120 + rand() % 10; }
      CK(hipMemcpy(da, ra.data(), 64 * 32, hipMemcpyHostToDevice));
      CK(hipMemcpy(db, rb.data(), 64 * 32, hipMemcpyHostToDevice));
      CK(hipMemcpy(dsa, s1.data(), 256, hipMemcpyHostToDevice));
      CK(hipMemcpy(dsb, s2.data(), 256, hipMemcpyHostToDevice));
      hipLaunchKernelGGL((mfma_probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
      float h[256];
      CK(hipMemcpy(h, dd, sizeof(h), hipMemcpyDeviceToHost));
      for (int l = 0; l < 64; ++l)
        for (int q = 0; q < 4; ++q) {
          const int col = l & 15, row = (l >> 4) * 4 + q;
          double ex = 0, ab = 0;
          for (int g = 0; g < 4; ++g)
            for (int j = 0; j < 32; ++j) {
              const int lane_a = row + 16 * g, lane_b = col + 16 * g;
              const int k = (j < 16) ? 16 * g + j : 64 + 16 * g + (j - 16);
              const int blk = k / 32;
              const double av = dec_e4m3(ra[lane_a * 32 + j]) * std::ldexp(1.0, s1[row + 16 * blk] - 127);
              const double bv = dec_e4m3(rb[lane_b * 32 + j]) * std::ldexp(1.0, s2[col + 16 * blk] - 127);
              ex += av * bv;
              ab += std::fabs(av * bv);
            }
          const double e = std::fabs(h[l * 4 + q] - ex);
          worst = std::fmax(worst, e / ab);
          worst_abs_rel = std::fmax(worst_abs_rel, e / std::fmax(std::fabs(ex), 1e-30));
        }
    }
    printf("scaled MFMA numerics: max |hw - exact| / sum|ab| = %.3g (2^%.1f); max rel to |exact| = %.3g\n", worst,
           std::log2(worst), worst_abs_rel);
  }
  // ---------------- conversion: every bf16-representable magnitude class + ties + saturation
  std::vector<float> xs;
  for (int i = 0; i < 200000; ++i) {
    const float m = (float)rand() / RAND_MAX * 2.f - 1.f;
    xs.push_back(std::ldexp(m, rand() % 24 - 14));
  }
  for (int b = 0; b < 256; ++b) {  // exact codes, midpoints between neighbours
    const float v = dec_e4m3((uint8_t)b);
    if (std::isnan(v)) continue;
    xs.push_back(v);
    const float w = dec_e4m3((uint8_t)(b + 1 < 256 ? b + 1 : b));
    if (!std::isnan(w) && ((b & 0x7f) != 0x7e)) xs.push_back(0.5f * (v + w));
  }
  xs.push_back(448.f); xs.push_back(460.f); xs.push_back(480.f); xs.push_back(-470.f); xs.push_back(1e-9f);
  if (xs.size() % 2) xs.push_back(0.f);
  const int n = (int)xs.size();
  float* dx;
  uint8_t* dy;
  CK(hipMalloc(&dx, n * 4));
  CK(hipMalloc(&dy, n));
  CK(hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(cvt_probe, dim3((n / 2 + 255) / 256), dim3(256), 0, 0, dx, dy, n);
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> y(n);
  CK(hipMemcpy(y.data(), dy, n, hipMemcpyDeviceToHost));
  int bad = 0, bad_sat = 0;
  for (int i = 0; i < n; ++i) {
    const float x = xs[i];
    const uint8_t r = enc_e4m3(std::fmax(-448.f, std::fmin(448.f, x)));
    if (y[i] != r) {
      if (std::fabs(x) > 448.f) {
        if (bad_sat < 4) printf("  sat: x=%g hw=0x%02x ref=0x%02x\n", x, y[i], r);
        ++bad_sat;
      } else {
        if (bad < 8) printf("  x=%.9g hw=0x%02x (%g) ref=0x%02x (%g)\n", x, y[i], dec_e4m3(y[i]), r, dec_e4m3(r));
        ++bad;
      }
    }
  }
  printf("cvt_pk_fp8_f32 vs RNE e4m3fn (|x|<=448): %s (%d / %d mismatches); |x|>448: %d differ from saturation\n",
         bad ? "FAIL" : "PASS", bad, n, bad_sat);
  return 0;
}
