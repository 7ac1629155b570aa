// fp32-I/O hot ops for --force-fp32 / --fp32-vae (the reference's default VAE dtype on ROCm is fp32,
// comfy/model_management.py:169-197; flags comfy/cli_args.py:55/:66): GEMM, implicit-GEMM conv,
// GroupNorm and LayerNorm on fp32 tensors, so an fp32 run stays on hand-written kernels instead of
// going to the vendor libraries.
//
// Matrix work runs on the f32-input MFMA (v_mfma_f32_16x16x4_f32): exact fp32 products, one rounding
// per fmaf step -- the numerics of an fp32 GEMM, at the f32 peak (157 TF, 1/16 of bf16). Block tile
// 128 x 128 x 32, four waves of 64 x 64 (16 independent 16x16 accumulators each, > the 40-cycle
// dependent latency). The k index inside each 16-deep slice is permuted so that a lane's four k-steps
// are four CONSECUTIVE floats: lane l at k-step s uses k = 4 * (l >> 4) + s for both operands (a dot
// product is order-free over k as long as A and B agree), so one ds_read_b128 feeds four MFMAs. LDS rows are
// 36 floats (144 B): the 16 rows a quarter-wave reads hit 16 distinct 4-bank groups. Register-prefetch
// double buffering: the next tile's global loads are in flight during the current tile's MFMAs, one
// barrier per tile.
#include "common.h"

namespace {
constexpr int FT_M = 128, FT_N = 128, FT_K = 32, FT_LD = FT_K + 4;
constexpr int FT_CPR = FT_K / 4;               // float4 chunks per tile row
constexpr int FT_RS = 256 / FT_CPR;            // row step between a thread's rows
constexpr int FT_RPT = FT_M / FT_RS;           // rows per thread (A and NT B)
constexpr int FT_BPT = FT_K * (FT_N / 4) / 256; // [K, N] B chunks per thread

struct F32Gemm {
  const float* A;    // dense: [M, K] rows of stride lda;  conv: NHWC input x (first C1 channels)
  const float* A2;   // conv: second input (channels C1..C1+C2), or null
  const float* B;    // [N, K] (stride ldb) or, with BKN, [K, N]
  float* C;
  const float* bias;
  const float* R;
  long long lda, ldb, ldc, ldr;
  long long sab, sbb, scb;   // batch strides (grid.y)
  int M, N, K, epi;
  float alpha;
  int tiles_n;
  // conv geometry (KIND 1)
  int H, W, C1, C2, Ho, Wo, kh, kw, stride, pad, up2;
};

constexpr int F_BIAS = 1, F_RES = 2, F_GELU = 4;

// 4 consecutive k of one row starting at k (k % 4 == 0, 16-B aligned); the elements at or past K read
// as zero (a K % 4 != 0 tail, e.g. attention probabilities over 77 keys)
__device__ __forceinline__ float4 ld_k4(const float* p, int k, int K) {
  if (k + 4 <= K) return *reinterpret_cast<const float4*>(p);
  float4 v = float4{0.f, 0.f, 0.f, 0.f};
  if (k < K) v.x = p[0];
  if (k + 1 < K) v.y = p[1];
  if (k + 2 < K) v.z = p[2];
  return v;
}

template <int KIND, bool BKN>
__global__ __launch_bounds__(256) void f32_gemm_kernel(const F32Gemm g) {
  __shared__ __attribute__((aligned(16))) float As[2][FT_M * FT_LD];
  __shared__ __attribute__((aligned(16))) float Bs[2][FT_N * FT_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = blockIdx.x;
  const int m0 = (tile / g.tiles_n) * FT_M, n0 = (tile % g.tiles_n) * FT_N;
  const long long bz = blockIdx.y;
  const float* Ab = g.A + bz * g.sab;
  const float* Bb = g.B + bz * g.sbb;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;

  // this thread's A rows / B rows (NT) and k-chunk of a tile
  const int r0 = tid / FT_CPR, kc = (tid % FT_CPR) * 4;
  int an[FT_RPT], ay[FT_RPT], ax[FT_RPT];
  bool am[FT_RPT];
#pragma unroll
  for (int i = 0; i < FT_RPT; ++i) {
    const int m = m0 + r0 + FT_RS * i;
    am[i] = m < g.M;
    if constexpr (KIND == 1) {
      const int mm = am[i] ? m : 0;
      const int hw = g.Ho * g.Wo;
      an[i] = mm / hw;
      const int rem = mm - an[i] * hw;
      const int oy = rem / g.Wo;
      ay[i] = oy * g.stride - g.pad;
      ax[i] = (rem - oy * g.Wo) * g.stride - g.pad;
    } else {
      an[i] = ay[i] = ax[i] = 0;
    }
  }
  const int Cin = g.C1 + g.C2;
  const int HH = g.up2 ? 2 * g.H : g.H, WW = g.up2 ? 2 * g.W : g.W;

  auto load_a = [&](int k0, float4 (&ra)[FT_RPT]) {
    const int k = k0 + kc;
    if constexpr (KIND == 0) {
#pragma unroll
      for (int i = 0; i < FT_RPT; ++i)
        ra[i] = am[i] ? ld_k4(Ab + (long long)(m0 + r0 + FT_RS * i) * g.lda + k, k, g.K) : float4{0.f, 0.f, 0.f, 0.f};
    } else {
      const int tap = k / Cin, ci = k - tap * Cin;
      const int ky = tap / g.kw, kx = tap - ky * g.kw;
#pragma unroll
      for (int i = 0; i < FT_RPT; ++i) {
        int iy = ay[i] + ky, ix = ax[i] + kx;
        const bool ok = am[i] && k < g.K && iy >= 0 && iy < HH && ix >= 0 && ix < WW;
        if (g.up2) { iy >>= 1; ix >>= 1; }
        float4 v = float4{0.f, 0.f, 0.f, 0.f};
        if (ok) {
          const long long pix = ((long long)an[i] * g.H + iy) * g.W + ix;
          v = ci < g.C1 ? *reinterpret_cast<const float4*>(g.A + pix * g.C1 + ci)
                        : *reinterpret_cast<const float4*>(g.A2 + pix * g.C2 + (ci - g.C1));
        }
        ra[i] = v;
      }
    }
  };
  auto load_b = [&](int k0, float4 (&rb)[FT_RPT]) {
    if constexpr (!BKN) {
      const int k = k0 + kc;
#pragma unroll
      for (int i = 0; i < FT_RPT; ++i) {
        const int n = n0 + r0 + FT_RS * i;
        rb[i] = n < g.N ? ld_k4(Bb + (long long)n * g.ldb + k, k, g.K) : float4{0.f, 0.f, 0.f, 0.f};
      }
    } else {   // [K, N]: a float4 of 4 consecutive n at one k
#pragma unroll
      for (int i = 0; i < FT_BPT; ++i) {
        const int e = tid + 256 * i;
        const int k = k0 + (e >> 5), n = n0 + (e & 31) * 4;
        rb[i] = (k < g.K && n < g.N) ? *reinterpret_cast<const float4*>(Bb + (long long)k * g.ldb + n)
                                     : float4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto store = [&](int buf, const float4 (&ra)[FT_RPT], const float4 (&rb)[FT_RPT]) {
#pragma unroll
    for (int i = 0; i < FT_RPT; ++i)
      *reinterpret_cast<float4*>(&As[buf][(r0 + FT_RS * i) * FT_LD + kc]) = ra[i];
    if constexpr (!BKN) {
#pragma unroll
      for (int i = 0; i < FT_RPT; ++i)
        *reinterpret_cast<float4*>(&Bs[buf][(r0 + FT_RS * i) * FT_LD + kc]) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < FT_BPT; ++i) {
        const int e = tid + 256 * i;
        const int kk = e >> 5, nn = (e & 31) * 4;
        Bs[buf][(nn + 0) * FT_LD + kk] = rb[i].x;
        Bs[buf][(nn + 1) * FT_LD + kk] = rb[i].y;
        Bs[buf][(nn + 2) * FT_LD + kk] = rb[i].z;
        Bs[buf][(nn + 3) * FT_LD + kk] = rb[i].w;
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + FT_K - 1) / FT_K;
  static_assert(FT_BPT <= FT_RPT, "rb holds the [K, N] chunks too");
  float4 ra[FT_RPT], rb[FT_RPT];
  load_a(0, ra);
  load_b(0, rb);
  store(0, ra, rb);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_a((kt + 1) * FT_K, ra);
      load_b((kt + 1) * FT_K, rb);
    }
#pragma unroll
    for (int h = 0; h < FT_K / 16; ++h) {      // 16-deep slices: one ds_read_b128 per operand fragment
      float4 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const float4*>(&As[cur][(wm + 16 * i + fr) * FT_LD + 16 * h + fk]);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bf[j] = *reinterpret_cast<const float4*>(&Bs[cur][(wn + 16 * j + fr) * FT_LD + 16 * h + fk]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    }
    if (more) store(cur ^ 1, ra, rb);
    __syncthreads();
  }

  float* Cb = g.C + bz * g.scb;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn + 16 * j + fr;
    if (n >= g.N) continue;
    const float bv = (g.epi & F_BIAS) ? g.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + (lane >> 4) * 4 + r;
        if (m >= g.M) continue;
        float v = __builtin_fmaf(acc[i][j][r], g.alpha, bv);
        if (g.epi & F_GELU) v = gelu_f(v);
        if (g.epi & F_RES) v += g.R[(long long)m * g.ldr + n];
        Cb[(long long)m * g.ldc + n] = v;
      }
  }
}

int launch(const F32Gemm& g0, int kind, bool bkn, int batch, hipStream_t stream) {
  F32Gemm g = g0;
  g.tiles_n = (g.N + FT_N - 1) / FT_N;
  const long long tiles = (long long)g.tiles_n * ((g.M + FT_M - 1) / FT_M);
  if (tiles > 0x7fffffffLL || batch > 65535) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)tiles, (unsigned)batch);
  if (kind == 1) f32_gemm_kernel<1, false><<<grid, 256, 0, stream>>>(g);
  else if (bkn) f32_gemm_kernel<0, true><<<grid, 256, 0, stream>>>(g);
  else f32_gemm_kernel<0, false><<<grid, 256, 0, stream>>>(g);
  return (int)hipGetLastError();
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
}  // namespace

// C[b] = act(alpha * A[b] . B[b]^T + bias) + R (fp32). A [M, K] (row stride lda), B [N, K] (ldb) or with
// bkn=1 B [K, N]; batch b offsets sab / sbb / scb (elements). epi: 1 bias, 2 residual (ldr), 4 GELU (erf).
// Row strides % 4 == 0 and 16-B aligned bases (float4 loads; any K); bkn needs N % 4 == 0.
CGS_EXPORT int cgs_gemm_f32(const float* A, const float* B, float* C, const float* bias, const float* R, int M,
                            int N, int K, long long lda, long long ldb, long long ldc, long long ldr, int epi,
                            float alpha, int bkn, int batch, long long sab, long long sbb, long long scb,
                            hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (K <= 0 || lda % 4 || ldb % 4 || sab % 4 || sbb % 4 || !al16(A) || !al16(B) || (bkn && N % 4))
    return (int)hipErrorInvalidValue;
  if (((epi & F_BIAS) && !bias) || ((epi & F_RES) && !R)) return (int)hipErrorInvalidValue;
  F32Gemm g{};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.R = R;
  g.lda = lda; g.ldb = ldb; g.ldc = ldc; g.ldr = ldr; g.sab = sab; g.sbb = sbb; g.scb = scb;
  g.M = M; g.N = N; g.K = K; g.epi = epi; g.alpha = alpha;
  return launch(g, 0, bkn != 0, batch, stream);
}

// NHWC fp32 convolution as an implicit GEMM on the same tile: x [N, H, W, C1] (+ x2 [N, H, W, C2]: the
// channel concat read in place), w [Cout, kh, kw, C1 + C2], y / R [N, Ho, Wo, Cout]; up2 reads x through a
// nearest-2x upsample (Ho, Wo computed by the caller on the upsampled size). (C1 + C2) % 4 == 0, C1 % 4 == 0.
CGS_EXPORT int cgs_conv_f32(const float* x, const float* x2, const float* w, const float* bias, const float* R,
                            float* y, int N, int H, int W, int C1, int C2, int Cout, int kh, int kw, int stride,
                            int pad, int up2, int Ho, int Wo, hipStream_t stream) {
  if (N <= 0 || Ho <= 0 || Wo <= 0 || Cout <= 0) return 0;
  const int Cin = C1 + C2;
  if (Cin <= 0 || C1 % 4 || C2 % 4 || (C2 && !x2) || !al16(x) || !al16(w) || (x2 && !al16(x2)) || stride <= 0)
    return (int)hipErrorInvalidValue;
  const long long M = (long long)N * Ho * Wo;
  if (M > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  F32Gemm g{};
  g.A = x; g.A2 = x2; g.B = w; g.C = y; g.bias = bias; g.R = R;
  g.ldb = (long long)kh * kw * Cin; g.ldc = Cout; g.ldr = Cout;
  g.M = (int)M; g.N = Cout; g.K = kh * kw * Cin;
  g.epi = (bias ? F_BIAS : 0) | (R ? F_RES : 0);
  g.alpha = 1.f;
  g.H = H; g.W = W; g.C1 = C1; g.C2 = C2; g.Ho = Ho; g.Wo = Wo; g.kh = kh; g.kw = kw; g.stride = stride;
  g.pad = pad; g.up2 = up2;
  return launch(g, 1, false, 1, stream);
}

// ---------------------------------------------------------------- GroupNorm (NHWC, fp32)
// Pass 1: per (image, pixel slice, channel) shifted sums -> (mean, M2) partials; pass 2: per (image,
// group) Chan combine of the partials -> per-channel (a, b) = (gamma * rstd, beta - mean * a); pass 3:
// y = x * a + b (+ SiLU). x may be the channel concat of x [.., C1] and x2 [.., C - C1]; pre_add [N, C]
// (a per-image channel bias) is added to x before the statistics.
namespace {
__device__ __forceinline__ float4 gn_ld(const float* x, const float* x2, const float* pa, int n, long long pix, int c,
                                        int C, int C1) {
  float4 v = c < C1 ? *reinterpret_cast<const float4*>(x + pix * C1 + c)
                    : *reinterpret_cast<const float4*>(x2 + pix * (C - C1) + (c - C1));
  if (pa) {
    const float4 p = *reinterpret_cast<const float4*>(pa + (long long)n * C + c);
    v.x += p.x; v.y += p.y; v.z += p.z; v.w += p.w;
  }
  return v;
}

__global__ __launch_bounds__(256) void gn_f32_partial_kernel(const float* __restrict__ x, const float* __restrict__ x2,
                                                             const float* __restrict__ pa, float* __restrict__ part,
                                                             int HW, int C, int C1, int S) {
  __shared__ float sh[256][9];
  const int n = blockIdx.y, s = blockIdx.x, tid = threadIdx.x;
  const int C4 = C >> 2;
  const long long p0 = (long long)HW * s / S, p1 = (long long)HW * (s + 1) / S;
  const int cnt = (int)(p1 - p0);
  const int P = C4 >= 256 ? 1 : 256 / C4;   // pixel lanes per channel chunk
  for (int cb = 0; cb < C4; cb += 256 / P) {
    const int c4 = cb + tid % (256 / P), pl = tid / (256 / P);
    const bool act = c4 < C4 && pl < P;
    float sum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f}, sft[4] = {0.f, 0.f, 0.f, 0.f};
    int k = 0;
    if (act && cnt > 0) {
      const float4 f = gn_ld(x, x2, pa, n, (long long)n * HW + p0, c4 * 4, C, C1);
      sft[0] = f.x; sft[1] = f.y; sft[2] = f.z; sft[3] = f.w;
      for (long long p = p0 + pl; p < p1; p += P, ++k) {
        const float4 v = gn_ld(x, x2, pa, n, (long long)n * HW + p, c4 * 4, C, C1);
        const float d[4] = {v.x - sft[0], v.y - sft[1], v.z - sft[2], v.w - sft[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) { sum[q] += d[q]; ssq[q] = __builtin_fmaf(d[q], d[q], ssq[q]); }
      }
    }
    // per-thread (count, mean, M2) for 4 channels, then Chan combine over the P pixel lanes in LDS
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float mu = k ? sum[q] / k : 0.f;
      sh[tid][2 * q] = sft[q] + mu;
      sh[tid][2 * q + 1] = k ? fmaxf(ssq[q] - sum[q] * mu, 0.f) : 0.f;
    }
    sh[tid][8] = (float)k;
    __syncthreads();
    if (act && pl == 0) {
      float nA = sh[tid][8], mA[4], MA[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) { mA[q] = sh[tid][2 * q]; MA[q] = sh[tid][2 * q + 1]; }
      for (int o = 1; o < P; ++o) {
        const int t2 = tid + o * (256 / P);
        const float nB = sh[t2][8];
        if (nB == 0.f) continue;
        const float nAB = nA + nB;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float d = sh[t2][2 * q] - mA[q];
          mA[q] += d * (nB / nAB);
          MA[q] += sh[t2][2 * q + 1] + d * d * (nA * nB / nAB);
        }
        nA = nAB;
      }
      float* o = part + (((long long)n * S + s) * C + c4 * 4) * 2;
#pragma unroll
      for (int q = 0; q < 4; ++q) { o[2 * q] = mA[q]; o[2 * q + 1] = MA[q]; }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void gn_f32_finalize_kernel(const float* __restrict__ part, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float* __restrict__ ab, int HW,
                                                              int C, int G, int S, float eps) {
  __shared__ float red[2][4];
  const int n = blockIdx.y, gi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cpg = C / G, c0 = gi * cpg, E = S * cpg;
  const float total = (float)HW * cpg;
  const float* P = part + (long long)n * S * C * 2;
  // pass a: grand mean = sum(count_s * mean) / total
  float s1 = 0.f;
  for (int e = tid; e < E; e += 256) {
    const int s = e / cpg, c = c0 + e - s * cpg;
    const float cnt = (float)((long long)HW * (s + 1) / S - (long long)HW * s / S);
    s1 += cnt * P[((long long)s * C + c) * 2];
  }
  s1 = wave_sum(s1);
  if (lane == 0) red[0][wave] = s1;
  __syncthreads();
  const float mean = (red[0][0] + red[0][1] + red[0][2] + red[0][3]) / total;
  // pass b: M2 = sum(M2_s + count_s * (mean_s - mean)^2)
  float s2 = 0.f;
  for (int e = tid; e < E; e += 256) {
    const int s = e / cpg, c = c0 + e - s * cpg;
    const float cnt = (float)((long long)HW * (s + 1) / S - (long long)HW * s / S);
    const float d = P[((long long)s * C + c) * 2] - mean;
    s2 += P[((long long)s * C + c) * 2 + 1] + cnt * d * d;
  }
  s2 = wave_sum(s2);
  if (lane == 0) red[1][wave] = s2;
  __syncthreads();
  const float var = (red[1][0] + red[1][1] + red[1][2] + red[1][3]) / total;
  const float rstd = rsqrtf(var + eps);
  for (int c = c0 + tid; c < c0 + cpg; c += 256) {
    const float a = (gamma ? gamma[c] : 1.f) * rstd;
    ab[((long long)n * C + c) * 2] = a;
    ab[((long long)n * C + c) * 2 + 1] = (beta ? beta[c] : 0.f) - mean * a;
  }
}

__global__ __launch_bounds__(256) void gn_f32_apply_kernel(const float* __restrict__ x, const float* __restrict__ x2,
                                                           const float* __restrict__ pa, const float* __restrict__ ab,
                                                           float* __restrict__ y, long long chunks, int HW, int C,
                                                           int C1, int silu) {
  const int C4 = C >> 2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < chunks; i += (long long)gridDim.x * 256) {
    const long long pix = i / C4;
    const int c = (int)(i - pix * C4) * 4;
    const int n = (int)(pix / HW);
    const float4 v = gn_ld(x, x2, pa, n, pix, c, C, C1);
    const float* q = ab + ((long long)n * C + c) * 2;
    float o[4] = {__builtin_fmaf(v.x, q[0], q[1]), __builtin_fmaf(v.y, q[2], q[3]), __builtin_fmaf(v.z, q[4], q[5]),
                  __builtin_fmaf(v.w, q[6], q[7])};
    if (silu) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = o[k] / (1.0f + expf(-o[k]));
    }
    reinterpret_cast<float4*>(y)[i] = float4{o[0], o[1], o[2], o[3]};
  }
}

int gn_slices(int N, int HW) {
  int S = (2048 + N - 1) / N;
  if (S > HW / 32) S = HW / 32;
  return S < 1 ? 1 : S;
}
}  // namespace

// Workspace floats for cgs_groupnorm_f32: partials [N, S, C, 2] + (a, b) [N, C, 2].
CGS_EXPORT long long cgs_groupnorm_f32_ws(int N, int HW, int C) {
  return (long long)N * gn_slices(N, HW) * C * 2 + (long long)N * C * 2;
}

CGS_EXPORT int cgs_groupnorm_f32(const float* x, const float* x2, int C1, float* y, const float* gamma,
                                 const float* beta, const float* pre_add, float* ws, int N, int HW, int C, int G,
                                 float eps, int silu, hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 4 || C1 % 4 || C1 > C || (C1 < C && !x2) || G <= 0 || C % G || !al16(x) || !al16(y) ||
      (x2 && !al16(x2)) || (pre_add && !al16(pre_add)) || N > 65535)
    return (int)hipErrorInvalidValue;
  const int S = gn_slices(N, HW);
  float* part = ws;
  float* ab = ws + (long long)N * S * C * 2;
  gn_f32_partial_kernel<<<dim3(S, N), 256, 0, stream>>>(x, x2, pre_add, part, HW, C, C1, S);
  gn_f32_finalize_kernel<<<dim3(G, N), 256, 0, stream>>>(part, gamma, beta, ab, HW, C, G, S, eps);
  const long long chunks = (long long)N * HW * (C / 4);
  const long long nb = (chunks + 255) / 256;
  gn_f32_apply_kernel<<<(unsigned)(nb > 16384 ? 16384 : nb), 256, 0, stream>>>(x, x2, pre_add, ab, y, chunks, HW, C,
                                                                               C1, silu);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- LayerNorm (fp32 rows)
// One wave per row: pass 1 the mean, pass 2 the centred sum of squares (exact two-pass variance; the
// second read of the row comes from L2), pass 3 the affine. C % 4 == 0.
namespace {
__global__ __launch_bounds__(256) void ln_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     long long rows, int C, float eps) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float4* xr = reinterpret_cast<const float4*>(x + row * C);
  const int C4 = C >> 2;
  float s = 0.f;
  for (int c = lane; c < C4; c += 64) {
    const float4 v = xr[c];
    s += (v.x + v.y) + (v.z + v.w);
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
  for (int c = lane; c < C4; c += 64) {
    const float4 v = xr[c];
    const float a = v.x - mean, bb = v.y - mean, cc = v.z - mean, d = v.w - mean;
    q += (a * a + bb * bb) + (cc * cc + d * d);
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  float4* yr = reinterpret_cast<float4*>(y + row * C);
  for (int c = lane; c < C4; c += 64) {
    const float4 v = xr[c];
    float o[4] = {(v.x - mean) * rstd, (v.y - mean) * rstd, (v.z - mean) * rstd, (v.w - mean) * rstd};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (w) o[k] *= w[4 * c + k];
      if (b) o[k] += b[4 * c + k];
    }
    yr[c] = float4{o[0], o[1], o[2], o[3]};
  }
}
}  // namespace

CGS_EXPORT int cgs_layernorm_f32(const float* x, float* y, const float* w, const float* b, long long rows, int C,
                                 float eps, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (C <= 0 || C % 4 || !al16(x) || !al16(y)) return (int)hipErrorInvalidValue;
  const long long blocks = (rows + 3) / 4;
  if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  ln_f32_kernel<<<(unsigned)blocks, 256, 0, stream>>>(x, y, w, b, rows, C, eps);
  return (int)hipGetLastError();
}
