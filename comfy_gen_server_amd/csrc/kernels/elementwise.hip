// Small fused element-wise kernels of the sampling loop and the UNet (K12, K13, K16, K08-standalone).
// All memory-bound: 16-byte vectors, grid-stride loops capped at 8192 blocks.
#include "common.h"

static inline int ew_blocks(long long n_vec) {
  long long b = (n_vec + 255) / 256;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

// ---------------------------------------------------------------- SiLU
template <int DT>
__global__ void silu_kernel(const u16* __restrict__ x, u16* __restrict__ y, long long n) {
  long long nv = n >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x) {
    s16x8 v = reinterpret_cast<const s16x8*>(x)[i];
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)cvt_out<DT>(silu_f(cvt_in<DT>((u16)v[j])));
    reinterpret_cast<s16x8*>(y)[i] = o;
  }
  long long tail = nv << 3;
  long long t = tail + blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && t < n) y[t] = cvt_out<DT>(silu_f(cvt_in<DT>(x[t])));
}

CGS_EXPORT int cgs_silu(const void* x, void* y, long long n, int dtype, hipStream_t stream) {
  int blocks = ew_blocks(n / 8 + 1);
  if (dtype == CGS_BF16) silu_kernel<CGS_BF16><<<blocks, 256, 0, stream>>>((const u16*)x, (u16*)y, n);
  else if (dtype == CGS_F16) silu_kernel<CGS_F16><<<blocks, 256, 0, stream>>>((const u16*)x, (u16*)y, n);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- CFG combine (fp32)
__global__ void cfg_combine_kernel(const float* __restrict__ c, const float* __restrict__ u, float* __restrict__ o,
                                   long long n, float s) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float uu = u[i];
    o[i] = uu + (c[i] - uu) * s;
  }
}

CGS_EXPORT int cgs_cfg_combine(const void* cond, const void* uncond, void* out, long long n, float scale, int dtype,
                               hipStream_t stream) {
  if (dtype != CGS_F32) return (int)hipErrorInvalidValue;
  cfg_combine_kernel<<<ew_blocks(n), 256, 0, stream>>>((const float*)cond, (const float*)uncond, (float*)out, n, scale);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- Euler / Euler-ancestral step (fp32, in place)
//  d = (x - den) / sigma ; x += d * (sigma_down - sigma) ; x += noise * sigma_up
__global__ void euler_step_kernel(float* __restrict__ x, const float* __restrict__ den, const float* __restrict__ noise,
                                  long long n, float inv_sigma, float dt, float s_up) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float xv = x[i];
    float d = (xv - den[i]) * inv_sigma;
    xv = fmaf(d, dt, xv);
    if (noise) xv = fmaf(noise[i], s_up, xv);
    x[i] = xv;
  }
}

CGS_EXPORT int cgs_euler_step(void* x, const void* denoised, const void* noise, long long n, float sigma,
                              float sigma_down, float sigma_up, hipStream_t stream) {
  euler_step_kernel<<<ew_blocks(n), 256, 0, stream>>>((float*)x, (const float*)denoised, (const float*)noise, n,
                                                     1.0f / sigma, sigma_down - sigma, sigma_up);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- timestep embedding [N, dim] fp32
__global__ void timestep_emb_kernel(const float* __restrict__ t, float* __restrict__ out, int n, int dim,
                                    float log_max_period, int flip) {
  int half = dim / 2;
  int total = n * half;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    int r = i / half, k = i % half;
    float freq = __expf(-log_max_period * (float)k / (float)half);
    float a = t[r] * freq;
    float c = cosf(a), s = sinf(a);
    out[(size_t)r * dim + k] = flip ? c : s;
    out[(size_t)r * dim + half + k] = flip ? s : c;
  }
}

CGS_EXPORT int cgs_timestep_embedding(const void* t, void* out, int n, int dim, float max_period, int flip,
                                      hipStream_t stream) {
  int total = n * (dim / 2);
  timestep_emb_kernel<<<(total + 255) / 256, 256, 0, stream>>>((const float*)t, (float*)out, n, dim,
                                                             logf(max_period), flip);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- nearest upsample x2, NHWC
// IDX = unsigned (32-bit index math, the common case) or unsigned long long (outputs >= 2^32 chunks):
// 64-bit integer division is emulated and dominated this memory-bound kernel.
template <class IDX>
__global__ void upsample2x_nhwc_kernel(const s16x8* __restrict__ x, s16x8* __restrict__ y, int N, int H, int W,
                                       int C8) {
  const IDX total = (IDX)N * 2 * H * 2 * W * C8;
  for (IDX i = (IDX)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (IDX)gridDim.x * blockDim.x) {
    const int c = (int)(i % (IDX)C8);
    const IDX p = i / (IDX)C8;
    const int ox = (int)(p % (IDX)(2 * W));
    const IDX q = p / (IDX)(2 * W);
    const int oy = (int)(q % (IDX)(2 * H));
    const int n = (int)(q / (IDX)(2 * H));
    y[i] = x[(((IDX)n * H + (oy >> 1)) * W + (ox >> 1)) * C8 + c];
  }
}

CGS_EXPORT int cgs_upsample_nearest2x_nhwc(const void* x, void* y, int N, int H, int W, int C, int dtype,
                                           hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  long long total = (long long)N * 4 * H * W * (C / 8);
  if (total < (1LL << 32) - (1LL << 24))
    upsample2x_nhwc_kernel<unsigned><<<ew_blocks(total), 256, 0, stream>>>((const s16x8*)x, (s16x8*)y, N, H, W, C / 8);
  else
    upsample2x_nhwc_kernel<unsigned long long><<<ew_blocks(total), 256, 0, stream>>>((const s16x8*)x, (s16x8*)y, N, H,
                                                                                     W, C / 8);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- standalone GEGLU: out = a * gelu(g)
// x rows: [a (N) | g (N)], out rows: N
__global__ void geglu_kernel(const u16* __restrict__ x, u16* __restrict__ out, int M, int N) {
  long long total = (long long)M * (N / 8);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    long long r = i / (N / 8);
    int c = (int)(i % (N / 8)) * 8;
    s16x8 a = *reinterpret_cast<const s16x8*>(x + r * 2 * N + c);
    s16x8 g = *reinterpret_cast<const s16x8*>(x + r * 2 * N + N + c);
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(bf2f((u16)a[j]) * gelu_sig(bf2f((u16)g[j])));
    *reinterpret_cast<s16x8*>(out + r * N + c) = o;
  }
}

CGS_EXPORT int cgs_geglu(const void* x, void* out, int M, int N, int dtype, hipStream_t stream) {
  if (dtype != CGS_BF16 || N % 8) return (int)hipErrorInvalidValue;
  geglu_kernel<<<ew_blocks((long long)M * N / 8), 256, 0, stream>>>((const u16*)x, (u16*)out, M, N);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- depthwise conv, NHWC, stride 1 (K11)
// y[n,h,w,c] = b[c] + sum_{i,j<k} x[n, h+i-p, w+j-p, c] * wt[(i*k+j)*C + c]; p = k/2.
// Out-of-range taps are zero ("zeros" padding) or clamped to the border (replicate=1, Stage A).
// One thread per 8 channels of one output pixel; neighbouring pixels of a wave share the same rows,
// so the k*k tap re-reads hit L1/L2 — the kernel streams x and y once from HBM.
template <int DT, int KF>   // KF: compile-time kernel size (3 / 7: unrolled taps), 0 = runtime k
__global__ __launch_bounds__(256) void dwconv_nhwc_kernel(const s16x8* __restrict__ x, const u16* __restrict__ wt,
                                                          const u16* __restrict__ b, s16x8* __restrict__ y, int N,
                                                          int H, int W, int C8, int kr, int replicate) {
  // 32-bit index math (the launcher checks N*H*W*C8 < 2^31): the 64-bit divisions / modulos of the
  // first version made this memory-bound kernel ALU-bound (~10x its streaming time at Cascade sizes)
  const unsigned total = (unsigned)N * H * W * C8;
  const int k = KF ? KF : kr;
  const int p = k >> 1;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % (unsigned)C8);
    const unsigned pix = i / (unsigned)C8;
    const int wo = (int)(pix % (unsigned)W);
    const unsigned t = pix / (unsigned)W;
    const int ho = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    float acc[8];
    if (b) {
      s16x8 bv = reinterpret_cast<const s16x8*>(b)[c8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = cvt_in<DT>((u16)bv[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    }
#pragma unroll
    for (int di = 0; di < (KF ? KF : 15); ++di) {
      if (!KF && di >= k) break;
      int hi = ho + di - p;
      if (replicate) hi = min(max(hi, 0), H - 1);
      else if (hi < 0 || hi >= H) continue;
#pragma unroll
      for (int dj = 0; dj < (KF ? KF : 15); ++dj) {
        if (!KF && dj >= k) break;
        int wi = wo + dj - p;
        if (replicate) wi = min(max(wi, 0), W - 1);
        else if (wi < 0 || wi >= W) continue;
        s16x8 xv = x[(((unsigned)n * H + hi) * W + wi) * (unsigned)C8 + c8];
        s16x8 wv = reinterpret_cast<const s16x8*>(wt + (size_t)(di * k + dj) * C8 * 8)[c8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += cvt_in<DT>((u16)xv[j]) * cvt_in<DT>((u16)wv[j]);
      }
    }
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)cvt_out<DT>(acc[j]);
    y[i] = o;
  }
}

// 3x3 form with PX = 2 or 4 output pixels along W per thread (W % PX == 0, zero padding): each of the three
// input rows is read once as PX + 2 chunks and reused by the three column taps of all four outputs (9 x 16-B
// loads of x and 9 of the weights per FOUR outputs instead of per one): the per-output kernel was bound by
// its L1 / L2 re-reads (~3x its HBM streaming time at Stable Cascade's 24 x 24 x 2048 maps).
template <int DT, int PX>
__global__ __launch_bounds__(256) void dwconv3_px_kernel(const s16x8* __restrict__ x, const u16* __restrict__ wt,
                                                          const u16* __restrict__ b, s16x8* __restrict__ y, int N,
                                                          int H, int W, int C8) {
  const int Wq = W / PX;
  const unsigned total = (unsigned)N * H * Wq * C8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % (unsigned)C8);
    const unsigned pq = i / (unsigned)C8;
    const int wq = (int)(pq % (unsigned)Wq);
    const unsigned t = pq / (unsigned)Wq;
    const int ho = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    const int w0 = wq * PX;
    float acc[PX][8];
    {
      float bb[8];
      if (b) {
        const s16x8 bv = reinterpret_cast<const s16x8*>(b)[c8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = cvt_in<DT>((u16)bv[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = 0.f;
      }
#pragma unroll
      for (int q = 0; q < PX; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[q][j] = bb[j];
    }
#pragma unroll
    for (int di = 0; di < 3; ++di) {
      const int hi = ho + di - 1;
      if (hi < 0 || hi >= H) continue;
      const unsigned rowb = ((unsigned)n * H + hi) * W;
      s16x8 xr[PX + 2];
#pragma unroll
      for (int q = 0; q < PX + 2; ++q) {
        const int wi = w0 + q - 1;
        xr[q] = (wi >= 0 && wi < W) ? x[(rowb + wi) * (unsigned)C8 + c8] : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int dj = 0; dj < 3; ++dj) {
        const s16x8 wv = reinterpret_cast<const s16x8*>(wt + (size_t)(di * 3 + dj) * C8 * 8)[c8];
        float wf[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) wf[j] = cvt_in<DT>((u16)wv[j]);
#pragma unroll
        for (int q = 0; q < PX; ++q)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[q][j] = __builtin_fmaf(cvt_in<DT>((u16)xr[q + dj][j]), wf[j], acc[q][j]);
      }
    }
    const unsigned ob = (((unsigned)n * H + ho) * W + w0) * (unsigned)C8 + c8;
#pragma unroll
    for (int q = 0; q < PX; ++q) {
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)cvt_out<DT>(acc[q][j]);
      y[ob + (unsigned)q * C8] = o;
    }
  }
}

static int g_dw_px = 4;
CGS_EXPORT void cgs_dwconv_set_px(int p) { g_dw_px = p == 1 ? 1 : p == 2 ? 2 : 4; }

CGS_EXPORT int cgs_dwconv_nhwc(const void* x, const void* wt, const void* b, void* y, int N, int H, int W, int C,
                               int k, int replicate, int dtype, hipStream_t stream) {
  if (C % 8 || (k & 1) == 0 || k > 15) return (int)hipErrorInvalidValue;
  long long total = (long long)N * H * W * (C / 8);
  if (total >= (1LL << 31)) return (int)hipErrorInvalidValue;
#define CGS_DW(DTV, KV)                                                                                           \
  dwconv_nhwc_kernel<DTV, KV><<<ew_blocks(total), 256, 0, stream>>>((const s16x8*)x, (const u16*)wt, (const u16*)b, \
                                                                    (s16x8*)y, N, H, W, C / 8, k, replicate)
  // Pixels per thread: 4 (measured best or tied from 1 x 24 x 24 x 2048 to 8 x 128 x 128 x 320: 1.4-2x the
  // one-pixel kernel on the large maps), 2 when W % 4 != 0; cgs_dwconv_set_px(1 / 2) overrides (A/B switch).
  int px = g_dw_px;
  if (W % px) px = (W % 2) ? 1 : 2;
  if (k == 3 && !replicate && px > 1) {
    const long long tq = total / px;
#define CGS_DWP(D, P)                                                                                           \
  dwconv3_px_kernel<D, P><<<ew_blocks(tq), 256, 0, stream>>>((const s16x8*)x, (const u16*)wt, (const u16*)b,       \
                                                            (s16x8*)y, N, H, W, C / 8)
    if (dtype == CGS_BF16) {
      if (px == 4) CGS_DWP(CGS_BF16, 4); else CGS_DWP(CGS_BF16, 2);
    } else {
      if (px == 4) CGS_DWP(CGS_F16, 4); else CGS_DWP(CGS_F16, 2);
    }
#undef CGS_DWP
    return (int)hipGetLastError();
  }
  if (dtype == CGS_BF16) {
    if (k == 3) CGS_DW(CGS_BF16, 3); else if (k == 7) CGS_DW(CGS_BF16, 7); else CGS_DW(CGS_BF16, 0);
  } else {
    if (k == 3) CGS_DW(CGS_F16, 3); else if (k == 7) CGS_DW(CGS_F16, 7); else CGS_DW(CGS_F16, 0);
  }
#undef CGS_DW
  return (int)hipGetLastError();
}
