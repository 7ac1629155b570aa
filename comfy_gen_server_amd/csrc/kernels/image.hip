// Image-space and small utility kernels (SURVEY §2.4 K25 resize, K28 GRN, K31 VQ codebook,
// K32 StyleGAN fused bias-act / upfirdn2d). All are bandwidth-bound: one thread per output
// element (grid-stride), fp32 accumulation, bf16 / fp16 / fp32 storage selected at run time.
#include "common.h"

namespace {

template <int DT>
__device__ __forceinline__ float ldv(const void* p, long long i) {
  if constexpr (DT == CGS_F32) return reinterpret_cast<const float*>(p)[i];
  else return cvt_in<DT>(reinterpret_cast<const u16*>(p)[i]);
}

template <int DT>
__device__ __forceinline__ void stv(void* p, long long i, float v) {
  if constexpr (DT == CGS_F32) reinterpret_cast<float*>(p)[i] = v;
  else reinterpret_cast<u16*>(p)[i] = cvt_out<DT>(v);
}

inline int grid_for(long long n, int block = 256) {
  long long g = (n + block - 1) / block;
  return (int)(g < 65535LL * 8 ? (g < 1 ? 1 : g) : 65535LL * 8);
}

#define CGS_DISPATCH_DT(dtype, KERNEL, ...)                                        \
  do {                                                                             \
    if ((dtype) == CGS_F32) KERNEL<CGS_F32> __VA_ARGS__;                           \
    else if ((dtype) == CGS_BF16) KERNEL<CGS_BF16> __VA_ARGS__;                    \
    else if ((dtype) == CGS_F16) KERNEL<CGS_F16> __VA_ARGS__;                      \
    else return (int)hipErrorInvalidValue;                                         \
  } while (0)

// ---------------------------------------------------------------------------------------------
// K32a: y = leaky_relu(x + bias[c], slope) * scale   (StyleGAN2 FusedLeakyReLU; c = (i / inner) % C)
// ---------------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) fused_bias_act_kernel(const void* x, const void* b, void* y, long long n,
                                                             int C, long long inner, float slope, float scale) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = ldv<DT>(x, i);
    if (b) v += ldv<DT>(b, (i / inner) % C);
    v = (v >= 0.f ? v : v * slope) * scale;
    stv<DT>(y, i, v);
  }
}

// ---------------------------------------------------------------------------------------------
// K32b: upfirdn2d on planar [NC, H, W]: zero-insert upsample, pad (negative = crop), FIR with the
// flipped kernel (true convolution), keep every down-th sample. Kernel taps staged in LDS.
// ---------------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) upfirdn2d_kernel(const void* x, const float* k, void* y, int NC, int H, int W,
                                                        int upx, int upy, int dnx, int dny, int px0, int py0,
                                                        int kh, int kw, int Ho, int Wo) {
  __shared__ float taps[32 * 32];
  for (int t = threadIdx.x; t < kh * kw; t += 256) taps[t] = k[t];
  __syncthreads();
  const long long total = (long long)NC * Ho * Wo;
  for (long long o = blockIdx.x * 256LL + threadIdx.x; o < total; o += (long long)gridDim.x * 256) {
    int ox = (int)(o % Wo);
    int oy = (int)((o / Wo) % Ho);
    long long nc = o / ((long long)Wo * Ho);
    const long long base = nc * H * W;
    float acc = 0.f;
    for (int i = 0; i < kh; ++i) {
      int uy = oy * dny + i - py0;
      if (uy < 0 || uy % upy) continue;
      int iy = uy / upy;
      if (iy >= H) continue;
      for (int j = 0; j < kw; ++j) {
        int ux = ox * dnx + j - px0;
        if (ux < 0 || ux % upx) continue;
        int ix = ux / upx;
        if (ix >= W) continue;
        acc += ldv<DT>(x, base + (long long)iy * W + ix) * taps[(kh - 1 - i) * kw + (kw - 1 - j)];
      }
    }
    stv<DT>(y, o, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// K25: resize planar [NC, H, W] -> [NC, Ho, Wo] with torch.nn.functional.interpolate semantics
// (size given, no scale_factor). mode 0 nearest, 1 nearest-exact, 2 bilinear, 3 bicubic (A=-0.75,
// clamped taps), 4 area (adaptive average pool).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float cubic1(float t, float A) { return ((A + 2.f) * t - (A + 3.f)) * t * t + 1.f; }
__device__ __forceinline__ float cubic2(float t, float A) { return ((A * t - 5.f * A) * t + 8.f * A) * t - 4.f * A; }

template <int DT>
__global__ void __launch_bounds__(256) resize_kernel(const void* x, void* y, int NC, int H, int W, int Ho, int Wo,
                                                     int mode, int align) {
  const long long total = (long long)NC * Ho * Wo;
  float sh, sw;
  if (align && mode >= 2 && mode <= 3) {
    sh = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
    sw = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  } else {
    sh = (float)H / (float)Ho;
    sw = (float)W / (float)Wo;
  }
  for (long long o = blockIdx.x * 256LL + threadIdx.x; o < total; o += (long long)gridDim.x * 256) {
    int ox = (int)(o % Wo);
    int oy = (int)((o / Wo) % Ho);
    long long base = (o / ((long long)Wo * Ho)) * H * W;
    float v;
    if (mode <= 1) {
      float off = mode == 1 ? 0.5f : 0.f;
      int iy = min((int)floorf((oy + off) * sh), H - 1);
      int ix = min((int)floorf((ox + off) * sw), W - 1);
      v = ldv<DT>(x, base + (long long)iy * W + ix);
    } else if (mode == 2) {
      float fy = align ? oy * sh : fmaxf((oy + 0.5f) * sh - 0.5f, 0.f);
      float fx = align ? ox * sw : fmaxf((ox + 0.5f) * sw - 0.5f, 0.f);
      int y0 = (int)fy, x0 = (int)fx;
      int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
      float ly = fy - y0, lx = fx - x0;
      v = (1.f - ly) * ((1.f - lx) * ldv<DT>(x, base + (long long)y0 * W + x0) + lx * ldv<DT>(x, base + (long long)y0 * W + x1)) +
          ly * ((1.f - lx) * ldv<DT>(x, base + (long long)y1 * W + x0) + lx * ldv<DT>(x, base + (long long)y1 * W + x1));
    } else if (mode == 3) {
      const float A = -0.75f;
      float fy = align ? oy * sh : (oy + 0.5f) * sh - 0.5f;
      float fx = align ? ox * sw : (ox + 0.5f) * sw - 0.5f;
      int iy = (int)floorf(fy), ix = (int)floorf(fx);
      float ty = fy - iy, tx = fx - ix;
      float wy[4] = {cubic2(ty + 1.f, A), cubic1(ty, A), cubic1(1.f - ty, A), cubic2(2.f - ty, A)};
      float wx[4] = {cubic2(tx + 1.f, A), cubic1(tx, A), cubic1(1.f - tx, A), cubic2(2.f - tx, A)};
      v = 0.f;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        int yy = min(max(iy - 1 + a, 0), H - 1);
        float row = 0.f;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          int xx = min(max(ix - 1 + b, 0), W - 1);
          row += wx[b] * ldv<DT>(x, base + (long long)yy * W + xx);
        }
        v += wy[a] * row;
      }
    } else {
      int y0 = (int)(((long long)oy * H) / Ho), y1 = (int)(((long long)(oy + 1) * H + Ho - 1) / Ho);
      int x0 = (int)(((long long)ox * W) / Wo), x1 = (int)(((long long)(ox + 1) * W + Wo - 1) / Wo);
      float s = 0.f;
      for (int yy = y0; yy < y1; ++yy)
        for (int xx = x0; xx < x1; ++xx) s += ldv<DT>(x, base + (long long)yy * W + xx);
      v = s / (float)((y1 - y0) * (x1 - x0));
    }
    stv<DT>(y, o, v);
  }
}

// ---------------------------------------------------------------------------------------------
// K31: nearest codebook entry. One wave per input row; lanes stride over the codebook computing
// sum_d (z_d - e_d)^2 in fp32, then a wave argmin (ties -> lowest index, like torch.argmin).
// Writes the index (int64) and the gathered entry.
// ---------------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) vq_nearest_kernel(const void* z, const void* cb, long long* idx, void* q,
                                                         int M, int n, int D) {
  extern __shared__ float zs[];               // [4 waves][D]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + wave;
  float* zr = zs + wave * D;
  if (row < M)
    for (int d = lane; d < D; d += 64) zr[d] = ldv<DT>(z, (long long)row * D + d);
  __syncthreads();
  if (row >= M) return;
  float best = 3.4e38f;
  int bi = 0x7fffffff;
  for (int j = lane; j < n; j += 64) {
    float s = 0.f;
    for (int d = 0; d < D; ++d) {
      float t = zr[d] - ldv<DT>(cb, (long long)j * D + d);
      s += t * t;
    }
    if (s < best) { best = s; bi = j; }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float ob = __shfl_xor(best, off, 64);
    int oi = __shfl_xor(bi, off, 64);
    if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (lane == 0) idx[row] = bi;
  for (int d = lane; d < D; d += 64) stv<DT>(q, (long long)row * D + d, ldv<DT>(cb, (long long)bi * D + d));
}

// ---------------------------------------------------------------------------------------------
// K28: ConvNeXt-V2 global response norm on NHWC x [N, HW, C]:
//   g[n,c] = ||x[n,:,c]||_2 ; nx = g / (mean_c g + 1e-6) ; y = beta + x * (1 + gamma * nx)
// pass 1: partial sum of squares over an HW slice (fp32 atomics into ws[N*C]);
// pass 2: per-sample mean over C, writes nx into ws[N*C ..]; pass 3: apply.
// ---------------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) grn_sumsq_kernel(const void* x, float* ss, int HW, int C, int rows_per) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int n = blockIdx.z;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(HW, r0 + rows_per);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) {
    float v = ldv<DT>(x, ((long long)n * HW + r) * C + c);
    s += v * v;
  }
  atomicAdd(ss + (long long)n * C + c, s);
}

__global__ void __launch_bounds__(256) grn_finalize_kernel(const float* ss, float* nx, int C) {
  __shared__ float red[256];
  const int n = blockIdx.x;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += 256) s += sqrtf(ss[(long long)n * C + c]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float inv = 1.f / (red[0] / (float)C + 1e-6f);
  for (int c = threadIdx.x; c < C; c += 256) nx[(long long)n * C + c] = sqrtf(ss[(long long)n * C + c]) * inv;
}

template <int DT>
__global__ void __launch_bounds__(256) grn_apply_kernel(const void* x, const float* nx, const void* gamma,
                                                        const void* beta, void* y, long long total, int HW, int C) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c = (int)(i % C);
    const long long n = i / ((long long)HW * C);
    const float v = ldv<DT>(x, i);
    stv<DT>(y, i, ldv<DT>(beta, c) + v * (1.f + ldv<DT>(gamma, c) * nx[n * C + c]));
  }
}


// K28 v2 (bf16 / fp16, C % 8 == 0): 16-B vectors, no atomics (per-row-slice partials, so no zero-fill
// pass), and an optional fused pre-GELU (Cascade's ChannelMLP is Linear -> GELU -> GRN: the GELU is
// recomputed in the two reads instead of being written and re-read).
//   pass 1: block = (512 channels, row slice, n), 4 row groups x 64 channel chunks -> part[n][c][slice]
//   pass 2: per n (1024 threads, a channel's S partials are contiguous: float4 reads),
//           g_c = sqrt(sum over slices), nx_c = g_c / (mean_c g + 1e-6)
//   pass 3: y = beta + a * (1 + gamma * nx), a = x or gelu(x)
template <int DT, bool GELU>
__global__ void __launch_bounds__(256) grn2_sumsq_kernel(const u16* __restrict__ x, float* __restrict__ part, int HW,
                                                         int C, int rows_per, int S) {
  __shared__ float red[4][64][8];
  const int n = blockIdx.z, sl = blockIdx.y;
  const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  const int nchunk = C >> 3;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ch < nchunk) {
    const int r0 = sl * rows_per, r1 = min(HW, r0 + rows_per);
    const u16* xb = x + (size_t)n * HW * C + ch * 8;
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += 4) {   // unrolled: several row loads in flight per thread
      const s16x8 v = *reinterpret_cast<const s16x8*>(xb + (size_t)r * C);
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2_t f = {cvt_in<DT>((u16)v[j]), cvt_in<DT>((u16)v[j + 1])};
        if (GELU) f = gelu_sig2(f);      // sigmoid-quintic GELU (|err| <= 2.6e-5): erff made GRN ALU-bound
        acc[j] += f.x * f.x;
        acc[j + 1] += f.y * f.y;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rg][lane][j] = acc[j];
  __syncthreads();
  if (rg == 0 && ch < nchunk) {
    float* o = part + ((size_t)n * C + ch * 8) * S + sl;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[(size_t)j * S] = (red[0][lane][j] + red[1][lane][j]) + (red[2][lane][j] + red[3][lane][j]);
  }
}

// gx[n][c] = ||x[n, :, c]||_2 from the slice partials, one thread per channel over a (C / 256, N) grid
// (a one-block-per-image form was latency-bound at batch 1-4: 2-8 workgroups); each block also
// leaves the sum of its 256 gx values in bsum[n][block] -- the apply pass forms mean_C(gx) from those.
__global__ void __launch_bounds__(256) grn2_finalize_kernel(const float* __restrict__ part, float* __restrict__ gx,
                                                            float* __restrict__ bsum, int C, int S) {
  __shared__ float red[4];
  const int n = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  float g = 0.f;
  if (c < C) {
    const float4* p = reinterpret_cast<const float4*>(part + ((size_t)n * C + c) * S);
    float ss = 0.f;
    for (int q = 0; q < S / 4; ++q) {
      const float4 v = p[q];
      ss += (v.x + v.y) + (v.z + v.w);
    }
    g = sqrtf(ss);
    gx[(size_t)n * C + c] = g;
  }
  g = wave_sum(g);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = g;
  __syncthreads();
  if (threadIdx.x == 0) bsum[(size_t)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// N <= GRN_MAXN images: each block first forms 1 / (mean_C gx + 1e-6) of every image from the
// finalize block sums (N x C/256 loads), then nx = gx * that inside the element loop.
#define GRN_MAXN 64
#define GRN_U 4
template <int DT, bool GELU>
__global__ void __launch_bounds__(256) grn2_apply_kernel(const u16* __restrict__ x, const float* __restrict__ gxp,
                                                         const float* __restrict__ bsum, int nblk, int N,
                                                         const u16* __restrict__ gamma, const u16* __restrict__ beta,
                                                         u16* __restrict__ y, long long chunks, int HW, int C) {
  __shared__ float inv_s[GRN_MAXN];
  // one wave per image, one finalize-block sum per lane (nblk <= 64: C <= 16384), then a wave sum: one
  // L2 round trip per block instead of nblk serial loads by one thread -- with one 16-B chunk per
  // thread that serial prologue was most of the kernel (33.7 us average per call in r03zl)
  {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (int n = wv; n < N; n += 4) {
      float t = 0.f;
      for (int b = ln; b < nblk; b += 64) t += bsum[(size_t)n * nblk + b];
      t = wave_sum(t);
      if (ln == 0) inv_s[n] = 1.f / (t / (float)C + 1e-6f);
    }
  }
  __syncthreads();
  const unsigned cpr = (unsigned)C >> 3;
  // GRN_U chunks per thread per step, all x loads issued before the math (more bytes in flight per CU:
  // the one-chunk loop ran at ~3 TB/s on the Stage C tensors)
  const long long step = (long long)gridDim.x * 256 * GRN_U;
  for (long long i0 = blockIdx.x * 256LL * GRN_U + threadIdx.x; i0 < chunks; i0 += step) {
    s16x8 v[GRN_U];
#pragma unroll
    for (int u = 0; u < GRN_U; ++u) {
      const long long i = i0 + 256LL * u;
      v[u] = i < chunks ? reinterpret_cast<const s16x8*>(x)[i] : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < GRN_U; ++u) {
      const long long i = i0 + 256LL * u;
      if (i >= chunks) break;
      // 32-bit index math (chunks < 2^32, checked by the launcher): 64-bit divisions cost ~10x
      const unsigned iu = (unsigned)i;
      const unsigned row = iu / cpr;
      const int c0 = (int)(iu - row * cpr) * 8;
      const int n = (int)(row / (unsigned)HW);
      const s16x8 gm = *reinterpret_cast<const s16x8*>(gamma + c0);
      const s16x8 bt = *reinterpret_cast<const s16x8*>(beta + c0);
      const float4* np = reinterpret_cast<const float4*>(gxp + (size_t)n * C + c0);
      const float4 n0 = np[0], n1 = np[1];
      const float iv = inv_s[n];
      const float nv[8] = {n0.x * iv, n0.y * iv, n0.z * iv, n0.w * iv, n1.x * iv, n1.y * iv, n1.z * iv, n1.w * iv};
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2_t f = {cvt_in<DT>((u16)v[u][j]), cvt_in<DT>((u16)v[u][j + 1])};
        if (GELU) f = gelu_sig2(f);
        o[j] = (short)cvt_out<DT>(cvt_in<DT>((u16)bt[j]) + f.x * (1.f + cvt_in<DT>((u16)gm[j]) * nv[j]));
        o[j + 1] = (short)cvt_out<DT>(cvt_in<DT>((u16)bt[j + 1]) + f.y * (1.f + cvt_in<DT>((u16)gm[j + 1]) * nv[j + 1]));
      }
      reinterpret_cast<s16x8*>(y)[i] = o;
    }
  }
}


// ---------------------------------------------------------------------------------------------
// K17 / K24: weighted accumulate of a piece into a region of an fp32 [B, C, Ho, Wo] accumulator
// pair (reference comfy/samplers.py:205-228 area/mask conds; comfy/utils.py tiled_scale feather):
//   out[b, c, oy + y, ox + x] += piece[b, c, y, x] * w(b, c, y, x);  div[...] += w(b, c, y, x)
// w = mult tensor [B, Cm, h, w] (Cm = 1 broadcasts over channels; any strides, any float dtype),
// times the separable feather ramp of the reference tiled blend when feather > 0 (rows / cols
// within `feather` of a tile edge scaled by (t+1)/feather, both edges when the tile is small),
// times `scale`. piece: any strides / float dtype. One thread per element of the piece.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float feather_ramp(int t, int n, int f) {
  float a = 1.f;
  if (t < f) a *= (float)(t + 1) / (float)f;
  if (n - 1 - t < f) a *= (float)(n - t) / (float)f;
  return a;
}

template <int DT>
__global__ void __launch_bounds__(256) region_acc_kernel(float* out, float* div, const void* piece, const void* mult,
                                                         int mdt, int B, int C, int Ho, int Wo, int h, int w, int oy,
                                                         int ox, long long ps0, long long ps1, long long ps2,
                                                         long long ps3, int Cm, long long ms0, long long ms1,
                                                         long long ms2, long long ms3, int feather, float scale) {
  const long long total = (long long)B * C * h * w;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int x = (int)(i % w);
    const int y = (int)((i / w) % h);
    const int c = (int)((i / ((long long)w * h)) % C);
    const int b = (int)(i / ((long long)w * h * C));
    const int Y = oy + y, X = ox + x;
    if (Y < 0 || Y >= Ho || X < 0 || X >= Wo) continue;
    float wt = scale;
    if (mult) {
      const long long mi = b * ms0 + (Cm == 1 ? 0 : c) * ms1 + y * ms2 + x * ms3;
      wt *= mdt == CGS_F32 ? ldv<CGS_F32>(mult, mi) : mdt == CGS_BF16 ? ldv<CGS_BF16>(mult, mi)
                                                                       : ldv<CGS_F16>(mult, mi);
    }
    if (feather > 0) wt *= feather_ramp(y, h, feather) * feather_ramp(x, w, feather);
    const float v = ldv<DT>(piece, b * ps0 + c * ps1 + y * ps2 + x * ps3);
    const long long o = (((long long)b * C + c) * Ho + Y) * Wo + X;
    out[o] += v * wt;
    if (div) div[o] += wt;
  }
}

// y = out / div (fp32 -> dtype of y), the final normalisation of both accumulations
template <int DT>
__global__ void __launch_bounds__(256) region_norm_kernel(const float* out, const float* div, void* y, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    stv<DT>(y, i, out[i] / div[i]);
}

// ---------------------------------------------------------------------------------------------
// K26: CLIP text embeddings (reference comfy/clip_model.py CLIPEmbeddings + the pooled gather of
// CLIPTextModel_): y[b, s, :] = tok[ids[b, s], :] + pos[s, :]; pooled[b, :] = x[b, argmax_s ids[b, s]]
// (first maximum, like torch.argmax). One thread per output element / one block per pooled row.
// ---------------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) clip_embed_kernel(const long long* ids, const void* tok, const void* pos,
                                                         void* y, int B, int S, int D, int vocab) {
  const long long total = (long long)B * S * D;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int d = (int)(i % D);
    const long long bs = i / D;
    const int s = (int)(bs % S);
    long long id = ids[bs];
    id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
    stv<DT>(y, i, ldv<DT>(tok, id * D + d) + ldv<DT>(pos, (long long)s * D + d));
  }
}

template <int DT>
__global__ void __launch_bounds__(256) pooled_gather_kernel(const long long* ids, const void* x, void* out, int S,
                                                            int D) {
  const int b = blockIdx.x;
  __shared__ long long best_v[256];
  __shared__ int best_i[256];
  long long bv = -(1ll << 62);
  int bi = 0;
  for (int s = threadIdx.x; s < S; s += 256) {
    const long long v = ids[(long long)b * S + s];
    if (v > bv) { bv = v; bi = s; }
  }
  best_v[threadIdx.x] = bv;
  best_i[threadIdx.x] = bi;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      const long long ov = best_v[threadIdx.x + w];
      const int oi = best_i[threadIdx.x + w];
      if (ov > best_v[threadIdx.x] || (ov == best_v[threadIdx.x] && oi < best_i[threadIdx.x])) {
        best_v[threadIdx.x] = ov;
        best_i[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  const int s = best_i[0];
  for (int d = threadIdx.x; d < D; d += 256)
    stv<DT>(out, (long long)b * D + d, ldv<DT>(x, ((long long)b * S + s) * D + d));
}

}  // namespace

CGS_EXPORT int cgs_fused_bias_act(const void* x, const void* b, void* y, long long n, int C, long long inner,
                                  float slope, float scale, int dtype, hipStream_t stream) {
  if (n <= 0) return 0;
  if (C <= 0 || inner <= 0) return (int)hipErrorInvalidValue;
  CGS_DISPATCH_DT(dtype, fused_bias_act_kernel, <<<grid_for(n), 256, 0, stream>>>(x, b, y, n, C, inner, slope, scale));
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_upfirdn2d(const void* x, const float* k, void* y, int NC, int H, int W, int upx, int upy, int dnx,
                             int dny, int px0, int px1, int py0, int py1, int kh, int kw, int dtype,
                             hipStream_t stream) {
  if (kh <= 0 || kw <= 0 || kh * kw > 32 * 32 || upx < 1 || upy < 1 || dnx < 1 || dny < 1)
    return (int)hipErrorInvalidValue;
  const int Ho = (H * upy + py0 + py1 - kh) / dny + 1;
  const int Wo = (W * upx + px0 + px1 - kw) / dnx + 1;
  if (Ho <= 0 || Wo <= 0) return (int)hipErrorInvalidValue;
  const long long total = (long long)NC * Ho * Wo;
  CGS_DISPATCH_DT(dtype, upfirdn2d_kernel, <<<grid_for(total), 256, 0, stream>>>(x, k, y, NC, H, W, upx, upy, dnx, dny,
                                                                                px0, py0, kh, kw, Ho, Wo));
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_resize(const void* x, void* y, int NC, int H, int W, int Ho, int Wo, int mode, int align,
                          int dtype, hipStream_t stream) {
  if (mode < 0 || mode > 4 || H <= 0 || W <= 0 || Ho <= 0 || Wo <= 0) return (int)hipErrorInvalidValue;
  const long long total = (long long)NC * Ho * Wo;
  if (total == 0) return 0;
  CGS_DISPATCH_DT(dtype, resize_kernel, <<<grid_for(total), 256, 0, stream>>>(x, y, NC, H, W, Ho, Wo, mode, align));
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_vq_nearest(const void* z, const void* cb, long long* idx, void* q, int M, int n, int D, int dtype,
                              hipStream_t stream) {
  if (M <= 0) return 0;
  if (n <= 0 || D <= 0 || D > 4096) return (int)hipErrorInvalidValue;
  const size_t lds = 4 * (size_t)D * sizeof(float);
  CGS_DISPATCH_DT(dtype, vq_nearest_kernel, <<<(M + 3) / 4, 256, lds, stream>>>(z, cb, idx, q, M, n, D));
  return (int)hipGetLastError();
}

// ws: fp32 workspace of 2*N*C floats, zeroed by the caller (first half: sum of squares).
CGS_EXPORT int cgs_grn_nhwc(const void* x, const void* gamma, const void* beta, void* y, float* ws, int N, int HW,
                            int C, int dtype, hipStream_t stream) {
  if (N <= 0 || HW <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  const int rows_per = 32;
  dim3 g1((C + 255) / 256, (HW + rows_per - 1) / rows_per, N);
  CGS_DISPATCH_DT(dtype, grn_sumsq_kernel, <<<g1, 256, 0, stream>>>(x, ws, HW, C, rows_per));
  grn_finalize_kernel<<<N, 256, 0, stream>>>(ws, ws + (long long)N * C, C);
  const long long total = (long long)N * HW * C;
  CGS_DISPATCH_DT(dtype, grn_apply_kernel, <<<grid_for(total), 256, 0, stream>>>(x, ws + (long long)N * C, gamma, beta,
                                                                                y, total, HW, C));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// K05: row softmax that materialises the probabilities (SAG / PAG need the attention map):
// y[r, :] = softmax(scale * x[r, :]) in fp32. One wave per row, three passes over the row
// (max, sum of exp, normalised write) straight from L2 for rows up to a few thousand columns.
// ---------------------------------------------------------------------------------------------
namespace {
template <int DT>
__global__ void __launch_bounds__(256) softmax_rows_kernel(const void* x, float* y, long long rows, int cols,
                                                           float scale) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long r = blockIdx.x * 4LL + wave;
  if (r >= rows) return;
  const long long base = r * cols;
  float mx = -INFINITY;
  for (int c = lane; c < cols; c += 64) mx = fmaxf(mx, ldv<DT>(x, base + c) * scale);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += __expf(ldv<DT>(x, base + c) * scale - mx);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float inv = 1.f / s;
  for (int c = lane; c < cols; c += 64) y[base + c] = __expf(ldv<DT>(x, base + c) * scale - mx) * inv;
}
}  // namespace

CGS_EXPORT int cgs_softmax_rows(const void* x, float* y, long long rows, int cols, float scale, int dtype,
                                hipStream_t stream) {
  if (rows <= 0) return 0;
  if (cols <= 0) return (int)hipErrorInvalidValue;
  const long long blocks = (rows + 3) / 4;
  if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  CGS_DISPATCH_DT(dtype, softmax_rows_kernel, <<<(unsigned)blocks, 256, 0, stream>>>(x, y, rows, cols, scale));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- K23: VAE output -> uint8 image
// The decoder's conv_out output (bf16, NHWC with C channels) straight to the uint8 HWC image the
// server encodes: v = clamp((x + 1) / 2, 0, 1); u8 = (uint8)(v * 255 + 0.5). One pass replaces the
// fp32 upcast, process_output, the NCHW->NHWC move and the uint8 conversion (sd.py VAE.decode +
// SaveImage's 255 scaling).
__global__ void vae_out_u8_kernel(const u16* __restrict__ x, uint8_t* __restrict__ y, long long n) {
  const long long n8 = n >> 3;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const s16x8 v = reinterpret_cast<const s16x8*>(x)[i];
    uint2 o;
    uint32_t w[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float f = fminf(fmaxf((bf2f((u16)v[j]) + 1.0f) * 0.5f, 0.0f), 1.0f);
      w[j >> 2] |= (uint32_t)(f * 255.0f + 0.5f) << (8 * (j & 3));
    }
    o.x = w[0];
    o.y = w[1];
    reinterpret_cast<uint2*>(y)[i] = o;
  }
  for (long long t = (n8 << 3) + blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n;
       t += (long long)gridDim.x * blockDim.x) {
    const float f = fminf(fmaxf((bf2f(x[t]) + 1.0f) * 0.5f, 0.0f), 1.0f);
    y[t] = (uint8_t)(f * 255.0f + 0.5f);
  }
}

CGS_EXPORT int cgs_vae_out_u8(const void* x, void* y, long long n, hipStream_t stream) {
  long long b = (n / 8 + 255) / 256;
  const int blocks = (int)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
  vae_out_u8_kernel<<<blocks, 256, 0, stream>>>((const u16*)x, (uint8_t*)y, n);
  return (int)hipGetLastError();
}

// K17 / K24 region accumulate (see region_acc_kernel). Strides in elements; mult may be null.
CGS_EXPORT int cgs_region_accumulate(float* out, float* div, const void* piece, int pdt, const void* mult, int mdt,
                                     int B, int C, int Ho, int Wo, int h, int w, int oy, int ox, long long ps0,
                                     long long ps1, long long ps2, long long ps3, int Cm, long long ms0, long long ms1,
                                     long long ms2, long long ms3, int feather, float scale, hipStream_t stream) {
  const long long n = (long long)B * C * h * w;
  if (n <= 0) return 0;
  if (!out || (Cm != 1 && Cm != C)) return (int)hipErrorInvalidValue;
  CGS_DISPATCH_DT(pdt, region_acc_kernel, <<<grid_for(n), 256, 0, stream>>>(out, div, piece, mult, mdt, B, C, Ho, Wo,
                                                                            h, w, oy, ox, ps0, ps1, ps2, ps3, Cm, ms0,
                                                                            ms1, ms2, ms3, feather, scale));
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_region_normalize(const float* out, const float* div, void* y, long long n, int ydt,
                                    hipStream_t stream) {
  if (n <= 0) return 0;
  CGS_DISPATCH_DT(ydt, region_norm_kernel, <<<grid_for(n), 256, 0, stream>>>(out, div, y, n));
  return (int)hipGetLastError();
}

// K26: token + position embeddings (ids int64 [B, S]; tok [vocab, D]; pos [>=S, D]; y [B, S, D])
CGS_EXPORT int cgs_clip_embed(const long long* ids, const void* tok, const void* pos, void* y, int B, int S, int D,
                              int vocab, int dtype, hipStream_t stream) {
  const long long n = (long long)B * S * D;
  if (n <= 0) return 0;
  CGS_DISPATCH_DT(dtype, clip_embed_kernel, <<<grid_for(n), 256, 0, stream>>>(ids, tok, pos, y, B, S, D, vocab));
  return (int)hipGetLastError();
}

// K26: pooled[b] = x[b, argmax(ids[b])] (x [B, S, D] contiguous)
CGS_EXPORT int cgs_pooled_gather(const long long* ids, const void* x, void* out, int B, int S, int D, int dtype,
                                 hipStream_t stream) {
  if (B <= 0) return 0;
  CGS_DISPATCH_DT(dtype, pooled_gather_kernel, <<<B, 256, 0, stream>>>(ids, x, out, S, D));
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- K29: FreeU Fourier filter
// Reference (comfy_extras/nodes_freelunch.py:6-23): fftn -> fftshift -> scale the 2t x 2t
// low-frequency square [H/2 - t, H/2 + t) x [W/2 - t, W/2 + t) -> ifftshift -> ifftn -> real.
// That square is the frequency set K = {-t .. t-1}^2, and the op is linear, so
//   y = x + (scale - 1) * Re( (1/HW) sum_{k in K} X_k e^{+2 pi i k.p} ),  X_k = sum_p x_p e^{-2 pi i k.p}
// -- exact, with (2t)^2 DFT coefficients per (b, c) instead of two full FFTs: pass 1 reduces the
// coefficients (one wave per 64 channels x 4 pixel lanes), pass 2 applies them. Any strides (NCHW or
// channels_last); t <= 4.
namespace {
constexpr int FF_MAXM = 64;

template <int DT>
__global__ __launch_bounds__(256) void fourier_coef_kernel(const u16* __restrict__ x, float* __restrict__ coef, int C,
                                                           int H, int W, long long sb, long long sc, long long sy,
                                                           long long sx, int t) {
  __shared__ float red[4][64][2];
  const int b = blockIdx.y, c = blockIdx.x * 64 + (threadIdx.x & 63), sub = threadIdx.x >> 6;
  const int n = 2 * t, nm = n * n;
  const float ty = 6.283185307179586f / H, tx = 6.283185307179586f / W;
  for (int m = 0; m < nm; ++m) {
    const int ky = m / n - t, kx = m % n - t;
    float re = 0.f, im = 0.f;
    if (c < C) {
      const u16* xb = x + b * sb + c * sc;
      for (int p = sub; p < H * W; p += 4) {
        const int py = p / W, px = p - py * W;
        const float v = cvt_in<DT>(xb[py * sy + px * sx]);
        float sn, cs;
        // angle reduced mod 1 turn before sincos (exact integer phase)
        const int ph_y = (ky * py) % H, ph_x = (kx * px) % W;
        __sincosf(ty * ph_y + tx * ph_x, &sn, &cs);
        re += v * cs;
        im -= v * sn;
      }
    }
    red[sub][threadIdx.x & 63][0] = re;
    red[sub][threadIdx.x & 63][1] = im;
    __syncthreads();
    if (sub == 0 && c < C) {
      const int l = threadIdx.x & 63;
      const float r = (red[0][l][0] + red[1][l][0]) + (red[2][l][0] + red[3][l][0]);
      const float i = (red[0][l][1] + red[1][l][1]) + (red[2][l][1] + red[3][l][1]);
      float* o = coef + (((long long)b * C + c) * nm + m) * 2;
      o[0] = r;
      o[1] = i;
    }
    __syncthreads();
  }
}

template <int DT>
__global__ __launch_bounds__(256) void fourier_apply_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                            const float* __restrict__ coef, int B, int C, int H, int W,
                                                            long long sb, long long sc, long long sy, long long sx,
                                                            long long ob, long long oc, long long oy, long long ox,
                                                            int t, float gain) {
  const long long total = (long long)B * C * H * W;
  const int n = 2 * t, nm = n * n;
  const float ty = 6.283185307179586f / H, tx = 6.283185307179586f / W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    // channel fastest: coalesced for channels_last, and a wave shares (b, py, px)
    const int c = (int)(i % C);
    long long r = i / C;
    const int px = (int)(r % W);
    r /= W;
    const int py = (int)(r % H);
    const int b = (int)(r / H);
    const float* cf = coef + ((long long)b * C + c) * nm * 2;
    float acc = 0.f;
    for (int m = 0; m < nm; ++m) {
      const int ky = m / n - t, kx = m % n - t;
      const int ph_y = (ky * py) % H, ph_x = (kx * px) % W;
      float sn, cs;
      __sincosf(ty * ph_y + tx * ph_x, &sn, &cs);
      acc += cf[2 * m] * cs - cf[2 * m + 1] * sn;
    }
    const float v = cvt_in<DT>(x[b * sb + c * sc + py * sy + px * sx]);
    y[b * ob + c * oc + py * oy + px * ox] = cvt_out<DT>(v + gain * acc);
  }
}
}  // namespace

CGS_EXPORT int cgs_fourier_filter(const void* x, void* y, float* coef, int B, int C, int H, int W, long long sb,
                                  long long sc, long long sy, long long sx, long long ob, long long oc, long long oy,
                                  long long ox, int t, float scale, int dtype, hipStream_t stream) {
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0) return 0;
  if (t < 1 || (2 * t) * (2 * t) > FF_MAXM || 2 * t > H || 2 * t > W || dtype == CGS_F32) return (int)hipErrorInvalidValue;
  dim3 g1((unsigned)((C + 63) / 64), (unsigned)B);
  const float gain = (scale - 1.0f) / ((float)H * (float)W);
  const long long total = (long long)B * C * H * W;
  long long nb = (total + 255) / 256;
  const int blocks = (int)(nb > 16384 ? 16384 : nb);
  if (dtype == CGS_BF16) {
    fourier_coef_kernel<CGS_BF16><<<g1, 256, 0, stream>>>((const u16*)x, coef, C, H, W, sb, sc, sy, sx, t);
    fourier_apply_kernel<CGS_BF16><<<blocks, 256, 0, stream>>>((const u16*)x, (u16*)y, coef, B, C, H, W, sb, sc, sy,
                                                                sx, ob, oc, oy, ox, t, gain);
  } else {
    fourier_coef_kernel<CGS_F16><<<g1, 256, 0, stream>>>((const u16*)x, coef, C, H, W, sb, sc, sy, sx, t);
    fourier_apply_kernel<CGS_F16><<<blocks, 256, 0, stream>>>((const u16*)x, (u16*)y, coef, B, C, H, W, sb, sc, sy,
                                                               sx, ob, oc, oy, ox, t, gain);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- K30: ToMe bipartite matching
// Reference (comfy_extras/nodes_tomesd.py:22-160): cosine similarity of every src token a_i with
// every dst token b_j, then (max_j, argmax_j) per src token. Fused here: 1/||row|| once per token
// (pass 1), then 64 x 64 score tiles from LDS-staged k-chunks, 4 x 4 per thread in fp32, folded into a
// running per-row (max, argmax) -- the [Na, Nb] score matrix never exists.
namespace {
template <int DT>
__global__ __launch_bounds__(256) void row_inv_norm_kernel(const u16* __restrict__ x, float* __restrict__ out,
                                                           long long rows, int C, long long ld) {
  const long long r = blockIdx.x * 4LL + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float v = cvt_in<DT>(x[r * ld + c]);
    s += v * v;
  }
  s = wave_sum(s);
  if (lane == 0) out[r] = s > 0.f ? rsqrtf(s) : 0.f;
}

template <int DT>
__global__ __launch_bounds__(256) void tome_match_kernel(const u16* __restrict__ a, const u16* __restrict__ b,
                                                         const float* __restrict__ ia, const float* __restrict__ ib,
                                                         float* __restrict__ vmax, long long* __restrict__ imax,
                                                         int Na, int Nb, int C, long long sab, long long sa,
                                                         long long sbb, long long sbr) {
  __shared__ float As[32][65], Bs[32][65];
  const int bt = blockIdx.y, r0 = blockIdx.x * 64;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const u16* ab = a + bt * sab;
  const u16* bb = b + bt * sbb;
  float best[4], inva[4];
  int bidx[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    best[i] = -INFINITY;
    bidx[i] = 0;
    const int r = r0 + ty * 4 + i;
    inva[i] = r < Na ? ia[(long long)bt * Na + r] : 0.f;
  }
  for (int c0 = 0; c0 < Nb; c0 += 64) {
    float acc[4][4] = {};
    for (int k0 = 0; k0 < C; k0 += 32) {
      // stage 64 rows x 32 k of A and B (transposed: [k][row])
      for (int e = tid; e < 64 * 32; e += 256) {
        const int row = e >> 5, k = e & 31;
        const int ra = r0 + row, rb = c0 + row, kk = k0 + k;
        As[k][row] = (ra < Na && kk < C) ? cvt_in<DT>(ab[ra * sa + kk]) : 0.f;
        Bs[k][row] = (rb < Nb && kk < C) ? cvt_in<DT>(bb[rb * sbr + kk]) : 0.f;
      }
      __syncthreads();
#pragma unroll 8
      for (int k = 0; k < 32; ++k) {
        float av[4], bv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) { av[i] = As[k][ty * 4 + i]; bv[i] = Bs[k][tx * 4 + i]; }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] += av[i] * bv[j];
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + tx * 4 + j;
      if (col >= Nb) continue;
      const float invb = ib[(long long)bt * Nb + col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float s = acc[i][j] * inva[i] * invb;
        if (s > best[i]) { best[i] = s; bidx[i] = col; }
      }
    }
  }
  // (max, argmax) over the 16 column lanes of each row group (lowest index on ties)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float ov = __shfl_xor(best[i], o, 64);
      const int oi = __shfl_xor(bidx[i], o, 64);
      if (ov > best[i] || (ov == best[i] && oi < bidx[i])) { best[i] = ov; bidx[i] = oi; }
    }
    const int r = r0 + ty * 4 + i;
    if (tx == 0 && r < Na) {
      vmax[(long long)bt * Na + r] = best[i];
      imax[(long long)bt * Na + r] = bidx[i];
    }
  }
}
}  // namespace

// a [B, Na, C] (row stride sa, batch stride sab), b [B, Nb, C]; ws: (B*Na + B*Nb) floats.
CGS_EXPORT int cgs_tome_match(const void* a, const void* b, float* ws, float* vmax, long long* imax, int B, int Na,
                              int Nb, int C, long long sab, long long sa, long long sbb, long long sbr, int dtype,
                              hipStream_t stream) {
  if (B <= 0 || Na <= 0) return 0;
  if (Nb <= 0 || C <= 0 || dtype == CGS_F32) return (int)hipErrorInvalidValue;
  float* ia = ws;
  float* ib = ws + (long long)B * Na;
  // row norms: rows of a batch are contiguous only per batch, so one launch per operand and batch stride
  for (int bt = 0; bt < B; ++bt) {
    const u16* ap = (const u16*)a + bt * sab;
    const u16* bp = (const u16*)b + bt * sbb;
    if (dtype == CGS_BF16) {
      row_inv_norm_kernel<CGS_BF16><<<(unsigned)((Na + 3) / 4), 256, 0, stream>>>(ap, ia + (long long)bt * Na, Na, C, sa);
      row_inv_norm_kernel<CGS_BF16><<<(unsigned)((Nb + 3) / 4), 256, 0, stream>>>(bp, ib + (long long)bt * Nb, Nb, C, sbr);
    } else {
      row_inv_norm_kernel<CGS_F16><<<(unsigned)((Na + 3) / 4), 256, 0, stream>>>(ap, ia + (long long)bt * Na, Na, C, sa);
      row_inv_norm_kernel<CGS_F16><<<(unsigned)((Nb + 3) / 4), 256, 0, stream>>>(bp, ib + (long long)bt * Nb, Nb, C, sbr);
    }
  }
  dim3 g((unsigned)((Na + 63) / 64), (unsigned)B);
  if (dtype == CGS_BF16)
    tome_match_kernel<CGS_BF16><<<g, 256, 0, stream>>>((const u16*)a, (const u16*)b, ia, ib, vmax, imax, Na, Nb, C, sab,
                                                        sa, sbb, sbr);
  else
    tome_match_kernel<CGS_F16><<<g, 256, 0, stream>>>((const u16*)a, (const u16*)b, ia, ib, vmax, imax, Na, Nb, C, sab,
                                                       sa, sbb, sbr);
  return (int)hipGetLastError();
}

// K28 v2 launcher: ws >= N * ((S + 1) * C + ceil(C / 256)) floats with S = cgs_grn_slices(N, HW, C), N <= 64.
CGS_EXPORT int cgs_grn_slices(int N, int HW, int C) {
  // ~512 pass-1 blocks, a multiple of 4 slices (pass 2 reads each channel's partials as float4s)
  const int cb = (C / 8 + 63) / 64;
  int s = (512 + N * cb - 1) / (N * cb);
  const int smax = (HW + 15) / 16;               // >= 16 rows per slice
  if (s > smax) s = smax;
  s = (s + 3) & ~3;
  return s < 4 ? 4 : s;
}

// Row-tiled GRN apply: a block owns 256 consecutive 8-channel chunks of ONE image and walks GRN_RT rows of
// it, so each thread forms its 8 per-channel coefficients a = 1 + gamma * nx[n], b = beta once and then only
// streams x -> y (one 16-B load, 8 FMAs, one 16-B store per chunk; GRN_RU rows in flight). The grid-stride
// form re-loaded gamma / beta / nx and re-derived (row, channel, image) with two divisions per chunk and ran
// the Stage C apply at ~3.5 TB/s.
template <int DT, bool GELU, int GRN_RT = 16, int GRN_RU = 4>
__global__ void __launch_bounds__(256) grn_apply_rows_kernel(const u16* __restrict__ x, const float* __restrict__ gxp,
                                                             const float* __restrict__ bsum, int nblk,
                                                             const u16* __restrict__ gamma,
                                                             const u16* __restrict__ beta, u16* __restrict__ y, int HW,
                                                             int C) {
  __shared__ float inv_s;
  const int n = blockIdx.z;
  if (threadIdx.x < 64) {
    float t = 0.f;
    for (int b = threadIdx.x; b < nblk; b += 64) t += bsum[(size_t)n * nblk + b];
    t = wave_sum(t);
    if (threadIdx.x == 0) inv_s = 1.f / (t / (float)C + 1e-6f);
  }
  __syncthreads();
  const int cpr = C >> 3;
  const int c8 = blockIdx.x * 256 + threadIdx.x;
  if (c8 >= cpr) return;
  const int c0 = c8 * 8;
  float a[8], bb[8];
  {
    const s16x8 gm = *reinterpret_cast<const s16x8*>(gamma + c0);
    const s16x8 bt = *reinterpret_cast<const s16x8*>(beta + c0);
    const float4* np = reinterpret_cast<const float4*>(gxp + (size_t)n * C + c0);
    const float4 n0 = np[0], n1 = np[1];
    const float iv = inv_s;
    const float nv[8] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, n1.z, n1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = 1.f + cvt_in<DT>((u16)gm[j]) * (nv[j] * iv);
      bb[j] = cvt_in<DT>((u16)bt[j]);
    }
  }
  const int r0 = blockIdx.y * GRN_RT;
  const int r1 = min(HW, r0 + GRN_RT);
  const s16x8* xr = reinterpret_cast<const s16x8*>(x) + (size_t)n * HW * cpr + c8;
  s16x8* yr = reinterpret_cast<s16x8*>(y) + (size_t)n * HW * cpr + c8;
  for (int r = r0; r < r1; r += GRN_RU) {
    s16x8 v[GRN_RU];
#pragma unroll
    for (int u = 0; u < GRN_RU; ++u)
      v[u] = r + u < r1 ? xr[(size_t)(r + u) * cpr] : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < GRN_RU; ++u) {
      if (r + u >= r1) break;
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        f32x2_t f = {cvt_in<DT>((u16)v[u][j]), cvt_in<DT>((u16)v[u][j + 1])};
        if (GELU) f = gelu_sig2(f);
        o[j] = (short)cvt_out<DT>(bb[j] + f.x * a[j]);
        o[j + 1] = (short)cvt_out<DT>(bb[j + 1] + f.y * a[j + 1]);
      }
      yr[(size_t)(r + u) * cpr] = o;
    }
  }
}

// 0: the grid-stride apply; 1: row-tiled, 16 rows per block, 4 in flight; 2: 32 / 8; 3: 64 / 8 (A/B switch)
static int g_grn_rows = 1;
CGS_EXPORT void cgs_grn_set_rows(int v) { g_grn_rows = v < 0 ? 0 : v > 3 ? 3 : v; }

template <int DT, bool GELU>
static void grn_apply_launch(const u16* x, const float* nx, const float* bsum, int nblk, int N, const u16* gamma,
                             const u16* beta, u16* y, int HW, int C, hipStream_t stream) {
  const int rt = g_grn_rows == 1 ? 16 : g_grn_rows == 2 ? 32 : 64;
  // a block spans 256 chunks of a row: only where that leaves <= 20 % of the threads idle (C = 2560 -> 320
  // chunks measured 8 % slower than the grid-stride form; 8192 / 5120 faster, profiles/r05/grn_apply_rows.md)
  const int cpr = C / 8, groups = (cpr + 255) / 256;
  if (g_grn_rows && (HW + rt - 1) / rt <= 65535 && cpr * 5 >= groups * 256 * 4) {
    const dim3 g((unsigned)((C / 8 + 255) / 256), (unsigned)((HW + rt - 1) / rt), (unsigned)N);
    if (g_grn_rows == 1)
      grn_apply_rows_kernel<DT, GELU, 16, 4><<<g, 256, 0, stream>>>(x, nx, bsum, nblk, gamma, beta, y, HW, C);
    else if (g_grn_rows == 2)
      grn_apply_rows_kernel<DT, GELU, 32, 8><<<g, 256, 0, stream>>>(x, nx, bsum, nblk, gamma, beta, y, HW, C);
    else
      grn_apply_rows_kernel<DT, GELU, 64, 8><<<g, 256, 0, stream>>>(x, nx, bsum, nblk, gamma, beta, y, HW, C);
    return;
  }
  const long long chunks = (long long)N * HW * (C / 8);
  const long long nb = (chunks + 256 * GRN_U - 1) / (256 * GRN_U);
  const int blocks = (int)(nb > 16384 ? 16384 : nb);
  grn2_apply_kernel<DT, GELU><<<blocks, 256, 0, stream>>>(x, nx, bsum, nblk, N, gamma, beta, y, chunks, HW, C);
}

CGS_EXPORT int cgs_grn_nhwc_v2(const void* x, const void* gamma, const void* beta, void* y, float* ws, int N, int HW,
                               int C, int pre_gelu, int dtype, hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 8 || dtype == CGS_F32 || (((uintptr_t)x | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15))
    return (int)hipErrorInvalidValue;
  const int S = cgs_grn_slices(N, HW, C);
  const int rows_per = (HW + S - 1) / S;
  if (N > GRN_MAXN) return (int)hipErrorInvalidValue;
  float* part = ws;
  float* nx = ws + (size_t)N * S * C;
  const int nblk = (C + 255) / 256;
  float* bsum = nx + (size_t)N * C;                 // ws >= N * ((S + 1) * C + nblk) floats
  dim3 g1((unsigned)((C / 8 + 63) / 64), (unsigned)S, (unsigned)N);
  const long long chunks = (long long)N * HW * (C / 8);
  if (chunks >= (1LL << 32)) return (int)hipErrorInvalidValue;
#define CGS_GRN2(DTV, GV)                                                                                        \
  grn2_sumsq_kernel<DTV, GV><<<g1, 256, 0, stream>>>((const u16*)x, part, HW, C, rows_per, S);                  \
  grn2_finalize_kernel<<<dim3((unsigned)nblk, (unsigned)N), 256, 0, stream>>>(part, nx, bsum, C, S);            \
  grn_apply_launch<DTV, GV>((const u16*)x, nx, bsum, nblk, N, (const u16*)gamma, (const u16*)beta, (u16*)y, HW, C, stream)
  if (dtype == CGS_BF16) {
    if (pre_gelu) { CGS_GRN2(CGS_BF16, true); } else { CGS_GRN2(CGS_BF16, false); }
  } else {
    if (pre_gelu) { CGS_GRN2(CGS_F16, true); } else { CGS_GRN2(CGS_F16, false); }
  }
#undef CGS_GRN2
  return (int)hipGetLastError();
}

// GRN pass 2 from the producing GEMM's partials (cgs_gemm_bf16_gelu_gns: part [N][HW / 64][C], the sum of
// squares over each 64-row block): sum_HW h^2 = their sum; then gx / bsum as grn2_finalize_kernel.
__global__ void __launch_bounds__(256) grn_gns_finalize_kernel(const float* __restrict__ part, float* __restrict__ gx,
                                                               float* __restrict__ bsum, int C, int nbk) {
  __shared__ float red[4];
  const int n = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  float g = 0.f;
  if (c < C) {
    const float* p = part + (size_t)n * nbk * C + c;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;   // four loads in flight per step
    int b = 0;
    for (; b + 4 <= nbk; b += 4) {
      s0 += p[(size_t)b * C];
      s1 += p[(size_t)(b + 1) * C];
      s2 += p[(size_t)(b + 2) * C];
      s3 += p[(size_t)(b + 3) * C];
    }
    for (; b < nbk; ++b) s0 += p[(size_t)b * C];
    g = sqrtf((s0 + s1) + (s2 + s3));
    gx[(size_t)n * C + c] = g;
  }
  g = wave_sum(g);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = g;
  __syncthreads();
  if (threadIdx.x == 0) bsum[(size_t)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// GRN apply with the statistics from GNS partials: y = beta + h * (1 + gamma * nx). ws >= N * (C + ceil(C / 256))
// floats. h bf16 [N, HW, C] (already GELU'd), HW % 64 == 0, C % 8 == 0, N <= 64.
CGS_EXPORT int cgs_grn_apply_gns(const void* h, const float* part, const void* gamma, const void* beta, void* y,
                                 float* ws, int N, int HW, int C, hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 8 || HW % 64 || N > GRN_MAXN || (((uintptr_t)h | (uintptr_t)y | (uintptr_t)gamma | (uintptr_t)beta) & 15) ||
      ((uintptr_t)part & 3))
    return (int)hipErrorInvalidValue;
  const int nblk = (C + 255) / 256;
  float* gx = ws;
  float* bsum = ws + (size_t)N * C;
  grn_gns_finalize_kernel<<<dim3((unsigned)nblk, (unsigned)N), 256, 0, stream>>>(part, gx, bsum, C, HW / 64);
  const long long chunks = (long long)N * HW * (C / 8);
  if (chunks >= (1LL << 32)) return (int)hipErrorInvalidValue;
  grn_apply_launch<CGS_BF16, false>((const u16*)h, gx, bsum, nblk, N, (const u16*)gamma, (const u16*)beta, (u16*)y, HW,
                                    C, stream);
  return (int)hipGetLastError();
}

// cgs_grn_stats from GNS partials instead of a pass over h: gx / bsum land where cgs_grn_stats puts them
// (ws + N * S * C, S = cgs_grn_slices), so cgs_grn_scale_weight reads them unchanged. HW % 64 == 0.
CGS_EXPORT int cgs_grn_stats_gns(const float* part, float* ws, int N, int HW, int C, hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 8 || HW % 64 || N > GRN_MAXN || ((uintptr_t)part & 3)) return (int)hipErrorInvalidValue;
  const int S = cgs_grn_slices(N, HW, C);
  float* gx = ws + (size_t)N * S * C;
  const int nblk = (C + 255) / 256;
  grn_gns_finalize_kernel<<<dim3((unsigned)nblk, (unsigned)N), 256, 0, stream>>>(part, gx, gx + (size_t)N * C, C,
                                                                                 HW / 64);
  return (int)hipGetLastError();
}

// GRN statistics only (passes 1-2 of cgs_grn_nhwc_v2, same ws layout): gx = ws + N * S * C ([N, C]) and the
// finalize block sums bsum = gx + N * C ([N, ceil(C / 256)]), for a consumer that folds the GRN scale into
// the next GEMM's weights (cgs_grn_scale_weight) instead of rewriting the activation.
CGS_EXPORT int cgs_grn_stats(const void* x, float* ws, int N, int HW, int C, int pre_gelu, int dtype,
                             hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 8 || dtype == CGS_F32 || ((uintptr_t)x & 15) || N > GRN_MAXN) return (int)hipErrorInvalidValue;
  const int S = cgs_grn_slices(N, HW, C);
  const int rows_per = (HW + S - 1) / S;
  float* part = ws;
  float* gx = ws + (size_t)N * S * C;
  const int nblk = (C + 255) / 256;
  float* bsum = gx + (size_t)N * C;
  dim3 g1((unsigned)((C / 8 + 63) / 64), (unsigned)S, (unsigned)N);
#define CGS_GRNS(DTV, GV)                                                                      \
  grn2_sumsq_kernel<DTV, GV><<<g1, 256, 0, stream>>>((const u16*)x, part, HW, C, rows_per, S); \
  grn2_finalize_kernel<<<dim3((unsigned)nblk, (unsigned)N), 256, 0, stream>>>(part, gx, bsum, C, S)
  if (dtype == CGS_BF16) {
    if (pre_gelu) { CGS_GRNS(CGS_BF16, true); } else { CGS_GRNS(CGS_BF16, false); }
  } else {
    if (pre_gelu) { CGS_GRNS(CGS_F16, true); } else { CGS_GRNS(CGS_F16, false); }
  }
#undef CGS_GRNS
  return (int)hipGetLastError();
}

// GRN folded into the following Linear (Cascade ChannelMLP: GRN -> Linear): for image n,
//   (beta + a * (1 + gamma * nx_n)) W^T = a (W * s_n)^T + W beta,   s_n[k] = 1 + gamma[k] * nx_n[k]
// so Wn[n] = W * s_n (bf16, [N, O, K]) replaces the rewrite of the [N, HW, K] activation -- the cheaper
// pass whenever O < HW. nx_n = gx[n] / (mean_k gx[n] + 1e-6) from cgs_grn_stats. One thread per 8-wide K
// chunk of W, looping over the images (W read once).
__global__ void __launch_bounds__(256) grn_scale_weight_kernel(const u16* __restrict__ W, const u16* __restrict__ gamma,
                                                               const float* __restrict__ gx,
                                                               const float* __restrict__ bsum, int nblk, int N,
                                                               u16* __restrict__ Wn, long long chunks, int K) {
  __shared__ float inv_s[GRN_MAXN];
  {
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    for (int n = wv; n < N; n += 4) {
      float t = 0.f;
      for (int b = ln; b < nblk; b += 64) t += bsum[(size_t)n * nblk + b];
      t = wave_sum(t);
      if (ln == 0) inv_s[n] = 1.f / (t / (float)K + 1e-6f);
    }
  }
  __syncthreads();
  const long long i = blockIdx.x * 256LL + threadIdx.x;
  if (i >= chunks) return;
  const unsigned kc = (unsigned)(K >> 3);
  const int k0 = (int)((unsigned long long)i % kc) * 8;
  const s16x8 w = reinterpret_cast<const s16x8*>(W)[i];
  const s16x8 gm = *reinterpret_cast<const s16x8*>(gamma + k0);
  float wf[8], gf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { wf[j] = bf2f((u16)w[j]); gf[j] = bf2f((u16)gm[j]); }
  for (int n = 0; n < N; ++n) {
    const float4* gp = reinterpret_cast<const float4*>(gx + (size_t)n * K + k0);
    const float4 g0 = gp[0], g1 = gp[1];
    const float iv = inv_s[n];
    const float nv[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (short)f2bf(wf[j] * (1.f + gf[j] * nv[j] * iv));
    reinterpret_cast<s16x8*>(Wn)[(size_t)n * chunks + i] = o;
  }
}

// W [O, K] bf16 (K % 8 == 0), gamma [K] bf16, stats = the ws of cgs_grn_stats(x, ws, N, HW, K, ...) -> Wn [N, O, K].
CGS_EXPORT int cgs_grn_scale_weight(const void* W, const void* gamma, const float* ws, int N, int HW, int O, int K,
                                    void* Wn, hipStream_t stream) {
  if (N <= 0 || O <= 0) return 0;
  if (K % 8 || N > GRN_MAXN || (((uintptr_t)W | (uintptr_t)gamma | (uintptr_t)Wn) & 15)) return (int)hipErrorInvalidValue;
  const int S = cgs_grn_slices(N, HW, K);
  const float* gx = ws + (size_t)N * S * K;
  const int nblk = (K + 255) / 256;
  const float* bsum = gx + (size_t)N * K;
  const long long chunks = (long long)O * (K / 8);
  grn_scale_weight_kernel<<<(unsigned)((chunks + 255) / 256), 256, 0, stream>>>(
      (const u16*)W, (const u16*)gamma, gx, bsum, nblk, N, (u16*)Wn, chunks, K);
  return (int)hipGetLastError();
}

// Per-(image, channel) affine on NHWC straight from a [N, ld] activation-dtype coefficient tensor:
// y = x * (add + s[n][c]) + t[n][c] (Stable Cascade TimestepBlock x * (1 + a) + b with a, b the two
// halves of the mapper GEMM output, comfy/ldm/cascade/common.py TimestepBlock) -- no fp32 cast /
// stack of the coefficients on the host side of the op.
template <int DT>
__global__ void __launch_bounds__(256) chan_affine_kernel(const u16* __restrict__ x, const u16* __restrict__ sc,
                                                          const u16* __restrict__ sh, long long ld,
                                                          u16* __restrict__ y, long long chunks, int HW, int C,
                                                          float add) {
  const unsigned cpr = (unsigned)C >> 3;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < chunks; i += (long long)gridDim.x * 256) {
    const unsigned iu = (unsigned)i;
    const unsigned row = iu / cpr;
    const int c0 = (int)(iu - row * cpr) * 8;
    const long long n = row / (unsigned)HW;
    const s16x8 v = reinterpret_cast<const s16x8*>(x)[i];
    const s16x8 a = *reinterpret_cast<const s16x8*>(sc + n * ld + c0);
    const s16x8 b = *reinterpret_cast<const s16x8*>(sh + n * ld + c0);
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      o[j] = (short)cvt_out<DT>(__builtin_fmaf(cvt_in<DT>((u16)v[j]), add + cvt_in<DT>((u16)a[j]), cvt_in<DT>((u16)b[j])));
    reinterpret_cast<s16x8*>(y)[i] = o;
  }
}

CGS_EXPORT int cgs_channel_affine2(const void* x, const void* scale, const void* shift, long long ld, void* y, int N,
                                   int HW, int C, float add, int dtype, hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  if (C % 8 || ld % 8 || dtype == CGS_F32 ||
      (((uintptr_t)x | (uintptr_t)y | (uintptr_t)scale | (uintptr_t)shift) & 15))
    return (int)hipErrorInvalidValue;
  const long long chunks = (long long)N * HW * (C / 8);
  if (chunks >= (1LL << 32)) return (int)hipErrorInvalidValue;
  long long nb = (chunks + 255) / 256;
  const int blocks = (int)(nb > 16384 ? 16384 : nb);
  if (dtype == CGS_BF16)
    chan_affine_kernel<CGS_BF16><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)scale, (const u16*)shift, ld,
                                                             (u16*)y, chunks, HW, C, add);
  else
    chan_affine_kernel<CGS_F16><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)scale, (const u16*)shift, ld,
                                                            (u16*)y, chunks, HW, C, add);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- K05: probability-output attention
// SAG / PAG read the attention map itself (comfy_extras/nodes_sag.py, reference fp32 bmm + softmax),
// so it is materialised: S = scale * Q K^T and O = P V as batched fp32 GEMMs on the f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact fp32 products, the reference's precision), P by the row softmax
// (K05 softmax_rows). C[b] = alpha * A[b] . B[b] with A(m, k) = A + b*sab + m*sam + k*sak and
// B(k, n) = B + b*sbb + k*sbk + n*sbn (any strides: B = K^T for the scores, B = V for PV);
// 64 x 64 tiles, 4 waves of 32 x 32, k-chunks of 16 staged through LDS as fp32.
namespace {
template <int DTA, int DTB>
__global__ __launch_bounds__(256) void bgemm_f32_kernel(const void* __restrict__ A, const void* __restrict__ Bm,
                                                        float* __restrict__ C, int M, int N, int K, long long sab,
                                                        long long sam, long long sak, long long sbb, long long sbk,
                                                        long long sbn, long long scb, long long scm, float alpha) {
  __shared__ float As[64][17], Bs[64][17];   // As[m][k], Bs[n][k]
  const int bt = blockIdx.z, m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 16) {
    for (int e = tid; e < 64 * 16; e += 256) {
      const int r = e >> 4, kk = e & 15, k = k0 + kk;
      const int m = m0 + r, n = n0 + r;
      As[r][kk] = (m < M && k < K) ? ldv<DTA>(A, bt * sab + m * sam + k * sak) : 0.f;
      Bs[r][kk] = (n < N && k < K) ? ldv<DTB>(Bm, bt * sbb + k * sbk + n * sbn) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float a = As[wm + 16 * i + (lane & 15)][kk];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[wn + 16 * j + (lane & 15)][kk], acc[i][j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + (lane >> 4) * 4 + r, n = n0 + wn + 16 * j + (lane & 15);
        if (m < M && n < N) C[bt * scb + (long long)m * scm + n] = acc[i][j][r] * alpha;
      }
}
}  // namespace

// dta / dtb: CgsDType of A / B (fp32, bf16 or fp16); C fp32 with row stride scm.
CGS_EXPORT int cgs_bgemm_f32(const void* A, const void* B, float* C, int batch, int M, int N, int K, long long sab,
                             long long sam, long long sak, long long sbb, long long sbk, long long sbn, long long scb,
                             long long scm, float alpha, int dta, int dtb, hipStream_t stream) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if (K <= 0 || batch > 65535 || (M + 63) / 64 > 65535) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64), (unsigned)batch);
#define CGS_BG(TA, TB) bgemm_f32_kernel<TA, TB><<<g, 256, 0, stream>>>(A, B, C, M, N, K, sab, sam, sak, sbb, sbk, sbn, scb, scm, alpha)
  if (dta == CGS_BF16 && dtb == CGS_BF16) CGS_BG(CGS_BF16, CGS_BF16);
  else if (dta == CGS_F32 && dtb == CGS_BF16) CGS_BG(CGS_F32, CGS_BF16);
  else if (dta == CGS_F16 && dtb == CGS_F16) CGS_BG(CGS_F16, CGS_F16);
  else if (dta == CGS_F32 && dtb == CGS_F16) CGS_BG(CGS_F32, CGS_F16);
  else if (dta == CGS_F32 && dtb == CGS_F32) CGS_BG(CGS_F32, CGS_F32);
  else return (int)hipErrorInvalidValue;
#undef CGS_BG
  return (int)hipGetLastError();
}
