// GroupNorm (+fused SiLU, +fused per-(n,c) pre-add) over NHWC activations, and LayerNorm.
// K06 / K07 of SURVEY §2.4. Reference semantics: comfy/ldm/modules/diffusionmodules/openaimodel.py
// ResBlock (GN -> SiLU -> conv, emb add before out_layers GN) and attention.py LayerNorms.
//
// GroupNorm = 3 small launches, every one fully coalesced on NHWC rows:
//   1. gn_partial : block = (pixel chunk, n); each lane owns fixed 8-channel chunks of the row and
//      accumulates shifted sums (shift = the block's first pixel; 4 rows of loads in flight per wave) -> per-wave (mean, M2) -> Chan combine over
//      the 4 waves in LDS -> per-(n, block, c) partial.
//   2. gn_finalize: one block per (n, g), one-pass Chan combine of the blocks x channels partials ->
//      mean/rstd -> per-(n,c) affine a, b (the pre-add shifts the channel mean only, so it folds into b).
//   3. gn_apply   : y = x*a + b (+SiLU), 16-byte vectors, per-thread channel chunk fixed (a, b in registers).
// LayerNorm: 8-64 lanes per row (sized to the row), two-pass mean/var from registers, 16-byte vectors.
#include "common.h"

#define GN_THREADS 256
#define GN_MAX_CHUNKS_PER_LANE 4   // <= 64*4*8 = 2048 channels of a row per block (wider rows: channel slices)

// statistics blocks over the batch: CGS_GN_BLOCKS (default 2048) / cgs_gn_set_blocks (A/B; a smaller count only
// shrinks the workspace cgs_groupnorm_workspace sized earlier)
static int g_gn_blocks = -1;
static int gn_blocks() {
  if (g_gn_blocks < 0) g_gn_blocks = getenv("CGS_GN_BLOCKS") ? atoi(getenv("CGS_GN_BLOCKS")) : 2048;
  return g_gn_blocks > 0 ? g_gn_blocks : 2048;
}
CGS_EXPORT void cgs_gn_set_blocks(int n) { g_gn_blocks = n; }

static inline int gn_pix_per_block(int N, int HW) {
  // ~2048 statistics blocks over the batch, >= 16 pixels each -- >= 64 at batch <= 4: there 16-pixel blocks
  // (1024 per image at 128^2) made the finalize pass (one block per (image, group)) walk 10-40 k partials
  // each (~16 us per GroupNorm at SDXL batch 1; profiles/r04/groupnorm_b1_r04ai.log)
  int target_blocks_per_n = (gn_blocks() + N - 1) / N;
  int ppb = (HW + target_blocks_per_n - 1) / target_blocks_per_n;
  if (ppb < 16) ppb = 16;
  if (N <= 4 && ppb < 64) ppb = 64;
  return ppb;
}

// Dual-source rows (K14: the UNet decoder's torch.cat([h, skip], 1) is never materialised): channel
// c < C1 of pixel `pix` lives in x (rows of C1), channel c >= C1 in x2 (rows of C - C1). Single-source
// calls pass C1 = C. C1 % 8 == 0, so an 8-channel vector never straddles the two sources.
__device__ __forceinline__ const u16* gn_src(const u16* __restrict__ x, const u16* __restrict__ x2, int C, int C1,
                                             size_t pix, int c) {
  return c < C1 ? x + pix * C1 + c : x2 + pix * (size_t)(C - C1) + (c - C1);
}

template <int DT, int KM, int PK = 1>
__global__ __launch_bounds__(GN_THREADS) void gn_partial_kernel(const u16* __restrict__ x, const u16* __restrict__ x2,
                                                               int C1, float* __restrict__ part,
                                                               int HW, int C, int ppb, int nb, int CS) {
  // blockIdx.z selects a channel slice [c0, c0 + CS) (CS <= 2048: the per-lane register budget; gn_slices).
  // KM = 16-byte chunk rounds per lane (ceil(CS / 512)); each wave keeps GN_UNROLL rows of loads in
  // flight before accumulating (one row per wave per trip left the HBM pipe half empty).
  // PK > 1 (narrow rows, CS / 8 <= 64 / PK chunks, KM = 1): the wave's lanes split into PK groups of
  // 64 / PK, each on its own pixel -- a 128-channel row (16 chunks) used a quarter of the lanes and ran
  // the VAE's 1024^2 GroupNorms at ~1.6 TB/s; the groups' sums are combined by shuffles at the end.
  constexpr int GN_UNROLL = 4;
  constexpr int LPG = 64 / PK;   // lanes per pixel group
  const int n = blockIdx.y;
  const int blk = blockIdx.x;
  const int c0 = blockIdx.z * CS;
  const int p0 = blk * ppb;
  const int p1 = min(HW, p0 + ppb);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int lch = PK > 1 ? lane % LPG : lane;   // chunk lane
  const int pg = PK > 1 ? lane / LPG : 0;       // pixel group
  const int nchunk = CS >> 3;
  const size_t pix0 = (size_t)n * HW;
  // shift = the block's first pixel (shared by all 4 waves): keeps the shifted sums well conditioned
  float s1[KM][8], s2[KM][8], sh[KM][8];
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    int ch = lch + 64 * k;
    s16x8 v = {};
    if (ch < nchunk && p0 < p1) v = *reinterpret_cast<const s16x8*>(gn_src(x, x2, C, C1, pix0 + p0, c0 + ch * 8));
#pragma unroll
    for (int j = 0; j < 8; ++j) { sh[k][j] = cvt_in<DT>((u16)v[j]); s1[k][j] = 0.f; s2[k][j] = 0.f; }
  }
  int cnt = 0;
  for (int p = p0 + wave * PK + pg; p < p1; p += 4 * PK * GN_UNROLL) {
    s16x8 buf[GN_UNROLL][KM];
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) {
      const int pu = p + 4 * PK * u;
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        int ch = lch + 64 * k;
        if (pu < p1 && ch < nchunk) buf[u][k] = *reinterpret_cast<const s16x8*>(gn_src(x, x2, C, C1, pix0 + pu, c0 + ch * 8));
      }
    }
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) {
      if (p + 4 * PK * u < p1) {
        cnt++;
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          if (lch + 64 * k < nchunk) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              float d = cvt_in<DT>((u16)buf[u][k][j]) - sh[k][j];
              s1[k][j] += d;
              s2[k][j] += d * d;
            }
          }
        }
      }
    }
  }
  if constexpr (PK > 1) {   // same channels, same shift in every pixel group: plain sums combine
#pragma unroll
    for (int off = LPG; off < 64; off <<= 1) {
      cnt += __shfl_xor(cnt, off);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[0][j] += __shfl_xor(s1[0][j], off);
        s2[0][j] += __shfl_xor(s2[0][j], off);
      }
    }
  }
  // per-wave (mean, M2) per channel -> LDS, then Chan-combine the 4 waves
  extern __shared__ __attribute__((aligned(16))) float gn_smem[];
  float* lmean = gn_smem;             // [4][CS]
  float* lm2 = gn_smem + 4 * CS;      // [4][CS]
  __shared__ int lcnt[4];
  if (lane == 0) lcnt[wave] = cnt;
#pragma unroll
  for (int k = 0; k < KM; ++k) {
    int ch = lch + 64 * k;
    if (ch < nchunk && pg == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float m = 0.f, m2 = 0.f;
        if (cnt > 0) {
          m = sh[k][j] + s1[k][j] / cnt;
          m2 = fmaxf(0.f, s2[k][j] - s1[k][j] * s1[k][j] / cnt);
        }
        lmean[wave * CS + ch * 8 + j] = m;
        lm2[wave * CS + ch * 8 + j] = m2;
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < CS; c += GN_THREADS) {
    float n_a = 0.f, mean = 0.f, m2 = 0.f;
    for (int w = 0; w < 4; ++w) {
      float n_b = (float)lcnt[w];
      if (n_b <= 0.f) continue;
      float mb = lmean[w * CS + c], m2b = lm2[w * CS + c];
      float nn = n_a + n_b;
      float d = mb - mean;
      mean += d * n_b / nn;
      m2 += m2b + d * d * n_a * n_b / nn;
      n_a = nn;
    }
    size_t o = (((size_t)n * nb + blk) * C + c0 + c) * 2;
    part[o] = mean;
    part[o + 1] = m2;
  }
}

// Chan's parallel combine of (count, mean, M2) triples (exact up to fp32 rounding, no cancellation)
__device__ __forceinline__ void chan_merge(float& na, float& ma, float& qa, float nb, float mb, float qb) {
  const float nn = na + nb;
  if (nn <= 0.f) return;
  const float d = mb - ma;
  const float f = nb / nn;
  ma += d * f;
  qa += qb + d * d * na * f;
  na = nn;
}

template <bool STATS_ONLY = false>
__global__ __launch_bounds__(256) void gn_finalize_kernel(const float* __restrict__ part, const void* __restrict__ gamma,
                                                         const void* __restrict__ beta, const void* __restrict__ pre_add,
                                                         float* __restrict__ ab, int HW, int C, int G, int ppb, int nb,
                                                         float eps, int wdt, int pld) {
  // STATS_ONLY (row-sharded GroupNorm, parallel/spatial.py): ab[(n G + g) * 2] = (mean, M2) of this rank's
  // band; the ranks' triples are Chan-combined on the host side and applied by gn_ab_from_stats_kernel.
  // one 256-thread block per (n, g): ONE pass over the per-(block, channel) (mean, M2) partials, each
  // thread Chan-combining its items (all loads of a round issued before any combine), then a Chan tree
  // over the wave (shuffles) and the 4 waves (LDS). (The two-pass form re-read every partial: at batch 1
  // -- 1024 pixel blocks per image -- it was L2-latency bound at ~20 us per GroupNorm.)
  const int g = blockIdx.x;
  const int n = blockIdx.y;
  const int tid = threadIdx.x;
  const int Cg = C / G;
  const int items = Cg * nb;
  __shared__ float red[3][4];
  auto chan_shift = [&](int c) -> float {
    if (!pre_add) return 0.f;
    const size_t i = (size_t)n * pld + c;     // pld: pre_add row stride (a column slice of a wider projection)
    return (wdt == CGS_BF16) ? bf2f(((const u16*)pre_add)[i])
                             : (wdt == CGS_F16 ? h2f(((const u16*)pre_add)[i]) : ((const float*)pre_add)[i]);
  };
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  constexpr int U = 8;
  for (int it0 = tid; it0 < items; it0 += 256 * U) {
    float2 v[U];
    float nbv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = it0 + 256 * u;
      v[u] = make_float2(0.f, 0.f);
      nbv[u] = 0.f;
      if (it < items) {
        const int b = it / Cg, cc = it - b * Cg;
        const int c = g * Cg + cc;
        v[u] = *reinterpret_cast<const float2*>(part + (((size_t)n * nb + b) * C + c) * 2);
        v[u].x += chan_shift(c);
        nbv[u] = (float)(min(HW, b * ppb + ppb) - b * ppb);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) chan_merge(cnt, mean, m2, nbv[u], v[u].x, v[u].y);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float on = __shfl_xor(cnt, off), om = __shfl_xor(mean, off), oq = __shfl_xor(m2, off);
    chan_merge(cnt, mean, m2, on, om, oq);
  }
  if ((tid & 63) == 0) { red[0][tid >> 6] = cnt; red[1][tid >> 6] = mean; red[2][tid >> 6] = m2; }
  __syncthreads();
  cnt = red[0][0]; mean = red[1][0]; m2 = red[2][0];
#pragma unroll
  for (int w = 1; w < 4; ++w) chan_merge(cnt, mean, m2, red[0][w], red[1][w], red[2][w]);
  if constexpr (STATS_ONLY) {
    if (tid == 0) {
      ab[((size_t)n * G + g) * 2] = mean;
      ab[((size_t)n * G + g) * 2 + 1] = m2;
    }
    return;
  }
  const float var = m2 / fmaxf(cnt, 1.f);
  const float rstd = rsqrtf(fmaxf(var, 0.f) + eps);
  for (int cc = tid; cc < Cg; cc += 256) {
    int c = g * Cg + cc;
    float gm = 1.f, bt = 0.f;
    if (gamma) gm = (wdt == CGS_BF16) ? bf2f(((const u16*)gamma)[c]) : (wdt == CGS_F16 ? h2f(((const u16*)gamma)[c]) : ((const float*)gamma)[c]);
    if (beta) bt = (wdt == CGS_BF16) ? bf2f(((const u16*)beta)[c]) : (wdt == CGS_F16 ? h2f(((const u16*)beta)[c]) : ((const float*)beta)[c]);
    float a = rstd * gm;
    ab[((size_t)n * C + c) * 2] = a;
    ab[((size_t)n * C + c) * 2 + 1] = (chan_shift(c) - mean) * a + bt;
  }
}

template <int DT, bool SILU>
__global__ __launch_bounds__(256) void gn_apply_kernel(const u16* __restrict__ x, const u16* __restrict__ x2, int C1,
                                                      u16* __restrict__ y,
                                                      const float* __restrict__ ab, int rows_total, int rows_per_iter,
                                                      int HW, int C) {
  // The grid stride is a whole number of rows, so every thread keeps ONE 8-channel chunk for its whole
  // life: its 16 affine coefficients stay in registers and are reloaded only when the image index n
  // changes (no 64-bit index divisions, no per-element coefficient loads).
  const int cpr = C >> 3;
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= rows_per_iter * cpr) return;
  const int ch = tid % cpr;
  int cur_n = -1;
  float a[8], bb[8];
  auto coef = [&](int n) {
    if (n != cur_n) {
      cur_n = n;
      const float4* abp = reinterpret_cast<const float4*>(ab + ((size_t)n * C + ch * 8) * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float4 t = abp[j];
        a[2 * j] = t.x; bb[2 * j] = t.y; a[2 * j + 1] = t.z; bb[2 * j + 1] = t.w;
      }
    }
  };
  auto apply = [&](int row, const s16x8& v) {
    coef(row / HW);
    s16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = cvt_in<DT>((u16)v[j]) * a[j] + bb[j];
      if (SILU) f = silu_f(f);
      o[j] = (short)cvt_out<DT>(f);
    }
    reinterpret_cast<s16x8*>(y)[(size_t)row * cpr + ch] = o;
  };
  // two rows per trip, both loads issued before either is used (one 16-B load in flight per lane left
  // the big VAE GroupNorms at ~2.3 TB/s)
  int row = tid / cpr;
  for (; row + rows_per_iter < rows_total; row += 2 * rows_per_iter) {
    const s16x8 v0 = *reinterpret_cast<const s16x8*>(gn_src(x, x2, C, C1, (size_t)row, ch * 8));
    const s16x8 v1 = *reinterpret_cast<const s16x8*>(gn_src(x, x2, C, C1, (size_t)(row + rows_per_iter), ch * 8));
    apply(row, v0);
    apply(row + rows_per_iter, v1);
  }
  if (row < rows_total) apply(row, *reinterpret_cast<const s16x8*>(gn_src(x, x2, C, C1, (size_t)row, ch * 8)));
}

// LayerNorm row statistics from GEMM-epilogue partials (pq::run RSO): part [M][P] (mean, M2) of 80 columns
// each -> rs [M] (mean, rstd) by Chan's combine (no cancellation), one thread per row.
// PV > 0 (P even, P <= 2 PV): the row's partials as PV 16-B loads, all issued before the combine (the loop form
// below waited one dependent 8-B load per chunk: ~5.6 us per call at SDXL sizes, one call per LayerNorm).
template <int PV>
__global__ __launch_bounds__(256) void ln_rs_from_partials_kernel(const float* __restrict__ part, float* __restrict__ rs,
                                                                  int M, int P, float eps) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= M) return;
  float n, mean, m2;
  auto chan = [&](float vm, float vq) {
    const float nn = n + 80.f, d = vm - mean, f = 80.f / nn;
    mean += d * f;
    m2 += vq + d * d * n * f;
    n = nn;
  };
  if constexpr (PV > 0) {
    const float4* p = reinterpret_cast<const float4*>(part) + (long long)row * (P >> 1);
    float4 v[PV];
#pragma unroll
    for (int c = 0; c < PV; ++c) v[c] = 2 * c < P ? p[c] : float4{0.f, 0.f, 0.f, 0.f};
    n = 80.f, mean = v[0].x, m2 = v[0].y;
    chan(v[0].z, v[0].w);
#pragma unroll
    for (int c = 1; c < PV; ++c)
      if (2 * c < P) {
        chan(v[c].x, v[c].y);
        chan(v[c].z, v[c].w);
      }
  } else {
    const float2* p = reinterpret_cast<const float2*>(part) + (long long)row * P;
    n = 80.f, mean = p[0].x, m2 = p[0].y;
    for (int c = 1; c < P; ++c) chan(p[c].x, p[c].y);
  }
  reinterpret_cast<float2*>(rs)[row] = float2{mean, rsqrtf(m2 / n + eps)};
}

CGS_EXPORT int cgs_ln_rs_from_partials(const float* part, float* rs, int M, int P, float eps, hipStream_t stream) {
  if (M <= 0 || P <= 0) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((M + 255) / 256);
  const bool vec = P % 2 == 0 && ((uintptr_t)part & 15) == 0;
  if (vec && P <= 8) ln_rs_from_partials_kernel<4><<<grid, 256, 0, stream>>>(part, rs, M, P, eps);
  else if (vec && P <= 16) ln_rs_from_partials_kernel<8><<<grid, 256, 0, stream>>>(part, rs, M, P, eps);
  else ln_rs_from_partials_kernel<0><<<grid, 256, 0, stream>>>(part, rs, M, P, eps);
  return (int)hipGetLastError();
}

CGS_EXPORT long long cgs_groupnorm_workspace(int N, int HW, int C) {
  int ppb = gn_pix_per_block(N, HW);
  int nb = (HW + ppb - 1) / ppb;
  return (long long)N * nb * C * 2 * 4 + (long long)N * C * 2 * 4 + 256;
}

static int gn_apply_launch(const void* x, const void* x2, int C1, void* y, const float* ab, int N, int HW, int C,
                           int silu, int dtype, hipStream_t stream);

// Channel slices of the statistics pass (blockIdx.z). Up to 512 channels a slice is the whole row, 513-1024 two
// halves (KM = 1 each); wider rows are cut into equal 8-aligned slices of <= 512 channels whose chunk count fills
// the wave (KM = 1, or the pixel-packed PK forms): the KM = 2..4 forms held 112-210 VGPRs. Full GroupNorm + SiLU
// at SDXL sizes (profiles/r06/gn_slices_ab.log, gn_mid_ab.log): C = 1920 at 64^2 269 -> 219 us, C = 2560 at
// 32^2 78 -> 68 us, C = 1280 48 -> 45 us, C = 640 68 -> 63 us (its 128-channel PK slices measured 71 us).
static int gn_slices(int C) {
  const int ns0 = (C + 2047) / 2048;
  if (C > 512 && C <= 1024 && C % 16 == 0) return 2;   // two KM = 1 slices: C = 640 68.2 -> 63.4 us (gn_mid_ab.log)
  if (C <= 1024 || C % 8) return ns0;
  const int tot = C / 8;
  int best = ns0;
  float bu = -1.f;
  for (int ns = (C + 511) / 512; ns <= tot; ++ns) {
    if (tot % ns) continue;
    const int nch = tot / ns;
    const int lanes = nch <= 8 ? 8 : nch <= 16 ? 16 : nch <= 32 ? 32 : 64;
    const float u = (float)nch / (float)lanes;
    if (u >= 0.9f) return ns;
    if (u > bu) { bu = u; best = ns; }
  }
  return best;
}

// x, y: [N, HW, C] (NHWC); gamma/beta [C] in the activation dtype; pre_add [N, C] (act dtype) or null.
// ws: workspace of cgs_groupnorm_workspace() bytes (torch-allocated so it is graph-capturable).
static int groupnorm_impl(const void* x, const void* x2, int C1, void* y, const void* gamma, const void* beta,
                          const void* pre_add, void* ws, int N, int HW, int C, int G, float eps, int silu, int dtype,
                          hipStream_t stream, int pld) {
  const int ns = gn_slices(C);      // equal, 8-aligned channel slices
  if (C % 8 || C % G || C % (8 * ns) || C > 8192 || C1 % 8 || C1 > C) return (int)hipErrorInvalidValue;
  const int CS = C / ns;
  int ppb = gn_pix_per_block(N, HW);
  int nb = (HW + ppb - 1) / ppb;
  float* part = (float*)ws;
  float* ab = part + (size_t)N * nb * C * 2;
  dim3 g1(nb, N, ns);
  const int km = (CS / 8 + 63) / 64;  // 1..4
#define CGS_GN_PARTIAL(KMV)                                                                                     \
  if (dtype == CGS_BF16)                                                                                        \
    gn_partial_kernel<CGS_BF16, KMV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS); \
  else                                                                                                          \
    gn_partial_kernel<CGS_F16, KMV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS);
#define CGS_GN_PARTIAL_PK(PKV)                                                                                  \
  if (dtype == CGS_BF16)                                                                                        \
    gn_partial_kernel<CGS_BF16, 1, PKV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS); \
  else                                                                                                          \
    gn_partial_kernel<CGS_F16, 1, PKV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS);
  const int nch = CS / 8;
  if (nch <= 8) { CGS_GN_PARTIAL_PK(8) }
  else if (nch <= 16) { CGS_GN_PARTIAL_PK(4) }
  else if (nch <= 32) { CGS_GN_PARTIAL_PK(2) }
  else if (km == 1) { CGS_GN_PARTIAL(1) } else if (km == 2) { CGS_GN_PARTIAL(2) } else if (km == 3) { CGS_GN_PARTIAL(3) } else { CGS_GN_PARTIAL(4) }
#undef CGS_GN_PARTIAL
#undef CGS_GN_PARTIAL_PK
  gn_finalize_kernel<<<dim3(G, N), 256, 0, stream>>>(part, gamma, beta, pre_add, ab, HW, C, G, ppb, nb, eps, dtype,
                                                    pld);
  return gn_apply_launch(x, x2, C1, y, ab, N, HW, C, silu, dtype, stream);
}

// The statistics half of groupnorm_impl: per-(n, g) (mean, M2) of the given rows into stats [N][G][2].
static int groupnorm_stats_impl(const void* x, const void* x2, int C1, const void* pre_add, void* ws, float* stats,
                                int N, int HW, int C, int G, int dtype, hipStream_t stream) {
  const int ns = gn_slices(C);
  if (C % 8 || C % G || C % (8 * ns) || C > 8192 || C1 % 8 || C1 > C) return (int)hipErrorInvalidValue;
  const int CS = C / ns;
  int ppb = gn_pix_per_block(N, HW);
  int nb = (HW + ppb - 1) / ppb;
  float* part = (float*)ws;
  dim3 g1(nb, N, ns);
  const int km = (CS / 8 + 63) / 64;
  const int nch = CS / 8;
#define CGS_GN_PARTIAL(KMV, PKV)                                                                                \
  if (dtype == CGS_BF16)                                                                                        \
    gn_partial_kernel<CGS_BF16, KMV, PKV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS); \
  else                                                                                                          \
    gn_partial_kernel<CGS_F16, KMV, PKV><<<g1, GN_THREADS, 8 * CS * sizeof(float), stream>>>((const u16*)x, (const u16*)x2, C1, part, HW, C, ppb, nb, CS);
  if (nch <= 8) { CGS_GN_PARTIAL(1, 8) }
  else if (nch <= 16) { CGS_GN_PARTIAL(1, 4) }
  else if (nch <= 32) { CGS_GN_PARTIAL(1, 2) }
  else if (km == 1) { CGS_GN_PARTIAL(1, 1) } else if (km == 2) { CGS_GN_PARTIAL(2, 1) }
  else if (km == 3) { CGS_GN_PARTIAL(3, 1) } else { CGS_GN_PARTIAL(4, 1) }
#undef CGS_GN_PARTIAL
  gn_finalize_kernel<true><<<dim3(G, N), 256, 0, stream>>>(part, nullptr, nullptr, pre_add, stats, HW, C, G, ppb, nb,
                                                          0.f, dtype, C);
  return (int)hipGetLastError();
}

// (mean, rstd) per (n, g) -> the per-(n, c) affine of gn_apply (gamma / beta / pre-add folded as in finalize).
__global__ __launch_bounds__(256) void gn_ab_from_stats_kernel(const float* __restrict__ mr, const void* __restrict__ gamma,
                                                               const void* __restrict__ beta,
                                                               const void* __restrict__ pre_add, float* __restrict__ ab,
                                                               int N, int C, int G, int wdt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C, g = c / (C / G);
  auto ld = [&](const void* p, int idx) -> float {
    return (wdt == CGS_BF16) ? bf2f(((const u16*)p)[idx]) : (wdt == CGS_F16 ? h2f(((const u16*)p)[idx]) : ((const float*)p)[idx]);
  };
  const float mean = mr[((size_t)n * G + g) * 2], rstd = mr[((size_t)n * G + g) * 2 + 1];
  const float gm = gamma ? ld(gamma, c) : 1.f, bt = beta ? ld(beta, c) : 0.f;
  const float sh = pre_add ? ld(pre_add, n * C + c) : 0.f;
  const float a = rstd * gm;
  ab[(size_t)i * 2] = a;
  ab[(size_t)i * 2 + 1] = (sh - mean) * a + bt;
}

// Row-sharded GroupNorm (latency mode, parallel/spatial.py), step 1: this rank's band statistics.
// x ([N, HW, C1]) / x2 ([N, HW, C - C1], or null: C1 = C) NHWC; pre_add [N, C] or null; ws of
// cgs_groupnorm_workspace(N, HW, C) bytes; stats out: [N][G] (mean, M2) over the band (count = HW * C / G).
CGS_EXPORT int cgs_groupnorm_band_stats(const void* x, const void* x2, int C1, const void* pre_add, void* ws,
                                        float* stats, int N, int HW, int C, int G, int dtype, hipStream_t stream) {
  if (!stats || !ws || HW <= 0) return (int)hipErrorInvalidValue;
  return groupnorm_stats_impl(x, x2 ? x2 : nullptr, x2 ? C1 : C, pre_add, ws, stats, N, HW, C, G, dtype, stream);
}

// Step 2 (after the ranks' (mean, M2) were combined): y = GN(x) with the given per-(n, g) (mean, rstd).
// ab: N * C * 2 floats of workspace.
CGS_EXPORT int cgs_groupnorm_apply_stats(const void* x, const void* x2, int C1, void* y, const void* gamma,
                                         const void* beta, const void* pre_add, const float* mean_rstd, float* ab,
                                         int N, int HW, int C, int G, int silu, int dtype, hipStream_t stream) {
  if (C % 8 || C % G || !mean_rstd || !ab || (x2 && (C1 % 8 || C1 > C))) return (int)hipErrorInvalidValue;
  gn_ab_from_stats_kernel<<<(unsigned)((N * C + 255) / 256), 256, 0, stream>>>(mean_rstd, gamma, beta, pre_add, ab, N,
                                                                              C, G, dtype);
  return gn_apply_launch(x, x2, x2 ? C1 : C, y, ab, N, HW, C, silu, dtype, stream);
}

static int gn_apply_launch(const void* x, const void* x2, int C1, void* y, const float* ab, int N, int HW, int C,
                           int silu, int dtype, hipStream_t stream) {
  const int cpr = C / 8;
  const long long rows_total = (long long)N * HW;
  if (rows_total == 0) return (int)hipGetLastError();
  if (rows_total * cpr >= (1LL << 31)) return (int)hipErrorInvalidValue;
  long long chunks = rows_total * cpr;
  long long nbk = (chunks + 255) / 256;
  int blocks = (int)(nbk < 8192 ? nbk : 8192);
  int rows_per_iter = (blocks * 256) / cpr;  // cpr <= 1024 <= blocks * 256 whenever chunks >= cpr
  if (rows_per_iter < 1) rows_per_iter = 1, blocks = (cpr + 255) / 256;
  if (dtype == CGS_BF16) {
    if (silu) gn_apply_kernel<CGS_BF16, true><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)x2, C1, (u16*)y, ab, (int)rows_total, rows_per_iter, HW, C);
    else gn_apply_kernel<CGS_BF16, false><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)x2, C1, (u16*)y, ab, (int)rows_total, rows_per_iter, HW, C);
  } else {
    if (silu) gn_apply_kernel<CGS_F16, true><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)x2, C1, (u16*)y, ab, (int)rows_total, rows_per_iter, HW, C);
    else gn_apply_kernel<CGS_F16, false><<<blocks, 256, 0, stream>>>((const u16*)x, (const u16*)x2, C1, (u16*)y, ab, (int)rows_total, rows_per_iter, HW, C);
  }
  return (int)hipGetLastError();
}

// GroupNorm whose statistics pass already ran in the producer's epilogue (cgs_conv2d_nhwc_gns): part =
// [N, HW / ppb, C] (mean, M2) partials of ppb pixels each; only finalize + apply run. ab: N * C * 2 floats.
CGS_EXPORT int cgs_groupnorm_nhwc_part(const void* x, void* y, const void* gamma, const void* beta, const void* pre_add,
                                       const float* part, float* ab, int N, int HW, int C, int G, int ppb, float eps,
                                       int silu, int dtype, hipStream_t stream) {
  if (C % 8 || C % G || ppb <= 0 || HW % ppb || !part || !ab) return (int)hipErrorInvalidValue;
  const int nb = HW / ppb;
  gn_finalize_kernel<<<dim3(G, N), 256, 0, stream>>>(part, gamma, beta, pre_add, ab, HW, C, G, ppb, nb, eps, dtype, C);
  return gn_apply_launch(x, nullptr, C, y, ab, N, HW, C, silu, dtype, stream);
}

CGS_EXPORT int cgs_groupnorm_nhwc_ws(const void* x, void* y, const void* gamma, const void* beta, const void* pre_add,
                                     void* ws, int N, int HW, int C, int G, float eps, int silu, int dtype,
                                     hipStream_t stream) {
  return groupnorm_impl(x, nullptr, C, y, gamma, beta, pre_add, ws, N, HW, C, G, eps, silu, dtype, stream, C);
}

// GroupNorm over the channel concat of x ([N, HW, C1]) and x2 ([N, HW, C - C1]) without materialising it.
CGS_EXPORT int cgs_groupnorm_nhwc_dual(const void* x, const void* x2, int C1, void* y, const void* gamma,
                                       const void* beta, const void* pre_add, void* ws, int N, int HW, int C, int G,
                                       float eps, int silu, int dtype, hipStream_t stream) {
  return groupnorm_impl(x, x2, C1, y, gamma, beta, pre_add, ws, N, HW, C, G, eps, silu, dtype, stream, C);
}

// The same three entry points with a row stride ``pld`` (elements, >= C) for pre_add: the UNet's ResBlock
// time-embedding projections are ONE GEMM per forward ([N, sum of the blocks' C]) and each block's GroupNorm
// reads its column slice in place (models/unet.py, UNetModel._emb_proj).
CGS_EXPORT int cgs_groupnorm_nhwc_ws_pld(const void* x, void* y, const void* gamma, const void* beta,
                                         const void* pre_add, int pld, void* ws, int N, int HW, int C, int G, float eps,
                                         int silu, int dtype, hipStream_t stream) {
  if (pre_add && pld < C) return (int)hipErrorInvalidValue;
  return groupnorm_impl(x, nullptr, C, y, gamma, beta, pre_add, ws, N, HW, C, G, eps, silu, dtype, stream, pld);
}

CGS_EXPORT int cgs_groupnorm_nhwc_dual_pld(const void* x, const void* x2, int C1, void* y, const void* gamma,
                                           const void* beta, const void* pre_add, int pld, void* ws, int N, int HW,
                                           int C, int G, float eps, int silu, int dtype, hipStream_t stream) {
  if (pre_add && pld < C) return (int)hipErrorInvalidValue;
  return groupnorm_impl(x, x2, C1, y, gamma, beta, pre_add, ws, N, HW, C, G, eps, silu, dtype, stream, pld);
}

CGS_EXPORT int cgs_groupnorm_nhwc_part_pld(const void* x, void* y, const void* gamma, const void* beta,
                                           const void* pre_add, int pld, const float* part, float* ab, int N, int HW,
                                           int C, int G, int ppb, float eps, int silu, int dtype, hipStream_t stream) {
  if (C % 8 || C % G || ppb <= 0 || HW % ppb || !part || !ab || (pre_add && pld < C)) return (int)hipErrorInvalidValue;
  const int nb = HW / ppb;
  gn_finalize_kernel<<<dim3(G, N), 256, 0, stream>>>(part, gamma, beta, pre_add, ab, HW, C, G, ppb, nb, eps, dtype,
                                                    pld);
  return gn_apply_launch(x, nullptr, C, y, ab, N, HW, C, silu, dtype, stream);
}

// ------------------------------------------------------------------------------------------------
// LayerNorm over the last dim; one wave per row.
// ------------------------------------------------------------------------------------------------
#define LN_MAXK 8  // chunks of 8 per lane -> C <= 4096 in registers

template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
  // butterfly over the LPR lanes of one row (LPR-aligned lane groups of the 64-wide wave)
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LPR lanes per row (64/LPR rows per wave): SDXL's C=640 rows are 80 16-byte chunks = 5 per lane at
// LPR=16 and C=1280 rows 5 per lane at LPR=32, so every lane slot carries data (one row per full wave
// would leave 37-75 % of the second chunk round idle) and the shuffle reductions are shorter.
template <int DT, int LPR>
__global__ __launch_bounds__(256) void layernorm_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                       const u16* __restrict__ w, const u16* __restrict__ b, int rows,
                                                       int C, float eps) {
  constexpr int RPB = 256 / LPR;  // rows per block
  const int lane = threadIdx.x % LPR;
  const int row = blockIdx.x * RPB + threadIdx.x / LPR;
  const bool live = row < rows;   // dead rows still join the shuffles (whole wave stays converged)
  const int nch = C >> 3;
  const u16* xr = x + (size_t)(live ? row : 0) * C;
  float v[LN_MAXK][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    int ch = lane + LPR * k;
    if (live && ch < nch) {
      s16x8 t = reinterpret_cast<const s16x8*>(xr)[ch];
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[k][j] = cvt_in<DT>((u16)t[j]); s += v[k][j]; }
    }
  }
  float mean = group_sum<LPR>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    int ch = lane + LPR * k;
    if (live && ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[k][j] - mean; q += d * d; }
    }
  }
  float rstd = rsqrtf(group_sum<LPR>(q) / C + eps);
  if (!live) return;
  u16* yr = y + (size_t)row * C;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    int ch = lane + LPR * k;
    if (ch < nch) {
      s16x8 wv, bv;
      if (w) wv = reinterpret_cast<const s16x8*>(w)[ch];
      if (b) bv = reinterpret_cast<const s16x8*>(b)[ch];
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = (v[k][j] - mean) * rstd * (w ? cvt_in<DT>((u16)wv[j]) : 1.f) + (b ? cvt_in<DT>((u16)bv[j]) : 0.f);
        o[j] = (short)cvt_out<DT>(f);
      }
      reinterpret_cast<s16x8*>(yr)[ch] = o;
    }
  }
}


// Per-image channel affine followed by a LayerNorm without affine, one pass: xa = x * (add + sc[n, c]) +
// sh[n, c] (rounded to the storage dtype: the tensor the block's residual path reads) is written, and
// y = LN(xa) from the same registers. Stable Cascade TimestepBlock -> AttnBlock (``x * (1 + a) + b``, then
// the attention's LayerNorm2d): one read of x instead of chan_affine's read + write and LayerNorm's
// second read. sc / sh: [N, C] rows with stride ld (the halves of the mapper GEMM output).
template <int DT, int LPR>
__global__ __launch_bounds__(256) void affine_layernorm_kernel(const u16* __restrict__ x, const u16* __restrict__ sc,
                                                               const u16* __restrict__ sh, long long ld, float add,
                                                               u16* __restrict__ xa, u16* __restrict__ y, int rows,
                                                               int HW, int C, float eps) {
  constexpr int RPB = 256 / LPR;
  const int lane = threadIdx.x % LPR;
  const int row = blockIdx.x * RPB + threadIdx.x / LPR;
  const bool live = row < rows;   // dead rows still join the shuffles (whole wave stays converged)
  const int nch = C >> 3;
  const size_t ro = (size_t)(live ? row : 0) * C;
  const long long n = (live ? row : 0) / HW;
  float v[LN_MAXK][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    const int ch = lane + LPR * k;
    if (live && ch < nch) {
      const s16x8 t = reinterpret_cast<const s16x8*>(x + ro)[ch];
      const s16x8 a = *reinterpret_cast<const s16x8*>(sc + n * ld + ch * 8);
      const s16x8 b = *reinterpret_cast<const s16x8*>(sh + n * ld + ch * 8);
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (short)cvt_out<DT>(__builtin_fmaf(cvt_in<DT>((u16)t[j]), add + cvt_in<DT>((u16)a[j]), cvt_in<DT>((u16)b[j])));
        v[k][j] = cvt_in<DT>((u16)o[j]);
        s += v[k][j];
      }
      reinterpret_cast<s16x8*>(xa + ro)[ch] = o;
    }
  }
  const float mean = group_sum<LPR>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    const int ch = lane + LPR * k;
    if (live && ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[k][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(group_sum<LPR>(q) / C + eps);
  if (!live) return;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    const int ch = lane + LPR * k;
    if (ch < nch) {
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (short)cvt_out<DT>((v[k][j] - mean) * rstd);
      reinterpret_cast<s16x8*>(y + ro)[ch] = o;
    }
  }
}

CGS_EXPORT int cgs_affine_layernorm(const void* x, const void* scale, const void* shift, long long ld, float add,
                                    void* xa, void* y, int N, int HW, int C, float eps, int dtype,
                                    hipStream_t stream) {
  if (N <= 0 || HW <= 0) return 0;
  const int nch = C / 8;
  if (C % 8 || ld % 8 || nch > 64 * LN_MAXK || dtype == CGS_F32 ||
      (((uintptr_t)x | (uintptr_t)xa | (uintptr_t)y | (uintptr_t)scale | (uintptr_t)shift) & 15))
    return (int)hipErrorInvalidValue;
  const long long rows = (long long)N * HW;
  if (rows >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int lpr = nch <= 8 * LN_MAXK ? 8 : nch <= 16 * LN_MAXK ? 16 : nch <= 32 * LN_MAXK ? 32 : 64;
  const dim3 grid((unsigned)((rows + 256 / lpr - 1) / (256 / lpr)));
#define CGS_ALN(L)                                                                                                  \
  if (dtype == CGS_BF16)                                                                                            \
    affine_layernorm_kernel<CGS_BF16, L><<<grid, 256, 0, stream>>>((const u16*)x, (const u16*)scale, (const u16*)shift, \
                                                                   ld, add, (u16*)xa, (u16*)y, (int)rows, HW, C, eps); \
  else                                                                                                              \
    affine_layernorm_kernel<CGS_F16, L><<<grid, 256, 0, stream>>>((const u16*)x, (const u16*)scale, (const u16*)shift, \
                                                                  ld, add, (u16*)xa, (u16*)y, (int)rows, HW, C, eps);
  if (lpr == 8) { CGS_ALN(8) } else if (lpr == 16) { CGS_ALN(16) } else if (lpr == 32) { CGS_ALN(32) } else { CGS_ALN(64) }
#undef CGS_ALN
  return (int)hipGetLastError();
}

// Row statistics only (the LayerNorm folded into the next GEMM's epilogue, MC_EPI_LNFOLD):
// rs[2r] = mean, rs[2r+1] = rstd of row r. Same row-group layout and reductions as layernorm_kernel.
template <int DT, int LPR>
__global__ __launch_bounds__(256) void ln_stats_kernel(const u16* __restrict__ x, float* __restrict__ rs, int rows,
                                                      int C, float eps) {
  constexpr int RPB = 256 / LPR;
  const int lane = threadIdx.x % LPR;
  const int row = blockIdx.x * RPB + threadIdx.x / LPR;
  const bool live = row < rows;
  const int nch = C >> 3;
  const u16* xr = x + (size_t)(live ? row : 0) * C;
  float v[LN_MAXK][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    int ch = lane + LPR * k;
    if (live && ch < nch) {
      s16x8 t = reinterpret_cast<const s16x8*>(xr)[ch];
#pragma unroll
      for (int j = 0; j < 8; ++j) { v[k][j] = cvt_in<DT>((u16)t[j]); s += v[k][j]; }
    }
  }
  const float mean = group_sum<LPR>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < LN_MAXK; ++k) {
    int ch = lane + LPR * k;
    if (live && ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = v[k][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(group_sum<LPR>(q) / C + eps);
  if (live && lane == 0) reinterpret_cast<float2*>(rs)[row] = float2{mean, rstd};
}

template <int DT>
__global__ __launch_bounds__(256) void layernorm_big_kernel(const u16* __restrict__ x, u16* __restrict__ y,
                                                           const u16* __restrict__ w, const u16* __restrict__ b,
                                                           int rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const u16* xr = x + (size_t)row * C;
  float s = 0.f;
  for (int i = lane; i < C; i += 64) s += cvt_in<DT>(xr[i]);
  float mean = wave_sum(s) / C;
  float q = 0.f;
  for (int i = lane; i < C; i += 64) { float d = cvt_in<DT>(xr[i]) - mean; q += d * d; }
  float rstd = rsqrtf(wave_sum(q) / C + eps);
  u16* yr = y + (size_t)row * C;
  for (int i = lane; i < C; i += 64)
    yr[i] = cvt_out<DT>((cvt_in<DT>(xr[i]) - mean) * rstd * (w ? cvt_in<DT>(w[i]) : 1.f) + (b ? cvt_in<DT>(b[i]) : 0.f));
}

CGS_EXPORT int cgs_layernorm(const void* x, void* y, const void* w, const void* b, int rows, int C, float eps,
                             int dtype, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  const int nch = C / 8;
  if (nch <= 64 * LN_MAXK) {
    // fewest lanes per row that still fits the row in LN_MAXK chunks per lane
    const int lpr = nch <= 8 * LN_MAXK ? 8 : nch <= 16 * LN_MAXK ? 16 : nch <= 32 * LN_MAXK ? 32 : 64;
    dim3 grid((rows + 256 / lpr - 1) / (256 / lpr));
#define CGS_LN_LAUNCH(L)                                                                                           \
  if (dtype == CGS_BF16)                                                                                           \
    layernorm_kernel<CGS_BF16, L><<<grid, 256, 0, stream>>>((const u16*)x, (u16*)y, (const u16*)w, (const u16*)b, rows, C, eps); \
  else                                                                                                             \
    layernorm_kernel<CGS_F16, L><<<grid, 256, 0, stream>>>((const u16*)x, (u16*)y, (const u16*)w, (const u16*)b, rows, C, eps);
    if (lpr == 8) { CGS_LN_LAUNCH(8) } else if (lpr == 16) { CGS_LN_LAUNCH(16) } else if (lpr == 32) { CGS_LN_LAUNCH(32) } else { CGS_LN_LAUNCH(64) }
#undef CGS_LN_LAUNCH
  } else {
    dim3 grid((rows + 3) / 4);
    if (dtype == CGS_BF16)
      layernorm_big_kernel<CGS_BF16><<<grid, 256, 0, stream>>>((const u16*)x, (u16*)y, (const u16*)w, (const u16*)b, rows, C, eps);
    else
      layernorm_big_kernel<CGS_F16><<<grid, 256, 0, stream>>>((const u16*)x, (u16*)y, (const u16*)w, (const u16*)b, rows, C, eps);
  }
  return (int)hipGetLastError();
}

// Depthwise k x k conv (stride 1, 'same' zeros / replicate padding) on NHWC with the LayerNorm statistics
// of every output pixel over C in the same pass (Stable Cascade ResBlock: depthwise -> LayerNorm2d ->
// ChannelMLP, common.py ResBlock): LPR lanes per pixel, each lane keeps its <= LN_MAXK 8-channel output
// chunks in registers (rounded to the output dtype, i.e. the values the next GEMM reads), writes them and
// forms (mean, rstd) by an exact two-pass over the registers -> rs [pixels, 2] (cgs_layernorm_stats layout).
// The folded-LayerNorm GEMM (MC_EPI_LNFOLD) then needs no separate statistics pass over the tensor.
template <int DT, int KF, int LPR>
__global__ __launch_bounds__(256) void dwconv_ln_stats_kernel(const u16* __restrict__ x, const u16* __restrict__ wt,
                                                              const u16* __restrict__ b, u16* __restrict__ y,
                                                              float* __restrict__ rs, int N, int H, int W, int C,
                                                              int kr, int replicate, float eps) {
  constexpr int RPB = 256 / LPR;
  const int lane = threadIdx.x % LPR;
  const unsigned npix = (unsigned)N * H * W;
  const unsigned pix = blockIdx.x * RPB + threadIdx.x / LPR;
  const bool live = pix < npix;
  const unsigned pp = live ? pix : 0u;
  const int wo = (int)(pp % (unsigned)W);
  const unsigned t = pp / (unsigned)W;
  const int ho = (int)(t % (unsigned)H);
  const int n = (int)(t / (unsigned)H);
  const int nch = C >> 3;
  const int k = KF ? KF : kr;
  const int p = k >> 1;
  float v[LN_MAXK][8];
  float s = 0.f;
#pragma unroll
  for (int kk = 0; kk < LN_MAXK; ++kk) {
    const int ch = lane + LPR * kk;
    if (live && ch < nch) {
      float acc[8];
      if (b) {
        const s16x8 bv = reinterpret_cast<const s16x8*>(b)[ch];
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
          const s16x8 xv = *reinterpret_cast<const s16x8*>(x + (((size_t)n * H + hi) * W + wi) * C + ch * 8);
          const s16x8 wv = *reinterpret_cast<const s16x8*>(wt + (size_t)(di * k + dj) * C + ch * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += cvt_in<DT>((u16)xv[j]) * cvt_in<DT>((u16)wv[j]);
        }
      }
      s16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = (short)cvt_out<DT>(acc[j]);
        v[kk][j] = cvt_in<DT>((u16)o[j]);
        s += v[kk][j];
      }
      *reinterpret_cast<s16x8*>(y + (size_t)pix * C + ch * 8) = o;
    }
  }
  const float mean = group_sum<LPR>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int kk = 0; kk < LN_MAXK; ++kk) {
    const int ch = lane + LPR * kk;
    if (live && ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = v[kk][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(group_sum<LPR>(q) / C + eps);
  if (live && lane == 0) reinterpret_cast<float2*>(rs)[pix] = float2{mean, rstd};
}

CGS_EXPORT int cgs_dwconv_ln_stats_nhwc(const void* x, const void* wt, const void* b, void* y, float* rs, int N, int H,
                                        int W, int C, int k, int replicate, float eps, int dtype, hipStream_t stream) {
  if (C % 8 || C / 8 > 32 * LN_MAXK || (k & 1) == 0 || k > 15 || dtype == CGS_F32) return (int)hipErrorInvalidValue;
  const long long npix = (long long)N * H * W;
  if (npix <= 0) return 0;
  if (npix * C >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int nch = C / 8;
  const int L = nch <= 8 * LN_MAXK ? 8 : (nch <= 16 * LN_MAXK ? 16 : 32);
#define CGS_DWL(DTV, KV, LPRV)                                                                                     \
  dwconv_ln_stats_kernel<DTV, KV, LPRV><<<(unsigned)((npix + 256 / LPRV - 1) / (256 / LPRV)), 256, 0, stream>>>( \
      (const u16*)x, (const u16*)wt, (const u16*)b, (u16*)y, rs, N, H, W, C, k, replicate, eps)
#define CGS_DWL_K(DTV, LPRV)                                          \
  do {                                                                \
    if (k == 3) CGS_DWL(DTV, 3, LPRV);                                \
    else if (k == 7) CGS_DWL(DTV, 7, LPRV);                           \
    else CGS_DWL(DTV, 0, LPRV);                                       \
  } while (0)
#define CGS_DWL_L(DTV)                                                \
  do {                                                                \
    if (L == 8) CGS_DWL_K(DTV, 8);                                    \
    else if (L == 16) CGS_DWL_K(DTV, 16);                             \
    else CGS_DWL_K(DTV, 32);                                          \
  } while (0)
  if (dtype == CGS_BF16) CGS_DWL_L(CGS_BF16);
  else CGS_DWL_L(CGS_F16);
#undef CGS_DWL_L
#undef CGS_DWL_K
#undef CGS_DWL
  return (int)hipGetLastError();
}

// (mean, rstd) per row of x [rows, C] (C % 8 == 0, C <= the register-resident LayerNorm limit)
CGS_EXPORT int cgs_layernorm_stats(const void* x, float* rs, int rows, int C, float eps, int dtype, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (C % 8 || C / 8 > 32 * LN_MAXK) return (int)hipErrorInvalidValue;
  const int nch = C / 8;
  const int L = nch <= 16 * LN_MAXK ? (nch <= 8 * LN_MAXK ? 8 : 16) : 32;
#define CGS_LNS(LPR) \
  do { \
    const int grid = (rows + (256 / LPR) - 1) / (256 / LPR); \
    if (dtype == CGS_BF16) ln_stats_kernel<CGS_BF16, LPR><<<grid, 256, 0, stream>>>((const u16*)x, rs, rows, C, eps); \
    else if (dtype == CGS_F16) ln_stats_kernel<CGS_F16, LPR><<<grid, 256, 0, stream>>>((const u16*)x, rs, rows, C, eps); \
    else return (int)hipErrorInvalidValue; \
  } while (0)
  if (L == 8) CGS_LNS(8);
  else if (L == 16) CGS_LNS(16);
  else CGS_LNS(32);
#undef CGS_LNS
  return (int)hipGetLastError();
}
