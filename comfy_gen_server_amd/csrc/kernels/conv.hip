// NHWC implicit-GEMM convolution for gfx950 (K09 conv3x3 s1/s2, K10 conv1x1, K12 upsample+conv,
// K14 skip-concat + conv, K15 residual epilogue). Reference semantics: torch.nn.Conv2d as used by
// comfy/ldm/modules/diffusionmodules/openaimodel.py (ResBlock, Down/Upsample) and model.py (VAE).
//
//   out[n,oy,ox,co] = bias[co] + sum_{ky,kx,ci} in[n, oy*s+ky-p, ox*s+kx-p, ci] * w[co,ky,kx,ci] (+ res)
// GEMM view: M = N*Ho*Wo output pixels, Ncols = Cout, K = kh*kw*Cin; weights pre-permuted to
// [Cout][kh][kw][Cin] (K-contiguous, like nn.Linear). Cin % 64 == 0 so every 64-wide K step lies in
// one filter tap: per step each lane computes ONE source pixel address (or the zero page for
// padding) and the 8-row x 128-B LDS-DMA pieces stream straight from the NHWC activation — im2col
// is never materialised. Same 256 x BN x 64 tile, 8 waves, MFMA 16x16x32, swizzled LDS ring and
// epilogue as the GEMM v2 kernel.
//
// Fusions (flags):
//   CONV_UP2X  : the input is read through a nearest-2x upsample (Upsample + conv, no 4x tensor);
//   dual input : channels [0, C1) come from in, [C1, Cin) from in2 — torch.cat([h, skip], 1) + conv
//                (the UNet decoder's skip concat is never materialised).
#include "common.h"
#include <stdlib.h>
#include "mfma_core.h"
#include "mfma_pp.h"
#include "mfma_pp160.h"
#include "mfma_ppk.h"

#define EPI_BIAS 1
#define EPI_RESIDUAL 2
#define CONV_UP2X 16
#ifndef CGS_CONV_PFE
#define CGS_CONV_PFE 0   // v6 conv epilogue-operand prefetch (pq::run PFE): off -- the in-loop bias prefetch measured +0.25 % per job (profiles/r06), the peeled form spilled
#endif

typedef __attribute__((address_space(3))) void lds_void;

__device__ __attribute__((aligned(16))) unsigned char g_conv_zero_page[256];

struct ConvArgs {
  const u16* in;
  const u16* in2;      // second input for the fused channel concat (or null)
  const u16* w;        // [Cout][kh][kw][Cin]
  const u16* bias;
  const u16* res;
  u16* out;
  int N, H, W, Cin, C1, Cout, kh, kw, stride, pad, Ho, Wo;
  int flags;
  int tiles_n;
  int group_m;
  unsigned cq_magic;   // ceil(2^32 / (Cin / 64)), 0 when Cin == 64 (ConvGatherK tap decode)
  int kw_m16;          // ceil(65536 / kw)
  ppk::Split sp;       // v7 split-K tail (S <= 1: none)
  float* gnp;          // v6 only: GroupNorm partial statistics out (pq::run GNS), or null
  int img_rsrc;        // ConvGatherKD: per-image buffer descriptors (an input >= 2 GiB; Ho*Wo % 256 == 0)
};

// Host: the multiply-shift constants of ConvGatherK (exact for k0 < kh*kw*Cin, kh*kw <= 32).
static void conv_magic(ConvArgs& a) {
  const unsigned cq = (unsigned)(a.Cin / 64);
  a.cq_magic = cq <= 1 ? 0u : (unsigned)(((1ull << 32) + cq - 1) / cq);
  a.kw_m16 = (65536 + a.kw - 1) / a.kw;
}

template <int BN>
__global__ __launch_bounds__(512, 1) void conv_nhwc_v2_kernel(ConvArgs a) {
  constexpr int BM = 256, BK = 64;
  constexpr int WN = BN / 4;
  constexpr int NJ = WN / 16;
  constexpr int NI = 8;
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 8 / 8;
  constexpr int B_INSTR = BN / 8 / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  const int nwg = gridDim.x;
  const int logical = xcd_remap(blockIdx.x, nwg);
  int tm, tn;
  grouped_tile(logical, nwg / a.tiles_n, a.tiles_n, a.group_m, tm, tn);
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 2) * 128;
  const int wn = (wave & 3) * WN;
  const int prow = lane >> 3;
  const int pchunk = lane & 7;
  const bool up = (a.flags & CONV_UP2X) != 0;
  const int Hin = up ? (a.H << 1) : a.H;   // logical (upsampled) input extent
  const int Win = up ? (a.W << 1) : a.W;

  // per-lane output pixel of each A piece
  int pn[A_INSTR], py[A_INSTR], px[A_INSTR], pswz[A_INSTR];
  bool pvalid[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    int r = (wave * A_INSTR + i) * 8 + prow;
    int m = m0 + r;
    pvalid[i] = m < M;
    m = min(m, M - 1);
    pn[i] = m / (a.Ho * a.Wo);
    int rem = m - pn[i] * a.Ho * a.Wo;
    py[i] = (rem / a.Wo) * a.stride - a.pad;
    px[i] = (rem % a.Wo) * a.stride - a.pad;
    pswz[i] = pchunk ^ ((r >> 1) & 7);
  }
  const u16* bsrc[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    int r = (wave * B_INSTR + i) * 8 + prow;
    int gr = min(n0 + r, a.Cout - 1);
    bsrc[i] = a.w + (long long)gr * K + 8 * (pchunk ^ ((r >> 1) & 7));
  }
  const int C2 = a.Cin - a.C1;
  auto issue = [&](int kt, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int k0 = kt * BK;
    const int tap = k0 / a.Cin;
    const int ci0 = k0 - tap * a.Cin;
    const int ky = tap / a.kw;
    const int kx = tap - ky * a.kw;
    const bool second = ci0 >= a.C1;
    const u16* src_t = second ? a.in2 : a.in;
    const int cstride = second ? C2 : a.C1;
    const int cbase = second ? ci0 - a.C1 : ci0;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) {
      int iy = py[i] + ky, ix = px[i] + kx;
      bool ok = pvalid[i] && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
      if (up) { iy >>= 1; ix >>= 1; }
      const void* src = ok ? (const void*)(src_t + (((long long)pn[i] * a.H + iy) * a.W + ix) * cstride + cbase + 8 * pswz[i])
                           : (const void*)(g_conv_zero_page + 16 * (lane & 15));
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(base + ((wave * A_INSTR + i) * 8) * 128), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + k0),
                                       (lds_void*)(base + A_BYTES + ((wave * B_INSTR + i) * 8) * 128), 16, 0, 0);
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  const int fr = lane & 15;
  const int fq = lane >> 4;
  issue(0, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < nk) issue(kt + 1, st ^ 1);
    const unsigned char* As = smem + st * STAGE;
    const unsigned char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[NI], bfr[NJ];
      const int c = kk * 4 + fq;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        int r = wm + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(As + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int r = wn + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + r * 128 + 16 * (c ^ ((r >> 1) & 7)));
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }

  const int er = fq * 4;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    int col = n0 + wn + j * 16 + fr;
    if (col >= a.Cout) continue;
    float bv = (a.flags & EPI_BIAS) ? bf2f(a.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = m0 + wm + i * 16 + er + r;
        if (row < M) {
          float v = acc[i][j][r] + bv;
          if (a.flags & EPI_RESIDUAL) v += bf2f(a.res[(long long)row * a.Cout + col]);
          a.out[(long long)row * a.Cout + col] = f2bf(v);
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// v3: the shared MFMA core (mfma_core.h) with an NHWC gather loader. BK = 32, so Cin % 32 == 0 and
// a 32-wide K step lies in one filter tap (and, for the fused concat, in one of the two inputs).
struct ConvGatherA {
  const ConvArgs* a;
  int pn[4], py[4], px[4];
  bool ok[4];
  int choff;   // this lane's source chunk (elements)
  __device__ __forceinline__ void setup(int p, int row) {
    const int M = a->N * a->Ho * a->Wo;
    ok[p] = row < M;
    row = row < M ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    pn[p] = row / hw;
    const int rem = row - pn[p] * hw;
    py[p] = (rem / a->Wo) * a->stride - a->pad;
    px[p] = (rem % a->Wo) * a->stride - a->pad;
    choff = 8 * mc::src_chunk(threadIdx.x & 63);
  }
  __device__ __forceinline__ const void* src(int p, int k0) const {
    const int tap = k0 / a->Cin;
    const int ci0 = k0 - tap * a->Cin;
    const int ky = tap / a->kw;
    const int kx = tap - ky * a->kw;
    const bool up = (a->flags & CONV_UP2X) != 0;
    const int Hin = up ? 2 * a->H : a->H, Win = up ? 2 * a->W : a->W;
    int iy = py[p] + ky, ix = px[p] + kx;
    const bool in = ok[p] && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
    if (!in) return (const void*)(g_conv_zero_page + 16 * (threadIdx.x & 15));
    if (up) { iy >>= 1; ix >>= 1; }
    const bool second = ci0 >= a->C1;
    const u16* t = second ? a->in2 : a->in;
    const int cs = second ? a->Cin - a->C1 : a->C1;
    const int cb = second ? ci0 - a->C1 : ci0;
    return (const void*)(t + (((long long)pn[p] * a->H + iy) * a->W + ix) * cs + cb + choff);
  }
};

template <int BN, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void conv_nhwc_v3_kernel(
    ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / a.tiles_n, a.tiles_n, a.group_m, tm, tn);
  ConvGatherA al;
  al.a = &a;
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  mc::tile<BN, NW>(al, a.w, K, M, a.Cout, K, tm * mc::BM, tn * BN, e, smem);
}

template <int BN, int NW>
static void conv_v3_go(ConvArgs& a, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v3_kernel<BN, NW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              mc::Cfg<BN, NW>::LDS);
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  const long long nwg = (long long)((M + mc::BM - 1) / mc::BM) * a.tiles_n;
  conv_nhwc_v3_kernel<BN, NW><<<(unsigned)nwg, 64 * NW, mc::Cfg<BN, NW>::LDS, stream>>>(a);
}

// v8: the v3 main loop on 128 x 128 tiles (two workgroups per CU) for short grids -- the level-2
// convs at UNet batch 2 (M = 2048) and Cascade's small token grids. Cin % 32 == 0 (v3 gather).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v8_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / a.tiles_n, a.tiles_n, a.group_m, tm, tn);
  ConvGatherA al;
  al.a = &a;
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  mc::tile<128, 4, ConvGatherA, 128>(al, a.w, K, M, a.Cout, K, tm * 128, tn * 128, e, smem);
}

static void conv_v8_go(ConvArgs& a, hipStream_t stream) {
  using Cf = mc::Cfg<128, 4, 128>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  a.tiles_n = (a.Cout + 127) / 128;
  const long long nwg = (long long)((M + 127) / 128) * a.tiles_n;
  conv_nhwc_v8_kernel<<<(unsigned)nwg, 256, Cf::LDS, stream>>>(a);
}

// v5: ping-pong schedule (mfma_pp.h), 256 x 256 x 64 tiles; Cin % 64 == 0 (one tap per K-tile).
struct ConvGatherA8 {
  const ConvArgs* a;
  int pn[4], py[4], px[4];
  bool ok[4];
  int choff[2];
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    ok[s] = row < M;
    row = row < M ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    pn[s] = row / hw;
    const int rem = row - pn[s] * hw;
    py[s] = (rem / a->Wo) * a->stride - a->pad;
    px[s] = (rem % a->Wo) * a->stride - a->pad;
    choff[s & 1] = 8 * pp::src_chunk8(s & 1);
  }
  __device__ __forceinline__ const void* src(int s, int k0) const {
    const int tap = k0 / a->Cin;
    const int ci0 = k0 - tap * a->Cin;
    const int ky = tap / a->kw;
    const int kx = tap - ky * a->kw;
    const bool up = (a->flags & CONV_UP2X) != 0;
    const int Hin = up ? 2 * a->H : a->H, Win = up ? 2 * a->W : a->W;
    int iy = py[s] + ky, ix = px[s] + kx;
    const bool in = ok[s] && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
    if (!in) return (const void*)(g_conv_zero_page + 16 * (threadIdx.x & 15));
    if (up) { iy >>= 1; ix >>= 1; }
    const bool second = ci0 >= a->C1;
    const u16* t = second ? a->in2 : a->in;
    const int cs = second ? a->Cin - a->C1 : a->C1;
    const int cb = second ? ci0 - a->C1 : ci0;
    return (const void*)(t + (((long long)pn[s] * a->H + iy) * a->W + ix) * cs + cb + choff[s & 1]);
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const { mc::lds_dma16(src(s, k0), dst); }
};

// Leaner gather for the v5/v7 main loops (no CONV_UP2X, kh*kw <= 32): per slot the lane keeps the
// pixel index of its output's top-left tap and a bit mask of in-bounds taps (built once per tile);
// per K-tile the uniform (tap, channel) decode is two multiply-shifts instead of two integer
// divisions, and the lane address is one 64-bit multiply-add -- the loader runs in the same waves
// as the MFMAs, so its VALU/SALU cost comes straight out of the matrix-core issue budget.
template <bool WIDE>   // WIDE: an input is >= 4 GiB (64-bit element offsets); else 32-bit byte offsets
struct ConvGatherK {
  const ConvArgs* a;
  int pix[4];
  uint32_t vm[4];
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    const bool ok = row < M;
    row = ok ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    const int n = row / hw;
    const int rem = row - n * hw;
    const int oy = rem / a->Wo;
    const int py = oy * a->stride - a->pad, px = (rem - oy * a->Wo) * a->stride - a->pad;
    pix[s] = (n * a->H + py) * a->W + px;
    uint32_t m = 0;
    if (ok) {
      for (int ky = 0; ky < a->kh; ++ky) {
        const bool ry = (unsigned)(py + ky) < (unsigned)a->H;
        for (int kx = 0; kx < a->kw; ++kx)
          if (ry && (unsigned)(px + kx) < (unsigned)a->W) m |= 1u << (ky * a->kw + kx);
      }
    }
    vm[s] = m;
  }
  __device__ __forceinline__ const void* src(int s, int k0) const {
    const unsigned kq = (unsigned)k0 >> 6;
    const unsigned tap = a->cq_magic ? __umulhi(kq, a->cq_magic) : kq;
    const int ci0 = k0 - (int)tap * a->Cin;
    const int ky = (int)((tap * (unsigned)a->kw_m16) >> 16);
    const int kx = (int)tap - ky * a->kw;
    if (!((vm[s] >> tap) & 1u)) return (const void*)(g_conv_zero_page + 16 * (threadIdx.x & 15));
    const bool second = ci0 >= a->C1;
    const unsigned char* t = reinterpret_cast<const unsigned char*>(second ? a->in2 : a->in);
    const int cs = second ? a->Cin - a->C1 : a->C1;
    const int cb = (second ? ci0 - a->C1 : ci0) + 8 * pp::src_chunk8(s & 1);
    const unsigned p = (unsigned)(pix[s] + ky * a->W + kx);
    if constexpr (WIDE) return (const void*)(t + 2 * ((size_t)p * (unsigned)cs + (unsigned)cb));
    else return (const void*)(t + 2u * (p * (unsigned)cs + (unsigned)cb));
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const { mc::lds_dma16(src(s, k0), dst); }
};

// v7's gather: the same decode, issued as buffer_load ... lds through one descriptor per input
// (built from kernel arguments only: wave-uniform). A padding tap gets an out-of-range voffset and
// the descriptor's range check returns zeros -- no zero page, no 64-bit VGPR address pairs (v7 runs
// at the 256-VGPR cap). Inputs must each span < 2 GiB.
struct ConvGatherKB {
  const ConvArgs* a;
  int pix[4];
  uint32_t vm[4];
  __amdgpu_buffer_rsrc_t r1, r2;
  __device__ __forceinline__ void init() {
    const unsigned px = (unsigned)(a->N * a->H * a->W);
    r1 = __builtin_amdgcn_make_buffer_rsrc((void*)a->in, 0, (int)(px * (unsigned)a->C1 * 2u), 0x00020000);
    r2 = __builtin_amdgcn_make_buffer_rsrc((void*)(a->in2 ? a->in2 : a->in), 0,
                                           (int)(px * (unsigned)(a->in2 ? a->Cin - a->C1 : a->C1) * 2u), 0x00020000);
  }
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    const bool ok = row < M;
    row = ok ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    const int n = row / hw;
    const int rem = row - n * hw;
    const int oy = rem / a->Wo;
    const int py = oy * a->stride - a->pad, px = (rem - oy * a->Wo) * a->stride - a->pad;
    pix[s] = (n * a->H + py) * a->W + px;
    uint32_t m = 0;
    if (ok) {
      for (int ky = 0; ky < a->kh; ++ky) {
        const bool ry = (unsigned)(py + ky) < (unsigned)a->H;
        for (int kx = 0; kx < a->kw; ++kx)
          if (ry && (unsigned)(px + kx) < (unsigned)a->W) m |= 1u << (ky * a->kw + kx);
      }
    }
    vm[s] = m;
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const {
    const unsigned kq = (unsigned)k0 >> 6;
    const unsigned tap = a->cq_magic ? __umulhi(kq, a->cq_magic) : kq;
    const int ci0 = k0 - (int)tap * a->Cin;
    const int ky = (int)((tap * (unsigned)a->kw_m16) >> 16);
    const int kx = (int)tap - ky * a->kw;
    const bool second = ci0 >= a->C1;
    const int cs = second ? a->Cin - a->C1 : a->C1;
    const int cb = (second ? ci0 - a->C1 : ci0) + 8 * pp::src_chunk8(s & 1);
    const unsigned p = (unsigned)(pix[s] + ky * a->W + kx);
    const unsigned off = ((vm[s] >> tap) & 1u) ? 2u * (p * (unsigned)cs + (unsigned)cb) : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? r2 : r1, (lds_void*)dst, 16, off, 0, 0, 0);
  }
};

// v6's gather: buffer_load ... lds like ConvGatherKB, with the per-lane work cut to the minimum -- per slot
// the lane keeps the byte offsets of its output pixel's top-left tap in each input (its 16-B chunk folded in)
// and the in-bounds tap mask; per K-tile the (tap, input, channel) decode is uniform (SALU) and the lane does
// one add, one bit test and one select. No 64-bit address math and no exec-mask branch per DMA (the old
// ConvGatherK source ran ~20 instructions with a divergent zero-page branch per slot, which made the conv
// loop 25-35 % slower than the same main loop on a dense A; profiles/r04/conv_table_r04t.md). A padding tap
// gets an offset past the descriptor's range and the DMA writes zeros. Offsets are 32-bit (they wrap mod
// 2^32: a negative top-left pixel offset plus an in-bounds tap offset is exact), so each descriptor spans
// < 2 GiB: the whole input, or -- img_rsrc, for the VAE's multi-GiB activations -- the one image a 256-row
// output tile lies in (host: Ho*Wo % 256 == 0), rebuilt per tile by tile().
struct ConvGatherKD {
  static constexpr bool kOwnDMA = true;
  const ConvArgs* a;
  uint32_t pb1[4], pb2[4], vm[4];
  __amdgpu_buffer_rsrc_t r1, r2;
  __device__ __forceinline__ void make(long long n_img, unsigned px) {
    const unsigned c2 = (unsigned)(a->in2 ? a->Cin - a->C1 : a->C1);
    r1 = __builtin_amdgcn_make_buffer_rsrc((void*)(a->in + n_img * px * a->C1), 0, (int)(px * (unsigned)a->C1 * 2u),
                                           0x00020000);
    r2 = __builtin_amdgcn_make_buffer_rsrc((void*)((a->in2 ? a->in2 : a->in) + n_img * px * c2), 0,
                                           (int)(px * c2 * 2u), 0x00020000);
  }
  __device__ __forceinline__ void init() {
    if (!a->img_rsrc) make(0, (unsigned)(a->N * a->H * a->W));
  }
  __device__ __forceinline__ void tile(int m0) {   // m0: the tile's first output row (uniform)
    if (a->img_rsrc) make(m0 / (a->Ho * a->Wo), (unsigned)(a->H * a->W));
  }
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    const bool ok = row < M;
    row = ok ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    const int n = row / hw;
    const int rem = row - n * hw;
    const int oy = rem / a->Wo;
    const int py = oy * a->stride - a->pad, px = (rem - oy * a->Wo) * a->stride - a->pad;
    const unsigned pix = (unsigned)(((a->img_rsrc ? 0 : n) * a->H + py) * a->W + px);
    uint32_t m = 0;
    if (ok) {
      for (int ky = 0; ky < a->kh; ++ky) {
        const bool ry = (unsigned)(py + ky) < (unsigned)a->H;
        for (int kx = 0; kx < a->kw; ++kx)
          if (ry && (unsigned)(px + kx) < (unsigned)a->W) m |= 1u << (ky * a->kw + kx);
      }
    }
    vm[s] = m;
    const unsigned ch = 16u * (unsigned)pp::src_chunk8(s & 1);
    pb1[s] = pix * (2u * (unsigned)a->C1) + ch;
    pb2[s] = pix * (2u * (unsigned)(a->Cin - a->C1)) + ch;
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const {
    // uniform decode, written select-free so the compiler keeps it scalar and branch-free
    const unsigned kq = (unsigned)k0 >> 6;
    const unsigned tap = __umulhi(kq, a->cq_magic) + (a->cq_magic ? 0u : kq);
    const int ci0 = k0 - (int)tap * a->Cin;
    const int ky = (int)((tap * (unsigned)a->kw_m16) >> 16);
    const int kx = (int)tap - ky * a->kw;
    const bool second = ci0 >= a->C1;
    const unsigned cs2 = 2u * (unsigned)(second ? a->Cin - a->C1 : a->C1);
    const unsigned so = (unsigned)(ky * a->W + kx) * cs2 + 2u * (unsigned)(second ? ci0 - a->C1 : ci0);
    // lane: bit `tap` of the mask moved to bit 31 and inverted -> a padding tap's offset has bit 31 set
    // (past every < 2 GiB descriptor range: the DMA writes zeros)
    const unsigned off = ((second ? pb2[s] : pb1[s]) + so) | (~(vm[s] << (31u - tap)) & 0x80000000u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? r2 : r1, (lds_void*)dst, 16, off, 0, 0, 0);
  }
};

// ConvGatherKD for the nearest-2x-upsampled input (CONV_UP2X, single input): the source pixel of tap (ky, kx)
// is ((py + ky) >> 1, (px + kx) >> 1) -- not an affine function of the tap, so the lane keeps its top-left
// (py, px) in upsampled coordinates and its image's base offset, and does two adds, two shifts and two
// 24-bit multiply-adds per DMA (still no branch; a padding tap sets bit 31 as in ConvGatherKD).
struct ConvGatherKU {
  static constexpr bool kOwnDMA = true;
  const ConvArgs* a;
  uint32_t pb[4], vm[4];
  int py[4], px[4];
  __amdgpu_buffer_rsrc_t r1;
  __device__ __forceinline__ void make(long long n_img, unsigned pixels) {
    r1 = __builtin_amdgcn_make_buffer_rsrc((void*)(a->in + n_img * pixels * a->C1), 0,
                                           (int)(pixels * (unsigned)a->C1 * 2u), 0x00020000);
  }
  __device__ __forceinline__ void init() {
    if (!a->img_rsrc) make(0, (unsigned)(a->N * a->H * a->W));
  }
  __device__ __forceinline__ void tile(int m0) {
    if (a->img_rsrc) make(m0 / (a->Ho * a->Wo), (unsigned)(a->H * a->W));
  }
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    const bool ok = row < M;
    row = ok ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    const int n = row / hw;
    const int rem = row - n * hw;
    const int oy = rem / a->Wo;
    const int y0 = oy * a->stride - a->pad, x0 = (rem - oy * a->Wo) * a->stride - a->pad;
    uint32_t m = 0;
    if (ok) {
      for (int ky = 0; ky < a->kh; ++ky) {
        const bool ry = (unsigned)(y0 + ky) < (unsigned)(2 * a->H);
        for (int kx = 0; kx < a->kw; ++kx)
          if (ry && (unsigned)(x0 + kx) < (unsigned)(2 * a->W)) m |= 1u << (ky * a->kw + kx);
      }
    }
    vm[s] = m;
    py[s] = y0;
    px[s] = x0;
    pb[s] = (unsigned)(a->img_rsrc ? 0 : n) * (unsigned)(a->H * a->W) * (2u * (unsigned)a->C1) +
            16u * (unsigned)pp::src_chunk8(s & 1);
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const {
    const unsigned kq = (unsigned)k0 >> 6;
    const unsigned tap = __umulhi(kq, a->cq_magic) + (a->cq_magic ? 0u : kq);
    const int ci0 = k0 - (int)tap * a->Cin;
    const int ky = (int)((tap * (unsigned)a->kw_m16) >> 16);
    const int kx = (int)tap - ky * a->kw;
    const unsigned iy = (unsigned)((py[s] + ky) >> 1) & 0xffffu, ix = (unsigned)((px[s] + kx) >> 1) & 0xffffu;
    const unsigned pix = __umul24(iy, (unsigned)a->W) + ix;
    const unsigned off = (pix * (2u * (unsigned)a->C1) + pb[s] + 2u * (unsigned)ci0) |
                         (~(vm[s] << (31u - tap)) & 0x80000000u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_void*)dst, 16, off, 0, 0, 0);
  }
};

// ConvGatherKD with 2 registers per slot instead of 3 (v7 runs at the 256-VGPR cap: KD spilled there): the
// lane keeps its top-left pixel index and tap mask, and multiplies by the input's row pitch per DMA (one
// 32-bit multiply, exact mod 2^32 like KD's offsets). Whole-input descriptors only (ppk re-points A per
// half-tile, so no per-image rebuild).
struct ConvGatherKL {
  static constexpr bool kOwnDMA = true;
  const ConvArgs* a;
  uint32_t pix[4], vm[4];
  __amdgpu_buffer_rsrc_t r1, r2;
  __device__ __forceinline__ void init() {
    const unsigned px = (unsigned)(a->N * a->H * a->W);
    r1 = __builtin_amdgcn_make_buffer_rsrc((void*)a->in, 0, (int)(px * (unsigned)a->C1 * 2u), 0x00020000);
    r2 = __builtin_amdgcn_make_buffer_rsrc((void*)(a->in2 ? a->in2 : a->in), 0,
                                           (int)(px * (unsigned)(a->in2 ? a->Cin - a->C1 : a->C1) * 2u), 0x00020000);
  }
  __device__ __forceinline__ void tile(int) {}
  __device__ __forceinline__ void setup(int s, int row) {
    const int M = a->N * a->Ho * a->Wo;
    const bool ok = row < M;
    row = ok ? row : M - 1;
    const int hw = a->Ho * a->Wo;
    const int n = row / hw;
    const int rem = row - n * hw;
    const int oy = rem / a->Wo;
    const int py = oy * a->stride - a->pad, px = (rem - oy * a->Wo) * a->stride - a->pad;
    pix[s] = (unsigned)((n * a->H + py) * a->W + px);
    uint32_t m = 0;
    if (ok) {
      for (int ky = 0; ky < a->kh; ++ky) {
        const bool ry = (unsigned)(py + ky) < (unsigned)a->H;
        for (int kx = 0; kx < a->kw; ++kx)
          if (ry && (unsigned)(px + kx) < (unsigned)a->W) m |= 1u << (ky * a->kw + kx);
      }
    }
    vm[s] = m;
  }
  __device__ __forceinline__ void dma(int s, int k0, unsigned char* dst) const {
    const unsigned kq = (unsigned)k0 >> 6;
    const unsigned tap = __umulhi(kq, a->cq_magic) + (a->cq_magic ? 0u : kq);
    const int ci0 = k0 - (int)tap * a->Cin;
    const int ky = (int)((tap * (unsigned)a->kw_m16) >> 16);
    const int kx = (int)tap - ky * a->kw;
    const bool second = ci0 >= a->C1;
    const unsigned cs2 = 2u * (unsigned)(second ? a->Cin - a->C1 : a->C1);
    const unsigned so = (unsigned)(ky * a->W + kx) * cs2 + 2u * (unsigned)(second ? ci0 - a->C1 : ci0) +
                        16u * (unsigned)pp::src_chunk8(s & 1);
    const unsigned off = (pix[s] * cs2 + so) | (~(vm[s] << (31u - tap)) & 0x80000000u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(second ? r2 : r1, (lds_void*)dst, 16, off, 0, 0, 0);
  }
};

static bool conv_fast_ok(const ConvArgs& a) { return !(a.flags & CONV_UP2X) && a.kh * a.kw <= 32; }
// an input tensor spans >= 2 GiB (v7's ConvGatherKB descriptors need < 2 GiB)
static bool conv_wide(const ConvArgs& a) {
  const long long px = (long long)a.N * a.H * a.W;
  return px * a.C1 * 2 >= (1ll << 31) || (a.in2 && px * (a.Cin - a.C1) * 2 >= (1ll << 31));
}
// ConvGatherKD applies (sets a.img_rsrc): every input < 2 GiB, or each image < 2 GiB with 256-row output
// tiles that never straddle two images
static bool conv_kd(ConvArgs& a) {
  a.img_rsrc = 0;
  if ((a.flags & CONV_UP2X) && (a.in2 || a.kh * a.kw > 32 || a.H >= 32768 || a.W >= 32768)) return false;
  if (!conv_wide(a)) return true;
  const long long px = (long long)a.H * a.W;
  const bool img_ok = ((long long)a.Ho * a.Wo) % 256 == 0 && px * a.C1 * 2 < (1ll << 31) &&
                      (!a.in2 || px * (a.Cin - a.C1) * 2 < (1ll << 31));
  a.img_rsrc = img_ok ? 1 : 0;
  return img_ok;
}

template <bool KD>   // KD: ConvGatherKD (buffer_load ... lds); else ConvGatherK with 64-bit offsets
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v5k_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / a.tiles_n, a.tiles_n, a.group_m, tm, tn);
  typename std::conditional<KD, ConvGatherKD, ConvGatherK<true>>::type al;
  al.a = &a;
  if constexpr (KD) al.init();
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  pp::tile(al, a.w, K, M, a.Cout, K, tm * pp::BM, tn * pp::BN, e, smem);
}

template <bool KU>   // KU: the upsample-aware buffer gather (ConvGatherKU); else the generic ConvGatherA8
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v5_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / a.tiles_n, a.tiles_n, a.group_m, tm, tn);
  typename std::conditional<KU, ConvGatherKU, ConvGatherA8>::type al;
  al.a = &a;
  if constexpr (KU) al.init();
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  pp::tile(al, a.w, K, M, a.Cout, K, tm * pp::BM, tn * pp::BN, e, smem);
}

// v5 / v6 loader override for A/B (-1 auto: KD / KU where legal; 1 forces ConvGatherK, 0 ConvGatherA8):
// CGS_CONV_LOADER at load, cgs_conv_v6_set_loader() after
static int conv_loader_env() {
  const char* v = getenv("CGS_CONV_LOADER");
  return v ? atoi(v) : -1;
}
static int g_conv_v6_ld = conv_loader_env();
CGS_EXPORT void cgs_conv_v6_set_loader(int ld) { g_conv_v6_ld = ld; }

static void conv_v5_go(ConvArgs& a, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v5_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              pp::LDS);
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v5_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              pp::LDS);
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  a.tiles_n = (a.Cout + pp::BN - 1) / pp::BN;
  const long long nwg = (long long)((M + pp::BM - 1) / pp::BM) * a.tiles_n;
  if (conv_fast_ok(a)) {
    static bool attr_k = false;
    if (!attr_k) {
      (void)hipFuncSetAttribute((const void*)conv_nhwc_v5k_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                pp::LDS);
      (void)hipFuncSetAttribute((const void*)conv_nhwc_v5k_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                pp::LDS);
      attr_k = true;
    }
    conv_magic(a);
    if (g_conv_v6_ld != 1 && conv_kd(a)) conv_nhwc_v5k_kernel<true><<<(unsigned)nwg, pp::THREADS, pp::LDS, stream>>>(a);
    else conv_nhwc_v5k_kernel<false><<<(unsigned)nwg, pp::THREADS, pp::LDS, stream>>>(a);
  } else if ((a.flags & CONV_UP2X) && g_conv_v6_ld != 0 && conv_kd(a)) {
    conv_magic(a);
    conv_nhwc_v5_kernel<true><<<(unsigned)nwg, pp::THREADS, pp::LDS, stream>>>(a);
  } else {
    conv_nhwc_v5_kernel<false><<<(unsigned)nwg, pp::THREADS, pp::LDS, stream>>>(a);
  }
}

// LD: 0 ConvGatherA8 (generic: UP2X, big filters), 1 ConvGatherK (64-bit offsets: an input >= 2 GiB),
// 2 ConvGatherKD (buffer_load ... lds, the default where it applies)
// NJ: 16-column MFMA tiles per wave group -- 5 (256 x 160 tiles) or 4 (256 x 128: Cout = 128 / 256 / 384 ...,
// variant 18)
template <int LD, int DS = 0, bool GNS = false, int NJ = 5, int PFE = CGS_CONV_PFE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v6_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  typename std::conditional<
      LD == 3, ConvGatherKU,
      typename std::conditional<LD == 2, ConvGatherKD,
                                typename std::conditional<LD == 1, ConvGatherK<true>, ConvGatherA8>::type>::type>::type al;
  al.a = &a;
  if constexpr (LD >= 2) al.init();
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  e.gnp = a.gnp;
  e.hw = a.Ho * a.Wo;
  pq::run<decltype(al), false, DS, GNS, false, false, false, PFE, NJ>(al, a.w, K, M, a.Cout, K, e, smem,
                                                                              (M + pq::BM - 1) / pq::BM, a.tiles_n,
                                                                              a.group_m);
}

// One-wave-group form (pq::run NW = 4, NI = 2): 128 x 80 tiles, 4 waves, two workgroups per CU -- variant 21,
// for the batch-1 grids (SDXL level 2 at batch 2: M = 2048 output pixels x Cout = 1280 is 256 tiles).
template <int LD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v6w4_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  typename std::conditional<
      LD == 3, ConvGatherKU,
      typename std::conditional<LD == 2, ConvGatherKD,
                                typename std::conditional<LD == 1, ConvGatherK<true>, ConvGatherA8>::type>::type>::type al;
  al.a = &a;
  if constexpr (LD >= 2) al.init();
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  using Gm = pq::Geo<5, 2, 4>;
  pq::run<decltype(al), false, 51, false, false, false, false, 0, 5, 2, 4>(al, a.w, K, M, a.Cout, K, e, smem,
                                                                          (M + Gm::BM - 1) / Gm::BM, a.tiles_n,
                                                                          a.group_m);
}

static int conv_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

int v6_conv_ds();   // gemm.hip: v6 DMA placement for convs (CGS_V6_CONV_DS / cgs_v6_set_mode)

template <int LD, int DS, bool GNS = false, int NJ = 5, int PFE = CGS_CONV_PFE>
static void conv_v6_launch(ConvArgs& a, int grid, hipStream_t stream) {
  constexpr int lds = pq::Geo<NJ>::LDS;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v6_kernel<LD, DS, GNS, NJ, PFE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  conv_nhwc_v6_kernel<LD, DS, GNS, NJ, PFE><<<grid, pq::THREADS, lds, stream>>>(a);
}



static void conv_v6w4_go(ConvArgs& a, hipStream_t stream) {
  using Gm = pq::Geo<5, 2, 4>;
  const int M = a.N * a.Ho * a.Wo;
  a.tiles_n = (a.Cout + Gm::BN - 1) / Gm::BN;
  const long long T = (long long)((M + Gm::BM - 1) / Gm::BM) * a.tiles_n;
  const int grid = (int)(T < 2 * conv_num_cus() ? T : 2 * conv_num_cus());
  int ld = conv_fast_ok(a) ? (conv_kd(a) ? 2 : 1) : ((a.flags & CONV_UP2X) && conv_kd(a) ? 3 : 0);
  if (g_conv_v6_ld >= 0 && g_conv_v6_ld < ld) ld = ld == 3 ? 0 : g_conv_v6_ld;
  if (ld) conv_magic(a);
  auto go = [&](auto lc) {
    constexpr int L = decltype(lc)::value;
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv_nhwc_v6w4_kernel<L>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                Gm::LDS);
      attr = true;
    }
    conv_nhwc_v6w4_kernel<L><<<grid, 256, Gm::LDS, stream>>>(a);
  };
  if (ld == 3) go(std::integral_constant<int, 3>{});
  else if (ld == 2) go(std::integral_constant<int, 2>{});
  else if (ld == 1) go(std::integral_constant<int, 1>{});
  else go(std::integral_constant<int, 0>{});
}

static void conv_v6_go(ConvArgs& a, hipStream_t stream, bool n128 = false) {
  const int M = a.N * a.Ho * a.Wo;
  if (a.gnp) n128 = false;   // the GroupNorm-statistics epilogue: 160-wide tiles only
  const int bn = n128 ? pq::Geo<4>::BN : pq::BN;
  a.tiles_n = (a.Cout + bn - 1) / bn;
  const long long T = (long long)((M + pq::BM - 1) / pq::BM) * a.tiles_n;
  const int grid = (int)(T < conv_num_cus() ? T : conv_num_cus());
  const int ds = v6_conv_ds();
  int ld = conv_fast_ok(a) ? (conv_kd(a) ? 2 : 1) : ((a.flags & CONV_UP2X) && conv_kd(a) ? 3 : 0);
  if (g_conv_v6_ld >= 0 && g_conv_v6_ld < ld) ld = ld == 3 ? 0 : g_conv_v6_ld;
  if (ld) conv_magic(a);
  auto go = [&](auto lc) {
    constexpr int L = decltype(lc)::value;
    if (a.gnp) {   // GroupNorm statistics epilogue (split-DMA main loop only)
      conv_v6_launch<L, 51, true>(a, grid, stream);
      return;
    }
    if (n128) {    // 256 x 128 tiles: the default DMA placement only; no epilogue-operand prefetch (NJ = 4 has
                   // the registers for the peeled form, but it measured 1-3 % slower, profiles/r06/conv_n128_ab.log)
      conv_v6_launch<L, 51, false, 4, 0>(a, grid, stream);
      return;
    }
    switch (ds) {
      case 0: conv_v6_launch<L, 0>(a, grid, stream); break;
      case 3: conv_v6_launch<L, 3>(a, grid, stream); break;
      case 17: conv_v6_launch<L, 17>(a, grid, stream); break;
      case 19: conv_v6_launch<L, 19>(a, grid, stream); break;
      case 1: conv_v6_launch<L, 1>(a, grid, stream); break;
      default: conv_v6_launch<L, 51>(a, grid, stream);
    }
  };
  if (ld == 3) go(std::integral_constant<int, 3>{});
  else if (ld == 2) go(std::integral_constant<int, 2>{});
  else if (ld == 1) go(std::integral_constant<int, 1>{});
  else go(std::integral_constant<int, 0>{});
}

// v7: the persistent 256 x 256 ping-pong with cross-tile prefetch and register epilogue (mfma_ppk.h)
// LOADER 0: ConvGatherA8 (generic: UP2X, big filters); 1: ConvGatherKB (buffer_load lds). (ConvGatherK
// with global_load_lds and 64-bit offsets measured 25-30 % slower here: it spills at the v7 VGPR cap.)
template <int LOADER>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv_nhwc_v7_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  typename std::conditional<LOADER == 2, ConvGatherKL,
                            typename std::conditional<LOADER == 1, ConvGatherKB, ConvGatherA8>::type>::type al;
  al.a = &a;
  if constexpr (LOADER >= 1) al.init();
  mc::Epi e{a.out, a.bias, a.res, a.Cout, a.Cout, a.flags & (EPI_BIAS | EPI_RESIDUAL), 1.0f};
  ppk::run<false>(al, a.w, K, M, a.Cout, K, e, smem, (M + ppk::BM - 1) / ppk::BM, a.tiles_n, a.group_m, a.sp);
}

static void conv_v7_go(ConvArgs& a, hipStream_t stream, void* ws = nullptr, long long ws_bytes = 0) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v7_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ppk::LDS);
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v7_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ppk::LDS);
    (void)hipFuncSetAttribute((const void*)conv_nhwc_v7_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ppk::LDS);
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  const int K = a.kh * a.kw * a.Cin;
  a.tiles_n = (a.Cout + ppk::BN - 1) / ppk::BN;
  const long long T = (long long)((M + ppk::BM - 1) / ppk::BM) * a.tiles_n;
  a.sp = ppk::Split{0, 1, nullptr, nullptr, 0};
  long long U = T;
  if (ws && ws_bytes >= ppk::split_ws_bytes(T, K / ppk::BK, conv_num_cus())) {
    a.sp.S = ppk::split_plan(T, K / ppk::BK, conv_num_cus(), a.sp.t_full);
    if (a.sp.S > 1) {
      const long long tail = T - a.sp.t_full;
      a.sp.part = (float4*)ws;
      a.sp.cnt = (int*)((char*)ws + tail * a.sp.S * 32ll * ppk::THREADS * 16);
      ppk::zero_counters_kernel<<<1, 256, 0, stream>>>(a.sp.cnt, (int)tail);
      if (hipGetLastError() != hipSuccess) a.sp.S = 1;
      else U = a.sp.t_full + tail * a.sp.S;
    }
  }
  const int grid = (int)(U < conv_num_cus() ? U : conv_num_cus());
  if (conv_fast_ok(a) && !conv_wide(a)) {
    conv_magic(a);
    a.img_rsrc = 0;
    if (g_conv_v6_ld == 1) conv_nhwc_v7_kernel<1><<<grid, ppk::THREADS, ppk::LDS, stream>>>(a);
    else conv_nhwc_v7_kernel<2><<<grid, ppk::THREADS, ppk::LDS, stream>>>(a);
  } else {
    conv_nhwc_v7_kernel<0><<<grid, ppk::THREADS, ppk::LDS, stream>>>(a);
  }
}

static int g_conv_group = 8;
CGS_EXPORT void cgs_conv_set_tile_group(int g) { g_conv_group = g < 1 ? 1 : g; }
static int g_conv_variant = -1;   // -1 auto (v3/8 waves where legal), 2 = v2 only, 3 = v3/4 waves, 4 = v3/8 waves
CGS_EXPORT void cgs_conv_set_variant(int v) { g_conv_variant = v; }

static int conv_v3_launch(ConvArgs& a, int variant, hipStream_t stream, void* ws = nullptr, long long ws_bytes = 0) {
  a.group_m = g_conv_group;
  if (variant == 5 && a.Cin % 64 == 0 && (a.in2 == nullptr || a.C1 % 64 == 0)) {
    conv_v5_go(a, stream);
    return (int)hipGetLastError();
  }
  if (variant == 7 && a.Cin % 64 == 0 && (a.in2 == nullptr || a.C1 % 64 == 0) && a.kh * a.kw * a.Cin >= 128 &&
      ((uintptr_t)a.bias % 8) == 0 && (long long)a.Cout * a.kh * a.kw * a.Cin * 2 < (1ll << 32)) {
    conv_v7_go(a, stream, ws, ws_bytes);
    return (int)hipGetLastError();
  }
  if (variant == 6 && a.Cin % 64 == 0 && (a.in2 == nullptr || a.C1 % 64 == 0) && a.kh * a.kw * a.Cin >= 128 &&
      ((uintptr_t)a.bias % 8) == 0) {
    conv_v6_go(a, stream);
    return (int)hipGetLastError();
  }
  if (variant == 21 && a.Cin % 64 == 0 && (a.in2 == nullptr || a.C1 % 64 == 0) && a.kh * a.kw * a.Cin >= 128 &&
      ((uintptr_t)a.bias % 8) == 0 && a.Cout % 80 == 0 && a.gnp == nullptr) {
    conv_v6w4_go(a, stream);
    return (int)hipGetLastError();
  }
  if (variant == 18 && a.Cin % 64 == 0 && (a.in2 == nullptr || a.C1 % 64 == 0) && a.kh * a.kw * a.Cin >= 128 &&
      ((uintptr_t)a.bias % 8) == 0 && a.Cout % 128 == 0) {
    conv_v6_go(a, stream, true);
    return (int)hipGetLastError();
  }
  if (variant == 8) {
    conv_v8_go(a, stream);
    return (int)hipGetLastError();
  }
  const int M = a.N * a.Ho * a.Wo;
  const int BN = mc::pick_bn(M, a.Cout);
  const bool w8 = variant != 3;
  if (BN == 256) { if (w8) conv_v3_go<256, 8>(a, stream); else conv_v3_go<256, 4>(a, stream); }
  else { if (w8) conv_v3_go<128, 8>(a, stream); else conv_v3_go<128, 4>(a, stream); }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Narrow-output conv (Cout <= 16): the UNet's conv_out (320 -> 4 latent channels, once per
// denoiser step) and the VAE decoder's conv_out (128 -> 3 at full image resolution). A 128/256-wide
// N tile wastes > 95 % of its MFMA columns and LDS traffic on these (they ran at ~1.7 ms per UNet
// step and ~10 ms per decode on v2). Here one wave owns SN_MB x 16 output pixels x 16 output
// channels: per 32-channel K step it issues SN_MB v_mfma_f32_16x16x32_bf16 whose A fragments are
// 16-B NHWC vectors loaded straight from global (lane l: pixel row l & 15, channels 8 (l >> 4) ..
// +7 -- the MFMA's own A layout, so no LDS) and whose B fragment is the same slice of the filter
// row of output channel l & 15 (the whole filter is a few 10s of KB and stays in L1/L2). No LDS,
// no barriers, 4 waves per workgroup and >= 1000 workgroups on the production shapes.
// Pixel mapping: a workgroup (4 waves) owns a 16 x 16 output patch of one image; wave w covers
// rows 4w .. 4w+3, one 16-pixel MFMA block per row (lane & 15 = x). The K loop runs channel-chunk
// outer, tap inner, so while a workgroup is on one 32-channel chunk it touches only its 18 x 18 x
// 64-B input halo (~21 KB): the nine taps' re-reads are L1 hits and HBM/L2 see ~one pass.
#define SN_MB 4
template <int KS>   // KS = kh = kw when 1 or 3 (taps unrolled), 0 = runtime kh / kw
__global__ __launch_bounds__(256) void conv_nhwc_smalln_kernel(ConvArgs a) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tiles_x = (a.Wo + 15) >> 4, tiles_y = (a.Ho + 15) >> 4;
  const int bid = blockIdx.x;
  const int n = bid / (tiles_x * tiles_y);
  const int trem = bid - n * tiles_x * tiles_y;
  const int ty = trem / tiles_x, tx = trem - ty * tiles_x;
  const int fr = lane & 15, fq = lane >> 4;
  const int kh = KS ? KS : a.kh, kw = KS ? KS : a.kw;
  const bool up = (a.flags & CONV_UP2X) != 0;
  const int Hin = up ? 2 * a.H : a.H, Win = up ? 2 * a.W : a.W;
  const int ox = tx * 16 + fr;
  const int px = ox * a.stride - a.pad;
  int py[SN_MB];
  bool pv[SN_MB];
#pragma unroll
  for (int b = 0; b < SN_MB; ++b) {
    const int oy = ty * 16 + wave * SN_MB + b;
    pv[b] = oy < a.Ho && ox < a.Wo;
    py[b] = oy * a.stride - a.pad;
  }
  const bool cv = fr < a.Cout;
  const int C2 = a.Cin - a.C1;
  const u16* wrow = a.w + (long long)(cv ? fr : 0) * kh * kw * a.Cin + 8 * fq;
  f32x4 acc[SN_MB];
#pragma unroll
  for (int b = 0; b < SN_MB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long long img = (long long)n * a.H;
  const bf16x8 zero = {};
  for (int c = 0; c < a.Cin; c += 32) {
    const bool second = c >= a.C1;
    const u16* src = second ? a.in2 : a.in;
    const int cs = second ? C2 : a.C1;
    const int cb = (second ? c - a.C1 : c) + 8 * fq;
    // Measured on the VAE 1024^2 shape (one image): this per-tap loop with predicated loads 287 us;
    // unconditional zero-page loads 337 us; all nine taps' loads hoisted ahead of the MFMAs (45 in
    // flight, 256 VGPRs, one wave per SIMD) 336 us; the 256-row v2 tile 443 us.
    {
#pragma unroll
      for (int ky = 0; ky < kh; ++ky) {
#pragma unroll
        for (int kx = 0; kx < kw; ++kx) {
          const bf16x8 bfr = cv ? *reinterpret_cast<const bf16x8*>(wrow + (ky * kw + kx) * a.Cin + c) : zero;
          int ix = px + kx;
          const bool okx = ix >= 0 && ix < Win;
          if (up) ix >>= 1;
          bf16x8 af[SN_MB];
#pragma unroll
          for (int b = 0; b < SN_MB; ++b) {
            int iy = py[b] + ky;
            const bool ok = pv[b] && okx && iy >= 0 && iy < Hin;
            if (up) iy >>= 1;
            af[b] = ok ? *reinterpret_cast<const bf16x8*>(src + ((img + iy) * a.W + ix) * cs + cb) : zero;
          }
#pragma unroll
          for (int b = 0; b < SN_MB; ++b) acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[b], bfr, acc[b], 0, 0, 0);
        }
      }
    }
  }
  // C/D layout: acc[b][r] = (pixel row 4 (lane >> 4) + r of block b, output channel lane & 15). Block b is
  // image row oy_b; its 16 MFMA rows are the 16 x positions tx*16 .. +15.
  if (!cv) return;
  const float bv = (a.flags & EPI_BIAS) ? bf2f(a.bias[fr]) : 0.f;
#pragma unroll
  for (int b = 0; b < SN_MB; ++b) {
    const int oy = ty * 16 + wave * SN_MB + b;
    if (oy >= a.Ho) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int x = tx * 16 + fq * 4 + r;
      if (x < a.Wo) {
        const long long row = ((long long)n * a.Ho + oy) * a.Wo + x;
        float v = acc[b][r] + bv;
        if (a.flags & EPI_RESIDUAL) v += bf2f(a.res[row * a.Cout + fr]);
        a.out[row * a.Cout + fr] = f2bf(v);
      }
    }
  }
}

// The same narrow-output conv for its production form -- 3 x 3, stride 1, pad 1, one source, Cin % 32 == 0 (the
// VAE decoder's conv_out, 128 -> 3 at full resolution; the UNet's 320 -> 4) -- with each 32-channel chunk of the
// workgroup's 18 x 18 input halo staged through LDS once (register-staged, double-buffered: the next chunk's loads
// are in flight while this one computes). The direct-load form re-read every input vector for each of the nine
// taps from L1 / L2, and with several workgroups per CU the halos did not stay in L1 (2.3 ms per 8-image decode,
// ~9x the input's bytes through L2). Pixel stride 80 B in LDS: the 16 lanes of a fragment read (16 consecutive
// pixels, one 16-B chunk) hit distinct banks.
#define SNL_PX 40   // u16 per staged pixel: 32 channels + 8 pad
__global__ __launch_bounds__(256) void conv_nhwc_smalln_lds_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) u16 halo[2][18 * 18 * SNL_PX];
  constexpr int NV = 18 * 18 * 4, NS = (NV + 255) / 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_x = (a.Wo + 15) >> 4, tiles_y = (a.Ho + 15) >> 4;
  const int bid = blockIdx.x;
  const int n = bid / (tiles_x * tiles_y);
  const int trem = bid - n * tiles_x * tiles_y;
  const int ty = trem / tiles_x, tx = trem - ty * tiles_x;
  const int fr = lane & 15, fq = lane >> 4;
  const int y0 = ty * 16 - 1, x0 = tx * 16 - 1;
  const u16* img = a.in + (long long)n * a.H * a.W * a.Cin;
  // staging slots of this thread: vector v = tid + 256 s -> (halo pixel v >> 2, 16-B chunk v & 3)
  long long soff[NS];
  bool sok[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int v = tid + 256 * s, p = v >> 2, ch = v & 3;
    const int py = p / 18, px = p - py * 18, iy = y0 + py, ix = x0 + px;
    sok[s] = v < NV && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    soff[s] = sok[s] ? ((long long)iy * a.W + ix) * a.Cin + 8 * ch : 0;
  }
  const s16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  s16x8 r[NS];
  auto load = [&](int c) {
#pragma unroll
    for (int s = 0; s < NS; ++s) r[s] = sok[s] ? *reinterpret_cast<const s16x8*>(img + soff[s] + c) : zero8;
  };
  auto put = [&](int buf) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int v = tid + 256 * s;
      if (v < NV) *reinterpret_cast<s16x8*>(&halo[buf][(v >> 2) * SNL_PX + 8 * (v & 3)]) = r[s];
    }
  };
  const bool cv = fr < a.Cout;
  const u16* wrow = a.w + (long long)(cv ? fr : 0) * 9 * a.Cin + 8 * fq;
  f32x4 acc[SN_MB];
#pragma unroll
  for (int b = 0; b < SN_MB; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16x8 zb = {};
  load(0);
  put(0);
  __syncthreads();
  int buf = 0;
  for (int c = 0; c < a.Cin; c += 32) {
    const bool more = c + 32 < a.Cin;
    if (more) load(c + 32);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const bf16x8 bfr = cv ? *reinterpret_cast<const bf16x8*>(wrow + (ky * 3 + kx) * a.Cin + c) : zb;
#pragma unroll
        for (int b = 0; b < SN_MB; ++b) {
          const int p = (wave * SN_MB + b + ky) * 18 + fr + kx;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(&halo[buf][p * SNL_PX + 8 * fq]);
          acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr, acc[b], 0, 0, 0);
        }
      }
    if (more) put(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  if (!cv) return;
  const float bv = (a.flags & EPI_BIAS) ? bf2f(a.bias[fr]) : 0.f;
#pragma unroll
  for (int b = 0; b < SN_MB; ++b) {
    const int oy = ty * 16 + wave * SN_MB + b;
    if (oy >= a.Ho) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int x = tx * 16 + fq * 4 + q;
      if (x < a.Wo) {
        const long long row = ((long long)n * a.Ho + oy) * a.Wo + x;
        float v = acc[b][q] + bv;
        if (a.flags & EPI_RESIDUAL) v += bf2f(a.res[row * a.Cout + fr]);
        a.out[row * a.Cout + fr] = f2bf(v);
      }
    }
  }
}

// CGS_SMALLN_LDS (default 1) / cgs_conv_smalln_set_lds: the LDS-staged form where it applies (A/B)
static int g_smalln_lds = -1;
static bool smalln_lds() {
  if (g_smalln_lds < 0) g_smalln_lds = getenv("CGS_SMALLN_LDS") ? atoi(getenv("CGS_SMALLN_LDS")) != 0 : 1;
  return g_smalln_lds != 0;
}
CGS_EXPORT void cgs_conv_smalln_set_lds(int on) { g_smalln_lds = on != 0; }

static int conv_smalln_launch(const ConvArgs& a, hipStream_t stream) {
  const long long nwg = (long long)a.N * ((a.Ho + 15) / 16) * ((a.Wo + 15) / 16);
  if (nwg > 0x7fffffffLL || nwg < 1) return (int)hipErrorInvalidValue;
  if (smalln_lds() && a.kh == 3 && a.kw == 3 && a.stride == 1 && a.pad == 1 && !(a.flags & CONV_UP2X) &&
      a.in2 == nullptr && a.Cin % 32 == 0 && a.Ho == a.H && a.Wo == a.W && a.Cout <= 16 &&
      (long long)a.H * a.W * a.Cin < (1ll << 31)) {
    conv_nhwc_smalln_lds_kernel<<<(unsigned)nwg, 256, 0, stream>>>(a);
    return (int)hipGetLastError();
  }
  if (a.kh == 3 && a.kw == 3) conv_nhwc_smalln_kernel<3><<<(unsigned)nwg, 256, 0, stream>>>(a);
  else if (a.kh == 1 && a.kw == 1) conv_nhwc_smalln_kernel<1><<<(unsigned)nwg, 256, 0, stream>>>(a);
  else conv_nhwc_smalln_kernel<0><<<(unsigned)nwg, 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

// variant 12 = the narrow-output kernel above (default for Cout <= 16); variant 2 keeps the
// 256-row v2 tile for A/B comparisons.
static int conv_launch(ConvArgs& a, hipStream_t stream, int variant = -2, void* ws = nullptr, long long ws_bytes = 0) {
  if (variant == -2) variant = g_conv_variant;
  if (a.Cout <= 16 && (variant != 2 || a.Cin % 64 || (a.in2 && a.C1 % 64))) return conv_smalln_launch(a, stream);
  // v3 needs Cout % 8 == 0 for the 16-B epilogue stores (SD/SDXL/VAE convs: all but the 3/4-channel
  // heads, which take v2).
  if (variant != 2 && a.Cout % 8 == 0) return conv_v3_launch(a, variant, stream, ws, ws_bytes);
  a.group_m = g_conv_group;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)conv_nhwc_v2_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        2 * (256 * 64 * 2 + 256 * 64 * 2));
    hipFuncSetAttribute((const void*)conv_nhwc_v2_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        2 * (256 * 64 * 2 + 128 * 64 * 2));
    attr = true;
  }
  const int M = a.N * a.Ho * a.Wo;
  const bool wide = a.Cout >= 1024;
  const int BN = wide ? 256 : 128;
  a.tiles_n = (a.Cout + BN - 1) / BN;
  long long nwg = (long long)((M + 255) / 256) * a.tiles_n;
  size_t lds = 2 * (256 * 64 * 2 + BN * 64 * 2);
  if (wide) conv_nhwc_v2_kernel<256><<<(unsigned)nwg, 512, lds, stream>>>(a);
  else conv_nhwc_v2_kernel<128><<<(unsigned)nwg, 512, lds, stream>>>(a);
  return (int)hipGetLastError();
}

// x [N,H,W,Cin] NHWC bf16, w [Cout,kh,kw,Cin], bias [Cout] | null, res [N,Ho,Wo,Cout] | null.
CGS_EXPORT int cgs_conv2d_nhwc(const void* x, const void* w, const void* bias, const void* res, void* out, int N, int H,
                               int W, int Cin, int Cout, int kh, int kw, int stride, int pad, int Ho, int Wo,
                               hipStream_t stream) {
  if (Cin % 32 || Cout < 1 || (Cout % 8 && Cout > 16 && Cin % 64)) return (int)hipErrorInvalidValue;
  ConvArgs a{(const u16*)x, nullptr, (const u16*)w, (const u16*)bias, (const u16*)res, (u16*)out, N, H, W, Cin, Cin,
             Cout, kh, kw, stride, pad, Ho, Wo, (bias ? EPI_BIAS : 0) | (res ? EPI_RESIDUAL : 0), 0, 1};
  return conv_launch(a, stream);
}

// Fused variants: flags may carry CONV_UP2X (input read through nearest-2x upsample); x2 != null
// concatenates x2's C2 = Cin - C1 channels after x's C1 channels (skip concat).
CGS_EXPORT int cgs_conv2d_nhwc_ex(const void* x, const void* x2, int C1, const void* w, const void* bias,
                                  const void* res, void* out, int N, int H, int W, int Cin, int Cout, int kh, int kw,
                                  int stride, int pad, int Ho, int Wo, int flags, hipStream_t stream) {
  if (Cin % 32 || (x2 && (C1 % 32)) || Cout < 1 || (Cout % 8 && Cout > 16 && (Cin % 64 || (x2 && C1 % 64))))
    return (int)hipErrorInvalidValue;
  ConvArgs a{(const u16*)x, (const u16*)x2, (const u16*)w, (const u16*)bias, (const u16*)res, (u16*)out, N, H, W,
             Cin, x2 ? C1 : Cin, Cout, kh, kw, stride, pad, Ho, Wo,
             (bias ? EPI_BIAS : 0) | (res ? EPI_RESIDUAL : 0) | (flags & CONV_UP2X), 0, 1};
  return conv_launch(a, stream);
}

// Per-call kernel choice for the autotuner (variant as in cgs_conv_set_variant; flags as _ex).
CGS_EXPORT int cgs_conv2d_nhwc_v(const void* x, const void* x2, int C1, const void* w, const void* bias,
                                 const void* res, void* out, int N, int H, int W, int Cin, int Cout, int kh, int kw,
                                 int stride, int pad, int Ho, int Wo, int flags, int variant, hipStream_t stream) {
  if (Cin % 32 || (x2 && (C1 % 32)) || Cout < 1 || (Cout % 8 && Cout > 16 && (Cin % 64 || (x2 && C1 % 64))))
    return (int)hipErrorInvalidValue;
  ConvArgs a{(const u16*)x, (const u16*)x2, (const u16*)w, (const u16*)bias, (const u16*)res, (u16*)out, N, H, W,
             Cin, x2 ? C1 : Cin, Cout, kh, kw, stride, pad, Ho, Wo,
             (bias ? EPI_BIAS : 0) | (res ? EPI_RESIDUAL : 0) | (flags & CONV_UP2X), 0, 1};
  return conv_launch(a, stream, variant);
}

// v6 conv whose epilogue also writes the GroupNorm partial statistics of its output (gnp: [N, Ho*Wo/64,
// Cout] (mean, M2) float pairs, the cgs_groupnorm_nhwc_part layout with 64 pixels per block), so the
// following GroupNorm skips its statistics pass. Needs (Ho * Wo) % 256 == 0 and the v6 conditions.
CGS_EXPORT int cgs_conv2d_nhwc_gns(const void* x, const void* x2, int C1, const void* w, const void* bias,
                                   const void* res, void* out, int N, int H, int W, int Cin, int Cout, int kh, int kw,
                                   int stride, int pad, int Ho, int Wo, int flags, float* gnp, hipStream_t stream) {
  if (!gnp || Cin % 64 || (x2 && C1 % 64) || Cout % 8 || kh * kw * Cin < 128 || (Ho * Wo) % 256 ||
      ((uintptr_t)bias % 8) || ((uintptr_t)gnp % 16))
    return (int)hipErrorInvalidValue;
  ConvArgs a{(const u16*)x, (const u16*)x2, (const u16*)w, (const u16*)bias, (const u16*)res, (u16*)out, N, H, W,
             Cin, x2 ? C1 : Cin, Cout, kh, kw, stride, pad, Ho, Wo,
             (bias ? EPI_BIAS : 0) | (res ? EPI_RESIDUAL : 0) | (flags & CONV_UP2X), 0, 1};
  a.gnp = gnp;
  a.group_m = g_conv_group;
  conv_v6_go(a, stream);
  return (int)hipGetLastError();
}

// v7 with the split-K tail workspace (>= cgs_v7_ws_bytes(N*Ho*Wo, Cout, kh*kw*Cin) bytes).
CGS_EXPORT int cgs_conv2d_nhwc_v7ws(const void* x, const void* x2, int C1, const void* w, const void* bias,
                                    const void* res, void* out, int N, int H, int W, int Cin, int Cout, int kh, int kw,
                                    int stride, int pad, int Ho, int Wo, int flags, void* ws, long long ws_bytes,
                                    hipStream_t stream) {
  if (Cin % 32 || (x2 && (C1 % 32)) || Cout < 1 || (Cout % 8 && Cout > 16 && (Cin % 64 || (x2 && C1 % 64))))
    return (int)hipErrorInvalidValue;
  ConvArgs a{(const u16*)x, (const u16*)x2, (const u16*)w, (const u16*)bias, (const u16*)res, (u16*)out, N, H, W,
             Cin, x2 ? C1 : Cin, Cout, kh, kw, stride, pad, Ho, Wo,
             (bias ? EPI_BIAS : 0) | (res ? EPI_RESIDUAL : 0) | (flags & CONV_UP2X), 0, 1};
  return conv_launch(a, stream, 7, ws, ws_bytes);
}
