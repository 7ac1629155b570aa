// bf16 GEMM with fused epilogues for gfx950 (K01 Linear, K08 GEGLU, K15-style residual adds).
//   C[M,N] = alpha * A[M,K] * W[N,K]^T (+ bias[N]) (+ residual[M,N])      (EPI_BIAS / EPI_RESIDUAL)
//   GEGLU: W rows interleaved in 16-row groups [a0..a15 | g0..g15 | a16..]; out[M, N/2] = a*gelu(g)
// Both operands are K-contiguous ("NT"), which is what nn.Linear weights and activations are.
//
// Structure: 128x128x64 block tile, 256 threads = 4 waves in 2x2, each wave 64x64 made of 4x4
// v_mfma_f32_16x16x32_bf16 tiles (the 16x16 shape holds a higher clock than 32x32 under load,
// MI355X_MICROARCH 'DVFS give-back' item 7). Register-staged global->LDS double buffer with the
// next tile's global loads issued before the current tile's MFMAs (one barrier per K step).
// LDS rows padded to 80 elements (160 B): conflict-free ds_read_b128 for the 16x16x32 operand
// lane groups and conflict-free ds_write_b128. 1-D grid with the XCD-aware bijective remap so
// neighbouring output tiles (sharing A / W panels) run on the same XCD L2.
#include "common.h"
#include <stdlib.h>
#include "mfma_core.h"
#include "mfma_pp.h"
#include "mfma_pp160.h"
#include "mfma_ppk.h"

#define G_BM 128
#define G_BN 128
#define G_BK 64
#define G_LDW 80
#define EPI_BIAS 1
#define EPI_RESIDUAL 2
#define EPI_GEGLU 4
#define EPI_LNFOLD 8
#define EPI_F32OUT 16   // fp32 C (v7 only; attention scores of the wide-head path)
#define EPI_GELU 32     // GELU(acc * alpha + bias) before the residual: v6 (ACT kernel), mc::tile kernels, skinny

// fp8 e4m3fn (OCP) -> bf16 bits, exact (every e4m3 value is a bf16 value); NaN stays NaN.
__device__ __forceinline__ u16 fp8e4m3_to_bf16(uint32_t b) {
  const uint32_t s = (b & 0x80u) << 8, e = (b >> 3) & 15u, m = b & 7u;
  uint32_t mag = e ? (((e + 120u) << 7) | (m << 4)) : (__float_as_uint((float)m * 0.001953125f) >> 16);
  if ((b & 0x7fu) == 0x7fu) mag = 0x7fc0u;
  return (u16)(s | mag);
}

__device__ __forceinline__ s16x8 fp8x8_to_bf16x8(uint2 w) {
  s16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = (short)fp8e4m3_to_bf16((w.x >> (8 * j)) & 0xffu);
    o[4 + j] = (short)fp8e4m3_to_bf16((w.y >> (8 * j)) & 0xffu);
  }
  return o;
}

// W8 = true: W is fp8 e4m3fn (K21: fp8-stored weights, e.g. --fp8_e4m3fn-unet), widened to bf16 in
// the global->register staging step, so LDS / MFMA see bf16 exactly as for bf16 weights and the
// weight stream from HBM is halved.
template <bool W8>
__global__ __launch_bounds__(256, 2) void gemm_bf16_nt_kernel(
    const u16* __restrict__ A, const void* __restrict__ Wv, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_n) {
  const u16* __restrict__ W = static_cast<const u16*>(Wv);
  const uint8_t* __restrict__ W8p = static_cast<const uint8_t*>(Wv);
  __shared__ __attribute__((aligned(16))) u16 As[2][G_BM * G_LDW];
  __shared__ __attribute__((aligned(16))) u16 Ws[2][G_BN * G_LDW];

  const int nwg = gridDim.x;
  const int logical = xcd_remap(blockIdx.x, nwg);
  const int tm = logical / tiles_n;
  const int tn = logical % tiles_n;
  const int m0 = tm * G_BM;
  const int n0 = tn * G_BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (wave >> 1) * 64;
  const int wn = (wave & 1) * 64;

  // global -> register staging: 128 rows x 8 chunks(16B) = 1024 chunks per operand, 4 per thread
  s16x8 ra[4], rw[4];
  auto gload = [&](int kt) {
    const int k0 = kt * G_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int idx = tid + i * 256;
      int r = idx >> 3, c = (idx & 7) * 8;
      int gk = k0 + c;
      s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      int gm = m0 + r;
      ra[i] = (gm < M && gk < K) ? *reinterpret_cast<const s16x8*>(A + gm * lda + gk) : z;
      int gn = n0 + r;
      if constexpr (W8)
        rw[i] = (gn < N && gk < K) ? fp8x8_to_bf16x8(*reinterpret_cast<const uint2*>(W8p + gn * ldw + gk)) : z;
      else
        rw[i] = (gn < N && gk < K) ? *reinterpret_cast<const s16x8*>(W + gn * ldw + gk) : z;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int idx = tid + i * 256;
      int r = idx >> 3, c = (idx & 7) * 8;
      *reinterpret_cast<s16x8*>(&As[buf][r * G_LDW + c]) = ra[i];
      *reinterpret_cast<s16x8*>(&Ws[buf][r * G_LDW + c]) = rw[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + G_BK - 1) / G_BK;
  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15;
  const int fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
#pragma unroll
    for (int kk = 0; kk < G_BK / 32; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(&As[buf][(wm + i * 16 + fr) * G_LDW + kk * 32 + fk]));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(&Ws[buf][(wn + j * 16 + fr) * G_LDW + kk * 32 + fk]));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) sstore(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue. C layout (16x16x32): col = lane&15, row = (lane>>4)*4 + reg
  const int er = (lane >> 4) * 4;
  if (epi & EPI_GEGLU) {
    const int NO = N >> 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        int ca = n0 + wn + (2 * jp) * 16 + fr;        // interleaved column of the "a" half
        int cg = ca + 16;                             // matching gate column
        int oc = (n0 + wn) / 2 + jp * 16 + fr;        // output column
        if (cg >= N) continue;
        float ba = 0.f, bg = 0.f;
        if (epi & EPI_BIAS) { ba = bf2f(bias[ca]); bg = bf2f(bias[cg]); }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + i * 16 + er + r;
          if (row < M) {
            float a = acc[i][2 * jp][r] * alpha + ba;
            float g = acc[i][2 * jp + 1][r] * alpha + bg;
            C[row * ldc + oc] = f2bf(a * gelu_sig(g));
          }
        }
      }
    }
    (void)NO;
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int col = n0 + wn + j * 16 + fr;
    if (col >= N) continue;
    float bv = (epi & EPI_BIAS) ? bf2f(bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = m0 + wm + i * 16 + er + r;
        if (row < M) {
          float v = acc[i][j][r] * alpha + bv;
          if (epi & EPI_RESIDUAL) v += bf2f(R[row * ldr + col]);
          C[row * ldc + col] = f2bf(v);
        }
      }
    }
  }
}


// ================================================================================================
// v2: 256 x BN x 64 block tile, 512 threads = 8 waves (2 in M x 4 in N), each wave 128 x BN/4 built
// from v_mfma_f32_16x16x32_bf16 tiles. Operands stream global -> LDS with global_load_lds
// (LDS-DMA, 16 B per lane, no VGPR round trip) into a 2-deep LDS ring; one barrier per K step.
// LDS image is lane-linear per wave-instruction (8 rows x 128 B); the bank-conflict swizzle is
// applied on the SOURCE address (LDS chunk c of row r holds logical chunk c ^ ((r >> 1) & 7)) and
// undone on the ds_read_b128 fragment reads — conflict-free for the 16x16x32 operand lane groups.
// ================================================================================================
typedef __attribute__((address_space(3))) void lds_void;

template <int BN>
__global__ __launch_bounds__(512, 1) void gemm_bf16_nt_v2_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_n, int group_m) {
  constexpr int BM = 256, BK = 64;
  constexpr int WN = BN / 4;          // wave N extent
  constexpr int NJ = WN / 16;         // 16-wide n tiles per wave
  constexpr int NI = 8;               // 16-high m tiles per wave (128 rows)
  constexpr int A_BYTES = BM * BK * 2;
  constexpr int B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 8 / 8;   // glds instrs per wave for A (8 rows each, 8 waves)
  constexpr int B_INSTR = BN / 8 / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int nwg = gridDim.x;
  const int logical = xcd_remap(blockIdx.x, nwg);
  int tm, tn;
  grouped_tile(logical, nwg / tiles_n, tiles_n, group_m, tm, tn);
  const int m0 = tm * BM;
  const int n0 = tn * BN;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = (wave >> 2) * 128;
  const int wn = (wave & 3) * WN;

  // per-lane source pointers for the glds pieces (row within the 8-row piece, swizzled chunk)
  const int prow = lane >> 3;
  const int pchunk = lane & 7;
  const u16* asrc[A_INSTR];
  const u16* bsrc[B_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    int r = (wave * A_INSTR + i) * 8 + prow;
    int gr = min(m0 + r, M - 1);
    asrc[i] = A + gr * lda + 8 * (pchunk ^ ((r >> 1) & 7));
  }
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    int r = (wave * B_INSTR + i) * 8 + prow;
    int gr = min(n0 + r, N - 1);
    bsrc[i] = W + gr * ldw + 8 * (pchunk ^ ((r >> 1) & 7));
  }
  auto issue = [&](int kt, int stage) {
    unsigned char* base = smem + stage * STAGE;
    const int koff = kt * BK;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(asrc[i] + koff),
                                       (lds_void*)(base + ((wave * A_INSTR + i) * 8) * 128), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(bsrc[i] + koff),
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
      const int c = kk * 4 + fq;   // logical 16-B chunk of the row
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

  // ---- epilogue (16x16x32 C layout: col = lane&15, row = (lane>>4)*4 + reg)
  const int er = fq * 4;
  if (epi & EPI_GEGLU) {
#pragma unroll
    for (int jp = 0; jp < NJ / 2; ++jp) {
      int ca = n0 + wn + (2 * jp) * 16 + fr;
      int cg = ca + 16;
      int oc = (n0 + wn) / 2 + jp * 16 + fr;
      if (cg >= N) continue;
      float ba = 0.f, bg = 0.f;
      if (epi & EPI_BIAS) { ba = bf2f(bias[ca]); bg = bf2f(bias[cg]); }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int row = m0 + wm + i * 16 + er + r;
          if (row < M) {
            float a = acc[i][2 * jp][r] * alpha + ba;
            float g = acc[i][2 * jp + 1][r] * alpha + bg;
            C[row * ldc + oc] = f2bf(a * gelu_sig(g));
          }
        }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    int col = n0 + wn + j * 16 + fr;
    if (col >= N) continue;
    float bv = (epi & EPI_BIAS) ? bf2f(bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = m0 + wm + i * 16 + er + r;
        if (row < M) {
          float v = acc[i][j][r] * alpha + bv;
          if (epi & EPI_RESIDUAL) v += bf2f(R[row * ldr + col]);
          C[row * ldc + col] = f2bf(v);
        }
      }
  }
}

static int g_tile_group = 4;   // grouped tile order (tile rows per group; 1 = row-major): 4 measured -0.3 % per headline job vs 8 (profiles/r05/tile_group_ab.json)
CGS_EXPORT void cgs_set_tile_group(int g) { g_tile_group = g < 1 ? 1 : g; }

static int gemm_v2_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                          hipStream_t stream) {
  const bool wide = N >= 1024;
  const int BN = wide ? 256 : 128;
  int tiles_m = (M + 255) / 256;
  int tiles_n = (N + BN - 1) / BN;
  long long nwg = (long long)tiles_m * tiles_n;
  size_t lds = 2 * (256 * 64 * 2 + BN * 64 * 2);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)gemm_bf16_nt_v2_kernel<256>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        2 * (256 * 64 * 2 + 256 * 64 * 2));
    hipFuncSetAttribute((const void*)gemm_bf16_nt_v2_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        2 * (256 * 64 * 2 + 128 * 64 * 2));
    attr_set = true;
  }
  if (wide) {
    gemm_bf16_nt_v2_kernel<256><<<(unsigned)nwg, 512, lds, stream>>>(
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi,
        alpha, tiles_n, g_tile_group);
  } else {
    gemm_bf16_nt_v2_kernel<128><<<(unsigned)nwg, 512, lds, stream>>>(
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi,
        alpha, tiles_n, g_tile_group);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// v3: 256 x BN x 32 tiles, 4 waves x (128 x BN/2) on 32x32x16 MFMA, 4-stage LDS-DMA ring
// (mfma_core.h). Needs K % 32 == 0 and 16-B aligned rows.
struct DenseA {
  const u16* A;
  long long lda;
  int M;
  const u16* p[4];
  __device__ __forceinline__ void setup(int pi, int row) {
    row = row < M ? row : M - 1;
    p[pi] = A + (long long)row * lda + 8 * mc::src_chunk(threadIdx.x & 63);
  }
  __device__ __forceinline__ const void* src(int pi, int k0) const { return p[pi] + k0; }
};

template <int BN, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW / 4, NW / 4))) void gemm_bf16_nt_v3_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_n, int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / tiles_n, tiles_n, group_m, tm, tn);
  DenseA al{A, lda, M, {}};
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha};
  mc::tile<BN, NW>(al, W, ldw, M, N, K, tm * mc::BM, tn * BN, e, smem);
}

// v8 / v10 / v11: the same main loop on 128 x 128 / 64 x 128 / 128 x 64 tiles (4 waves), two
// workgroups per CU, for the short-M / short-N shapes whose 256-row grids leave most CUs idle (the
// batch-1 UNet: M = 2048 tokens at level 2 gives 40 256x256 tiles, 160 128x128 tiles, 320 64x128
// tiles). K % 32 == 0, 16-B aligned rows. rs / cs: the MC_EPI_LNFOLD operands.
template <int BN, int BMV, int NS = mc::STAGES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v8_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_n, int group_m, const float* rs, const float* cs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / tiles_n, tiles_n, group_m, tm, tn);
  DenseA al{A, lda, M, {}};
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  mc::tile<BN, 4, DenseA, BMV, NS>(al, W, ldw, M, N, K, tm * BMV, tn * BN, e, smem);
}

template <int BN, int BMV, int NS = mc::STAGES>
static int gemm_small_tile_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                  int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                  float alpha, hipStream_t stream, const float* rs, const float* cs) {
  using Cf = mc::Cfg<BN, 4, BMV, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v8_kernel<BN, BMV, NS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Cf::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + BN - 1) / BN;
  const long long nwg = (long long)((M + BMV - 1) / BMV) * tiles_n;
  if (nwg > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  gemm_bf16_nt_v8_kernel<BN, BMV, NS><<<(unsigned)nwg, 256, Cf::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_n, g_tile_group, rs, cs);
  return (int)hipGetLastError();
}

// variant 8 = 128 x 128, 10 = 64 x 128, 11 = 128 x 64 (4-stage ring); 12 = 64 x 128 and 13 = 128 x 64 with
// a 6-stage ring (72 / 72 KiB: still two workgroups per CU), 14 = 128 x 128 with 5 stages (80 KiB)
static int gemm_v8_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                          hipStream_t stream, int variant = 8, const float* rs = nullptr, const float* cs = nullptr) {
  if (variant == 10)
    return gemm_small_tile_launch<128, 64>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
  if (variant == 11)
    return gemm_small_tile_launch<64, 128>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
  if (variant == 12)
    return gemm_small_tile_launch<128, 64, 6>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
  if (variant == 13)
    return gemm_small_tile_launch<64, 128, 6>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
  if (variant == 14)
    return gemm_small_tile_launch<128, 128, 5>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
  return gemm_small_tile_launch<128, 128>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs);
}

// Split-K form of the v8 family (K13, batch-1 grids): blockIdx.y = K slice z, the tile computes
// A[:, z Ks : (z + 1) Ks] . W[:, same]^T into the fp32 partial ws[z] (MC_EPI_F32RAW); splitk_reduce_kernel
// then sums the slices and applies the whole epilogue (alpha, LayerNorm fold, bias, GELU, residual) once.
// For the under-filled shapes of SDXL batch 1 (M = 2048: FF-out K = 5120, out-proj K = 1280) a 160-tile
// grid becomes 320-640 workgroups.
template <int BN, int BMV, int NS = mc::STAGES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v8sk_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, float* __restrict__ ws, int M, int N, int Ks,
    long long lda, long long ldw, int tiles_n, int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / tiles_n, tiles_n, group_m, tm, tn);
  const long long kb = (long long)blockIdx.y * Ks;
  DenseA al{A + kb, lda, M, {}};
  mc::Epi e{reinterpret_cast<u16*>(ws + (long long)blockIdx.y * M * N), nullptr, nullptr, N, 0, MC_EPI_F32RAW, 1.f};
  mc::tile<BN, 4, DenseA, BMV, NS>(al, W + kb, ldw, M, N, Ks, tm * BMV, tn * BN, e, smem);
}

// out = epilogue(alpha * sum_z ws[z]) per 8-column chunk: LN fold (rs / cs), bias, GELU, residual -> bf16
template <bool LNF, bool ACT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S, u16* __restrict__ C,
                                                            const u16* __restrict__ bias, const u16* __restrict__ R,
                                                            const float* __restrict__ rs, const float* __restrict__ cs,
                                                            int M, int N, long long ldc, long long ldr, float alpha,
                                                            int flags) {
  const unsigned cpr = (unsigned)N >> 3;
  const long long chunks = (long long)M * cpr;
  const long long MN = (long long)M * N;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < chunks; i += (long long)gridDim.x * 256) {
    const unsigned row = (unsigned)(i / cpr);
    const int c0 = (int)(i - (long long)row * cpr) * 8;
    const float* p = ws + (long long)row * N + c0;
    float4 a0 = *reinterpret_cast<const float4*>(p), a1 = *reinterpret_cast<const float4*>(p + 4);
    for (int z = 1; z < S; ++z) {
      const float4 b0 = *reinterpret_cast<const float4*>(p + z * MN), b1 = *reinterpret_cast<const float4*>(p + z * MN + 4);
      a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
      a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
    }
    float v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    if constexpr (LNF) {
      const float2 st = *reinterpret_cast<const float2*>(rs + 2 * (long long)row);
      const float4 q0 = *reinterpret_cast<const float4*>(cs + c0), q1 = *reinterpret_cast<const float4*>(cs + c0 + 4);
      const float q[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = st.y * (v[t] - st.x * q[t]);
    } else {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] *= alpha;
    }
    if (flags & MC_EPI_BIAS) {
      const uint4 b = *reinterpret_cast<const uint4*>(bias + c0);
      const float4 lo = unpack4_bf16(uint2{b.x, b.y}), hi = unpack4_bf16(uint2{b.z, b.w});
      v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w; v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
    }
    if constexpr (ACT) {
#pragma unroll
      for (int t = 0; t < 8; ++t) v[t] = gelu_sig(v[t]);
    }
    if (flags & MC_EPI_RESIDUAL) {
      const uint4 rr = *reinterpret_cast<const uint4*>(R + (long long)row * ldr + c0);
      const float4 lo = unpack4_bf16(uint2{rr.x, rr.y}), hi = unpack4_bf16(uint2{rr.z, rr.w});
      v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w; v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
    }
    const uint2 o0 = pack4_bf16(v[0], v[1], v[2], v[3]), o1 = pack4_bf16(v[4], v[5], v[6], v[7]);
    *reinterpret_cast<uint4*>(C + (long long)row * ldc + c0) = uint4{o0.x, o0.y, o1.x, o1.y};
  }
}

template <int BN, int BMV, int NS = mc::STAGES>
static int gemm_splitk_go(const void* A, const void* W, float* ws, int M, int N, int Ks, int S, long long lda,
                          long long ldw, hipStream_t stream) {
  using Cf = mc::Cfg<BN, 4, BMV, NS>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v8sk_kernel<BN, BMV, NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, Cf::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + BN - 1) / BN;
  const long long nwg = (long long)((M + BMV - 1) / BMV) * tiles_n;
  if (nwg > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  gemm_bf16_nt_v8sk_kernel<BN, BMV, NS><<<dim3((unsigned)nwg, (unsigned)S), 256, Cf::LDS, stream>>>(
      (const u16*)A, (const u16*)W, ws, M, N, Ks, lda, ldw, tiles_n, g_tile_group);
  return (int)hipGetLastError();
}

// Bytes of fp32 workspace cgs_gemm_bf16_splitk needs.
CGS_EXPORT long long cgs_splitk_ws_bytes(int M, int N, int splits) { return 4LL * splits * M * N; }

// Split-K GEMM (see gemm_bf16_nt_v8sk_kernel): variant 8 / 10 / 11 / 14 = the v8 tile shapes; splits
// 2..8 with K % (32 * splits) == 0. epi: bias, residual, LN fold (rs / cs, alpha ignored), GELU -- no GEGLU.
CGS_EXPORT int cgs_gemm_bf16_splitk(const void* A, const void* W, void* C, const void* bias, const void* R,
                                    const float* rs, const float* cs, int M, int N, int K, long long lda,
                                    long long ldw, long long ldc, long long ldr, int epi, float alpha, int splits,
                                    int variant, float* ws, long long ws_bytes, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (splits < 2 || splits > 8 || K % (32 * splits) || N % 8 || lda % 8 || ldw % 8 || ldc % 8 ||
      (epi & ~(EPI_BIAS | EPI_RESIDUAL | EPI_LNFOLD | EPI_GELU)) || ((epi & EPI_RESIDUAL) && (!R || ldr % 8)) ||
      ((epi & EPI_BIAS) && !bias) || ((epi & EPI_LNFOLD) && (!rs || !cs)) || !ws ||
      ws_bytes < cgs_splitk_ws_bytes(M, N, splits) ||
      (((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)bias | (uintptr_t)R | (uintptr_t)ws) & 15))
    return (int)hipErrorInvalidValue;
  const int Ks = K / splits;
  int rc;
  switch (variant) {
    case 10: rc = gemm_splitk_go<128, 64>(A, W, ws, M, N, Ks, splits, lda, ldw, stream); break;
    case 11: rc = gemm_splitk_go<64, 128>(A, W, ws, M, N, Ks, splits, lda, ldw, stream); break;
    case 14: rc = gemm_splitk_go<128, 128, 5>(A, W, ws, M, N, Ks, splits, lda, ldw, stream); break;
    default: rc = gemm_splitk_go<128, 128>(A, W, ws, M, N, Ks, splits, lda, ldw, stream);
  }
  if (rc) return rc;
  const long long chunks = (long long)M * (N / 8);
  const long long nb = (chunks + 255) / 256;
  const unsigned blocks = (unsigned)(nb > 8192 ? 8192 : nb);
  const bool lnf = (epi & EPI_LNFOLD) != 0, act = (epi & EPI_GELU) != 0;
#define CGS_SKR(L, G) splitk_reduce_kernel<L, G><<<blocks, 256, 0, stream>>>(ws, splits, (u16*)C, (const u16*)bias, \
      (const u16*)R, rs, cs, M, N, ldc, ldr, alpha, epi)
  if (lnf) { if (act) CGS_SKR(true, true); else CGS_SKR(true, false); }
  else { if (act) CGS_SKR(false, true); else CGS_SKR(false, false); }
#undef CGS_SKR
  return (int)hipGetLastError();
}

template <int BN, int NW>
static void gemm_v3_go(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                       long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                       hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v3_kernel<BN, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, mc::Cfg<BN, NW>::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + BN - 1) / BN;
  const long long nwg = (long long)((M + mc::BM - 1) / mc::BM) * tiles_n;
  gemm_bf16_nt_v3_kernel<BN, NW><<<(unsigned)nwg, 64 * NW, mc::Cfg<BN, NW>::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_n, g_tile_group);
}

static int gemm_v3_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha, int nw,
                          hipStream_t stream) {
  const int BN = mc::pick_bn(M, N);
  if (nw == 8) {
    if (BN == 256) gemm_v3_go<256, 8>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    else gemm_v3_go<128, 8>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  } else {
    if (BN == 256) gemm_v3_go<256, 4>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    else gemm_v3_go<128, 4>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// v5: 256 x 256 x 64 ping-pong schedule (mfma_pp.h). Needs K % 64 == 0, N % 8 == 0, aligned rows.
struct DenseA8 {
  const u16* A;
  long long lda;
  int M;
  const u16* p[4];
  __device__ __forceinline__ void setup(int slot, int row) {
    row = row < M ? row : M - 1;
    p[slot] = A + (long long)row * lda + 8 * pp::src_chunk8(slot & 1);
  }
  __device__ __forceinline__ const void* src(int slot, int k0) const { return p[slot] + k0; }
};

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v5_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_n, int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  int tm, tn;
  grouped_tile(logical, gridDim.x / tiles_n, tiles_n, group_m, tm, tn);
  DenseA8 al{A, lda, M, {}};
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha};
  pp::tile(al, W, ldw, M, N, K, tm * pp::BM, tn * pp::BN, e, smem);
}

static int gemm_v5_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                          hipStream_t stream) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v5_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              pp::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + pp::BN - 1) / pp::BN;
  const long long nwg = (long long)((M + pp::BM - 1) / pp::BM) * tiles_n;
  gemm_bf16_nt_v5_kernel<<<(unsigned)nwg, pp::THREADS, pp::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_n, g_tile_group);
  return (int)hipGetLastError();
}

// Dense A loader with 32-bit byte offsets from one uniform base (global_load_lds saddr + voffset form:
// one VGPR per slot instead of a 64-bit pointer pair -- the v7 kernel runs at the 256-VGPR cap).
struct DenseA32 {
  const unsigned char* A;
  long long lda;
  int M;
  uint32_t off[4];
  __device__ __forceinline__ void setup(int slot, int row) {
    row = row < M ? row : M - 1;
    off[slot] = (uint32_t)(((long long)row * lda + 8 * pp::src_chunk8(slot & 1)) * 2);
  }
  __device__ __forceinline__ const void* src(int slot, int k0) const { return A + (off[slot] + (uint32_t)(k0 * 2)); }
  __device__ __forceinline__ void dma(int slot, int k0, unsigned char* dst) const { mc::lds_dma16(src(slot, k0), dst); }
};

// DenseA8's buffer-descriptor form (v6 DS & 64): per-slot row byte offsets fixed per tile, the K offset in
// the SGPR soffset -- the DMA needs no address VALU. Host: M * lda * 2 < 2 GiB. Measured against the
// pointer form (with DS & 128, the same for B): -5..+8 % per shape, no consistent gain on the GEMMs
// (profiles/r04/v6_buffer_dma_ab_r04ae.log; unlike the conv gathers, whose per-DMA address work was 5x
// larger) -- kept as CGS_V6_DS modes 65 / 129 / 193, default off.
struct DenseKB {
  static constexpr bool kOwnDMA = true;
  const u16* A;
  long long lda;
  int M;
  uint32_t off[4];
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ void init() {
    r = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((long long)M * lda * 2), 0x00020000);
  }
  __device__ __forceinline__ void tile(int) {}
  __device__ __forceinline__ void setup(int slot, int row) {
    row = row < M ? row : M - 1;
    off[slot] = (uint32_t)(((long long)row * lda + 8 * pp::src_chunk8(slot & 1)) * 2);
  }
  __device__ __forceinline__ void dma(int slot, int k0, unsigned char* dst) const {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (mc_lds_void*)dst, 16, off[slot], k0 * 2, 0, 0);
  }
};

// ------------------------------------------------------------------------------------------------
// v6: 256 x 160 x 64 ping-pong (mfma_pp160.h): whole-round tile counts on the SDXL channel widths.
// NI: 16-row MFMA blocks per wave -- 4 (256 x 160 tiles) or 2 (128 x 160: variant 19, the short-M grids)
template <bool LN = false, int DS = 0, bool GG = false, bool ACT = false, bool RSO = false, int NI = 4>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v6_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m, const float* rs = nullptr, const float* cs = nullptr,
    float* rso = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // 64-bit operand pointers: the 32-bit-offset (saddr) DMA form measured 3-10 % slower on v6
  // (profiles/r03/v6_offsets32.log)
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  e.gnp = rso;    // RSO: per-row LayerNorm statistics partials out
  if constexpr ((DS & 64) != 0) {
    DenseKB al;
    al.A = A;
    al.lda = lda;
    al.M = M;
    al.init();
    pq::run<DenseKB, LN, DS, false, GG, ACT, RSO, 1, 5, NI>(al, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
  } else {
    DenseA8 al{A, lda, M, {}};
    pq::run<DenseA8, LN, DS, false, GG, ACT, RSO, 1, 5, NI>(al, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
  }
}
// The one-wave-group form (pq::run W = 4): 128 x 80 tiles, 4 waves, two workgroups per CU -- variant 20 (the
// batch-1 grids: M = 2048 x N = 1280 is 256 tiles, one per CU, where 256 x 160 gives 64 and 128 x 160 128).
template <bool LN = false, bool RSO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v6w4_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m, const float* rs = nullptr, const float* cs = nullptr,
    float* rso = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  e.gnp = rso;
  DenseA8 al{A, lda, M, {}};
  pq::run<DenseA8, LN, 1, false, false, false, RSO, 1, 5, 2, 4>(al, W, ldw, M, N, K, e, smem, tiles_m, tiles_n,
                                                                 group_m);
}
static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// v6 DMA placement (pq::run DS): CGS_V6_DS at first use, cgs_v6_set_mode() after (in-process A/B).
// Default 1 (A parts in phase 0, B parts in phase 1): +4..11 % over all-in-phase-0 on the SDXL
// N = 640 / 1280 GEMMs and +2..4 % on the Cout = 320 convs (profiles/r03/v6_dma_split.log).
// Convs default to 51 = 19 | 32 (balanced split, phase 0 without the read drain: +1.5..6 % over 1 on
// the Cout = 320 convs, profiles/r03/v6_phase0_nodrain.log; 8-B column-tile-4 stores, which measured
// 1.5..5 % faster there than the permlane16-paired 16-B stores the GEMMs use,
// profiles/r03/v6_tile4_store_pairing.log); GEMMs keep 1 (19 / 17 within -6..+3 %).
static int g_v6_ds = -1, g_v6_conv_ds = -1;
int v6_ds() {
  if (g_v6_ds < 0) g_v6_ds = getenv("CGS_V6_DS") ? atoi(getenv("CGS_V6_DS")) : 1;
  return g_v6_ds;
}
int v6_conv_ds() {
  if (g_v6_conv_ds < 0) g_v6_conv_ds = getenv("CGS_V6_CONV_DS") ? atoi(getenv("CGS_V6_CONV_DS")) : 51;
  return g_v6_conv_ds;
}
CGS_EXPORT void cgs_v6_set_mode(int m) { g_v6_ds = m; g_v6_conv_ds = m; }

template <bool LN, int DS, bool GG = false, bool ACT = false, bool RSO = false, int NI = 4>
static void gemm_v6_go(int grid, const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                       int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                       int tiles_m, int tiles_n, hipStream_t stream, const float* rs, const float* cs,
                       float* rso = nullptr) {
  constexpr int lds = pq::Geo<5, NI>::LDS;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v6_kernel<LN, DS, GG, ACT, RSO, NI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  gemm_bf16_nt_v6_kernel<LN, DS, GG, ACT, RSO, NI><<<grid, pq::THREADS, lds, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_m, tiles_n, g_tile_group, rs, cs, rso);
}

template <bool LN, bool RSO>
static int gemm_v6w4_go(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                        long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                        hipStream_t stream, const float* rs, const float* cs, float* rso) {
  using Gm = pq::Geo<5, 2, 4>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v6w4_kernel<LN, RSO>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, Gm::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + Gm::BN - 1) / Gm::BN;
  const int tiles_m = (M + Gm::BM - 1) / Gm::BM;
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < 2 * num_cus() ? T : 2 * num_cus());
  gemm_bf16_nt_v6w4_kernel<LN, RSO><<<grid, 256, Gm::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_m, tiles_n, g_tile_group, rs, cs, rso);
  return (int)hipGetLastError();
}

static int gemm_v6_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                          hipStream_t stream, const float* rs = nullptr, const float* cs = nullptr, int ni = 4) {
  if (ni == 1) {   // variant 20: 128 x 80 tiles, one wave group (plain / bias / residual or LayerNorm-folded)
    if (epi & (EPI_GELU | EPI_GEGLU)) return (int)hipErrorInvalidValue;
    if (epi & EPI_LNFOLD)
      return gemm_v6w4_go<true, false>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs,
                                       nullptr);
    return gemm_v6w4_go<false, false>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, rs, cs,
                                      nullptr);
  }
  const int tiles_n = (N + pq::BN - 1) / pq::BN;
  const int tiles_m = (M + 64 * ni - 1) / (64 * ni);
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < num_cus() ? T : num_cus());
  if (ni == 2) {   // 128 x 160 tiles (variant 19): plain / bias / residual or LayerNorm-folded, default DMA split
    if (epi & (EPI_GELU | EPI_GEGLU)) return (int)hipErrorInvalidValue;
    if (epi & EPI_LNFOLD)
      gemm_v6_go<true, 1, false, false, false, 2>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
                                                  tiles_m, tiles_n, stream, rs, cs);
    else
      gemm_v6_go<false, 1, false, false, false, 2>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
                                                   tiles_m, tiles_n, stream, rs, cs);
    return (int)hipGetLastError();
  }
  int ds = v6_ds();
  if ((long long)M * lda * 2 >= (1ll << 31)) ds &= ~64;    // buffer-descriptor forms need < 2 GiB operands
  if ((long long)N * ldw * 2 >= (1ll << 31)) ds &= ~128;
  if (epi & EPI_GELU) {    // GELU epilogue: plain or LayerNorm-folded form (no GEGLU)
    if (epi & EPI_GEGLU) return (int)hipErrorInvalidValue;
    if (epi & EPI_LNFOLD)
      gemm_v6_go<true, 1, false, true>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m,
                                       tiles_n, stream, rs, cs);
    else
      gemm_v6_go<false, 1, false, true>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m,
                                        tiles_n, stream, rs, cs);
    return (int)hipGetLastError();
  }
  if (epi & EPI_GEGLU) {   // GEGLU epilogue (pq::run GG): split-DMA main loop, N % 160 == 0 (host-checked)
    if (epi & EPI_LNFOLD)
      gemm_v6_go<true, 1, true>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n,
                                stream, rs, cs);
    else
      gemm_v6_go<false, 1, true>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n,
                                 stream, rs, cs);
    return (int)hipGetLastError();
  }
  auto go = [&](auto lnc) {
    constexpr bool L = decltype(lnc)::value;
    switch (ds) {
      case 0: gemm_v6_go<L, 0>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 3: gemm_v6_go<L, 3>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 17: gemm_v6_go<L, 17>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 19: gemm_v6_go<L, 19>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 65: gemm_v6_go<L, 65>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 129: gemm_v6_go<L, 129>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      case 193: gemm_v6_go<L, 193>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs); break;
      default: gemm_v6_go<L, 1>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, stream, rs, cs);
    }
  };
  if (epi & EPI_LNFOLD) go(std::true_type{});
  else go(std::false_type{});
  return (int)hipGetLastError();
}


// v6 GEMM whose epilogue also writes per-(image, 64-row block, column) sums of squares of its bf16 output
// (pq::run GNS = 2, the sum-of-squares form of the conv GroupNorm-statistics epilogue) -- for Stable
// Cascade's ChannelMLP, where the GlobalResponseNorm after Linear -> GELU needs sum_HW h^2 per (image,
// channel): cgs_grn_apply_gns sums these partials instead of a statistics pass over h.
template <bool LN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v6_gns_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias, int M,
    int N, int K, long long lda, long long ldw, long long ldc, int epi, int tiles_m, int tiles_n, int group_m,
    const float* rs, const float* cs, float* gnp, int hw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, nullptr, ldc, 0, epi, 1.0f, rs, cs};
  e.gnp = gnp;
  e.hw = hw;
  DenseA8 al{A, lda, M, {}};
  pq::run<DenseA8, LN, 1, 2, false, true, false, 0>(al, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
}

// y = gelu(A W^T + bias) (LN-folded with rs / cs when epi has EPI_LNFOLD) + the sum-of-squares partials:
// part = [M / 64][N] floats. hw = rows per image, hw % 64 == 0; N % 8 == 0, K % 64 == 0, K >= 128.
CGS_EXPORT int cgs_gemm_bf16_gelu_gns(const void* A, const void* W, void* C, const void* bias, const float* rs,
                                      const float* cs, int M, int N, int K, long long lda, long long ldw,
                                      long long ldc, int epi, float* part, int hw, hipStream_t stream) {
  if (!part || !bias || hw <= 0 || hw % 64 || M % hw || N % 8 || K % 64 || K < 128 || lda % 8 || ldw % 8 ||
      ldc % 8 || (epi & ~(EPI_BIAS | EPI_GELU | EPI_LNFOLD)) != 0 || !(epi & EPI_GELU) || !(epi & EPI_BIAS) ||
      ((epi & EPI_LNFOLD) && (!rs || !cs)) || ((uintptr_t)bias % 8) ||
      ((((uintptr_t)A | (uintptr_t)W | (uintptr_t)C)) % 16) || ((uintptr_t)part % 16))
    return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  const int tiles_n = (N + pq::BN - 1) / pq::BN, tiles_m = (M + pq::BM - 1) / pq::BM;
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < num_cus() ? T : num_cus());
  static bool attr[2] = {false, false};
  const bool ln = (epi & EPI_LNFOLD) != 0;
  if (!attr[ln]) {
    (void)hipFuncSetAttribute(ln ? (const void*)gemm_bf16_nt_v6_gns_kernel<true> : (const void*)gemm_bf16_nt_v6_gns_kernel<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, pq::LDS);
    attr[ln] = true;
  }
  if (ln)
    gemm_bf16_nt_v6_gns_kernel<true><<<grid, pq::THREADS, pq::LDS, stream>>>(
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, M, N, K, lda, ldw, ldc, epi, tiles_m, tiles_n,
        g_tile_group, rs, cs, part, hw);
  else
    gemm_bf16_nt_v6_gns_kernel<false><<<grid, pq::THREADS, pq::LDS, stream>>>(
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, M, N, K, lda, ldw, ldc, epi, tiles_m, tiles_n,
        g_tile_group, rs, cs, part, hw);
  return (int)hipGetLastError();
}

// v6 GEMM (bias / residual epilogue) that also writes per-row LayerNorm statistics partials of its output
// (pq::run RSO): part = [M][N / 80] (mean, M2) float pairs; cgs_ln_rs_from_partials turns them into the
// (mean, rstd) rows a LayerNorm-folded GEMM reads. N % 160 == 0, K % 64 == 0, K >= 128.
static int gemm_rowstats(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                         long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha, float* part,
                         int ni, hipStream_t stream);
CGS_EXPORT int cgs_gemm_bf16_rowstats(const void* A, const void* W, void* C, const void* bias, const void* R, int M,
                                      int N, int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                      float alpha, float* part, hipStream_t stream) {
  return gemm_rowstats(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, part, 4, stream);
}
// variant 6 (256 x 160) or 19 (128 x 160 tiles)
CGS_EXPORT int cgs_gemm_bf16_rowstats_v(const void* A, const void* W, void* C, const void* bias, const void* R, int M,
                                        int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
                                        int epi, float alpha, float* part, int variant, hipStream_t stream) {
  if (variant != 6 && variant != 19 && variant != 20) return (int)hipErrorInvalidValue;
  return gemm_rowstats(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, part,
                       variant == 20 ? 1 : variant == 19 ? 2 : 4, stream);
}
static int gemm_rowstats(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                         long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha, float* part,
                         int ni, hipStream_t stream) {
  if (!part || N % 160 || K % 64 || K < 128 || (epi & ~(EPI_BIAS | EPI_RESIDUAL)) || lda % 8 || ldw % 8 ||
      ldc % 8 || ((epi & EPI_RESIDUAL) && ldr % 8) || ((uintptr_t)bias % 8) ||
      ((((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)R)) % 16) || ((uintptr_t)part % 8))
    return (int)hipErrorInvalidValue;
  if (M == 0) return 0;
  if (ni == 1) return gemm_v6w4_go<false, true>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream,
                                                nullptr, nullptr, part);
  const int tiles_n = N / pq::BN;
  const int tiles_m = (M + 64 * ni - 1) / (64 * ni);
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < num_cus() ? T : num_cus());
  if (ni == 2)
    gemm_v6_go<false, 1, false, false, true, 2>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
                                                tiles_m, tiles_n, stream, nullptr, nullptr, part);
  else
    gemm_v6_go<false, 1, false, false, true>(grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m,
                                             tiles_n, stream, nullptr, nullptr, part);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// v7: persistent 256 x 256 x 64 ping-pong with cross-tile prefetch and a register epilogue (mfma_ppk.h)
template <bool GG, bool LN = false, bool F32 = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm_bf16_nt_v7_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m, ppk::Split sp, const float* rs = nullptr,
    const float* cs = nullptr) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  DenseA32 al{reinterpret_cast<const unsigned char*>(A), lda, M, {}};
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  ppk::run<GG, LN, DenseA32, F32>(al, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m, sp);
}

// Timing-probe bits of the v7 loop (ppk::run): CGS_V7_SPLIT_DBG at first use, cgs_v7_set_dbg() after.
static int g_v7_dbg = -1;
static int v7_dbg() {
  if (g_v7_dbg < 0) g_v7_dbg = getenv("CGS_V7_SPLIT_DBG") ? atoi(getenv("CGS_V7_SPLIT_DBG")) : 0;
  return g_v7_dbg;
}
CGS_EXPORT void cgs_v7_set_dbg(int d) { g_v7_dbg = d; }

// ws (may be null): split-K tail workspace of >= cgs_v7_ws_bytes(M, N, K) bytes; without it the
// tail round runs whole tiles.
static int gemm_v7_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                          long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                          void* ws, long long ws_bytes, hipStream_t stream, const float* rs = nullptr,
                          const float* cs = nullptr) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v7_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ppk::LDS);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v7_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ppk::LDS);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v7_kernel<false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, ppk::LDS);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v7_kernel<true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, ppk::LDS);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_v7_kernel<false, false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, ppk::LDS);
    attr_set = true;
  }
  const int tiles_n = (N + ppk::BN - 1) / ppk::BN;
  const int tiles_m = (M + ppk::BM - 1) / ppk::BM;
  const long long T = (long long)tiles_m * tiles_n;
  ppk::Split sp{0, 1, nullptr, nullptr, v7_dbg()};
  long long U = T;
  if (ws && ws_bytes >= ppk::split_ws_bytes(T, K / ppk::BK, num_cus())) {
    sp.S = ppk::split_plan(T, K / ppk::BK, num_cus(), sp.t_full);
    if (sp.S > 1) {
      const long long tail = T - sp.t_full;
      sp.part = (float4*)ws;
      sp.cnt = (int*)((char*)ws + tail * sp.S * 32ll * ppk::THREADS * 16);
      if (!(sp.dbg & 2)) {
        ppk::zero_counters_kernel<<<1, 256, 0, stream>>>(sp.cnt, (int)tail);
        hipError_t err = hipGetLastError();
        if (err != hipSuccess) return (int)err;
      }
      U = sp.t_full + tail * sp.S;
    }
  }
  static const int grid_cap = getenv("CGS_V7_GRID") ? atoi(getenv("CGS_V7_GRID")) : 0;   // diagnostics only
  int grid = (int)(U < num_cus() ? U : num_cus());
  if (grid_cap > 0 && grid > grid_cap) grid = grid_cap;
  const bool ln = (epi & EPI_LNFOLD) != 0;
#define CGS_V7L(GG, LNF)                                                                                            \
  gemm_bf16_nt_v7_kernel<GG, LNF><<<grid, ppk::THREADS, ppk::LDS, stream>>>(                                        \
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, \
      tiles_m, tiles_n, g_tile_group, sp, rs, cs)
  if (epi & EPI_F32OUT) {
    gemm_bf16_nt_v7_kernel<false, false, true><<<grid, ppk::THREADS, ppk::LDS, stream>>>(
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
        tiles_m, tiles_n, g_tile_group, sp, rs, cs);
  } else if (epi & EPI_GEGLU) {
    if (ln) CGS_V7L(true, true);
    else CGS_V7L(true, false);
  } else {
    if (ln) CGS_V7L(false, true);
    else CGS_V7L(false, false);
  }
#undef CGS_V7L
  return (int)hipGetLastError();
}

// Split-K tail workspace size of the v7 GEMM / conv for an M x N x K problem (0: no split).
CGS_EXPORT long long cgs_v7_ws_bytes(int M, int N, int K) {
  if (K % ppk::BK || K < 2 * ppk::BK) return 0;
  const long long T = (long long)((M + ppk::BM - 1) / ppk::BM) * ((N + ppk::BN - 1) / ppk::BN);
  return ppk::split_ws_bytes(T, K / ppk::BK, num_cus());
}

// ------------------------------------------------------------------------------------------------
// Skinny GEMM (M <= 128): CLIP text-encoder layers at one prompt (M = 77), the ResBlock time-
// embedding projections (M = UNet batch). A 256x256 tile per workgroup leaves ~15 CUs busy there and
// runs each call at a few TF/s; these calls are weight-bandwidth bound instead. One workgroup per 16
// output columns (N / 16 workgroups), all M rows as MR 16-row MFMA tiles (16x16x32 bf16), the K
// range split over the 8 waves (K-steps interleaved), fragments loaded straight from global memory
// (16 B per lane, next K-step's loads issued before this one's MFMAs), partial accumulators summed
// through LDS, bias / residual epilogue. Needs K % 32 == 0 and 16-B aligned rows.
constexpr int SK_WAVES = 8;

// Split-K form (part != null): gridDim.y = S slices of the K-steps; slice s writes its fp32 partial sums to
// part[s][row][col] and gemm_skinny_reduce_kernel adds the S slices and applies the epilogue. The 16-column
// grid alone is N / 16 workgroups -- 80 for N = 1280 (CLIP-G fc2 / out-proj at K = 5120 / 1280 ran ~30 % of
// the CUs for 40-80 us); the slices fill the chip.
template <int MR>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_kernel(const u16* __restrict__ A, const u16* __restrict__ W,
                                                          u16* __restrict__ C, const u16* __restrict__ bias,
                                                          const u16* __restrict__ R, int M, int N, int K, long long lda,
                                                          long long ldw, long long ldc, long long ldr, int epi,
                                                          float alpha, float* __restrict__ part = nullptr) {
  __shared__ f32x4 red[SK_WAVES][MR][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int fr = lane & 15, fq = lane >> 4;
  const int ncol = min(n0 + fr, N - 1);
  const u16* wp = W + (long long)ncol * ldw + 8 * fq;
  const u16* ap[MR];
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) ap[mr] = A + (long long)min(mr * 16 + fr, M - 1) * lda + 8 * fq;
  f32x4 acc[MR];
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) acc[mr] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nks_all = K / 32;
  const int per = (nks_all + gridDim.y - 1) / gridDim.y;
  const int ks0 = blockIdx.y * per;
  const int nks = min(nks_all, ks0 + per);
  int ks = ks0 + wave;
  if (ks < nks) {
    bf16x8 a[MR], b;
    b = *reinterpret_cast<const bf16x8*>(wp + ks * 32);
#pragma unroll
    for (int mr = 0; mr < MR; ++mr) a[mr] = *reinterpret_cast<const bf16x8*>(ap[mr] + ks * 32);
    for (; ks < nks; ks += SK_WAVES) {
      const int kn = ks + SK_WAVES < nks ? ks + SK_WAVES : ks;
      const bf16x8 bn = *reinterpret_cast<const bf16x8*>(wp + kn * 32);
      bf16x8 an[MR];
#pragma unroll
      for (int mr = 0; mr < MR; ++mr) an[mr] = *reinterpret_cast<const bf16x8*>(ap[mr] + kn * 32);
#pragma unroll
      for (int mr = 0; mr < MR; ++mr) acc[mr] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mr], b, acc[mr], 0, 0, 0);
      b = bn;
#pragma unroll
      for (int mr = 0; mr < MR; ++mr) a[mr] = an[mr];
    }
  }
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) red[wave][mr][lane] = acc[mr];
  __syncthreads();
  const int col = n0 + fr;
  float bv = 0.f;
  if (!part && (epi & EPI_BIAS) && col < N) bv = bf2f(bias[col]);
#pragma unroll
  for (int mr = 0; mr < MR; ++mr) {
    if ((mr % SK_WAVES) != wave) continue;
    f32x4 v = red[0][mr][lane];
#pragma unroll
    for (int w = 1; w < SK_WAVES; ++w) v += red[w][mr][lane];
    if (part) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mr * 16 + fq * 4 + r;
        if (row < M && col < N) part[((long long)blockIdx.y * M + row) * N + col] = v[r];
      }
      continue;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = mr * 16 + fq * 4 + r;
      if (row < M && col < N) {
        float o = v[r] * alpha + bv;
        if (epi & EPI_GELU) o = gelu_sig(o);
        if (epi & EPI_RESIDUAL) o += bf2f(R[(long long)row * ldr + col]);
        C[(long long)row * ldc + col] = f2bf(o);
      }
    }
  }
}

// S partial slices + epilogue: out[row][col] = epi(sum_s part[s][row][col])
__global__ __launch_bounds__(256) void gemm_skinny_reduce_kernel(const float* __restrict__ part, u16* __restrict__ C,
                                                                 const u16* __restrict__ bias, const u16* __restrict__ R,
                                                                 int M, int N, int S, long long ldc, long long ldr,
                                                                 int epi, float alpha) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)M * N) return;
  const int row = (int)(i / N), col = (int)(i - (long long)row * N);
  float o = 0.f;
  for (int s = 0; s < S; ++s) o += part[(long long)s * M * N + i];
  o *= alpha;
  if (epi & EPI_BIAS) o += bf2f(bias[col]);
  if (epi & EPI_GELU) o = gelu_sig(o);
  if (epi & EPI_RESIDUAL) o += bf2f(R[(long long)row * ldr + col]);
  C[(long long)row * ldc + col] = f2bf(o);
}

// K-slices for the skinny kernel: fill ~2 waves of workgroups per CU, >= 8 K-steps per slice, <= 8 slices.
// Only for long K (>= 4096: CLIP-G fc2 29 -> 22 us); below that the second launch costs more than the
// slices save (profiles/r04/skinny_split_ab.log).
static int skinny_splits(int M, int N, int K) {
  if (M > 128 || K % 32 || K < 4096) return 1;
  const int wgs = (N + 15) / 16, nks = K / 32;
  int S = (512 + wgs - 1) / wgs;
  S = S < nks / 8 ? S : nks / 8;
  return S < 2 ? 1 : (S > 8 ? 8 : S);
}

CGS_EXPORT long long cgs_gemm_skinny_ws_bytes(int M, int N, int K) {
  const int S = skinny_splits(M, N, K);
  return S > 1 ? (long long)S * M * N * 4 : 0;
}

static int gemm_skinny_launch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                              int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                              hipStream_t stream, void* ws = nullptr, long long ws_bytes = 0) {
  const int S = skinny_splits(M, N, K);
  const bool split = S > 1 && ws && ws_bytes >= (long long)S * M * N * 4;
  const dim3 g((unsigned)((N + 15) / 16), split ? (unsigned)S : 1u);
  float* part = split ? (float*)ws : nullptr;
  const int mr = (M + 15) / 16;
#define CGS_SKINNY(MRV)                                                                                          \
  gemm_skinny_kernel<MRV><<<g, 64 * SK_WAVES, 0, stream>>>((const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias,         \
                                                 (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, part)
  switch (mr) {
    case 0: CGS_SKINNY(1); break;
    case 2: CGS_SKINNY(2); break;
    case 3: CGS_SKINNY(3); break;
    case 4: CGS_SKINNY(4); break;
    case 5: CGS_SKINNY(5); break;
    case 6: CGS_SKINNY(6); break;
    case 7: CGS_SKINNY(7); break;
    default: CGS_SKINNY(8); break;
  }
#undef CGS_SKINNY
  if (split) {
    const long long n = (long long)M * N;
    gemm_skinny_reduce_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(
        part, (u16*)C, (const u16*)bias, (const u16*)R, M, N, S, ldc, ldr, epi, alpha);
  }
  return (int)hipGetLastError();
}

// The skinny GEMM with its split-K workspace (ws from the caller's allocator, >= cgs_gemm_skinny_ws_bytes).
CGS_EXPORT int cgs_gemm_skinny_ws(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                  int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                  float alpha, void* ws, long long ws_bytes, hipStream_t stream) {
  if (M > 128 || K % 32 || lda % 8 || ldw % 8 || (((uintptr_t)A | (uintptr_t)W) % 16) ||
      (epi & (EPI_GEGLU | EPI_F32OUT | EPI_LNFOLD)))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  return gemm_skinny_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, ws, ws_bytes);
}

static int g_gemm_variant = -1;   // -1 auto, 1 = v1 only, 2 = v2, 3 = v3 (4 waves), 4 = v3 (8 waves), 5 = v5 ping-pong

CGS_EXPORT void cgs_gemm_set_variant(int v) { g_gemm_variant = v; }

// w6 (gemm_w6.hip): one-wave-per-SIMD 256x256x64 persistent kernel with full-line LDS-DMA; variant 16.
// variant 17: its 256x160 form (128 x 80 wave tiles).
CGS_EXPORT int cgs_gemm_w6_ok(int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                              int bn);
CGS_EXPORT int cgs_gemm_bf16_w6(const void* A, const void* W, void* C, const void* bias, const void* R, const float* rs,
                                const float* cs, int M, int N, int K, long long lda, long long ldw, long long ldc,
                                long long ldr, int epi, float alpha, int dbg, int group_m, int grid_cap, int bn,
                                hipStream_t stream);
constexpr int kVariantW6 = 16, kVariantW6n160 = 17;

// w6's pointer alignment (cgs_gemm_bf16_w6 returns hipErrorInvalidValue otherwise)
static bool w6_ptrs_ok(const void* A, const void* W, const void* C, const void* bias, const void* R, int epi) {
  return ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 == 0 && (!(epi & EPI_RESIDUAL) || (uintptr_t)R % 16 == 0) &&
         (!(epi & EPI_BIAS) || (uintptr_t)bias % 16 == 0);
}

static int gemm_dispatch(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                         long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                         int variant, hipStream_t stream, void* ws = nullptr, long long ws_bytes = 0) {
  if (K % 8 || lda % 8 || ldw % 8) return (int)hipErrorInvalidValue;
  if ((epi & EPI_GEGLU) && (N % 32)) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  if (epi & EPI_GELU) {
    // GELU epilogue kernels: skinny (M <= 128), v6 (variant 6), the mc::tile family (v3 / v4, v8 and the
    // small tiles; auto = v8). No GEGLU / LayerNorm-fold / fp32-out combination.
    if (epi & (EPI_GEGLU | EPI_LNFOLD | EPI_F32OUT)) return (int)hipErrorInvalidValue;
    const bool ok = (K % 32 == 0) && (N % 8 == 0) && (ldc % 8 == 0) && (!(epi & EPI_RESIDUAL) || ldr % 8 == 0) &&
                    ((((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)R)) % 16 == 0);
    if (!ok) return (int)hipErrorInvalidValue;
    if (M <= 128 && (variant == -1 || variant == 9))
      return gemm_skinny_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    if (variant == 6) {
      if (K % 64 || K < 128 || ((uintptr_t)bias % 8)) return (int)hipErrorInvalidValue;
      return gemm_v6_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    }
    if (variant == 3 || variant == 4)
      return gemm_v3_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, variant == 3 ? 4 : 8, stream);
    if (variant == -1 || variant == 8 || (variant >= 10 && variant <= 14))
      return gemm_v8_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream,
                            variant == -1 ? 8 : variant);
    return (int)hipErrorInvalidValue;
  }
  // v2 needs K % 64 == 0 and 16-B aligned rows; it pays off once there are >= ~256 big tiles'
  // worth of work (otherwise the 128x128 kernel keeps more CUs busy).
  bool v2_ok = (K % 64 == 0) && (lda % 8 == 0) && (ldw % 8 == 0) && M >= 256 && N >= 128 &&
               (((uintptr_t)A | (uintptr_t)W) % 16 == 0);
  const int nout = (epi & EPI_GEGLU) ? N / 2 : N;
  bool v3_ok = (K % 32 == 0) && (lda % 8 == 0) && (ldw % 8 == 0) && (nout % 8 == 0) && (ldc % 8 == 0) &&
               (!(epi & EPI_RESIDUAL) || ldr % 8 == 0) &&
               ((((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)R)) % 16 == 0);
  // skinny M (<= 128 rows): weight-bandwidth bound, one workgroup per 16 columns (variant 9, or auto)
  if (M <= 128 && K % 32 == 0 && !(epi & (EPI_GEGLU | EPI_F32OUT | EPI_LNFOLD)) && (variant == -1 || variant == 9) &&
      lda % 8 == 0 && ldw % 8 == 0 && (((uintptr_t)A | (uintptr_t)W) % 16 == 0))
    return gemm_skinny_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  if (epi & EPI_F32OUT) {   // fp32 output: v7 only, plain / bias epilogue
    if ((epi & (EPI_GEGLU | EPI_RESIDUAL | EPI_LNFOLD)) || !v3_ok || K % 64 || K < 128 || ((uintptr_t)bias % 8) ||
        (long long)M * lda * 2 >= (1ll << 32) || (long long)N * ldw * 2 >= (1ll << 32))
      return (int)hipErrorInvalidValue;
    return gemm_v7_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, ws, ws_bytes, stream);
  }
  if (variant == kVariantW6 || variant == kVariantW6n160) {
    // a table choice made by shape: a call outside w6's stride / alignment domain (16-B bias / residual
    // pointers, views with lda != K) runs on the auto path instead of failing
    const int bn = variant == kVariantW6 ? 256 : 160;
    if (cgs_gemm_w6_ok(M, N, K, lda, ldw, ldc, ldr, epi, bn) && w6_ptrs_ok(A, W, C, bias, R, epi))
      return cgs_gemm_bf16_w6(A, W, C, bias, R, nullptr, nullptr, M, N, K, lda, ldw, ldc, ldr, epi, alpha, 0, 4, 0,
                              bn, stream);
    variant = -1;
  }
  if (v3_ok && K % 64 == 0 && K >= 128 && variant == 6 && (!(epi & EPI_GEGLU) || (N % 160 == 0 && !(epi & EPI_RESIDUAL))) &&
      ((uintptr_t)bias % 8 == 0))
    return gemm_v6_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  if (v3_ok && K % 64 == 0 && K >= 128 && (variant == 19 || variant == 20) && !(epi & EPI_GEGLU) &&
      ((uintptr_t)bias % 8 == 0))
    return gemm_v6_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, nullptr, nullptr,
                          variant == 20 ? 1 : 2);
  if (v3_ok && K % 64 == 0 && K >= 128 && variant == 7 && !((epi & EPI_GEGLU) && (epi & EPI_RESIDUAL)) &&
      ((uintptr_t)bias % 8 == 0) && (long long)M * lda * 2 < (1ll << 32) && (long long)N * ldw * 2 < (1ll << 32))
    return gemm_v7_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, ws, ws_bytes, stream);
  if (v3_ok && (variant == 8 || (variant >= 10 && variant <= 14)) && !(epi & EPI_LNFOLD))
    return gemm_v8_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream, variant);
  if (v3_ok && K % 64 == 0 && variant == 5)
    return gemm_v5_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  if (v3_ok && (variant >= 3 || variant == -1)) {
    long long t3 = (long long)((M + 255) / 256) * ((N + 127) / 128);
    if (variant >= 3 || t3 >= 128)
      return gemm_v3_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
                            variant == 3 ? 4 : 8, stream);
  }
  if (v2_ok && variant != 1 && variant < 3) {
    const int BN = N >= 1024 ? 256 : 128;
    long long t2 = (long long)((M + 255) / 256) * ((N + BN - 1) / BN);
    if (variant == 2 || t2 >= 128)
      return gemm_v2_launch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
  }
  int tiles_m = (M + G_BM - 1) / G_BM;
  int tiles_n = (N + G_BN - 1) / G_BN;
  long long nwg = (long long)tiles_m * tiles_n;
  gemm_bf16_nt_kernel<false><<<(unsigned)nwg, 256, 0, stream>>>((const u16*)A, W, (u16*)C, (const u16*)bias,
                                                               (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
                                                               tiles_n);
  return (int)hipGetLastError();
}

// C = A (bf16) x W^T (fp8 e4m3fn, ldw in elements = bytes) with the same epilogues.
CGS_EXPORT int cgs_gemm_bf16_w8(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                float alpha, hipStream_t stream) {
  if (K % 8 || lda % 8 || ldw % 8 || ((uintptr_t)W & 7) || ((uintptr_t)A & 15)) return (int)hipErrorInvalidValue;
  if ((epi & EPI_GEGLU) && (N % 32)) return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  const int tiles_m = (M + G_BM - 1) / G_BM, tiles_n = (N + G_BN - 1) / G_BN;
  gemm_bf16_nt_kernel<true><<<(unsigned)((long long)tiles_m * tiles_n), 256, 0, stream>>>(
      (const u16*)A, W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_n);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_gemm_bf16(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                             int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                             hipStream_t stream) {
  return gemm_dispatch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, g_gemm_variant, stream);
}

// Per-call kernel choice (used by the op-layer autotuner): variant as in cgs_gemm_set_variant.
CGS_EXPORT int cgs_gemm_bf16_v(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                               int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                               int variant, hipStream_t stream) {
  if (variant == -2) variant = g_gemm_variant;   // -2: the process-wide override (default auto)
  return gemm_dispatch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, variant, stream);
}

// v7 with the split-K tail workspace (ws from the caller's allocator, >= cgs_v7_ws_bytes bytes).
CGS_EXPORT int cgs_gemm_bf16_v7ws(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                  int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                  float alpha, void* ws, long long ws_bytes, hipStream_t stream) {
  return gemm_dispatch(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, 7, stream, ws, ws_bytes);
}

// LayerNorm folded into the GEMM (MC_EPI_LNFOLD): C = rstd_r * (A W'^T - mean_r * cs) + bias, with
// rs = per-row (mean, rstd) of A (cgs_layernorm_stats) and W' / cs / bias precomputed by the caller
// (W' = W * gamma, cs = rowsum(W'), bias = b + W beta). v7 only (+ optional GEGLU, split-K tail).
static int gemm_lnfold(const void* A, const void* W, void* C, const void* bias, const float* rs, const float* cs,
                       int M, int N, int K, long long lda, long long ldw, long long ldc, int epi, void* ws,
                       long long ws_bytes, int variant, hipStream_t stream) {
  const int nout = (epi & EPI_GEGLU) ? N / 2 : N;
  if (!rs || !cs || K % 64 || K < 128 || lda % 8 || ldw % 8 || ldc % 8 || nout % 8 || (epi & EPI_RESIDUAL) ||
      ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 || ((uintptr_t)bias % 8) || ((uintptr_t)cs % 16) ||
      ((uintptr_t)rs % 8) || (long long)M * lda * 2 >= (1ll << 32) || (long long)N * ldw * 2 >= (1ll << 32))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  if (epi & EPI_GELU) {    // LayerNorm -> Linear -> GELU (Cascade ChannelMLP): v6 ACT or the mc::tile kernels
    if ((epi & EPI_GEGLU) || variant == 7) return (int)hipErrorInvalidValue;
    if (variant == 6 || (variant < 0 && N % 160 == 0))
      return gemm_v6_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, stream, rs, cs);
    return gemm_v8_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, stream,
                          variant < 0 ? 8 : variant, rs, cs);
  }
  if (variant == kVariantW6 || variant == kVariantW6n160) {    // outside w6's domain: the v6 / v7 choice below
    const int bn = variant == kVariantW6 ? 256 : 160;
    if (cgs_gemm_w6_ok(M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, bn) && w6_ptrs_ok(A, W, C, bias, nullptr, epi))
      return cgs_gemm_bf16_w6(A, W, C, bias, nullptr, rs, cs, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, 0, 4,
                              0, bn, stream);
    variant = -1;
  }
  // v6 (256x160) for the N = 640 / 1280 projections (the cross-attention query), v7 otherwise
  if (variant == 8 || (variant >= 10 && variant <= 14))
    return gemm_v8_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, stream, variant,
                          rs, cs);
  const bool v6_ok = N % 160 == 0;   // incl. GEGLU (pq::run GG)
  if (variant == 6 && !v6_ok) return (int)hipErrorInvalidValue;
  if (variant == 19 || variant == 20) {     // 128 x 160 / 128 x 80 tiles: no GEGLU form
    if (N % 80 || (variant == 19 && !v6_ok) || (epi & EPI_GEGLU)) return (int)hipErrorInvalidValue;
    return gemm_v6_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, stream, rs, cs,
                          variant == 20 ? 1 : 2);
  }
  if (variant == 6 || (variant < 0 && v6_ok && !(epi & EPI_GEGLU) && N <= 1280))
    return gemm_v6_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, stream, rs, cs);
  return gemm_v7_launch(A, W, C, bias, nullptr, M, N, K, lda, ldw, ldc, 0, epi | EPI_LNFOLD, 1.0f, ws, ws_bytes, stream,
                        rs, cs);
}

CGS_EXPORT int cgs_gemm_bf16_lnfold(const void* A, const void* W, void* C, const void* bias, const float* rs,
                                    const float* cs, int M, int N, int K, long long lda, long long ldw, long long ldc,
                                    int epi, void* ws, long long ws_bytes, hipStream_t stream) {
  return gemm_lnfold(A, W, C, bias, rs, cs, M, N, K, lda, ldw, ldc, epi, ws, ws_bytes, -1, stream);
}

// Per-call kernel choice for the LayerNorm-folded GEMM (op-layer autotuner): -1 = v6 / v7 by shape,
// 6 / 7 = v6 / v7 explicitly, 8 / 10..14 = the small-tile kernels for under-filled grids.
CGS_EXPORT int cgs_gemm_bf16_lnfold_v(const void* A, const void* W, void* C, const void* bias, const float* rs,
                                      const float* cs, int M, int N, int K, long long lda, long long ldw, long long ldc,
                                      int epi, void* ws, long long ws_bytes, int variant, hipStream_t stream) {
  return gemm_lnfold(A, W, C, bias, rs, cs, M, N, K, lda, ldw, ldc, epi, ws, ws_bytes, variant, stream);
}
