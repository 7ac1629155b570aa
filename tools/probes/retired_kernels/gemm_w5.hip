// "w5" GEMM (experiment): C[M,N] = A[M,K] W[N,K]^T (+ bias) (+ residual), bf16 in / out, fp32 accumulate.
//
// One wave per SIMD (4 waves, one 256 x 256 tile per workgroup, 128 x 128 per wave = 8 x 8
// v_mfma_f32_16x16x32_bf16 tiles, 256 accumulator registers in the AGPR half of the 512-entry file) with
// a 4-slot ring of 32-deep K stages (4 x 32 KiB of LDS): stage s+3 is DMA'd into the slot stage s-1
// vacated while stage s computes, so ONE barrier per 64 MFMAs and every stage's loads have two whole
// stages (~2000 MFMA cycles) to land. Per stage and wave: 64 MFMAs on the fragments read during the
// previous stage, interleaved 1:4 with the 16 fragment reads of the next stage and 1:8 with the 8 LDS
// DMAs of stage s+3, in one basic block (reads and DMAs alternate in program order: a DMA writes LDS,
// so the scheduler keeps it ordered against every ds_read and the interleave pins must follow that order).
// The structure follows the loop of hipBLASLt's 256 x 256 x 64 MI16x16 kernel on gfx950 (4 waves,
// 128 x 128 wave tile, accumulators in AGPRs, every MFMA separated by one other instruction;
// profiles/r04/hipblaslt_kernels.md) with a deeper ring instead of its 4-barrier double buffer.
//
// LDS rows are 64 B (one 32-deep K stage of a row); chunk c (8 bf16) of row r lives at
// c ^ ((-(r >> 2)) & 3): for the 16x16x32 fragment read (lane l: row l & 15, chunk l >> 4) every
// ds_read_b128 lane group of 16 lanes then hits 16 distinct 16-B bank slots. One DMA instruction fills
// one 16-row piece (1 KiB, lane l -> slot l), so the swizzle is applied on the source chunk.
// Operands stream through buffer descriptors (rows past M / N read as zeros; operands < 2 GiB).
// Needs K % 128 == 0, K >= 128, N % 4 == 0, 16-B aligned rows. Epilogue: 8-B stores (4 columns per lane).
#include "common.h"
#include "mfma_core.h"

namespace w5 {

constexpr int BM = 256, BN = 256, BK = 32, NS = 4;
constexpr int THREADS = 256;
constexpr int AIMG = BM * 64;             // A stage image: 256 rows x 64 B
constexpr int STAGE = AIMG + BN * 64;     // 32 KiB
constexpr int LDS = NS * STAGE;           // 128 KiB

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

__device__ __forceinline__ int swz(int r) { return (-(r >> 2)) & 3; }

// DBG (ablation probes, tools/probes/w5_ablate.py): bit 0 = no main-loop DMAs, bit 1 = no main-loop
// fragment reads (the MFMAs re-use stale fragments), bit 2 = no per-stage wait + barrier.
template <int DBG>
__device__ __forceinline__ void run(const u16* __restrict__ A, long long lda, const u16* __restrict__ W, long long ldw,
                                    int M, int N, int K, const mc::Epi& e, unsigned char* smem, int tiles_m,
                                    int tiles_n, int group_m) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  grouped_tile(xcd_remap(blockIdx.x, gridDim.x), tiles_m, tiles_n, group_m, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int ns = K / BK;

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((long long)M * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)((long long)N * ldw * 2), 0x00020000);
  // DMA piece p of this wave (p 0..3): image rows 16 * (4 p + wave) + (lane >> 2), slot lane
  const int prow = lane >> 2;
  const uint32_t sch = 16u * (uint32_t)((lane & 3) ^ swz(prow));
  uint32_t aoff[4], boff[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = 16 * (4 * p + wave) + prow;
    aoff[p] = m0 + r < M ? (uint32_t)(m0 + r) * (uint32_t)(lda * 2) + sch : 0x80000000u;
    boff[p] = n0 + r < N ? (uint32_t)(n0 + r) * (uint32_t)(ldw * 2) + sch : 0x80000000u;
  }
  auto dma = [&](int q, int slot, int st) {   // q 0..7: A pieces 0..3, then B pieces 0..3
    const int p = q & 3;
    unsigned char* dst = smem + slot * STAGE + (q < 4 ? 0 : AIMG) + (4 * p + wave) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 4 ? ra : rw, (lds_void*)dst, 16, q < 4 ? aoff[p] : boff[p],
                                             st * BK * 2, 0, 0);
  };

  // fragment g (0..15): A row block g (g < 8) / B column block g - 8, rows 16 g' + (lane & 15)
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t fcb = 16u * (uint32_t)(fq ^ swz(fr));
  auto frag_addr = [&](int slot, int g) -> const bf16x8* {
    const int base = g < 8 ? (wr * 128 + 16 * g) : (wc * 128 + 16 * (g - 8));
    return reinterpret_cast<const bf16x8*>(smem + slot * STAGE + (g < 8 ? 0 : AIMG) + (base + fr) * 64 + fcb);
  };

  f32x4 acc[8][8];
  bf16x8 fx[16], fy[16];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: stages 0, 1, 2 in flight; fragments of stage 0 in registers
#pragma unroll
  for (int st = 0; st < 3; ++st)
#pragma unroll
    for (int q = 0; q < 8; ++q) dma(q, st, st < ns ? st : ns - 1);
  mc::wait_vmcnt<16>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int g = 0; g < 16; ++g) fx[g] = *frag_addr(0, g);

  // stage s: MFMAs on `cur`; reads of stage s+1 into `nxt`; DMAs of stage s+3 into slot (s+3) % 4
  auto stage = [&](auto slot_c, const bf16x8 (&cur)[16], bf16x8 (&nxt)[16], int s) {
    constexpr int SL = decltype(slot_c)::value;
    constexpr int NX = (SL + 1) & 3, DS = (SL + 3) & 3;
    fence();
    if constexpr (!(DBG & 4)) {
      mc::wait_vmcnt<8>();              // stage s+1 landed (this wave); stage s+2 may stay in flight
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of `cur` are done
      __builtin_amdgcn_s_barrier();     // ... and every wave's: slot DS is dead, stage s+1 is visible
    }
    fence();
    const int sd = s + 3 < ns ? s + 3 : ns - 1;   // past the end: harmless reload into the dead slot
    // program order = issue order: r0 r1 d0 r2 r3 d1 ... (16 reads, 8 DMAs)
    mc::static_for<0, 16>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (!(DBG & 2)) nxt[g] = *frag_addr(NX, g);
      if constexpr ((g & 1) && !(DBG & 1)) dma(g >> 1, DS, sd);
    });
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur[8 + j], cur[i], acc[i][j], 0, 0, 0);
    // pin: MFMA groups of 3 for the first 48 MFMAs, each followed by one read (and a DMA after every
    // second read), then the last 16 MFMAs
    mc::static_for<0, 16>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);   // 3 MFMA
      if constexpr (!(DBG & 2)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 DS read
      if constexpr ((g & 1) && !(DBG & 1)) __builtin_amdgcn_sched_group_barrier(0x010, 1, 0);   // 1 VMEM (DMA)
    });
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    fence();
  };

  for (int s = 0; s < ns; s += 4) {
    stage(std::integral_constant<int, 0>{}, fx, fy, s);
    stage(std::integral_constant<int, 1>{}, fy, fx, s + 1);
    stage(std::integral_constant<int, 2>{}, fx, fy, s + 2);
    stage(std::integral_constant<int, 3>{}, fy, fx, s + 3);
  }
  mc::wait_vmcnt<0>();

  // epilogue: acc[i][j][t] = C[m0 + wr*128 + 16 i + fr][n0 + wc*128 + 16 j + 4 fq + t]
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = n0 + wc * 128 + 16 * j + 4 * fq;
    if (col >= N) continue;
    float4 bv = float4{0.f, 0.f, 0.f, 0.f};
    if (hb) bv = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = m0 + wr * 128 + 16 * i + fr;
      if (row >= M) continue;
      const f32x4 a = acc[i][j];
      float v0 = a[0] * e.alpha + bv.x, v1 = a[1] * e.alpha + bv.y, v2 = a[2] * e.alpha + bv.z,
            v3 = a[3] * e.alpha + bv.w;
      if (hr) {
        const float4 r = unpack4_bf16(*reinterpret_cast<const uint2*>(e.R + (long long)row * e.ldr + col));
        v0 += r.x; v1 += r.y; v2 += r.z; v3 += r.w;
      }
      *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + col) = pack4_bf16(v0, v1, v2, v3);
    }
  }
}

}  // namespace w5

template <int DBG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_bf16_nt_w5_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha};
  w5::run<DBG>(A, lda, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
}

static int g_w5_group = -1;


// epi: 1 bias, 2 residual (no GEGLU / LayerNorm fold / fp32 out).
template <int DBG>
static int launch_w5(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                     long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                     hipStream_t stream) {
  if (K % 128 || K < 128 || N % 4 || lda % 8 || ldw % 8 || ldc % 4 || ((epi & MC_EPI_RESIDUAL) && ldr % 4) ||
      (epi & (MC_EPI_GEGLU | MC_EPI_LNFOLD | MC_EPI_F32OUT | MC_EPI_GELU)) ||
      ((uintptr_t)A | (uintptr_t)W) % 16 || ((uintptr_t)C | (uintptr_t)R | (uintptr_t)bias) % 8 ||
      (long long)M * lda * 2 >= (1ll << 31) || (long long)N * ldw * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_w5_kernel<DBG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              w5::LDS);
    attr_set = true;
  }
  if (g_w5_group < 0) g_w5_group = getenv("CGS_W5_GROUP") ? atoi(getenv("CGS_W5_GROUP")) : 4;
  const int tiles_m = (M + w5::BM - 1) / w5::BM, tiles_n = (N + w5::BN - 1) / w5::BN;
  const long long T = (long long)tiles_m * tiles_n;
  if (T > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  gemm_bf16_nt_w5_kernel<DBG><<<(unsigned)T, w5::THREADS, w5::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_m, tiles_n, g_w5_group);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_gemm_bf16_w5(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                                hipStream_t stream) {
  return launch_w5<0>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
}

// ablation probes (results are wrong by design for dbg != 0)
CGS_EXPORT int cgs_gemm_bf16_w5_dbg(const void* A, const void* W, void* C, const void* bias, const void* R, int M,
                                    int N, int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                                    float alpha, int dbg, hipStream_t stream) {
  switch (dbg) {
    case 0: return launch_w5<0>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    case 1: return launch_w5<1>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    case 2: return launch_w5<2>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    case 3: return launch_w5<3>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    case 4: return launch_w5<4>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    case 7: return launch_w5<7>(A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, stream);
    default: return (int)hipErrorInvalidValue;
  }
}
