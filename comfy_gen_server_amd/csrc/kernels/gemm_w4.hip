// "w4" GEMM: persistent 256 x 256 x 64 bf16 GEMM with ONE wave per SIMD (4 waves per workgroup, one
// workgroup per CU), each wave owning a 128 x 128 output tile (8 x 8 v_mfma_f32_16x16x32_bf16 tiles,
// 256 accumulator registers), ONE barrier per K-tile. Same fused epilogues as the 8-wave kernels (bias,
// residual, GEGLU, folded LayerNorm).
//
// Why a second structure next to the 8-wave ping-pong kernels (mfma_pp.h / mfma_ppk.h): PMC on MI355X
// (profiles/r04/gemm_pmc.md) shows hipBLASLt's 256x256 kernel keeping the MFMA pipes ~88 % busy at
// 8192^3 with 4 waves, a 128 x 128 wave tile and the same LDS / VMEM instruction counts as this
// structure, against 59-65 % for a 4-barrier-per-K-tile version of it and for the ping-pong v7: at one
// wave per SIMD every barrier drains the matrix pipe, so the K-tile must carry as few as possible.
// A 128 x 128 wave tile also reads 16 fragments (16 KiB of LDS) per 64 MFMAs instead of 24 for the
// 8-wave 128 x 64 tile: fewer LDS bytes per FLOP, which the power-capped chip turns into clock.
//
// K-tile t (64 deep, LDS buffer u = t & 1, 64 KiB: A [256 rows][128 B] then B [256 rows][128 B]):
//   A : 64 MFMAs, k 0..31  (fragment set F0)  | read F1(t) (k 32..63) from buffer u
//   B1: 32 MFMAs, k 32..63 (F1, row tiles 0-3)
//   --- s_waitcnt vmcnt(0) lgkmcnt(0) + s_barrier: K-tile t+1 landed for every wave, buffer u is dead
//   B2: 32 MFMAs, k 32..63 (F1, row tiles 4-7) | read F0(t+1) from buffer u^1 | DMA K-tile t+2 -> buffer u
// so each K-tile's DMAs have one whole K-tile (~2000 MFMA-cycles) to land, and the fragment reads of a
// step are always issued one step ahead. Buffer u can be re-staged right after the barrier because its
// last readers (F0(t) in B2(t-1), F1(t) in A(t)) all retired before it.
//
// Operands stream by buffer_load ... lds (16 B per lane, 1 KiB per wave-instruction) through one buffer
// descriptor per operand: the lane's row offset is a VGPR fixed per work unit, the K offset an SGPR --
// no per-DMA address arithmetic. Rows past M / N get an out-of-range offset, so the descriptor's range
// check returns zeros (operands must each span < 2 GiB). Chunk c of an LDS row r lives at
// c ^ ((r >> 1) & 7) (conflict-free ds_read_b128 fragment reads; applied on the source offsets).
//
// Persistent: workgroup b walks units b, b + G, ... (XCD-aware order, grouped_tile). The DMA stream
// runs across unit boundaries (the loaders switch to the next unit right before its first DMA), so a
// unit starts with its first fragments in registers; the first K-tile of a unit issues its MFMAs with
// a zero accumulator operand (no accumulator clearing).
//
// C^T form (W fragment as the MFMA A operand): a lane's accumulator holds 4 consecutive output COLUMNS of
// one row; B rows are staged in a permuted order so that column tiles 2p, 2p+1 give the lane 8
// consecutive columns -> 16-B stores (GEGLU: 'a' and 'g' weight rows of the same outputs in tiles 2p /
// 2p+1). Needs K % 64 == 0, K >= 128, N % 8 == 0 (GEGLU: N % 32), 16-B aligned rows, operands < 2 GiB.
#include "common.h"
#include "mfma_core.h"
#include <type_traits>

namespace w4 {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int THREADS = 256;
constexpr int HALF = 256 * 128;          // A or B image of one K-tile (32 KiB)
constexpr int BUF = 2 * HALF;            // one K-tile
constexpr int LDS = 2 * BUF;             // 128 KiB

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(4))) uint32_t* cptr_u32;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// Tile column (GEGLU: weight row within the tile's 256) staged at B row r. Wave wc reads rows
// wc*128 + s; MFMA column tile j = s >> 4 holds lane fq = (s >> 2) & 3, element t = s & 3.
template <bool GG>
__device__ __forceinline__ int b_col(int r) {
  const int wc = r >> 7, s = r & 127, j = s >> 4, fq = (s >> 2) & 3, t = s & 3;
  if constexpr (GG) {
    // output column o (0..63 within the wave's 64) = 32 (j >> 2) + 8 fq + 4 ((j >> 1) & 1) + t;
    // 'a' rows in even tiles, the matching 'g' rows in odd tiles ([a0..a15, g0..g15] weight interleave)
    const int o = wc * 64 + 32 * (j >> 2) + 8 * fq + 4 * ((j >> 1) & 1) + t;
    return (o >> 4) * 32 + 16 * (j & 1) + (o & 15);
  } else {
    return wc * 128 + 32 * (j >> 1) + 8 * fq + 4 * (j & 1) + t;
  }
}

template <bool GG, bool LN>
__device__ __forceinline__ void run(const u16* __restrict__ A, long long lda, const u16* __restrict__ W,
                                    long long ldw, int M, int N, int K, const mc::Epi& e,
                                    unsigned char* smem, int tiles_m, int tiles_n, int group_m) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = K / BK;
  const int T = tiles_m * tiles_n;
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= T) return;

  auto coords = [&](int l, int& m0, int& n0) {
    int tm, tn;
    grouped_tile(l, tiles_m, tiles_n, group_m, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };

  // ---- loaders: DMA g (0..7) of this wave covers image rows g*32 + (tid >> 3), stored chunk tid & 7
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((long long)M * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)((long long)N * ldw * 2), 0x00020000);
  const int lrow = tid >> 3;
  const int lch = tid & 7;
  uint32_t aoff[8], boff[8];
  auto setup = [&](int m0, int n0) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int r = g * 32 + lrow;
      const uint32_t ch = 16u * (uint32_t)(lch ^ ((r >> 1) & 7));
      const int m = m0 + r;
      aoff[g] = m < M ? (uint32_t)m * (uint32_t)(lda * 2) + ch : 0x80000000u;
      const int n = n0 + b_col<GG>(r);
      boff[g] = n < N ? (uint32_t)n * (uint32_t)(ldw * 2) + ch : 0x80000000u;
    }
  };
  auto dma = [&](int g, int sbuf, int kt) {   // DMA pair g (A and B rows g*32..+32) of K-tile kt
    unsigned char* base = smem + sbuf * BUF + g * 4096 + wave * 1024;
    const int ko = kt * BK * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)base, 16, aoff[g], ko, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(base + HALF), 16, boff[g], ko, 0, 0);
  };

  // ---- fragments: A row wr*128 + 16 i + (lane & 15), B row wc*128 + 16 j + (lane & 15); chunk 4 kk + (lane >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  const int swz = (fr >> 1) & 7;                        // (row >> 1) & 7 is the same for every fragment row
  const uint32_t c0 = 16u * (uint32_t)(fq ^ swz);       // kk = 0 chunk byte offset
  const uint32_t c1 = 16u * (uint32_t)((4 + fq) ^ swz); // kk = 1
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  auto read_set = [&](int sbuf, uint32_t cb, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
    const unsigned char* P = smem + sbuf * BUF;
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(P + (wr * 128 + 16 * i + fr) * 128 + cb);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(P + HALF + (wc * 128 + 16 * j + fr) * 128 + cb);
  };

  f32x4 acc[8][8];
  // MFMAs over row tiles [I0, I1) of fragment set (fa, fb); Z: first K-tile (zero accumulator operand)
  auto mma = [&](auto i0c, auto i1c, auto zc, const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
    constexpr int I0 = decltype(i0c)::value, I1 = decltype(i1c)::value;
    constexpr bool Z = decltype(zc)::value;
#pragma unroll
    for (int i = I0; i < I1; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if constexpr (Z)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
  };
  // pin the interleave: after MFMA q of Q, issue its share of R fragment reads and V DMAs
  auto pin = [&](auto qc, auto rc, auto vc) {
    constexpr int Q = decltype(qc)::value, R = decltype(rc)::value, V = decltype(vc)::value;
    mc::static_for<0, Q>([&](auto kc) {
      constexpr int q = decltype(kc)::value;
      constexpr int nds = ((q + 1) * R) / Q - (q * R) / Q;
      constexpr int nvm = ((q + 1) * V) / Q - (q * V) / Q;
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if constexpr (nds > 0) __builtin_amdgcn_sched_group_barrier(0x100, nds, 0);
      if constexpr (nvm > 0) __builtin_amdgcn_sched_group_barrier(0x010, nvm, 0);
    });
  };

  // ---- epilogue from registers. acc[i][j][t]: row m0 + wr*128 + 16 i + fr; column (staged order, b_col)
  // n0 + wc*128 + 32 (j >> 1) + 8 fq + 4 (j & 1) + t; GEGLU output column (n0 >> 1) + wc*64 + 32 (j >> 2) +
  // 8 fq + 4 ((j >> 1) & 1) + t with a = tile j even, g = j + 1. Half h = j >> 2 of the wave's tiles covers
  // staged columns / weight rows wc*128 + 64 h + [0, 64) in both layouts.
  auto loc = [&](int j, int f) {   // column / weight row of acc[.][j][0] for fq = f, within its 64-half
    if constexpr (GG) {
      const int o = 8 * f + 4 * ((j >> 1) & 1);
      return (o >> 4) * 32 + 16 * (j & 1) + (o & 15);
    } else {
      return 32 * ((j >> 1) & 1) + 8 * f + 4 * (j & 1);
    }
  };
  auto epilogue_t = [&](int m0, int n0, auto hbc, auto hrc) {
    constexpr bool HB = decltype(hbc)::value, HR = decltype(hrc)::value;
    const int ncw = n0 + wc * 128;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c0h = ncw + 64 * h;
      float4 bv[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) bv[jj] = float4{0.f, 0.f, 0.f, 0.f};
      if constexpr (HB) {
        if (c0h + 64 <= N) {
          // 64 bias values = 32 dwords through the scalar cache (no vmcnt wait behind the in-flight DMAs)
          cptr_u32 bp = (cptr_u32)(e.bias + c0h);
          uint32_t sbv[32];
#pragma unroll
          for (int k = 0; k < 32; ++k) sbv[k] = __builtin_amdgcn_readfirstlane(bp[k]);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int d0 = loc(jj, 0) >> 1, d1 = loc(jj, 1) >> 1, d2 = loc(jj, 2) >> 1, d3 = loc(jj, 3) >> 1;
            const uint32_t w0 = fq == 0 ? sbv[d0] : fq == 1 ? sbv[d1] : fq == 2 ? sbv[d2] : sbv[d3];
            const uint32_t w1 = fq == 0 ? sbv[d0 + 1] : fq == 1 ? sbv[d1 + 1] : fq == 2 ? sbv[d2 + 1] : sbv[d3 + 1];
            bv[jj] = unpack4_bf16(uint2{w0, w1});
          }
        } else {
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            int col = c0h + loc(jj, fq);
            col = col < N ? col : N - 4;
            bv[jj] = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
          }
        }
      }
      if constexpr (LN) {
        // LayerNorm folded in: acc = rstd_r * (acc - mean_r * cs[c]) (+ bias below)
        float4 cv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          int col = c0h + loc(jj, fq);
          col = col < N ? col : N - 4;
          cv[jj] = *reinterpret_cast<const float4*>(e.cs + col);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          int row = m0 + wr * 128 + 16 * i + fr;
          row = row < M ? row : M - 1;
          const float2 st = *reinterpret_cast<const float2*>(e.rs + 2 * (long long)row);
          const float mr = st.x * st.y;
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            f32x4& v = acc[i][4 * h + jj];
            v[0] = st.y * v[0] - mr * cv[jj].x;
            v[1] = st.y * v[1] - mr * cv[jj].y;
            v[2] = st.y * v[2] - mr * cv[jj].z;
            v[3] = st.y * v[3] - mr * cv[jj].w;
          }
        }
      }
      if constexpr (GG) {
        const int ocol = (n0 >> 1) + wc * 64 + 32 * h + 8 * fq;
        const int Nout = N >> 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = m0 + wr * 128 + 16 * i + fr;
          uint2 o2[2];
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const f32x4 av = acc[i][4 * h + 2 * p], gv = acc[i][4 * h + 2 * p + 1];
            const float4 ba = bv[2 * p], bg = bv[2 * p + 1];
            const f32x2_t g01 = gelu_sig2(f32x2_t{gv[0], gv[1]} * e.alpha + f32x2_t{bg.x, bg.y});
            const f32x2_t g23 = gelu_sig2(f32x2_t{gv[2], gv[3]} * e.alpha + f32x2_t{bg.z, bg.w});
            const f32x2_t o01 = (f32x2_t{av[0], av[1]} * e.alpha + f32x2_t{ba.x, ba.y}) * g01;
            const f32x2_t o23 = (f32x2_t{av[2], av[3]} * e.alpha + f32x2_t{ba.z, ba.w}) * g23;
            o2[p] = pack4_bf16(o01.x, o01.y, o23.x, o23.y);
          }
          if (row < M && ocol < Nout)
            *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + ocol) =
                u32x4_t{o2[0].x, o2[0].y, o2[1].x, o2[1].y};
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = m0 + wr * 128 + 16 * i + fr;
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            const int col = c0h + 32 * p + 8 * fq;
            uint4 rq = uint4{0u, 0u, 0u, 0u};
            if constexpr (HR) {
              const int rr = row < M ? row : M - 1, cc = col < N ? col : N - 8;
              rq = *reinterpret_cast<const uint4*>(e.R + (long long)rr * e.ldr + cc);
            }
            uint2 hv[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const f32x4 v = acc[i][4 * h + 2 * p + q];
              const float4 bb = bv[2 * p + q];
              float v0 = v[0] * e.alpha + bb.x, v1 = v[1] * e.alpha + bb.y;
              float v2 = v[2] * e.alpha + bb.z, v3 = v[3] * e.alpha + bb.w;
              if constexpr (HR) {
                const float4 r4 = unpack4_bf16(q ? uint2{rq.z, rq.w} : uint2{rq.x, rq.y});
                v0 += r4.x; v1 += r4.y; v2 += r4.z; v3 += r4.w;
              }
              hv[q] = pack4_bf16(v0, v1, v2, v3);
            }
            if (row < M && col < N)
              *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + col) =
                  u32x4_t{hv[0].x, hv[0].y, hv[1].x, hv[1].y};
          }
        }
      }
    }
  };
  using F_ = std::false_type;
  using T_ = std::true_type;
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
  auto epilogue = [&](int m0, int n0) {
    if constexpr (LN || GG) {
      if (hb) epilogue_t(m0, n0, T_{}, F_{});
      else epilogue_t(m0, n0, F_{}, F_{});
    } else {
      if (hr) {
        if (hb) epilogue_t(m0, n0, T_{}, T_{});
        else epilogue_t(m0, n0, F_{}, T_{});
      } else {
        if (hb) epilogue_t(m0, n0, T_{}, F_{});
        else epilogue_t(m0, n0, F_{}, F_{});
      }
    }
  };

  // ---- unit state + prologue (K-tiles 0 and 1 of the first unit, F0 of K-tile 0)
  int m0, n0;
  coords(u, m0, n0);
  int un = u + G;
  bool has_next = un < T;
  int nm0 = m0, nn0 = n0;
  if (has_next) coords(un, nm0, nn0);
  setup(m0, n0);
#pragma unroll
  for (int g = 0; g < 8; ++g) dma(g, 0, 0);
#pragma unroll
  for (int g = 0; g < 8; ++g) dma(g, 1, 1);
  mc::wait_vmcnt<16>();
  __builtin_amdgcn_s_barrier();
  read_set(0, c0, fa0, fb0);
  int sb = 0;                   // LDS buffer of the current K-tile

  using I0 = std::integral_constant<int, 0>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;
  auto ktile = [&](auto zc, int kt) {
    // A: k 0..31 | read F1(t)
    fence();
    wait_lgkm0();               // F0(t) landed (read in the previous B2 / the prologue)
    fence();
    read_set(sb, c1, fa1, fb1);
    mma(I0{}, I8{}, zc, fa0, fb0);
    pin(std::integral_constant<int, 64>{}, std::integral_constant<int, 16>{}, I0{});
    fence();
    // B1: k 32..63 of row tiles 0-3
    wait_lgkm0();
    fence();
    mma(I0{}, I4{}, F_{}, fa1, fb1);
    fence();
    // K-tile t+1 landed (every wave's DMAs), buffer sb dead for every wave
    mc::wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    fence();
    // B2: k 32..63 of row tiles 4-7 | read F0(t+1) | DMA K-tile t+2 (this unit's or the next unit's; after
    // the last unit a dummy reload of K-tile nk-1 into the dead buffer keeps the block branch-free)
    const int k2 = kt + 2;
    if (k2 == nk && has_next) setup(nm0, nn0);
    const int kd = k2 < nk ? k2 : (has_next ? k2 - nk : nk - 1);
    fence();
    read_set(sb ^ 1, c0, fa0, fb0);
#pragma unroll
    for (int g = 0; g < 8; ++g) dma(g, sb, kd);
    mma(I4{}, I8{}, F_{}, fa1, fb1);
    pin(std::integral_constant<int, 32>{}, std::integral_constant<int, 16>{}, std::integral_constant<int, 16>{});
    fence();
    sb ^= 1;
  };

  while (true) {
    ktile(T_{}, 0);
    for (int kt = 1; kt < nk; ++kt) ktile(F_{}, kt);
    epilogue(m0, n0);
    if (!has_next) break;
    u = un;
    m0 = nm0;
    n0 = nn0;
    un = u + G;
    has_next = un < T;
    if (has_next) coords(un, nm0, nn0);
  }
  mc::wait_vmcnt<0>();
}

}  // namespace w4

template <bool GG, bool LN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_bf16_nt_w4_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m, const float* rs, const float* cs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  w4::run<GG, LN>(A, lda, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
}

namespace {
int w4_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}
int g_w4_group = -1;
}  // namespace

// Tile-group height of the w4 grouped order (CGS_W4_GROUP; default 4 tile rows).
CGS_EXPORT void cgs_w4_set_group(int g) { g_w4_group = g; }

// epi: 1 bias, 2 residual, 4 GEGLU, 8 LayerNorm fold (rs / cs as in cgs_gemm_bf16_lnfold).
CGS_EXPORT int cgs_gemm_bf16_w4(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                                const float* rs, const float* cs, hipStream_t stream) {
  const bool gg = (epi & MC_EPI_GEGLU) != 0, ln = (epi & MC_EPI_LNFOLD) != 0;
  const int nout = gg ? N / 2 : N;
  if (K % 64 || K < 128 || lda % 8 || ldw % 8 || ldc % 8 || nout % 8 || (gg && N % 32) ||
      ((epi & MC_EPI_RESIDUAL) && (gg || ln || ldr % 8)) || (epi & MC_EPI_F32OUT) ||
      ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)R) % 16 || ((uintptr_t)bias % 8) ||
      (ln && (!rs || !cs || ((uintptr_t)cs % 16) || ((uintptr_t)rs % 8))) ||
      (long long)M * lda * 2 >= (1ll << 31) || (long long)N * ldw * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  if (g_w4_group < 0) g_w4_group = getenv("CGS_W4_GROUP") ? atoi(getenv("CGS_W4_GROUP")) : 4;
  const int tiles_m = (M + w4::BM - 1) / w4::BM, tiles_n = (N + w4::BN - 1) / w4::BN;
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < w4_num_cus() ? T : w4_num_cus());
#define W4L(GG_, LN_)                                                                                            \
  do {                                                                                                           \
    static bool attr = false;                                                                                    \
    if (!attr) {                                                                                                 \
      (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_w4_kernel<GG_, LN_>,                                   \
                                hipFuncAttributeMaxDynamicSharedMemorySize, w4::LDS);                            \
      attr = true;                                                                                               \
    }                                                                                                            \
    gemm_bf16_nt_w4_kernel<GG_, LN_><<<grid, w4::THREADS, w4::LDS, stream>>>(                                    \
        (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, \
        alpha, tiles_m, tiles_n, g_w4_group, rs, cs);                                                            \
  } while (0)
  if (gg) {
    if (ln) W4L(true, true);
    else W4L(true, false);
  } else {
    if (ln) W4L(false, true);
    else W4L(false, false);
  }
#undef W4L
  return (int)hipGetLastError();
}
