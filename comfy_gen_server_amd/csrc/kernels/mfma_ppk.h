// Persistent ping-pong GEMM main loop ("v7"): the mfma_pp.h 256 x 256 x 64 schedule (8 waves in two
// barrier-staggered groups, 4 phases per K-tile, LDS-DMA parts restaged one phase after their last
// read) turned into a persistent kernel whose K-tile DMA stream never stops at a tile boundary.
//
// Why: on the SDXL shapes K is short (640 / 1280 -> 10 / 20 K-tiles per output tile), so a
// one-tile-per-workgroup kernel pays, per tile, a cold pipeline fill (~2 us of HBM latency before
// the first MFMA) and an LDS-staged epilogue during which the MFMA pipes idle -- 15-30 % of the
// tile. Here:
//   * the grid is one workgroup per CU; workgroup b walks work units b, b + G, ... (XCD-aware
//     order, grouped_tile() so XCD-mates share A/W panels in their L2);
//   * the loaders target the global K-tile sequence: while the last two K-tiles of unit t are
//     consumed, the parts of unit t+1's first two K-tiles are DMA'd (each loader slot is re-pointed
//     to the next unit right before its first next-unit stage), so unit t+1 starts with its data
//     already in LDS;
//   * the MFMAs compute C^T (W fragment as the A operand), so a lane's accumulator holds 4
//     consecutive output COLUMNS of one row; the W rows are staged in a permuted order so that the
//     lane's two MFMA column tiles hold 8 consecutive columns -> the epilogue writes 16 B per lane
//     and every store instruction covers 64 contiguous bytes of 16 rows (full 64-B L2 requests:
//     measured +6..13 % over 8-B stores on the K = 640 / 1280 shapes, where the output write is as
//     large as the operand reads). Straight from registers (the LDS keeps prefetching), bias from
//     scalar loads (no vmcnt drain of the in-flight DMAs), GEGLU pairs in-lane, residual via 16-B
//     loads;
//   * output stores leave in full 128-B lines: one dwordx4 store instruction = 8 rows x 128 B (the
//     MFMA layout gives a lane 16 B of 16 different rows per instruction = 16 half lines). The
//     accumulators pass through the 32 KiB LDS staging area (wave-local for plain outputs; for GEGLU,
//     whose wave slice is only 64 B wide, the two waves of a column pair exchange halves behind a
//     barrier). Measured on MI355X (tools/probes/store_probe.hip): one CU writes a 128 KiB tile at
//     99 GB/s this way vs 35 GB/s with half lines; with every CU storing at once both meet the
//     chip's ~5.7 TB/s write limit, which is why the workgroups are also de-synchronised;
//   * the epilogue's stores sit in the vmcnt order between two DMA stages: the waits of the next
//     K-tile allow STORES more outstanding ops (a full tile issues every store; a partial tile keeps
//     the plain counts, which over-wait and are therefore safe);
//   * split-K tail (wave quantisation): with T tiles on G CUs the last round holds T mod G tiles,
//     e.g. 64 of 256 for every SDXL level-2 1280-wide GEMM / conv (M = 16384: 320 tiles) -- 2
//     rounds for 1.25 rounds of work. When a workspace is given, those tail tiles are cut into S
//     K-ranges (S*tail <= G, chosen on the host); each range unit writes its fp32 partial tile,
//     and the LAST unit of a tile to arrive (agent-scope release/acquire + one atomic counter per
//     tile, no spin-waiting anywhere) sums the other partials and runs the normal epilogue.
// Needs K % 64 == 0, K >= 128, N % 8 == 0, 16-B aligned rows, operands < 4 GiB (32-bit byte offsets).
#pragma once
#include "common.h"
#include "mfma_core.h"
#include "mfma_pp.h"
#include <algorithm>

namespace ppk {

using pp::BM;
using pp::BN;
using pp::BK;
using pp::THREADS;
using pp::PART;
using pp::BUF;
// Full-line epilogue (kFullLine): outputs leave as 8 rows x 128 B per store instruction through a 32 KiB
// LDS staging area. Measured on MI355X (profiles/r03_gemm_epilogue.md): one CU stores a 128 KiB tile
// 3x faster that way when the chip is otherwise idle, but inside this kernel the LDS round trip (and,
// for GEGLU, the pair exchange behind barriers) costs what the faster stores save -- in-process A/B
// within +-2 % of the register epilogue on all 7 shapes. Compiled out; kept for the next structure.
constexpr bool kFullLine = false;
constexpr int STG = kFullLine ? 32768 : 0;
constexpr int LDS = pp::LDS + STG;

using pp::P_A0;
using pp::P_A1;
using pp::P_B0;
using pp::P_B1;

typedef const __attribute__((address_space(4))) uint32_t* cptr_u32;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// 16-B output store (non-temporal stores measured no better: tools/gemm_sweep.py history)
__device__ __forceinline__ void store16(u16* p, uint2 lo, uint2 hi, int) {
  *reinterpret_cast<u32x4_t*>(p) = u32x4_t{lo.x, lo.y, hi.x, hi.y};
}

template <bool GG>
struct Stores {
  static constexpr int N = GG ? 8 : 16;   // global stores per lane per full tile
};

// Split-K tail plan (host and device agree on it through these fields).
struct Split {
  int t_full;        // tiles computed whole (a multiple of the CU count)
  int S;             // K-ranges per tail tile (1: no split)
  float4* part;      // [tail * S][32][512] fp32 partial tiles
  int* cnt;          // [tail] arrival counters (zeroed before the launch)
  int dbg;           // timing probes (CGS_V7_SPLIT_DBG): 1 no fences, 4 no partial reads
};

template <int EXTRA>
__device__ __forceinline__ void wait_window(bool after_epilogue) {
  if (after_epilogue) mc::wait_vmcnt<10 + EXTRA>();
  else mc::wait_vmcnt<10>();
}

// tile column (0..255) staged at row r (0..127) of B part nq: the lane holding MFMA column tile j,
// row 4*fq + t of wave wc's 32-row slice must see output column wc*64 + nq*32 + 8*fq + 4*j + t
// (GEGLU: output column oc = wc*32 + 8*fq + 4*nq + t of the a (j = 0) / g (j = 1) half, whose
// weight row sits at (oc / 16) * 32 + 16 * j + oc % 16 in the interleaved layout).
template <bool GG>
__device__ __forceinline__ int b_col_perm(int nq, int r) {
  const int wc = r >> 5, j = (r >> 4) & 1, fq = (r >> 2) & 3, t = r & 3;
  if constexpr (GG) {
    const int oc = wc * 32 + 8 * fq + 4 * nq + t;
    return (oc >> 4) * 32 + 16 * j + (oc & 15);
  } else {
    return wc * 64 + nq * 32 + 8 * fq + 4 * j + t;
  }
}

template <bool GG, bool LN = false, class AL, bool F32 = false>
__device__ __forceinline__ void run(AL& al, const u16* __restrict__ W, long long ldw, int M, int N, int K,
                                    const mc::Epi& e, unsigned char* smem, int tiles_m, int tiles_n, int group_m,
                                    Split sp = Split{0, 1, nullptr, nullptr, 0}) {
  constexpr int E = Stores<GG>::N;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / BK;
  const int T = tiles_m * tiles_n;
  const int S = sp.S;
  const int U = S > 1 ? sp.t_full + (T - sp.t_full) * S : T;   // work units
  const int G = gridDim.x;
  const int u0 = xcd_remap(blockIdx.x, G);
  if (u0 >= U) return;
  // timing probes (CGS_V7_SPLIT_DBG / cgs_v7_set_dbg): bit 8 = no epilogue stores. (Start-delay
  // desynchronisation probes -- 2, 4 and 8 phases per XCD, with and without full-line stores --
  // measured slower at every spread and were removed: profiles/r03_gemm_epilogue.md.)
  const bool nostore = (sp.dbg & 8) != 0;
  constexpr bool legacy = !kFullLine;         // register epilogue: 16 B per lane, 16 rows x 64 B per store

  // unit -> (tile origin, K range, partial slot or -1)
  auto unit = [&](int u, int& m0, int& n0, int& kb, int& ke, int& slot) {
    int l;
    if (S <= 1 || u < sp.t_full) {
      l = u;
      kb = 0;
      ke = nk;
      slot = -1;
    } else {
      const int v = u - sp.t_full;
      const int q = v / S, r = v - q * S;
      l = sp.t_full + q;
      kb = r * nk / S;
      ke = (r + 1) * nk / S;
      slot = v;
    }
    int tm, tn;
    grouped_tile(l, tiles_m, tiles_n, group_m, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };

  const int lrow = tid >> 3;
  const int lch = tid & 7;
  uint32_t boff[2][2];           // byte offsets from W (32-bit: the saddr + voffset load form)
  const unsigned char* Wb = reinterpret_cast<const unsigned char*>(W);
  auto setup_a = [&](int mq, int m0) {
#pragma unroll
    for (int g = 0; g < 2; ++g) al.setup(mq * 2 + g, m0 + pp::a_row(mq, g * 64 + lrow));
  };
  auto setup_b = [&](int n0) {
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int r = g * 64 + lrow;
        int n = n0 + b_col_perm<GG>(nq, r);
        n = n < N ? n : N - 1;
        boff[nq][g] = (uint32_t)(((long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7))) * 2);
      }
  };
  // stage part `part` of the K-tile with global sequence number s (-> LDS buffer s & 1), taking
  // K offset kt * BK from whatever unit the part's loader slots currently point at
  auto stage = [&](int part, long long s, int kt) {
    const int k0 = kt * BK;
    unsigned char* base = smem + (int)(s & 1) * BUF + part * PART + wave * 1024;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if (part == P_A0) al.dma(0 * 2 + g, k0, base + g * 8192);
      else if (part == P_A1) al.dma(1 * 2 + g, k0, base + g * 8192);
      else if (part == P_B0) mc::lds_dma16((const void*)(Wb + (boff[0][g] + (uint32_t)(k0 * 2))), base + g * 8192);
      else mc::lds_dma16((const void*)(Wb + (boff[1][g] + (uint32_t)(k0 * 2))), base + g * 8192);
    }
  };

  f32x4 acc[8][4];
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  auto read_a = [&](int buf, int mq) {
    const unsigned char* P = smem + buf * BUF + (mq ? P_A1 : P_A0) * PART;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r = wr * 64 + 16 * i + fr;
        const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
        af[i][kk] = *reinterpret_cast<const bf16x8*>(P + r * 128 + 16 * c);
      }
  };
  auto read_b = [&](int buf, int nq, bf16x8 (&b)[2][2]) {
    const unsigned char* P = smem + buf * BUF + (nq ? P_B1 : P_B0) * PART;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r = wc * 32 + 16 * j + fr;
        const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
        b[j][kk] = *reinterpret_cast<const bf16x8*>(P + r * 128 + 16 * c);
      }
  };
  // C^T tiles: lane (fr, fq) accumulates C[row 16i + fr][4 columns, see b_col_perm] of its quadrant
  auto mma = [&](auto mqc, auto nqc, const bf16x8 (&b)[2][2]) {
    constexpr int mq = decltype(mqc)::value, nq = decltype(nqc)::value;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mq * 4 + i][nq * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][kk], af[i][kk], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // ---- epilogue straight from registers. Row of acc[mq*4+i][.] = m0 + wr*128 + mq*64 + 16i + fr;
  // acc[.][nq*2+j][t] is column n0 + wc*64 + nq*32 + 8fq + 4j + t (GEGLU: see b_col_perm).
  auto epilogue_t = [&](int m0, int n0, auto hb_c, auto hr_c) {
    constexpr bool HB = decltype(hb_c)::value, HR = decltype(hr_c)::value;
    // lane-dependent indices re-derived here, opaque to the compiler (as in gemm_w6.hip): hoisted copies
    // live across the K loop were spilled, and a scratch reload in the epilogue waits vmcnt(0) -- also for
    // the next unit's in-flight DMAs
    int lane_e;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
    const int lane = lane_e, fr = lane_e & 15, fq = lane_e >> 4;
    const int ncw = n0 + wc * 64;                 // first (staged) column of this wave
    // bias column offset (from ncw) of acc[.][nq*2+j][0] for this lane
    auto bcol = [&](int nq, int j) {
      if constexpr (GG) return (fq >> 1) * 32 + 16 * j + 8 * (fq & 1) + 4 * nq;
      else return nq * 32 + 8 * fq + 4 * j;
    };
    if constexpr (LN) {
      // LayerNorm folded in (MC_EPI_LNFOLD): the GEMM ran on the raw rows x with W' = W * gamma;
      // LN(x) W^T = rstd_r * (x W'^T - mean_r * colsum(W')) (+ W beta, folded into the bias)
      float4 cv[2][2];
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          int col = ncw + bcol(nq, j);
          col = col < N ? col : N - 4;
          cv[nq][j] = *reinterpret_cast<const float4*>(e.cs + col);
        }
      // one 4-row batch of statistics at a time (all 8 at once spill at the 256-VGPR cap)
#pragma unroll
      for (int mq = 0; mq < 2; ++mq) {
        float2 st[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
          row = row < M ? row : M - 1;
          st[i] = *reinterpret_cast<const float2*>(e.rs + 2 * (long long)row);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              f32x4& a = acc[mq * 4 + i][nq * 2 + j];
              const float4 c = cv[nq][j];
              const float mr = st[i].x * st[i].y;
              a[0] = st[i].y * a[0] - mr * c.x;
              a[1] = st[i].y * a[1] - mr * c.y;
              a[2] = st[i].y * a[2] - mr * c.z;
              a[3] = st[i].y * a[3] - mr * c.w;
            }
        asm volatile("" ::: "memory");      // keep the two batches' loads apart
      }
    }
    float4 bv[2][2];
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[nq][j] = float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (HB) {
      if (ncw + 64 <= N) {
        // 64 bias values of the wave = 32 dwords through the scalar cache (lgkm, not vmcnt)
        cptr_u32 bp = (cptr_u32)(e.bias + ncw);
        uint32_t sb[32];
#pragma unroll
        for (int k = 0; k < 32; ++k) sb[k] = __builtin_amdgcn_readfirstlane(bp[k]);
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            // dword of column bcol(nq, j) for fq = 0..3 (compile-time per fq, selected per lane)
            int d[4];
#pragma unroll
            for (int f = 0; f < 4; ++f)
              d[f] = (GG ? (f >> 1) * 32 + 16 * j + 8 * (f & 1) + 4 * nq : nq * 32 + 8 * f + 4 * j) >> 1;
            const uint32_t w0 = fq == 0 ? sb[d[0]] : fq == 1 ? sb[d[1]] : fq == 2 ? sb[d[2]] : sb[d[3]];
            const uint32_t w1 = fq == 0 ? sb[d[0] + 1] : fq == 1 ? sb[d[1] + 1] : fq == 2 ? sb[d[2] + 1] : sb[d[3] + 1];
            bv[nq][j] = unpack4_bf16(uint2{w0, w1});
          }
      } else {
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            int col = ncw + bcol(nq, j);
            col = col < N ? col : N - 4;
            bv[nq][j] = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
          }
      }
    }
    if constexpr (GG) {
     if constexpr (legacy) {
      const int Nout = N >> 1;
      const int ocol = (n0 >> 1) + wc * 32 + 8 * fq;   // 8 output columns of this lane
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
          uint2 h[2];
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            const f32x4 a = acc[mq * 4 + i][nq * 2 + 0], g = acc[mq * 4 + i][nq * 2 + 1];
            const float4 ba = bv[nq][0], bg = bv[nq][1];
            f32x2_t g01 = f32x2_t{g[0], g[1]} * e.alpha + f32x2_t{bg.x, bg.y};
            f32x2_t g23 = f32x2_t{g[2], g[3]} * e.alpha + f32x2_t{bg.z, bg.w};
            g01 = gelu_sig2(g01);
            g23 = gelu_sig2(g23);
            const f32x2_t o01 = (f32x2_t{a[0], a[1]} * e.alpha + f32x2_t{ba.x, ba.y}) * g01;
            const f32x2_t o23 = (f32x2_t{a[2], a[3]} * e.alpha + f32x2_t{ba.z, ba.w}) * g23;
            h[nq] = pack4_bf16(o01.x, o01.y, o23.x, o23.y);
          }
          if (row < M && ocol < Nout && !nostore) store16(e.C + (long long)row * e.ldc + ocol, h[0], h[1], e.flags);
        }
     } else {
      // The wave's output slice is 128 rows x 32 columns (64 B). Waves wc = 2p, 2p + 1 (same group,
      // so the group's barriers order their exchange) own adjacent 64-B halves of the same rows:
      // per 64-row round both write their halves into the pair's 8 KiB region ([64 rows][128 B], 16-B
      // chunk c of row r at c ^ (r & 7)), then each stores 32 whole rows.
      const int Nout = N >> 1;
      unsigned char* reg = smem + pp::LDS + (wr * 2 + (wc >> 1)) * 8192;
      const int half = wc & 1;
      const int gcol = (n0 >> 1) + (wc >> 1) * 64 + 8 * (lane & 7);
#pragma unroll
      for (int mq = 0; mq < 2; ++mq) {
        if (mq) {
          pp::wait_lgkm0();
          pp::barrier();           // WAR: the pair read round 0 before round 1 overwrites it
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          uint2 h[2];
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            const f32x4 a = acc[mq * 4 + i][nq * 2 + 0], g = acc[mq * 4 + i][nq * 2 + 1];
            const float4 ba = bv[nq][0], bg = bv[nq][1];
            const f32x2_t g01 = gelu_sig2(f32x2_t{g[0], g[1]} * e.alpha + f32x2_t{bg.x, bg.y});
            const f32x2_t g23 = gelu_sig2(f32x2_t{g[2], g[3]} * e.alpha + f32x2_t{bg.z, bg.w});
            const f32x2_t o01 = (f32x2_t{a[0], a[1]} * e.alpha + f32x2_t{ba.x, ba.y}) * g01;
            const f32x2_t o23 = (f32x2_t{a[2], a[3]} * e.alpha + f32x2_t{ba.z, ba.w}) * g23;
            h[nq] = pack4_bf16(o01.x, o01.y, o23.x, o23.y);
          }
          const int r = 16 * i + fr;
          *reinterpret_cast<u32x4_t*>(reg + r * 128 + 16 * ((half * 4 + fq) ^ (r & 7))) =
              u32x4_t{h[0].x, h[0].y, h[1].x, h[1].y};
        }
        pp::wait_lgkm0();
        pp::barrier();             // RAW: the partner's half is in the region
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int r = half * 32 + 8 * t + (lane >> 3);
          const u32x4_t v = *reinterpret_cast<const u32x4_t*>(reg + r * 128 + 16 * ((lane & 7) ^ (r & 7)));
          const int row = m0 + wr * 128 + mq * 64 + r;
          if (row < M && gcol < Nout && !nostore) *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + gcol) = v;
        }
      }
     }
    } else if constexpr (F32 && !HR) {
      // fp32 output (materialised attention scores): two 16-B stores per (row, nq) -- 32 per lane
      // per tile, so the caller keeps the plain vmcnt windows (stores_pending stays false)
      float* Cf = reinterpret_cast<float*>(e.C);
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            const int col = ncw + nq * 32 + 8 * fq;
            if (row < M && col < N) {
              float* p = Cf + (long long)row * e.ldc + col;
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                const f32x4 v = acc[mq * 4 + i][nq * 2 + j];
                const float4 b = bv[nq][j];
                *reinterpret_cast<float4*>(p + 4 * j) =
                    float4{v[0] * e.alpha + b.x, v[1] * e.alpha + b.y, v[2] * e.alpha + b.z, v[3] * e.alpha + b.w};
              }
            }
          }
        }
    } else if constexpr (legacy) {
      uint4 rw[2][4][2];
      if constexpr (HR) {
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
            row = row < M ? row : M - 1;
#pragma unroll
            for (int nq = 0; nq < 2; ++nq) {
              int col = ncw + nq * 32 + 8 * fq;
              col = col < N ? col : N - 8;
              rw[mq][i][nq] = *reinterpret_cast<const uint4*>(e.R + (long long)row * e.ldr + col);
            }
          }
      }
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            uint2 h[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 v = acc[mq * 4 + i][nq * 2 + j];
              const float4 b = bv[nq][j];
              float v0 = v[0] * e.alpha + b.x, v1 = v[1] * e.alpha + b.y;
              float v2 = v[2] * e.alpha + b.z, v3 = v[3] * e.alpha + b.w;
              if constexpr (HR) {
                const uint4 rq = rw[mq][i][nq];
                const float4 rv = unpack4_bf16(j ? uint2{rq.z, rq.w} : uint2{rq.x, rq.y});
                v0 += rv.x; v1 += rv.y; v2 += rv.z; v3 += rv.w;
              }
              h[j] = pack4_bf16(v0, v1, v2, v3);
            }
            const int col = ncw + nq * 32 + 8 * fq;
            if (row < M && col < N && !nostore) store16(e.C + (long long)row * e.ldc + col, h[0], h[1], e.flags);
          }
        }
    } else {
      // The wave's slice is 128 rows x 64 columns = 128-B rows: per 16-row block i, the lane's two
      // 16-B chunks (nq = 0, 1) of row fr go to the wave's 2 KiB staging block ([16 rows][128 B], chunk
      // c of row r at c ^ (r & 7): conflict-free b128 writes and reads), then come back as two full
      // 8-row x 128-B store instructions (lane -> row lane >> 3, chunk lane & 7). The residual is read
      // in that output layout (16 loads issued before the first store) and added to the rounded
      // GEMM output in fp32 -- the reference's bf16 linear + bf16 residual add.
      unsigned char* stg = smem + pp::LDS + wave * 2048;
      const int sr = lane >> 3, sc = lane & 7;
      const int gcol = ncw + 8 * sc;
      uint4 rw[2][4][2];
      if constexpr (HR) {
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              int row = m0 + wr * 128 + mq * 64 + 16 * i + 8 * hh + sr;
              row = row < M ? row : M - 1;
              const int col = gcol < N ? gcol : N - 8;
              rw[mq][i][hh] = *reinterpret_cast<const uint4*>(e.R + (long long)row * e.ldr + col);
            }
      }
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            uint2 h[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 v = acc[mq * 4 + i][nq * 2 + j];
              const float4 b = bv[nq][j];
              h[j] = pack4_bf16(v[0] * e.alpha + b.x, v[1] * e.alpha + b.y, v[2] * e.alpha + b.z,
                                v[3] * e.alpha + b.w);
            }
            *reinterpret_cast<u32x4_t*>(stg + fr * 128 + 16 * ((nq * 4 + fq) ^ (fr & 7))) =
                u32x4_t{h[0].x, h[0].y, h[1].x, h[1].y};
          }
          asm volatile("" ::: "memory");     // the wave's chunk writes precede its row reads (LDS in order)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int r = 8 * hh + sr;
            u32x4_t v = *reinterpret_cast<const u32x4_t*>(stg + r * 128 + 16 * (sc ^ (r & 7)));
            if constexpr (HR) {
              const uint4 rq = rw[mq][i][hh];
              const float4 a0 = unpack4_bf16(uint2{v[0], v[1]}), a1 = unpack4_bf16(uint2{v[2], v[3]});
              const float4 r0 = unpack4_bf16(uint2{rq.x, rq.y}), r1 = unpack4_bf16(uint2{rq.z, rq.w});
              const uint2 p0 = pack4_bf16(a0.x + r0.x, a0.y + r0.y, a0.z + r0.z, a0.w + r0.w);
              const uint2 p1 = pack4_bf16(a1.x + r1.x, a1.y + r1.y, a1.z + r1.z, a1.w + r1.w);
              v = u32x4_t{p0.x, p0.y, p1.x, p1.y};
            }
            const int row = m0 + wr * 128 + mq * 64 + 16 * i + r;
            if (row < M && gcol < N && !nostore) *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + gcol) = v;
          }
          asm volatile("" ::: "memory");     // this block's reads precede the next block's writes
        }
    }
  };
  using F = std::false_type;
  using Tt = std::true_type;
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
  auto epilogue = [&](int m0, int n0) {
    if constexpr (LN) {                     // folded LayerNorm: no residual form (host-checked)
      if (hb) epilogue_t(m0, n0, Tt{}, F{});
      else epilogue_t(m0, n0, F{}, F{});
      return;
    }
    if (hr) {
      if (hb) epilogue_t(m0, n0, Tt{}, Tt{});
      else epilogue_t(m0, n0, F{}, Tt{});
    } else {
      if (hb) epilogue_t(m0, n0, Tt{}, F{});
      else epilogue_t(m0, n0, F{}, F{});
    }
  };
  __shared__ int last_flag_static;
  int& last_flag = last_flag_static;
  // split unit: publish the fp32 partial; the tile's last arriver reduces and runs the epilogue
  auto split_epilogue = [&](int m0, int n0, int slot) {
    float4* mine = sp.part + (size_t)slot * (32 * THREADS);
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const f32x4 v = acc[q >> 2][q & 3];
      mine[q * THREADS + tid] = float4{v[0], v[1], v[2], v[3]};
    }
    // Publish: the workgroup barrier orders every wave's partial stores (all in this XCD's L2 once
    // the barrier's vmcnt(0) retires them) before ONE agent-scope release by thread 0 -- a per-wave
    // release would write the L2 back once per wave; then the arrival count. The last arriver's
    // thread 0 acquires (invalidates this CU's caches) before the barrier that lets every wave
    // read the other units' partials.
    mc::wait_vmcnt<0>();         // this wave's partial stores have reached the L2
    __syncthreads();
    const int tile = slot / S;
    if (tid == 0) {
      if (!(sp.dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      mc::wait_vmcnt<0>();       // keep: the fence's own wait may be dropped, and it must precede the ticket
      const int old = __hip_atomic_fetch_add(sp.cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_flag = old == S - 1;
      if (old == S - 1) {
        __hip_atomic_store(sp.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // self-reset
        if (!(sp.dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        mc::wait_vmcnt<0>();
      }
    }
    __syncthreads();
    const bool last = last_flag;
    __syncthreads();               // every wave has read the flag before the epilogue reuses its LDS word
    if (!last) return;
    const int r0 = tile * S;
    for (int r = 0; r < S; ++r) {
      if (r0 + r == slot || (sp.dbg & 4)) continue;
      const float4* o = sp.part + (size_t)(r0 + r) * (32 * THREADS);
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const float4 w = o[q * THREADS + tid];
        acc[q >> 2][q & 3] += f32x4{w.x, w.y, w.z, w.w};
      }
    }
    epilogue(m0, n0);
  };

  // ---- prologue: A0 B0 B1 A1 of the first K-tile, A0 B0 B1 of the second -> wait for A0, B0
  int u = u0, m0, n0, kb, ke, slot;
  unit(u, m0, n0, kb, ke, slot);
  setup_a(0, m0);
  setup_a(1, m0);
  setup_b(n0);
  stage(P_A0, 0, kb);
  stage(P_B0, 0, kb);
  stage(P_B1, 0, kb);
  stage(P_A1, 0, kb);
  stage(P_A0, 1, kb + 1);
  stage(P_B0, 1, kb + 1);
  stage(P_B1, 1, kb + 1);
  mc::wait_vmcnt<10>();
  pp::barrier();
  if (wr == 1) pp::barrier();   // stagger: group 1 runs one segment behind group 0

  long long s = 0;              // global K-tile sequence number of this workgroup
  bool stores_pending = false;  // the previous tile's full set of epilogue stores is in the vmcnt window
  while (true) {
    const int un = u + G;
    const bool has_next = un < U;
    int nm0 = m0, nn0 = n0, nkb = kb, nke = ke, nslot = -1;
    if (has_next) unit(un, nm0, nn0, nkb, nke, nslot);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = kb; kt < ke; ++kt) {
      const int buf = (int)(s & 1);
      const bool after = stores_pending && kt == kb;
      // K-tiles one and two ahead in this workgroup's sequence (the next unit's first two, or a
      // dummy reload of this unit's last one after the final unit); every unit spans >= 2 K-tiles
      const int kt1 = kt + 1 < ke ? kt + 1 : (has_next ? nkb + (kt + 1 - ke) : ke - 1);
      const int kt2 = kt + 2 < ke ? kt + 2 : (has_next ? nkb + (kt + 2 - ke) : ke - 1);
      // phase 1 (mq0, nq0): read A0, B0; DMA A1 of sequence s+1
      read_a(buf, 0);
      read_b(buf, 0, bf0);
      if (kt + 1 == ke && has_next) setup_a(1, nm0);
      stage(P_A1, s + 1, kt1);
      wait_window<E>(after);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I0{}, I0{}, bf0);
      pp::barrier();
      // phase 2 (mq0, nq1): read B1; DMA A0 of s+2
      read_b(buf, 1, bf1);
      if (kt + 2 == ke && has_next) setup_a(0, nm0);
      stage(P_A0, s + 2, kt2);
      wait_window<E>(after);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I0{}, I1{}, bf1);
      pp::barrier();
      // phase 3 (mq1, nq1): read A1; DMA B0 of s+2
      read_a(buf, 1);
      if (kt + 2 == ke && has_next) setup_b(nn0);
      stage(P_B0, s + 2, kt2);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I1{}, I1{}, bf1);
      pp::barrier();
      // phase 4 (mq1, nq0): DMA B1 of s+2; retire A0(s+1), B0(s+1) for the next phase 1
      stage(P_B1, s + 2, kt2);
      wait_window<E>(after);
      pp::barrier();
      mma(I1{}, I0{}, bf0);
      pp::barrier();
      ++s;
    }
    if (slot >= 0) {
      // a split unit is its workgroup's last (S * tail <= G): drain, then reduce / publish
      mc::wait_vmcnt<0>();
      if (wr == 0) pp::barrier();   // balance the stagger before the workgroup barriers
      split_epilogue(m0, n0, slot);
      return;
    }
    epilogue(m0, n0);
    // a full tile issued every one of its E stores (partial tiles may skip some: keep plain waits)
    stores_pending = (m0 + BM <= M) && (n0 + BN <= N) && !F32;
    if (!has_next) break;
    u = un;
    m0 = nm0;
    n0 = nn0;
    kb = nkb;
    ke = nke;
    slot = nslot;
  }
  if (wr == 0) pp::barrier();   // balance the stagger
  mc::wait_vmcnt<0>();          // trailing dummy DMAs must land before the workgroup's LDS is released
}

// Host: split-K tail plan for T tiles of nk K-tiles on G CUs. Returns S (1 = no split) and the
// number of whole tiles; the workspace needs tail * S * 256 KiB of partials + tail counters.
// Cost of the last round in K-tile times (one K-tile = 256x256x64 on one CU, ~1.5 us), calibrated
// on MI355X (tools/split_probe.py): nk / S of MFMA work + ~19 fixed (release fence + partial-slab
// write + restart) + ~4.7 per extra slab the last arriver reads (256 KiB at one block's ~100 GB/s).
// Short K (<= 32 K-tiles) never pays; the level-2 convs (nk = 90..360) and K = 5120 do.
inline int split_plan(long long T, int nk, int G, int& t_full) {
  const long long tail = T % G;
  t_full = (int)(T - tail);
  if (tail == 0 || tail * 2 > G || nk < 4) return 1;
  // CGS_V7_SPLIT_FORCE=S (diagnostics): split every tail tile S ways when it fits (S * tail <= G)
  static const int force = getenv("CGS_V7_SPLIT_FORCE") ? atoi(getenv("CGS_V7_SPLIT_FORCE")) : 0;
  if (force > 1 && force * tail <= G && nk / force >= 2) return force;
  int best = 1;
  double best_cost = nk;
  const int smax = (int)std::min<long long>(std::min<long long>(G / tail, nk / 2), 16);
  for (int S = 2; S <= smax; ++S) {
    const double c = (double)nk / S + 4.7 * (S - 1) + 19.0;
    if (c < best_cost) { best_cost = c; best = S; }
  }
  return best;
}

// Zero the tail-tile arrival counters ahead of the launch with a kernel, not hipMemsetAsync: a
// memset issued on a capturing stream did not replay as part of the hipGraph here (replays with new
// inputs saw stale counters -> unreduced tail tiles), while a kernel launch is captured like the
// GEMM itself.
static __global__ void zero_counters_kernel(int* cnt, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) cnt[i] = 0;
}

inline long long split_ws_bytes(long long T, int nk, int G) {
  int t_full;
  const int S = split_plan(T, nk, G, t_full);
  if (S <= 1) return 0;
  const long long tail = T - t_full;
  return tail * S * 32ll * THREADS * 16 + ((tail * 4 + 255) / 256) * 256;
}

}  // namespace ppk
