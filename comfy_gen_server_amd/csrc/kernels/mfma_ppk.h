// Persistent ping-pong GEMM main loop ("v7"): the mfma_pp.h 256 x 256 x 64 schedule (8 waves in two
// barrier-staggered groups, 4 phases per K-tile, LDS-DMA parts restaged one phase after their last
// read) turned into a persistent kernel whose K-tile DMA stream never stops at a tile boundary.
//
// Why: on the SDXL shapes K is short (640 / 1280 -> 10 / 20 K-tiles per output tile), so a
// one-tile-per-workgroup kernel pays, per tile, a cold pipeline fill (~2 us of HBM latency before
// the first MFMA) and an LDS-staged epilogue during which the MFMA pipes idle -- 15-30 % of the
// tile. Here:
//   * the grid is one workgroup per CU; workgroup b walks logical tiles b, b + G, ... (XCD-aware
//     order, grouped_tile() so XCD-mates share A/W panels in their L2);
//   * the loaders target the global K-tile sequence: while the last two K-tiles of tile t are
//     consumed, the parts of tile t+1's first two K-tiles are DMA'd (each loader slot is re-pointed
//     to the next tile right before its first next-tile stage), so tile t+1 starts with its data
//     already in LDS;
//   * the MFMAs compute C^T (W fragment as the A operand), so a lane's accumulator holds 4
//     consecutive output COLUMNS of one row -> the epilogue stores 8 B per lane straight from
//     registers (no LDS round trip: the LDS keeps prefetching), with bias from scalar loads (no
//     vector load, so no vmcnt drain of the in-flight DMAs), GEGLU pairs in-lane (interleaved
//     16-row groups: MFMA col tiles 2p / 2p+1 = a / g of the same columns), residual via 8-B loads;
//   * the epilogue's stores sit in the vmcnt order between two DMA stages: the waits of the next
//     K-tile allow STORES more outstanding ops (a full tile issues every store; a partial tile keeps
//     the plain counts, which over-wait and are therefore safe).
// Needs K % 64 == 0, K >= 128, N % 8 == 0, 16-B aligned rows, operands < 4 GiB (32-bit byte offsets).
#pragma once
#include "common.h"
#include "mfma_core.h"
#include "mfma_pp.h"

namespace ppk {

using pp::BM;
using pp::BN;
using pp::BK;
using pp::THREADS;
using pp::PART;
using pp::BUF;
using pp::LDS;
using pp::P_A0;
using pp::P_A1;
using pp::P_B0;
using pp::P_B1;

typedef const __attribute__((address_space(4))) uint32_t* cptr_u32;

template <bool GG>
struct Stores {
  static constexpr int N = GG ? 16 : 32;   // global stores per lane per tile
};

template <int EXTRA>
__device__ __forceinline__ void wait_window(bool after_epilogue, bool probe = false) {
  if (probe) mc::wait_vmcnt<63>();     // EXPERIMENT flag 256: ignore the stores (timing probe; unsafe)
  else if (after_epilogue) mc::wait_vmcnt<10 + EXTRA>();
  else mc::wait_vmcnt<10>();
}

template <bool GG, class AL>
__device__ __forceinline__ void run(AL& al, const u16* __restrict__ W, long long ldw, int M, int N, int K,
                                    const mc::Epi& e, unsigned char* smem, int tiles_m, int tiles_n, int group_m) {
  constexpr int E = Stores<GG>::N;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / BK;
  const int T = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int l0 = xcd_remap(blockIdx.x, G);
  if (l0 >= T) return;

  auto coords = [&](int l, int& m0, int& n0) {
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
        int n = n0 + pp::b_col(nq, r);
        n = n < N ? n : N - 1;
        boff[nq][g] = (uint32_t)(((long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7))) * 2);
      }
  };
  // stage part `part` of the K-tile with global sequence number s (-> LDS buffer s & 1), taking
  // K offset kt * BK from whatever tile the part's loader slots currently point at
  auto stage = [&](int part, long long s, int kt) {
    const int k0 = kt * BK;
    unsigned char* base = smem + (int)(s & 1) * BUF + part * PART + wave * 1024;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const void* src;
      if (part == P_A0) src = al.src(0 * 2 + g, k0);
      else if (part == P_A1) src = al.src(1 * 2 + g, k0);
      else if (part == P_B0) src = (const void*)(Wb + (boff[0][g] + (uint32_t)(k0 * 2)));
      else src = (const void*)(Wb + (boff[1][g] + (uint32_t)(k0 * 2)));
      mc::lds_dma16(src, base + g * 8192);
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
  // C^T tiles: lane (fr, fq) accumulates C[row 16i + fr][col 16j + 4fq + 0..3] of its quadrant
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
  // col of acc[.][nq*2+j] = n0 + wc*64 + nq*32 + 16j + 4fq + (0..3).
  auto epilogue_t = [&](int m0, int n0, auto hb_c, auto hr_c) {
    constexpr bool HB = decltype(hb_c)::value, HR = decltype(hr_c)::value;
    const int ncw = n0 + wc * 64;                 // first column of this wave
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
            const int b0 = nq * 16 + 8 * j;
            const uint32_t w0 = fq == 0 ? sb[b0] : fq == 1 ? sb[b0 + 2] : fq == 2 ? sb[b0 + 4] : sb[b0 + 6];
            const uint32_t w1 = fq == 0 ? sb[b0 + 1] : fq == 1 ? sb[b0 + 3] : fq == 2 ? sb[b0 + 5] : sb[b0 + 7];
            bv[nq][j] = unpack4_bf16(uint2{w0, w1});
          }
      } else {
#pragma unroll
        for (int nq = 0; nq < 2; ++nq)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            int col = ncw + nq * 32 + 16 * j + 4 * fq;
            col = col < N ? col : N - 4;
            bv[nq][j] = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
          }
      }
    }
    if constexpr (GG) {
      const int Nout = N >> 1;
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
#pragma unroll
          for (int nq = 0; nq < 2; ++nq) {
            const f32x4 a = acc[mq * 4 + i][nq * 2 + 0], g = acc[mq * 4 + i][nq * 2 + 1];
            const float4 ba = bv[nq][0], bg = bv[nq][1];
            const float o0 = (a[0] * e.alpha + ba.x) * gelu_fast(g[0] * e.alpha + bg.x);
            const float o1 = (a[1] * e.alpha + ba.y) * gelu_fast(g[1] * e.alpha + bg.y);
            const float o2 = (a[2] * e.alpha + ba.z) * gelu_fast(g[2] * e.alpha + bg.z);
            const float o3 = (a[3] * e.alpha + ba.w) * gelu_fast(g[3] * e.alpha + bg.w);
            const int ocol = ((ncw + nq * 32) >> 1) + 4 * fq;
            if (row < M && ocol < Nout)
              *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + ocol) = pack4_bf16(o0, o1, o2, o3);
          }
        }
    } else {
      // residual words: all 32 loads issued before the first store (one wait, one drain)
      uint2 rw[2][4][2][2];
      if constexpr (HR) {
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
            row = row < M ? row : M - 1;
#pragma unroll
            for (int nq = 0; nq < 2; ++nq)
#pragma unroll
              for (int j = 0; j < 2; ++j) {
                int col = ncw + nq * 32 + 16 * j + 4 * fq;
                col = col < N ? col : N - 4;
                rw[mq][i][nq][j] = *reinterpret_cast<const uint2*>(e.R + (long long)row * e.ldr + col);
              }
          }
      }
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = m0 + wr * 128 + mq * 64 + 16 * i + fr;
#pragma unroll
          for (int nq = 0; nq < 2; ++nq)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const f32x4 v = acc[mq * 4 + i][nq * 2 + j];
              const float4 b = bv[nq][j];
              float v0 = v[0] * e.alpha + b.x, v1 = v[1] * e.alpha + b.y;
              float v2 = v[2] * e.alpha + b.z, v3 = v[3] * e.alpha + b.w;
              if constexpr (HR) {
                const float4 rv = unpack4_bf16(rw[mq][i][nq][j]);
                v0 += rv.x; v1 += rv.y; v2 += rv.z; v3 += rv.w;
              }
              const int col = ncw + nq * 32 + 16 * j + 4 * fq;
              // EXPERIMENT flag 64: store only one quadrant (timing probe of the store-drain cost)
              if (row < M && col < N && (!(e.flags & 64) || (mq == 0 && nq == 0)))
                *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + col) = pack4_bf16(v0, v1, v2, v3);
            }
        }
    }
  };
  using F = std::false_type;
  using Tt = std::true_type;
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
  auto epilogue = [&](int m0, int n0) {
    if (hr) {
      if (hb) epilogue_t(m0, n0, Tt{}, Tt{});
      else epilogue_t(m0, n0, F{}, Tt{});
    } else {
      if (hb) epilogue_t(m0, n0, Tt{}, F{});
      else epilogue_t(m0, n0, F{}, F{});
    }
  };

  // EXPERIMENT flag 128: odd workgroups start ~half a tile later (store-burst desync probe)
  if ((e.flags & 128) && (blockIdx.x & 1)) {
    for (int t = 0; t < nk * 3000 / 8128 / 2 + 1; ++t) __builtin_amdgcn_s_sleep(127);
  }
  // ---- prologue: A0 B0 B1 A1 of K-tile 0, A0 B0 B1 of K-tile 1 -> wait for A0(0), B0(0)
  int l = l0, m0, n0;
  coords(l, m0, n0);
  setup_a(0, m0);
  setup_a(1, m0);
  setup_b(n0);
  stage(P_A0, 0, 0);
  stage(P_B0, 0, 0);
  stage(P_B1, 0, 0);
  stage(P_A1, 0, 0);
  stage(P_A0, 1, 1);
  stage(P_B0, 1, 1);
  stage(P_B1, 1, 1);
  mc::wait_vmcnt<10>();
  pp::barrier();
  if (wr == 1) pp::barrier();   // stagger: group 1 runs one segment behind group 0

  long long s = 0;              // global K-tile sequence number of this workgroup
  bool stores_pending = false;  // the previous tile's full set of epilogue stores is in the vmcnt window
  while (true) {
    const int ln = l + G;
    const bool has_next = ln < T;
    int nm0 = m0, nn0 = n0;
    if (has_next) coords(ln, nm0, nn0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = (int)(s & 1);
      const bool after = stores_pending && kt == 0;
      const bool probe = (e.flags & 256) && stores_pending && kt < 3;
      const int kt1 = kt + 1 < nk ? kt + 1 : (has_next ? 0 : nk - 1);
      const int kt2 = kt + 2 < nk ? kt + 2 : (has_next ? kt + 2 - nk : nk - 1);
      // phase 1 (mq0, nq0): read A0, B0; DMA A1 of sequence s+1
      read_a(buf, 0);
      read_b(buf, 0, bf0);
      if (kt + 1 == nk && has_next) setup_a(1, nm0);
      stage(P_A1, s + 1, kt1);
      wait_window<E>(after, probe);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I0{}, I0{}, bf0);
      pp::barrier();
      // phase 2 (mq0, nq1): read B1; DMA A0 of s+2
      read_b(buf, 1, bf1);
      if (kt + 2 == nk && has_next) setup_a(0, nm0);
      stage(P_A0, s + 2, kt2);
      wait_window<E>(after, probe);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I0{}, I1{}, bf1);
      pp::barrier();
      // phase 3 (mq1, nq1): read A1; DMA B0 of s+2
      read_a(buf, 1);
      if (kt + 2 == nk && has_next) setup_b(nn0);
      stage(P_B0, s + 2, kt2);
      pp::wait_lgkm0();
      pp::barrier();
      mma(I1{}, I1{}, bf1);
      pp::barrier();
      // phase 4 (mq1, nq0): DMA B1 of s+2; retire A0(s+1), B0(s+1) for the next phase 1
      stage(P_B1, s + 2, kt2);
      wait_window<E>(after, probe);
      pp::barrier();
      mma(I1{}, I0{}, bf0);
      pp::barrier();
      ++s;
    }
    epilogue(m0, n0);
    // a full tile issued every one of its E stores (partial tiles may skip some: keep plain waits)
    stores_pending = (m0 + BM <= M) && (n0 + BN <= N);
    if (!has_next) break;
    l = ln;
    m0 = nm0;
    n0 = nn0;
  }
  if (wr == 0) pp::barrier();   // balance the stagger
  mc::wait_vmcnt<0>();          // trailing dummy DMAs must land before the workgroup's LDS is released
}

}  // namespace ppk
