// Ping-pong MFMA main loop with a 256 x 160 block tile ("v6") for GEMM and implicit-GEMM conv.
//
// Why 160: every SDXL channel count is a multiple of 160 (640, 1280, 1920, 2560, 3840, 5120,
// 10240), so a 160-wide tile never wastes columns, and the tile counts come out as whole rounds of
// the 256 CUs: [16384 x 1280] -> 64 x 8 = 512 tiles (2 rounds; 256 x 256 tiles give 320 = 1.25
// rounds, i.e. 62.5 % of the chip in the last round), [65536 x 640] -> 1024 tiles (256-wide tiles
// waste 1/6 of the last column tile).
//
// 8 waves (512 threads): wave w -> stagger group g = w >> 2 (one wave of each group per SIMD),
// output sub-tile rows (w & 3) * 64, cols g * 80 = 4 x 5 tiles of v_mfma_f32_16x16x32_bf16
// (80 accumulator VGPRs). Group 1 runs one barrier behind group 0, so on every SIMD one wave's
// 20-MFMA segment overlaps its partner's fragment ds_reads / LDS-DMA issue (as in mfma_pp.h).
//
// K-tile (64 deep) = 2 phases (k 0..31, 32..63). LDS: 3-slot ring of whole K-tiles
// (A 256 x 128 B + B 160 x 128 B = 52 KiB, 156 KiB total); tile t+2 is DMA'd in phase 0 of tile t
// into the slot tile t-1 vacated (its last reads retired one phase earlier: every load segment ends
// with lgkmcnt(0) before its barrier), and each wave's DMAs of tile t+1 are retired (counted
// vmcnt: only tile t+2's are younger) in phase 1 of tile t, one barrier before they are read.
// Rows are 128 B with 16-B chunk c stored at c ^ ((row >> 1) & 7) (conflict-free fragment reads;
// applied on the DMA source addresses). No GEGLU epilogue (the interleaved a/g column pairs of
// the 256-wide kernel would straddle waves here).
#pragma once
#include "common.h"
#include "mfma_core.h"
#include "mfma_pp.h"

namespace pq {

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
// Loads the compiler does not track: no s_waitcnt is inserted for their results, so the caller must retire
// them with its own counted wait before reading the registers (pq::run's epilogue-operand prefetch).
__device__ __forceinline__ void untracked_load(u32x4v& d, const void* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(d) : "v"(p));
}
__device__ __forceinline__ void untracked_load(u32x2v& d, const void* p) {
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(d) : "v"(p));
}

constexpr int BM = 256, BN = 160, BK = 64;
constexpr int THREADS = 512;
constexpr int A_BYTES = BM * 128;
constexpr int B_BYTES = BN * 128;
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int LDS = 3 * STAGE;     // 156 KiB
// NJ = 4 (run<..., NJ>): the 256 x 128 form -- 2 groups x 64 columns, no column tile 4 -- for Cout = 128 convs
// (the VAE's full-resolution ResnetBlocks: a 160-wide tile wastes 20 % of its columns there, a 256-wide one half).
// NI = 2 (run<..., NI>): 128-row tiles (the 4 row waves 32 rows each) -- twice the tiles where M is short (SDXL
// batch 1: M = 2048 tokens at level 2 gives 64 256 x 160 tiles, 128 of 128 x 160).
// W = 4 (run<..., W>): one wave group (4 waves, 256 threads) -- 128 x 80 tiles with NI = 2, two workgroups per CU
// (each SIMD pairs waves of two workgroups); the batch-1 grids (M = 2048 x N = 1280: 256 tiles, one per CU).
template <int NJ, int NI = 4, int W = 8>
struct Geo {
  static constexpr int GW = 16 * NJ, BN = GW * (W / 4);         // wave-group / tile columns
  static constexpr int BM = 64 * NI;                            // tile rows (4 row waves x 16 NI)
  static constexpr int PR = 8 * W;                              // rows per DMA piece (W waves x 8 rows x 128 B)
  static constexpr int NA = BM / PR;                            // A DMA pieces
  static constexpr int A_BYTES = BM * 128;
  static constexpr int B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES, LDS = 3 * STAGE;
  static constexpr int NBG = (BN + PR - 1) / PR;                // B DMA pieces; the last one, when BN % PR != 0,
  static constexpr int REM = BN % PR;                           //   only by the waves below REM / 8
  static constexpr bool B_HALF = REM != 0;
};

// Tile column staged at B row r. Wave group g reads rows g*80 + 16j + (4fq + t) as MFMA column tile
// j; the tile pairs (0,1) and (2,3) are interleaved so that the lane holds 8 consecutive columns
// (32p + 8fq + 4(j&1) + t) -> 16-B epilogue stores covering 64 contiguous bytes per row; tile 4
// keeps its 16 plain columns (8-B stores).
template <int NJ = 5>
__device__ __forceinline__ int b_col160(int r) {
  constexpr int GW = 16 * NJ;
  const int g = r >= GW, l = r - GW * g, j = l >> 4, q = l & 15;
  if (j >= 4) return GW * g + 64 + q;
  return GW * g + 32 * (j >> 1) + 8 * (q >> 2) + 4 * (j & 1) + (q & 3);
}

// GEGLU staging (run<..., GG>): staged B row r of group g = r / 80, tile j, row q in the tile -> output column
// c = 40 g + 8 j + (q & 7) of the tile, 'a' (q < 8) or 'g' (q >= 8) weight row of the 16-row interleave.
__device__ __forceinline__ int gg_row160(int r) {
  const int g = r >= 80, l = r - 80 * g, j = l >> 4, q = l & 15;
  const int c = 40 * g + 8 * j + (q & 7);
  return 32 * (c >> 4) + (c & 15) + 16 * (q >> 3);
}

// AL: loader with setup(slot, global_row) for slots 0..3 (tile rows slot*64 + (tid >> 3)) and
// src(slot, k0) -> this lane's 16-B source for K offset k0 (swizzled chunk already applied).
//
// Persistent: the grid is one workgroup per CU; workgroup b walks logical tiles b, b + G, ...
// (G = gridDim.x; XCD-mates take consecutive logical tiles, grouped_tile() orders them). The
// K-tile stream runs ACROSS tiles: the DMAs of the next tile's first two K-tiles are issued during
// the current tile's last two, and the epilogue (direct 8-B stores from registers, no LDS) runs
// while they are in flight -- no per-tile prologue bubble, no LDS-staged epilogue (16-B stores for
// 4 of the 5 column tiles, see b_col160). Needs K >= 128, N % 8 == 0.
// DS: where a K-tile's DMAs are issued (the per-phase interleave): bits 0-1 the split over the two
// phases (see stage_part), bit 2 DMAs before / after the phase's fragment reads. Phase-1 DMAs are
// issued before that phase's counted wait, so the vmcnt counts are the same in every mode.
// GNS: the epilogue also writes GroupNorm partial statistics of the stored (bf16) outputs -- per image,
// 64-row block (one wave's rows) and column, (mean, M2) by an exact two-pass over the wave's registers
// (DPP row sums) -- into e.gnp in the gn_partial layout with 64 pixels per block, so the next GroupNorm
// skips its statistics pass over the tensor (host: rows per image % 256 == 0). GNS == 2: the sum of squares
// only (one float per image, 64-row block and column: Cascade's GlobalResponseNorm needs sum_HW h^2, and the
// one-pass form skips the mean pass and half the DPP reductions).
// GG: GEGLU epilogue (out = a * gelu(g), N / 2 output columns) from the 16-row-interleaved weights of the
// 256-wide kernels ([a0..a15, g0..g15, ...], geglu_interleave): the B staging puts, in every 16-column MFMA
// tile, 8 'a' rows in lanes fq = 0, 1 and their 8 'g' rows in fq = 2, 3, so one v_permlane32_swap of row
// blocks i / i + 1 hands every lane 4 (a, g) pairs (lower lanes: row block i, upper: i + 1). 160 weight
// rows = 5 interleave groups = 80 output columns per tile (whole rounds where the 256-wide tiles leave a
// partial one, e.g. SDXL batch 1: M = 2048, N = 10240 -> 512 tiles vs 320). Host: N % 160 == 0.
// ACT: GELU on (acc * alpha + bias) before the residual add (MC_EPI_GELU: Cascade's ChannelMLP Linear -> GELU).
// RSO: the epilogue also writes per-row LayerNorm statistics partials of the stored (bf16) outputs -- per row
// and 80-column chunk (one wave's columns), (mean, M2) shifted by the row's first value in the chunk -- into
// e.gnp as [M][N / 80][2] floats; a LayerNorm over these rows then needs only cgs_ln_rs_from_partials
// instead of a statistics pass over the tensor. Host: N % 160 == 0.
// PFE: epilogue operands (bias, LayerNorm-fold statistics, residual) prefetched one K-tile ahead -- see
// `prefetch` -- with the last two K-tiles peeled (1), or only bias / LN statistics, inside the K loop (2: the
// conv gathers, whose peeled loop and whose prefetched residual spilled), or loaded in the epilogue (0).
template <class AL, bool LN = false, int DS = 0, int GNS = 0, bool GG = false, bool ACT = false,
          bool RSO = false, int PFE = 1, int NJ = 5, int NI = 4, int NW = 8>
__device__ __forceinline__ void run(AL& al, const u16* __restrict__ W, long long ldw, int M, int N, int K,
                                    const mc::Epi& e, unsigned char* smem, int tiles_m, int tiles_n, int group_m) {
  static_assert(NJ == 5 || NJ == 4, "column tiles per wave group");
  static_assert(NJ == 5 || (!GG && !RSO && !LN), "NJ = 4: plain / residual / GroupNorm-statistics epilogues");
  static_assert(NI == 4 || NI == 2, "16-row MFMA blocks per wave");
  static_assert(NI == 4 || GNS == 0, "NI = 2: the GroupNorm partials are laid out in 64-row blocks");
  static_assert(NW == 8 || NW == 4, "waves per workgroup");
  using Gm = Geo<NJ, NI, NW>;
  constexpr int BN = Gm::BN, GW = Gm::GW, STAGE = Gm::STAGE, BMv = Gm::BM, A_BYTESv = Gm::A_BYTES;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = NW == 8 ? wave >> 2 : 0;
  const int wm = wave & 3;
  const int nk = K / BK;
  const int T = tiles_m * tiles_n;
  const int G = gridDim.x;
  const int base_l = xcd_remap(blockIdx.x, G);
  if (base_l >= T) return;

  auto coords = [&](int l, int& m0, int& n0) {
    int tm, tn;
    grouped_tile(l, tiles_m, tiles_n, group_m, tm, tn);
    m0 = tm * BMv;
    n0 = tn * BN;
  };

  const int lrow = tid >> 3;
  const int lch = tid & 7;
  const u16* bsrc[3];
  // DS & 128: B DMAs through a buffer descriptor (per-row byte offsets fixed per tile, the K offset in the
  // SGPR soffset: no per-DMA address VALU). Host: N * ldw * 2 < 2 GiB.
  uint32_t boff[3];
  __amdgpu_buffer_rsrc_t wr;
  if constexpr ((DS & 128) != 0)
    wr = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)((long long)N * ldw * 2 < 0x7fffffffll ? N * ldw * 2
                                                                                               : 0x7fffffff),
                                           0x00020000);
  auto setup = [&](int m0, int n0) {
    if constexpr (mc::own_dma<AL>::value) al.tile(m0);
#pragma unroll
    for (int g = 0; g < Gm::NA; ++g) al.setup(g, m0 + g * Gm::PR + lrow);
#pragma unroll
    for (int g = 0; g < Gm::NBG; ++g) {
      const int r = g * Gm::PR + lrow;
      int n = n0 + (GG ? gg_row160(r < BN ? r : BN - 1) : b_col160<NJ>(r < BN ? r : BN - 1));
      n = n < N ? n : N - 1;
      if constexpr ((DS & 128) != 0) boff[g] = (uint32_t)(((long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7))) * 2);
      else bsrc[g] = W + (long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7));
    }
  };
  // A slot g / B row group g of K-tile kt into ring slot `slot`
  auto dma_a = [&](int g, int kt, int slot) {
    if (g >= Gm::NA) return;
    if constexpr (mc::own_dma<AL>::value) al.dma(g, kt * BK, smem + slot * STAGE + wave * 1024 + g * (Gm::PR * 128));
    else mc::lds_dma16(al.src(g, kt * BK), smem + slot * STAGE + wave * 1024 + g * (Gm::PR * 128));
  };
  auto dma_b = [&](int g, int kt, int slot) {
    if (g >= Gm::NBG) return;
    if (!Gm::B_HALF || g < Gm::NBG - 1 || wave < Gm::REM / 8) {  // BN = 160: B rows 128..159 by group 0 only
      if constexpr ((DS & 128) != 0)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, (mc_lds_void*)(smem + slot * STAGE + wave * 1024 + A_BYTESv + g * (Gm::PR * 128)),
                                                 16, boff[g], kt * BK * 2, 0, 0);
      else
        mc::lds_dma16((const void*)(bsrc[g] + kt * BK), smem + slot * STAGE + wave * 1024 + A_BYTESv + g * (Gm::PR * 128));
    }
  };
  // the phase-0 (part 0) / phase-1 (part 1) DMAs of K-tile kt: DS & 3 = 0 all in phase 0, 1 A | B,
  // 2 B | A, 3 balanced (A0 A1 B0 | A2 A3 B1 B2)
  auto stage_part = [&](int part, int kt, int slot) {
    constexpr int D = DS & 3;
    if constexpr (D == 0) {
      if (part == 0) {
#pragma unroll
        for (int g = 0; g < 4; ++g) dma_a(g, kt, slot);
#pragma unroll
        for (int g = 0; g < 3; ++g) dma_b(g, kt, slot);
      }
    } else if constexpr (D == 1 || D == 2) {
      if ((part == 0) == (D == 1)) {
#pragma unroll
        for (int g = 0; g < 4; ++g) dma_a(g, kt, slot);
      } else {
#pragma unroll
        for (int g = 0; g < 3; ++g) dma_b(g, kt, slot);
      }
    } else {
      if (part == 0) {
        dma_a(0, kt, slot);
        dma_a(1, kt, slot);
        dma_b(0, kt, slot);
      } else {
        dma_a(2, kt, slot);
        dma_a(3, kt, slot);
        dma_b(1, kt, slot);
        dma_b(2, kt, slot);
      }
    }
  };
  auto stage = [&](int kt, int slot) {
    stage_part(0, kt, slot);
    if constexpr ((DS & 3) != 0) stage_part(1, kt, slot);
  };
  auto wait_tile = [&]() {   // all but one K-tile's DMAs (BN = 160: 7 in group 0, 6 in group 1) retired
    if (!Gm::B_HALF || wave < Gm::REM / 8) mc::wait_vmcnt<Gm::NA + Gm::NBG>();
    else mc::wait_vmcnt<Gm::NA + Gm::NBG - 1>();
  };

  f32x4 acc[NI][NJ];
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[NI], bfr[NJ];
  auto read_frags = [&](const unsigned char* S, int kk) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r = wm * (16 * NI) + 16 * i + fr;
      const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
      af[i] = *reinterpret_cast<const bf16x8*>(S + r * 128 + 16 * c);
    }
    const unsigned char* SB = S + A_BYTESv;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int r = grp * GW + 16 * j + fr;
      const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
      bfr[j] = *reinterpret_cast<const bf16x8*>(SB + r * 128 + 16 * c);
    }
  };
  auto mma = [&]() {   // C^T tiles: lane (fr, fq) accumulates C[16i + fr][16j + 4fq + 0..3]
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // column of acc[.][j][0] for this lane (b_col160): pairs (0,1), (2,3) interleaved, tile 4 plain;
  // GEGLU: the weight row of acc[.][j][0] relative to the wave's first column (gg_row160 of staged row 16 j + 4 fq)
  auto colj = [&](int j) {
    if constexpr (GG) return gg_row160(grp * 80 + 16 * j + 4 * fq) - grp * 80;
    return j < 4 ? 32 * (j >> 1) + 8 * fq + 4 * (j & 1) : 64 + 4 * fq;
  };
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
  // Epilogue operands. PFE: loaded right after the counted wait of the unit's second-to-last K-tile, by loads
  // the compiler does not track. They then sit in the vmcnt queue between the next unit's first K-tile
  // (issued before them) and its second (issued after), so the last K-tile's own counted wait (wait_tile)
  // retires them and the epilogue reads registers. Loaded in the epilogue they were younger than both of the
  // next unit's prefetched K-tiles and waited for all of them (the residual shapes ran 17-23 % slower than
  // store-only, docs/OPEN_ITEMS.md round 5); compiler-tracked prefetch loads still got a vmcnt(0) (its
  // wait-count analysis does not credit the counted waits behind the per-group LDS-DMAs).
  u32x2v pbias[NJ];
  u32x4v pcs[NJ];
  u32x2v prs[NI];
  u32x4v prw4[NI][2];
  u32x2v prw2[NI];
  auto prefetch = [&](int m0, int n0, bool hb, bool hr, bool tracked = PFE == 0) {
    const int m_w = m0 + wm * (16 * NI), n_w = n0 + grp * GW;
    if (hb) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int col = n_w + colj(j);
        col = col < N ? col : N - 4;
        if (!tracked) untracked_load(pbias[j], e.bias + col);
        else pbias[j] = *reinterpret_cast<const u32x2v*>(e.bias + col);
      }
    }
    if constexpr (LN) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int col = n_w + colj(j);
        col = col < N ? col : N - 4;
        if (!tracked) untracked_load(pcs[j], e.cs + col);
        else pcs[j] = *reinterpret_cast<const u32x4v*>(e.cs + col);
      }
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        int row = m_w + 16 * i + fr;
        row = row < M ? row : M - 1;
        if (!tracked) untracked_load(prs[i], e.rs + 2 * (long long)row);
        else prs[i] = *reinterpret_cast<const u32x2v*>(e.rs + 2 * (long long)row);
      }
    } else if (hr) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        int row = m_w + 16 * i + fr;
        row = row < M ? row : M - 1;
        const u16* rrow = e.R + (long long)row * e.ldr;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          int col = n_w + 32 * p + 8 * fq;
          col = col < N ? col : N - 8;
          if (!tracked) untracked_load(prw4[i][p], rrow + col);
          else prw4[i][p] = *reinterpret_cast<const u32x4v*>(rrow + col);
        }
        if constexpr (NJ == 5) {
          int col = n_w + 64 + 4 * fq;
          col = col < N ? col : N - 4;
          if (!tracked) untracked_load(prw2[i], rrow + col);
          else prw2[i] = *reinterpret_cast<const u32x2v*>(rrow + col);
        }
      }
    }
  };
  // epilogue variants are separate straight-line paths (flags are wave-uniform)
  auto epilogue_t = [&](int m0, int n0, auto has_bias_c, auto has_res_c) {
    constexpr bool HB = decltype(has_bias_c)::value, HR = decltype(has_res_c)::value;
    const int m_w = m0 + wm * (16 * NI), n_w = n0 + grp * GW;
    if constexpr (PFE == 0) prefetch(m0, n0, HB, HR);
    else if constexpr (PFE == 2) prefetch(m0, n0, false, HR, true);    // the residual
    // column tile 4 (8 B per lane and row): row blocks i / i+1 are paired with v_permlane16_swap so a
    // lane stores 16 B (fq even: row block i, cols 64 + 8 (fq / 2) .. + 7; fq odd: row block i + 1)
    auto store_t4 = [&](int i, uint2 a, uint2 b) {
      const auto rx = __builtin_amdgcn_permlane16_swap(a.x, b.x, false, false);
      const auto ry = __builtin_amdgcn_permlane16_swap(a.y, b.y, false, false);
      const int row = m_w + 16 * (i + (fq & 1)) + fr;
      const int col = n_w + 64 + 8 * (fq >> 1);
      if (row < M && col < N)
        *reinterpret_cast<uint4*>(e.C + (long long)row * e.ldc + col) = uint4{rx[0], ry[0], rx[1], ry[1]};
    };
    float4 bv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) bv[j] = HB ? unpack4_bf16(uint2{pbias[j].x, pbias[j].y}) : float4{0.f, 0.f, 0.f, 0.f};
    if constexpr (LN) {
      // LayerNorm folded in (MC_EPI_LNFOLD, see mfma_ppk.h): acc = rstd_r * (acc - mean_r * cs[c])
      float4 cv[5];
#pragma unroll
      for (int j = 0; j < 5; ++j)
        cv[j] = float4{__uint_as_float(pcs[j].x), __uint_as_float(pcs[j].y), __uint_as_float(pcs[j].z),
                       __uint_as_float(pcs[j].w)};
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float2 st = float2{__uint_as_float(prs[i].x), __uint_as_float(prs[i].y)};
        const float mr = st.x * st.y;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          acc[i][j][0] = st.y * acc[i][j][0] - mr * cv[j].x;
          acc[i][j][1] = st.y * acc[i][j][1] - mr * cv[j].y;
          acc[i][j][2] = st.y * acc[i][j][2] - mr * cv[j].z;
          acc[i][j][3] = st.y * acc[i][j][3] - mr * cv[j].w;
        }
      }
    }
    uint2 rw[NI][NJ];   // residual words
    if (HR) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          rw[i][2 * p] = uint2{prw4[i][p].x, prw4[i][p].y};
          rw[i][2 * p + 1] = uint2{prw4[i][p].z, prw4[i][p].w};
        }
        if constexpr (NJ == 5) rw[i][4] = uint2{prw2[i].x, prw2[i].y};
      }
    }
    auto val = [&](int i, int j) {
      float v0 = acc[i][j][0] * e.alpha + bv[j].x, v1 = acc[i][j][1] * e.alpha + bv[j].y;
      float v2 = acc[i][j][2] * e.alpha + bv[j].z, v3 = acc[i][j][3] * e.alpha + bv[j].w;
      if constexpr (ACT) {
        const f32x2_t g01 = gelu_sig2(f32x2_t{v0, v1}), g23 = gelu_sig2(f32x2_t{v2, v3});
        v0 = g01.x; v1 = g01.y; v2 = g23.x; v3 = g23.y;
      }
      if (HR) {
        const float4 rv = unpack4_bf16(rw[i][j]);
        v0 += rv.x; v1 += rv.y; v2 += rv.z; v3 += rv.w;
      }
      return pack4_bf16(v0, v1, v2, v3);
    };
    if constexpr (GG) {
      // bias / LN already applied per weight row; pair row blocks (i, i+1) across the half-waves
      const int oc0 = n0 / 2 + grp * 40 + 4 * (fq & 1);
      const int Nout = N / 2;
#pragma unroll
      for (int i = 0; i < NI; i += 2) {
        const int row = m_w + 16 * (i + (fq >> 1)) + fr;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          float o[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float bt = t == 0 ? bv[j].x : t == 1 ? bv[j].y : t == 2 ? bv[j].z : bv[j].w;
            const float x0 = acc[i][j][t] * e.alpha + bt, x1 = acc[i + 1][j][t] * e.alpha + bt;
            const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x0), __float_as_uint(x1), false, false);
            o[t] = __uint_as_float(r[0]) * gelu_sig(__uint_as_float(r[1]));
          }
          const int col = oc0 + 8 * j;
          if (row < M && col < Nout)
            *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + col) = pack4_bf16(o[0], o[1], o[2], o[3]);
        }
      }
      return;
    }
    if constexpr (GNS) {
      uint2 pk[NI][NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) pk[i][j] = val(i, j);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = m_w + 16 * i + fr;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int col = n_w + 32 * p + 8 * fq;
          if (row < M && col < N)
            *reinterpret_cast<uint4*>(e.C + (long long)row * e.ldc + col) =
                uint4{pk[i][2 * p].x, pk[i][2 * p].y, pk[i][2 * p + 1].x, pk[i][2 * p + 1].y};
        }
      }
      if constexpr (NJ == 5) {
#pragma unroll
        for (int i = 0; i < NI; i += 2) store_t4(i, pk[i][4], pk[i + 1][4]);
      }
      if (m_w >= M) return;       // a partial last tile (GEMM rows: M % 256 != 0) -- no block past the tensor
      const int img = m_w / e.hw;
      const int nbk = e.hw >> 6;
      if constexpr (GNS == 2) {
        float* dq = e.gnp + (size_t)(img * nbk + ((m_w - img * e.hw) >> 6)) * N;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          float4 q = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int i = 0; i < NI; ++i) {
            const float4 u = unpack4_bf16(pk[i][j]);
            q.x += u.x * u.x; q.y += u.y * u.y; q.z += u.z * u.z; q.w += u.w * u.w;
          }
          q = float4{row16_sum(q.x), row16_sum(q.y), row16_sum(q.z), row16_sum(q.w)};
          const int col = n_w + colj(j);
          if (fr == 0 && col < N) *reinterpret_cast<float4*>(dq + col) = q;
        }
        return;
      }
      float* dst = e.gnp + (size_t)(img * nbk + ((m_w - img * e.hw) >> 6)) * N * 2;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float4 u[4];
#pragma unroll
        for (int i = 0; i < NI; ++i) u[i] = unpack4_bf16(pk[i][j]);
        float4 mu = u[0];
#pragma unroll
        for (int i = 1; i < 4; ++i) { mu.x += u[i].x; mu.y += u[i].y; mu.z += u[i].z; mu.w += u[i].w; }
        constexpr float inv = 1.f / 64.f;
        mu = float4{row16_sum(mu.x) * inv, row16_sum(mu.y) * inv, row16_sum(mu.z) * inv, row16_sum(mu.w) * inv};
        float4 q = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const float dx = u[i].x - mu.x, dy = u[i].y - mu.y, dz = u[i].z - mu.z, dw = u[i].w - mu.w;
          q.x += dx * dx; q.y += dy * dy; q.z += dz * dz; q.w += dw * dw;
        }
        q = float4{row16_sum(q.x), row16_sum(q.y), row16_sum(q.z), row16_sum(q.w)};
        const int col = n_w + colj(j);
        if (fr == 0 && col < N) {
          float4* d4 = reinterpret_cast<float4*>(dst + (size_t)col * 2);
          d4[0] = float4{mu.x, q.x, mu.y, q.y};
          d4[1] = float4{mu.z, q.z, mu.w, q.w};
        }
      }
      return;
    }
    if constexpr (RSO) {
      uint2 pk[NI][5];
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < 5; ++j) pk[i][j] = val(i, j);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = m_w + 16 * i + fr;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int col = n_w + 32 * p + 8 * fq;
          if (row < M && col < N)
            *reinterpret_cast<uint4*>(e.C + (long long)row * e.ldc + col) =
                uint4{pk[i][2 * p].x, pk[i][2 * p].y, pk[i][2 * p + 1].x, pk[i][2 * p + 1].y};
        }
      }
#pragma unroll
      for (int i = 0; i < NI; i += 2) store_t4(i, pk[i][4], pk[i + 1][4]);
      // row (16 i + fr) of this wave's 80 columns: 20 values in each of the 4 lanes fr + 16 fq. Each lane takes
      // (mean, M2) of its 20 (shifted by its own first value), then Chan-combines with lane l ^ 16 and l ^ 32
      // through v_permlane16/32_swap (VALU; the former __shfl_xor / __shfl broadcast were 5 LDS permutes per row
      // block: the epilogue cost 5-15 us per GEMM on the SDXL residual shapes, profiles/r06/rso_cost.log).
      // Both lanes of a pair see the (lower, upper) operands in the same order: identical results.
      const int P = N / 80;
      const int chunk = n_w / 80;
      auto comb = [](float& mean, float& m2, float n, auto swp) {   // two equal halves of n values each
        const auto rm = swp(__float_as_uint(mean));
        const auto rq = swp(__float_as_uint(m2));
        const float ma = __uint_as_float(rm[0]), mb = __uint_as_float(rm[1]), d = mb - ma;
        mean = 0.5f * (ma + mb);
        m2 = __uint_as_float(rq[0]) + __uint_as_float(rq[1]) + d * d * (0.5f * n);
      };
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float sh = unpack4_bf16(pk[i][0]).x;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const float4 u = unpack4_bf16(pk[i][j]);
          const float d0 = u.x - sh, d1 = u.y - sh, d2 = u.z - sh, d3 = u.w - sh;
          s1 += (d0 + d1) + (d2 + d3);
          s2 += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
        }
        constexpr float i20 = 1.f / 20.f;
        float mean = sh + s1 * i20, m2 = fmaxf(s2 - s1 * s1 * i20, 0.f);
        comb(mean, m2, 20.f, [](unsigned v) { return __builtin_amdgcn_permlane16_swap(v, v, false, false); });
        comb(mean, m2, 40.f, [](unsigned v) { return __builtin_amdgcn_permlane32_swap(v, v, false, false); });
        const int row = m_w + 16 * i + fr;
        if (fq == 0 && row < M)
          *reinterpret_cast<float2*>(e.gnp + ((long long)row * P + chunk) * 2) = float2{mean, m2};
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int row = m_w + 16 * i + fr;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int col = n_w + 32 * p + 8 * fq;
        const uint2 lo = val(i, 2 * p), hi = val(i, 2 * p + 1);
        if (row < M && col < N)
          *reinterpret_cast<uint4*>(e.C + (long long)row * e.ldc + col) = uint4{lo.x, lo.y, hi.x, hi.y};
      }
    }
    if constexpr (NJ == 4) {
    } else if constexpr ((DS & 32) != 0) {   // A/B reference: 8-B stores for column tile 4
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = m_w + 16 * i + fr, col = n_w + 64 + 4 * fq;
        const uint2 w4 = val(i, 4);
        if (row < M && col < N) *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + col) = w4;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; i += 2) store_t4(i, val(i, 4), val(i + 1, 4));
    }
  };
  using T0 = std::false_type;
  using T1 = std::true_type;
  auto epilogue = [&](int m0, int n0) {
    if constexpr (LN) {                     // folded LayerNorm: no residual form (host-checked)
      if (hb) epilogue_t(m0, n0, T1{}, T0{});
      else epilogue_t(m0, n0, T0{}, T0{});
      return;
    }
    if (hr) {
      if (hb) epilogue_t(m0, n0, T1{}, T1{});
      else epilogue_t(m0, n0, T0{}, T1{});
    } else {
      if (hb) epilogue_t(m0, n0, T1{}, T0{});
      else epilogue_t(m0, n0, T0{}, T0{});
    }
  };

  int l = base_l;
  int m0, n0;
  coords(l, m0, n0);
  setup(m0, n0);
  stage(0, 0);
  stage(nk > 1 ? 1 : 0, 1);
  wait_tile();
  pp::barrier();
  if (NW == 8 && grp == 1) pp::barrier();   // stagger: group 1 runs one segment behind group 0

  int slot = 0;                  // ring slot of the K-tile being consumed
  while (true) {
    const int ln = l + G;
    const bool has_next = ln < T;
    int nm0 = 0, nn0 = 0;
    if (has_next) coords(ln, nm0, nn0);
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one K-tile; PF: the unit's second-to-last, which issues the epilogue-operand prefetch after its counted wait
    auto ktile = [&](int kt, bool PF) {
      const unsigned char* S = smem + slot * STAGE;
      const int slot2 = slot >= 1 ? slot - 1 : 2;      // (slot + 2) % 3
      // phase 0: fragments k 0..31; DMA the K-tile two ahead in the stream into the slot vacated
      const int kst = kt + 2 < nk ? kt + 2 : (has_next ? kt + 2 - nk : nk - 1);
      if (kt + 2 == nk && has_next) setup(nm0, nn0);   // switch the loaders to the next tile
      // past the last tile: reload the last K-tile into a dead slot (keeps the vmcnt pattern);
      // DS & 4: the DMAs go out ahead of the phase's fragment reads
      if constexpr ((DS & 4) != 0) stage_part(0, kst, slot2);
      read_frags(S, 0);
      if constexpr ((DS & 4) == 0) stage_part(0, kst, slot2);
      // DS & 16: phase 0 does not drain its fragment reads before the barrier (the MFMAs wait for them
      // one by one). WAR-safe: slot kt is next restaged three phases on; phase 1 keeps the drain because
      // the other group restages the slot it reads one segment later.
      if constexpr ((DS & 16) == 0) pp::wait_lgkm0();
      pp::barrier();
      mma();
      pp::barrier();
      // phase 1: fragments k 32..63; retire this wave's DMAs of the next K-tile in the stream
      if constexpr ((DS & 4) != 0) stage_part(1, kst, slot2);
      read_frags(S, 1);
      if constexpr ((DS & 4) == 0) stage_part(1, kst, slot2);
      wait_tile();
      if (PFE && PF) prefetch(m0, n0, hb, PFE == 1 && hr);
      pp::wait_lgkm0();
      pp::barrier();
      mma();
      pp::barrier();
      slot = slot == 2 ? 0 : slot + 1;
    };
    if constexpr (PFE == 2) {   // not peeled: the prefetch registers stay allocated through the K loop
      for (int kt = 0; kt < nk; ++kt) ktile(kt, kt == nk - 2);
    } else if constexpr (PFE) {   // the last two K-tiles peeled: the prefetched registers live only from there on
      for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, false);
      ktile(nk - 2, true);
      ktile(nk - 1, false);
    } else {
      for (int kt = 0; kt < nk; ++kt) ktile(kt, false);
    }
    epilogue(m0, n0);
    if (!has_next) break;
    l = ln;
    m0 = nm0;
    n0 = nn0;
  }
  if (NW == 8 && grp == 0) pp::barrier();   // balance the stagger
  mc::wait_vmcnt<0>();           // the trailing dummy DMAs must land before the LDS is released
}

}  // namespace pq
