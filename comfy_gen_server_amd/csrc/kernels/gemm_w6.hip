// "w6" GEMM: C[M,N] = A[M,K] W[N,K]^T, bf16 in / out, fp32 accumulate, persistent, with the fused
// epilogues of the SDXL transformer (bias, residual, LayerNorm fold, GEGLU gate).
//
// Main loop: one wave per SIMD (4 waves, a 256 x 256 tile per workgroup, 128 x 128 per wave = 8 x 8
// v_mfma_f32_16x16x32_bf16 tiles, 256 accumulators in the AGPR half of the 512-entry file) over
// 64-deep K tiles in TWO LDS buffers (2 x 64 KiB).
//
// Why 64-deep tiles: every LDS-DMA instruction then moves 8 whole 128-B lines (8 rows x 128 B) instead
// of 16 half lines (the 32-deep ring of the retired w5 loop, tools/probes/retired_kernels/gemm_w5.hip).
// Measured on MI355X (profiles/r05/gemm_w6.md):
// the w5 loop with its DMAs removed ran 1.25x faster (1379 -> 1724 TF/s at 8192^3, above hipBLASLt's
// 1652) while removing its fragment reads or its barriers was worth <= 4 %; with full-line DMAs the
// same loop shape reaches 1510 at 8192^3 (w5 1396).
//
// Schedule per K-tile t (buffer b = t & 1; fragments of the two 32-deep halves kk = 0 / 1 in two
// register sets f0 / f1, 128 MFMAs per wave in four chunks of 32):
//   chunk 0  MFMAs (f0, rows 0-63)   + the 16 fragment reads of f1 (tile t, buffer b)
//   -- lgkmcnt(0) + barrier Y: every wave is done reading buffer b
//   chunk 1  MFMAs (f0, rows 64-127) + the 8 A-operand DMAs of tile t+2 into buffer b
//   -- vmcnt(8) + barrier X: tile t+1 (issued during chunks 1-2 of tile t-1) has landed for every wave
//   chunk 2  MFMAs (f1, rows 0-63)   + the 8 B-operand DMAs of tile t+2 + 8 B-fragment reads of f0 (t+1)
//   chunk 3  MFMAs (f1, rows 64-127) + the 8 A-fragment reads of f0 (tile t+1), front-loaded
// so a DMA has >= 1.5 chunks (~1500 MFMA cycles) before its wait, and two barriers per 128 MFMAs.
//
// Persistent: one workgroup per CU walks work units u0, u0 + G, ... (XCD-remapped, grouped tile order).
// "Tile t+2" runs on into the next unit: the last two K-tiles of a unit DMA the next unit's first two
// (the DMA offsets are re-pointed right before), so a unit starts with its operands in LDS and its
// first fragments in registers, and the epilogue's stores overlap those DMAs (the first barrier X of
// the next unit then allows the epilogue's stores in its vmcnt window).
//
// LDS: [A buf 0 | A buf 1 | B buf 0 | B buf 1], each rows [256][128 B]; 16-B chunk c of row r at
// c ^ (r & 7): the 16x16x32 fragment read (lane l: row l & 15, chunk 4 kk + (l >> 4)) hits 16 distinct
// 16-B slots in every ds_read_b128 lane group. LDS-DMA writes lane-linear (lane l -> row l >> 3,
// slot l & 7), so the swizzle is applied on the source chunk: (l & 7) ^ (l >> 3).
//
// Output layout: the MFMAs compute C^T (W fragment as the A operand), so a lane holds 4 consecutive
// output columns of one row per MFMA tile; the W rows are staged in a permuted order (b_src_row) so that
// a lane's tiles (2P, 2P+1) hold 8 consecutive columns -> 16-B stores (GEGLU: tiles 4Q..4Q+3 hold the
// a / g values of 8 consecutive outputs).
// Operands stream through buffer descriptors (rows past M / N read as zeros; operands < 2 GiB).
// Needs K % 128 == 0 (an even number of K-tiles), N % 16 == 0, 16-B aligned rows.
#include "common.h"
#include "mfma_core.h"

namespace w6 {

constexpr int BM = 256, BK = 64;
constexpr int THREADS = 256;
constexpr int HALF = 256 * 128;           // the A operand of one K-tile: 256 rows x 128 B
// BN = 256 (wave tile 128 x 128, 8 B fragments per 32-deep half) or 160 (128 x 80, 5: the N = 640 / 1280 /
// 1920 / 3840 projections fill whole rounds of 256 CUs, as hipBLASLt's MT256x160 "MIWT8_5" kernel does)
template <int BN>
struct Geo {
  static constexpr int NB = BN / 32;                 // B fragments per half per wave (= B DMAs per wave)
  static constexpr int WN = BN / 2;                  // wave tile columns
  static constexpr int HALF_B = BN * 128;
  static constexpr int LDS = 2 * (HALF + HALF_B);    // [A buf 0 | A buf 1 | B buf 0 | B buf 1]
  static constexpr int NF = 8 + NB;                  // fragments per half
};

// Interleave NM MFMAs with NR other instructions (one per group, evenly spread; kind(i) = the i-th one's
// sched_group_barrier mask), for the instruction order pinned by the surrounding sched_barriers.
template <int NM, int NR, class Kind>
__device__ __forceinline__ void pin(Kind kind) {
  mc::static_for<0, NR>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    constexpr int m = (i + 1) * NM / NR - i * NM / NR;
    if constexpr (m > 0) __builtin_amdgcn_sched_group_barrier(0x008, m, 0);
    __builtin_amdgcn_sched_group_barrier(kind(ic), 1, 0);
  });
}

typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// W row (within the 256-row tile) staged at LDS row RB: plain -- wave half wc = RB >> 7, MFMA tile
// j = (RB >> 4) & 7 = 2P + h, row x = 4 fq + r -> column 32 P + 8 fq + 4 h + r of the half; GEGLU
// (a / g rows interleaved in groups of 16) -- j = 4 Q + 2 hh + isg -> output o = wc * 64 + 32 Q + 8 fq
// + 4 hh + r, weight row (o / 16) * 32 + 16 isg + o % 16.
template <bool GG, int BN = 256>
__device__ __forceinline__ int b_src_row(int RB) {
  if constexpr (BN != 256) return RB;     // 80-column wave tiles: natural order, 8-B stores
  const int wc = RB >> 7, j = (RB >> 4) & 7, fq = (RB >> 2) & 3, r = RB & 3;
  if constexpr (GG) {
    const int o = wc * 64 + 32 * (j >> 2) + 8 * fq + 4 * ((j >> 1) & 1) + r;
    return (o >> 4) * 32 + 16 * (j & 1) + (o & 15);
  } else {
    return wc * 128 + 32 * (j >> 1) + 8 * fq + 4 * (j & 1) + r;
  }
}

__device__ __forceinline__ void unpack8(uint4 w, float (&v)[8]) {
  const float4 lo = unpack4_bf16(uint2{w.x, w.y}), hi = unpack4_bf16(uint2{w.z, w.w});
  v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
}

__device__ __forceinline__ u32x4_t pack8(const float (&v)[8]) {
  const uint2 lo = pack4_bf16(v[0], v[1], v[2], v[3]), hi = pack4_bf16(v[4], v[5], v[6], v[7]);
  return u32x4_t{lo.x, lo.y, hi.x, hi.y};
}

// DBG (ablation probes): bit 0 = no main-loop DMAs, bit 1 = no main-loop fragment reads.
// GG: GEGLU epilogue (N/2 outputs). LN: LayerNorm folded in (MC_EPI_LNFOLD: e.rs row stats, e.cs colsums).
template <int DBG, bool GG, bool LN, int BN>
__device__ __forceinline__ void run(const u16* __restrict__ A, long long lda, const u16* __restrict__ W, long long ldw,
                                    int M, int N, int K, const mc::Epi& e, unsigned char* smem, int tiles_m,
                                    int tiles_n, int group_m) {
  using Gm = Geo<BN>;
  constexpr int NB = Gm::NB, WN = Gm::WN, HB = Gm::HALF_B, NF = Gm::NF;
  static_assert(!GG || BN == 256, "GEGLU: 256-wide tiles");
  constexpr int E = GG ? 16 : (BN == 256 ? 32 : 8 * NB);   // global stores per lane per full tile
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int nk = K / BK;
  const int T = tiles_m * tiles_n;
  const int G = gridDim.x;
  int u = xcd_remap(blockIdx.x, G);
  if (u >= T) return;
  auto unit_origin = [&](int uu, int& m0_, int& n0_) {
    int tm, tn;
    grouped_tile(uu, tiles_m, tiles_n, group_m, tm, tn);
    m0_ = tm * BM;
    n0_ = tn * BN;
  };
  int m0, n0;
  unit_origin(u, m0, n0);

  // Operand descriptors start at the unit's first row, with the unit's remaining rows as their size
  // (rows past M / N read as zeros); the per-lane DMA offsets are then the same for every unit and a
  // switch to the next unit rebuilds only the (scalar) descriptors.
  __amdgpu_buffer_rsrc_t ra, rw;
  auto set_a = [&](int mm0) {
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + (long long)mm0 * lda), 0, (int)((long long)(M - mm0) * lda * 2),
                                           0x00020000);
  };
  auto set_b = [&](int nn0) {
    rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (long long)nn0 * ldw), 0, (int)((long long)(N - nn0) * ldw * 2),
                                           0x00020000);
  };
  set_a(m0);
  set_b(n0);
  // DMA q (0..7) of this wave per operand: piece p = 8 wave + q = LDS rows 8 p + (lane >> 3)
  const int lr = lane >> 3;
  const uint32_t lcs = 16u * (uint32_t)((lane & 7) ^ lr);
  // B piece q of this wave: rows 8 (NB wave + q) + (lane >> 3)
  uint32_t aoff[8], boff[NB];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int r = 8 * (8 * wave + q) + lr;
    aoff[q] = (uint32_t)r * (uint32_t)(lda * 2) + lcs;
  }
#pragma unroll
  for (int q = 0; q < NB; ++q) {
    const int r = 8 * (NB * wave + q) + lr;
    boff[q] = (uint32_t)b_src_row<GG, BN>(r) * (uint32_t)(ldw * 2) + lcs;
  }
  // LDS-DMA destinations: the wave's first piece + immediates. `dbase` is re-materialised per K-tile
  // (opaque to the compiler) so that the 32 destinations are one s_add each instead of 32 hoisted SGPRs.
  const uint32_t dbase0 = (uint32_t)(uintptr_t)smem;
  uint32_t dbase = dbase0;
  auto dma = [&](int q, int buf, int kt) {   // q 0..7: A pieces, 8..8+NB-1: B pieces
    // an LDS address -> LDS pointer (inttoptr; a generic-pointer round trip would map offset 0 to null)
    const uint32_t off = q < 8 ? buf * HALF + (8 * wave + q) * 1024 : 2 * HALF + buf * HB + (NB * wave + q - 8) * 1024;
    lds_void* dst = (lds_void*)(uintptr_t)(dbase + off);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(q < 8 ? ra : rw, dst, 16, q < 8 ? aoff[q] : boff[q - 8],
                                             kt * BK * 2, 0, 0);
  };

  // fragment g (0..15) of half kk: A row block g (g < 8) / B row block g - 8. LDS layout [A buf 0 | A buf 1 |
  // B buf 0 | B buf 1] (32 KiB each): one per-lane base per (operand, half) and every buffer / block offset an
  // immediate (<= 32 KiB + 14 KiB, inside the 16-bit DS offset).
  const int fr = lane & 15, fq = lane >> 4;
  uint32_t fbase[2][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const uint32_t sw = 16u * (uint32_t)((4 * kk + fq) ^ (fr & 7));
    fbase[0][kk] = (uint32_t)(uintptr_t)smem + (wr * 128 + fr) * 128 + sw;
    fbase[1][kk] = (uint32_t)(uintptr_t)smem + 2 * HALF + (wc * WN + fr) * 128 + sw;
  }
  auto frag = [&](int buf, int kk, int g) -> bf16x8 {
    const uint32_t a = g < 8 ? fbase[0][kk] + (uint32_t)(buf * HALF + g * 2048)
                             : fbase[1][kk] + (uint32_t)(buf * HB + (g - 8) * 2048);
    return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>((uintptr_t)a);
  };

  f32x4 acc[8][NB];
  bf16x8 f0[NF], f1[NF];

  // prologue: tiles 0 and 1 of the first unit in flight, tile 0's kk = 0 fragments in registers
#pragma unroll
  for (int q = 0; q < NF; ++q) dma(q, 0, 0);
#pragma unroll
  for (int q = 0; q < NF; ++q) dma(q, 1, 1);
  mc::wait_vmcnt<NF>();
  __builtin_amdgcn_s_barrier();

  // MFMAs of rows [4 ih, 4 ih + 4) of half-set f (ZERO: first K-tile, the accumulators start at 0)
  auto mfma_rows = [&](const bf16x8 (&f)[NF], int ih, auto zc) {
    constexpr bool ZERO = decltype(zc)::value;
#pragma unroll
    for (int i = 4 * ih; i < 4 * ih + 4; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[8 + j], f[i], ZERO ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][j],
                                                            0, 0, 0);
  };
  using Fz = std::false_type;
  using Tz = std::true_type;

  int nm0 = m0, nn0 = n0;      // next unit's origin
  bool has_next = false;

  // one K-tile; b (the tile's LDS buffer) is a compile-time constant so every LDS address is a
  // per-lane base + immediate. FIRST: the unit's first K-tile (zeroed accumulators; `after` = the
  // previous unit's full set of epilogue stores sits in the vmcnt window of barrier X).
  auto ktile = [&](auto bc, auto firstc, auto lastc, int t, bool after) {
    constexpr int b = decltype(bc)::value;
    constexpr bool FIRST = decltype(firstc)::value;
    constexpr bool LAST = decltype(lastc)::value;     // the unit's last K-tile: no f0 reads (they would
                                                      // stay live across the epilogue)
    dbase = dbase0;
    asm volatile("" : "+s"(dbase));
    // tile t+2: this unit's, the next unit's first two, or (last unit) a harmless reload of tile nk-1
    // into the dead buffer
    int kt2 = t + 2;
    if (t + 2 >= nk) kt2 = has_next ? t + 2 - nk : nk - 1;
    kt2 = __builtin_amdgcn_readfirstlane(kt2);      // uniform: keeps the DMAs' soffset in an SGPR
    constexpr int CM = 4 * NB;                      // MFMAs per chunk
    constexpr auto DS = [](auto) { return 0x100; };
    constexpr auto VM = [](auto) { return 0x010; };
    // chunk 0: f0 rows 0-63; read f1 of tile t
    fence();
    mc::static_for<0, NF>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (!(DBG & 2)) f1[g] = frag(b, 1, g);
    });
    mfma_rows(f0, 0, std::integral_constant<bool, FIRST>{});
    if constexpr (!(DBG & 2)) pin<CM, NF>(DS);
    fence();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();         // Y: buffer b is free
    if (t + 2 == nk && has_next) set_a(nm0);
    fence();
    // chunk 1: f0 rows 64-127; A DMAs of tile t+2 into buffer b
    mc::static_for<0, 8>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      if constexpr (!(DBG & 1)) dma(q, b, kt2);
    });
    mfma_rows(f0, 1, std::integral_constant<bool, FIRST>{});
    if constexpr (!(DBG & 1)) pin<CM, 8>(VM);
    fence();
    if constexpr (DBG & 1) {
      mc::wait_vmcnt<0>();
    } else if constexpr (FIRST) {
      if (after) mc::wait_vmcnt<8 + E>();   // tile t+1 landed; the epilogue's E stores may stay in flight
      else mc::wait_vmcnt<8>();
    } else {
      mc::wait_vmcnt<8>();                  // tile t+1 landed (this wave)
    }
    __builtin_amdgcn_s_barrier();         // X: ... for every wave
    if (t + 2 == nk && has_next) set_b(nn0);
    fence();
    // chunk 2: f1 rows 0-63; B DMAs of tile t+2; reads of the B fragments of f0 (tile t+1), alternating
    // (a DMA writes LDS: program order between it and the reads is kept, so the pins follow it)
    mc::static_for<0, NB>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      if constexpr (!(DBG & 1)) dma(8 + q, b, kt2);
      if constexpr (!(DBG & 2) && !LAST) f0[8 + q] = frag(b ^ 1, 0, 8 + q);
    });
    mfma_rows(f1, 0, Fz{});
    if constexpr (!(DBG & 1) && !(DBG & 2) && !LAST) {
      pin<CM, 2 * NB>([](auto ic) { return (decltype(ic)::value & 1) ? 0x100 : 0x010; });
    } else if constexpr (!(DBG & 1)) {
      pin<CM, NB>(VM);
    } else if constexpr (!(DBG & 2) && !LAST) {
      pin<CM, NB>(DS);
    }
    fence();
    // chunk 3: f1 rows 64-127; the A fragments of f0 (tile t+1), front-loaded so that the next
    // tile's first MFMAs do not wait for them
    mc::static_for<0, 8>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      if constexpr (!(DBG & 2) && !LAST) f0[g] = frag(b ^ 1, 0, g);
    });
    mfma_rows(f1, 1, Fz{});
    if constexpr (!(DBG & 2) && !LAST) pin<CM / 2, 8>(DS);
    __builtin_amdgcn_sched_group_barrier(0x008, CM - (DBG & 2 || LAST ? 0 : CM / 2), 0);
    fence();
  };

  // ---- epilogue straight from registers: acc[i][j][r] of row m0 + wr*128 + 16 i + fr; plain: tiles
  // (2P, 2P+1) = columns n0 + wc*128 + 32 P + 8 fq + [0, 8); GEGLU: tiles 4Q + {0 a-lo, 1 g-lo, 2 a-hi,
  // 3 g-hi} = outputs n0/2 + wc*64 + 32 Q + 8 fq + [0, 8).
  const bool hb = (e.flags & MC_EPI_BIAS) != 0, hr = (e.flags & MC_EPI_RESIDUAL) != 0;
  // One row block i at a time, each closed by a scheduling fence: the accumulator reads, the LN fold and the
  // stores of one block do not get hoisted together (a spill here reloads through vmcnt, which would also
  // wait for the next unit's in-flight DMAs). LN fold per element: v = acc * (alpha rstd) + (b - alpha
  // mean rstd cs) -- two FMAs.
  auto epilogue = [&]() {
    // lane-dependent indices re-derived here, opaque to the compiler: copies hoisted out of the K loop (all
    // 256 VGPRs taken) were spilled, and the scratch reload at the epilogue's start waited vmcnt(0) -- for
    // the next unit's in-flight DMAs as well
    int lane_e;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_e));
    const int fr = lane_e & 15, fq = lane_e >> 4;
    const long long ld16 = 16 * e.ldc;
    float2 st[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) st[i] = float2{0.f, 1.f};
    if constexpr (LN) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wr * 128 + 16 * i + fr;
        st[i] = *reinterpret_cast<const float2*>(e.rs + 2 * (long long)(row < M ? row : M - 1));
      }
    }
    const int row0 = m0 + wr * 128 + fr;
    if constexpr (GG) {
      const int Nout = N >> 1;
#pragma unroll
      for (int Q = 0; Q < 2; ++Q) {
        fence();
        const int oc = (n0 >> 1) + wc * 64 + 32 * Q + 8 * fq;     // first of 8 outputs
        const int ra_ = n0 + (((wc * 64 + 32 * Q + 8 * fq) >> 4) << 5) + ((8 * fq) & 15);   // its a row
        float ba[8], bg[8], ca[8], cg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) ba[k] = bg[k] = ca[k] = cg[k] = 0.f;
        if (oc < Nout) {
          if (hb) {
            unpack8(*reinterpret_cast<const uint4*>(e.bias + ra_), ba);
            unpack8(*reinterpret_cast<const uint4*>(e.bias + ra_ + 16), bg);
          }
          if constexpr (LN) {
            const float4* cp = reinterpret_cast<const float4*>(e.cs + ra_);
            const float4 c0 = cp[0], c1 = cp[1], c2 = cp[4], c3 = cp[5];
            ca[0] = c0.x; ca[1] = c0.y; ca[2] = c0.z; ca[3] = c0.w; ca[4] = c1.x; ca[5] = c1.y; ca[6] = c1.z; ca[7] = c1.w;
            cg[0] = c2.x; cg[1] = c2.y; cg[2] = c2.z; cg[3] = c2.w; cg[4] = c3.x; cg[5] = c3.y; cg[6] = c3.z; cg[7] = c3.w;
          }
        }
        u16* cp = e.C + (long long)row0 * e.ldc + oc;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = row0 + 16 * i;
          const float ar = e.alpha * st[i].y, amr = ar * st[i].x;
          float va[8], vg[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            va[r] = acc[i][4 * Q][r];
            va[4 + r] = acc[i][4 * Q + 2][r];
            vg[r] = acc[i][4 * Q + 1][r];
            vg[4 + r] = acc[i][4 * Q + 3][r];
          }
          float o[8];
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            f32x2_t ta = f32x2_t{ba[k], ba[k + 1]}, tg = f32x2_t{bg[k], bg[k + 1]};
            if constexpr (LN) {
              ta = ta - amr * f32x2_t{ca[k], ca[k + 1]};
              tg = tg - amr * f32x2_t{cg[k], cg[k + 1]};
            }
            const f32x2_t g2 = gelu_sig2(f32x2_t{vg[k], vg[k + 1]} * ar + tg);
            const f32x2_t a2 = f32x2_t{va[k], va[k + 1]} * ar + ta;
            o[k] = a2.x * g2.x;
            o[k + 1] = a2.y * g2.y;
          }
          if (row < M && oc < Nout) *reinterpret_cast<u32x4_t*>(cp) = pack8(o);
          cp += ld16;
          fence();
        }
      }
    } else if constexpr (BN != 256) {
      // 80-column wave tiles: lane (fr, fq) holds columns 16 j + 4 fq + [0, 4) of each MFMA tile j
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        fence();
        const int col = n0 + wc * WN + 16 * j + 4 * fq;
        float4 bv = float4{0.f, 0.f, 0.f, 0.f}, cv = float4{0.f, 0.f, 0.f, 0.f};
        if (col < N) {
          if (hb) bv = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
          if constexpr (LN) cv = *reinterpret_cast<const float4*>(e.cs + col);
        }
        u16* cp = e.C + (long long)row0 * e.ldc + col;
        const u16* rp = hr ? e.R + (long long)row0 * e.ldr + col : nullptr;
        const long long lr16 = 16 * e.ldr;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = row0 + 16 * i;
          const float ar = e.alpha * st[i].y, amr = ar * st[i].x;
          const f32x4 a = acc[i][j];
          float v0 = a[0] * ar + bv.x, v1 = a[1] * ar + bv.y, v2 = a[2] * ar + bv.z, v3 = a[3] * ar + bv.w;
          if constexpr (LN) {
            v0 -= amr * cv.x; v1 -= amr * cv.y; v2 -= amr * cv.z; v3 -= amr * cv.w;
          }
          if (row < M && col < N) {
            if (hr) {
              const float4 rv = unpack4_bf16(*reinterpret_cast<const uint2*>(rp));
              v0 += rv.x; v1 += rv.y; v2 += rv.z; v3 += rv.w;
            }
            *reinterpret_cast<uint2*>(cp) = pack4_bf16(v0, v1, v2, v3);
          }
          cp += ld16;
          if (hr) rp += lr16;
          fence();
        }
      }
    } else {
#pragma unroll
      for (int P = 0; P < 4; ++P) {
        fence();
        const int col = n0 + wc * 128 + 32 * P + 8 * fq;
        float bv[8], cv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) bv[k] = cv[k] = 0.f;
        if (col < N) {
          if (hb) unpack8(*reinterpret_cast<const uint4*>(e.bias + col), bv);
          if constexpr (LN) {
            const float4* cp4 = reinterpret_cast<const float4*>(e.cs + col);
            const float4 c0 = cp4[0], c1 = cp4[1];
            cv[0] = c0.x; cv[1] = c0.y; cv[2] = c0.z; cv[3] = c0.w; cv[4] = c1.x; cv[5] = c1.y; cv[6] = c1.z; cv[7] = c1.w;
          }
        }
        u16* cp = e.C + (long long)row0 * e.ldc + col;
        const u16* rp = hr ? e.R + (long long)row0 * e.ldr + col : nullptr;
        const long long lr16 = 16 * e.ldr;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = row0 + 16 * i;
          const float ar = e.alpha * st[i].y, amr = ar * st[i].x;
          float v[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[i][2 * P][r];
            v[4 + r] = acc[i][2 * P + 1][r];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float t = bv[k];
            if constexpr (LN) t -= amr * cv[k];
            v[k] = v[k] * ar + t;
          }
          if (row < M && col < N) {
            if (hr) {
              float rv[8];
              unpack8(*reinterpret_cast<const uint4*>(rp), rv);
#pragma unroll
              for (int k = 0; k < 8; ++k) v[k] += rv[k];
            }
            *reinterpret_cast<u32x4_t*>(cp) = pack8(v);
          }
          cp += ld16;
          if (hr) rp += lr16;
          fence();
        }
      }
    }
  };

  using B0 = std::integral_constant<int, 0>;
  using B1 = std::integral_constant<int, 1>;
  bool after = false;
  while (true) {
    const int un = u + G;
    has_next = un < T;
    if (has_next) unit_origin(un, nm0, nn0);
    // the unit's first fragments (tile 0 landed before the previous barrier X / the prologue barrier)
#pragma unroll
    for (int g = 0; g < NF; ++g) f0[g] = frag(0, 0, g);
    ktile(B0{}, Tz{}, Fz{}, 0, after);
    for (int t = 1; t + 1 < nk - 1 + 1 && t < nk - 1; t += 2) {     // nk is even (host-checked)
      ktile(B1{}, Fz{}, Fz{}, t, false);
      ktile(B0{}, Fz{}, Fz{}, t + 1, false);
    }
    ktile(B1{}, Fz{}, Tz{}, nk - 1, false);
    epilogue();
    // a full tile issued every one of its E stores (partial tiles may skip some: keep the plain wait)
    after = (m0 + BM <= M) && (n0 + BN <= N);
    if (!has_next) break;
    u = un;
    m0 = nm0;
    n0 = nn0;
  }
  mc::wait_vmcnt<0>();   // the trailing reload DMAs land before the workgroup's LDS is released
}

}  // namespace w6

template <int DBG, bool GG, bool LN, int BN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_bf16_nt_w6_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, const float* __restrict__ rs, const float* __restrict__ cs, int M, int N, int K,
    long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha, int tiles_m, int tiles_n,
    int group_m) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha};
  e.rs = rs;
  e.cs = cs;
  w6::run<DBG, GG, LN, BN>(A, lda, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
}

static int g_w6_cus = 0;

template <int DBG, bool GG, bool LN, int BN>
static int launch_w6(const void* A, const void* W, void* C, const void* bias, const void* R, const float* rs,
                     const float* cs, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
                     int epi, float alpha, int group_m, int grid_cap, hipStream_t stream) {
  constexpr int LDS = w6::Geo<BN>::LDS;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_w6_kernel<DBG, GG, LN, BN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr_set = true;
  }
  const int tiles_m = (M + w6::BM - 1) / w6::BM, tiles_n = (N + BN - 1) / BN;
  const long long T = (long long)tiles_m * tiles_n;
  if (T > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (g_w6_cus <= 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&g_w6_cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_w6_cus <= 0) g_w6_cus = 256;
  }
  const int cap = grid_cap > 0 ? grid_cap : g_w6_cus;     // one workgroup per CU
  const unsigned grid = (unsigned)(T < cap ? T : cap);
  gemm_bf16_nt_w6_kernel<DBG, GG, LN, BN><<<grid, w6::THREADS, LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, rs, cs, M, N, K, lda, ldw, ldc, ldr, epi,
      alpha, tiles_m, tiles_n, group_m);
  return (int)hipGetLastError();
}

// Shape / alignment domain of the w6 kernel (the dispatcher asks before choosing it); bn = 256 or 160.
CGS_EXPORT int cgs_gemm_w6_ok(int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr, int epi,
                              int bn) {
  const bool gg = (epi & MC_EPI_GEGLU) != 0;
  if (bn != 256 && bn != 160) return 0;
  if (K % 128 || K < 128 || N % 16 || lda % 8 || ldw % 8 || ldc % 8 || ((epi & MC_EPI_RESIDUAL) && ldr % 8)) return 0;
  if (epi & (MC_EPI_F32OUT | MC_EPI_GELU)) return 0;
  if (gg && ((epi & MC_EPI_RESIDUAL) || N % 32 || bn != 256)) return 0;
  if ((epi & MC_EPI_LNFOLD) && (epi & MC_EPI_RESIDUAL)) return 0;
  if ((long long)M * lda * 2 >= (1ll << 31) || (long long)N * ldw * 2 >= (1ll << 31)) return 0;
  return 1;
}

// epi: MC_EPI_BIAS / RESIDUAL / GEGLU / LNFOLD (rs: [M][2] (mean, rstd), cs: [N] colsums of W' = W * gamma).
// dbg: ablation probes (results wrong by design for dbg & 3). grid_cap: persistent grid (0 = one workgroup
// per CU; >= tiles = one tile per workgroup). bn: tile width 256 or 160.
CGS_EXPORT int cgs_gemm_bf16_w6(const void* A, const void* W, void* C, const void* bias, const void* R, const float* rs,
                                const float* cs, int M, int N, int K, long long lda, long long ldw, long long ldc,
                                long long ldr, int epi, float alpha, int dbg, int group_m, int grid_cap, int bn,
                                hipStream_t stream) {
  if (!cgs_gemm_w6_ok(M, N, K, lda, ldw, ldc, ldr, epi, bn) || ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C) % 16 ||
      ((epi & MC_EPI_RESIDUAL) && (uintptr_t)R % 16) || ((epi & MC_EPI_BIAS) && (uintptr_t)bias % 16) ||
      ((epi & MC_EPI_LNFOLD) && (!rs || !cs || (uintptr_t)cs % 16)))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  if (group_m <= 0) group_m = 4;
  const bool gg = (epi & MC_EPI_GEGLU) != 0, ln = (epi & MC_EPI_LNFOLD) != 0;
#define W6_CASE(D, GGV, LNV, BNV)                                                                                 \
  if (dbg == D && gg == GGV && ln == LNV && bn == BNV)                                                            \
    return launch_w6<D, GGV, LNV, BNV>(A, W, C, bias, R, rs, cs, M, N, K, lda, ldw, ldc, ldr, epi, alpha, group_m, \
                                       grid_cap, stream);
  W6_CASE(0, false, false, 256) W6_CASE(0, true, false, 256) W6_CASE(0, false, true, 256) W6_CASE(0, true, true, 256)
  W6_CASE(0, false, false, 160) W6_CASE(0, false, true, 160)
  W6_CASE(1, false, false, 256) W6_CASE(2, false, false, 256) W6_CASE(3, false, false, 256)
#undef W6_CASE
  return (int)hipErrorInvalidValue;
}
