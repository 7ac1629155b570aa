// STATUS (measured, profiles/r04/gemm_hip_vs_hipblaslt.md): 0.5-0.8x of the production v6 / v7 kernels on
// every SDXL shape and its GEGLU form off by ~0.1 relative error -- an experiment the dispatcher never
// selects (tools/gemm_ab.py / gemm_probe.py only); GEGLU is refused at the entry point.
//
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

constexpr int BM = 256, BK = 64;
constexpr int THREADS = 256;
constexpr int AIMG = 256 * 128;          // A image of one K-tile (32 KiB)

// NJ = MFMA column tiles per wave: 8 -> 256-wide tiles (wave tile 128 x 128), 5 -> 160-wide tiles
// (128 x 80: every SDXL width is a multiple of 160, so 1280 / 640-wide GEMMs get whole rounds of tiles)
template <int NJ>
struct Geo {
  static constexpr int BN = 32 * NJ;          // tile columns
  static constexpr int WN = 16 * NJ;          // wave columns
  static constexpr int BIMG = BN * 128;       // B image of one K-tile
  static constexpr int BUF = AIMG + BIMG;     // one K-tile
  static constexpr int LDS = 2 * BUF;         // 128 / 104 KiB
  static constexpr int NP = NJ / 2;           // column-tile pairs (16-B stores); NJ odd: one 8-B tail tile
};

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(4))) uint32_t* cptr_u32;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

// Tile column (GEGLU: weight row within the tile) staged at B row r. Wave wc reads rows wc*WN + s;
// MFMA column tile j = s >> 4 holds lane fq = (s >> 2) & 3, element t = s & 3. Tiles 2p / 2p+1 give a lane
// 8 consecutive columns; an odd last tile keeps its 16 plain columns.
template <int NJ, bool GG>
__device__ __forceinline__ int b_col(int r) {
  constexpr int WN = Geo<NJ>::WN;
  const int wc = r / WN, s = r - wc * WN, j = s >> 4, fq = (s >> 2) & 3, t = s & 3;
  if constexpr (GG) {
    // (NJ == 8) output column o (0..63 within the wave's 64) = 32 (j >> 2) + 8 fq + 4 ((j >> 1) & 1) + t;
    // 'a' rows in even tiles, the matching 'g' rows in odd tiles ([a0..a15, g0..g15] weight interleave)
    const int o = wc * 64 + 32 * (j >> 2) + 8 * fq + 4 * ((j >> 1) & 1) + t;
    return (o >> 4) * 32 + 16 * (j & 1) + (o & 15);
  } else {
    if ((NJ & 1) && j == NJ - 1) return wc * WN + 16 * (NJ - 1) + 4 * fq + t;
    return wc * WN + 32 * (j >> 1) + 8 * fq + 4 * (j & 1) + t;
  }
}

template <int NJ, bool GG, bool LN>
__device__ __forceinline__ void run(const u16* __restrict__ A, long long lda, const u16* __restrict__ W,
                                    long long ldw, int M, int N, int K, const mc::Epi& e,
                                    unsigned char* smem, int tiles_m, int tiles_n, int group_m) {
  using Gm = Geo<NJ>;
  static_assert(!GG || NJ == 8, "GEGLU staging needs 256-wide tiles");
  constexpr int BN = Gm::BN, WN = Gm::WN, BUF = Gm::BUF, NP = Gm::NP;
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

  // ---- loaders: DMA g of this wave covers image rows g*32 + (tid >> 3), stored chunk tid & 7
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((long long)M * lda * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)((long long)N * ldw * 2), 0x00020000);
  const int lrow = tid >> 3;
  const int lch = tid & 7;
  uint32_t aoff[8], boff[NJ];
  auto setup = [&](int m0, int n0) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int r = g * 32 + lrow;
      const int m = m0 + r;
      aoff[g] = m < M ? (uint32_t)m * (uint32_t)(lda * 2) + 16u * (uint32_t)(lch ^ ((r >> 1) & 7)) : 0x80000000u;
    }
#pragma unroll
    for (int g = 0; g < NJ; ++g) {
      const int r = g * 32 + lrow;
      const int n = n0 + b_col<NJ, GG>(r);
      boff[g] = n < N ? (uint32_t)n * (uint32_t)(ldw * 2) + 16u * (uint32_t)(lch ^ ((r >> 1) & 7)) : 0x80000000u;
    }
  };
  auto dma_a = [&](int g, int sbuf, int kt) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(smem + sbuf * BUF + g * 4096 + wave * 1024), 16,
                                             aoff[g], kt * BK * 2, 0, 0);
  };
  auto dma_b = [&](int g, int sbuf, int kt) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (lds_void*)(smem + sbuf * BUF + AIMG + g * 4096 + wave * 1024), 16,
                                             boff[g], kt * BK * 2, 0, 0);
  };
  auto dma_tile = [&](int sbuf, int kt) {   // interleaved A / B so both operands arrive together
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      dma_a(g, sbuf, kt);
      if (g < NJ) dma_b(g, sbuf, kt);
    }
  };

  // ---- fragments: A row wr*128 + 16 i + (lane & 15), B row wc*WN + 16 j + (lane & 15); chunk 4 kk + (lane >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  const int swz = (fr >> 1) & 7;                        // (row >> 1) & 7 is the same for every fragment row
  const uint32_t c0 = 16u * (uint32_t)(fq ^ swz);       // kk = 0 chunk byte offset
  const uint32_t c1 = 16u * (uint32_t)((4 + fq) ^ swz); // kk = 1
  bf16x8 fa0[8], fb0[NJ], fa1[8], fb1[NJ];
  auto read_set = [&](int sbuf, uint32_t cb, bf16x8 (&fa)[8], bf16x8 (&fb)[NJ]) {
    const unsigned char* P = smem + sbuf * BUF;
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(P + (wr * 128 + 16 * i + fr) * 128 + cb);
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(P + AIMG + (wc * WN + 16 * j + fr) * 128 + cb);
  };

  // F0(t+1) reads from buffer rb interleaved with the DMAs of K-tile kd into buffer db (8 + NJ each)
  auto read_dma = [&](int rb, uint32_t cb, bf16x8 (&fa)[8], bf16x8 (&fb)[NJ], int db, int kd) {
    const unsigned char* P = smem + rb * BUF;
    mc::static_for<0, 8 + NJ>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i < 8)
        fa[i] = *reinterpret_cast<const bf16x8*>(P + (wr * 128 + 16 * i + fr) * 128 + cb);
      else
        fb[i - 8] = *reinterpret_cast<const bf16x8*>(P + AIMG + (wc * WN + 16 * (i - 8) + fr) * 128 + cb);
      // DMA i: A pieces first, then B (the same 8 + NJ loads as dma_tile)
      if constexpr (i < 8)
        dma_a(i, db, kd);
      else
        dma_b(i - 8, db, kd);
    });
  };

  f32x4 acc[8][NJ];
  // MFMAs over row tiles [I0, I1) of fragment set (fa, fb); Z: first K-tile (zero accumulator operand)
  auto mma = [&](auto i0c, auto i1c, auto zc, const bf16x8 (&fa)[8], const bf16x8 (&fb)[NJ]) {
    constexpr int I0 = decltype(i0c)::value, I1 = decltype(i1c)::value;
    constexpr bool Z = decltype(zc)::value;
#pragma unroll
    for (int i = I0; i < I1; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
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

  // ---- epilogue from registers. acc[i][j][t]: row m0 + wr*128 + 16 i + fr; column b_col order:
  // pair p (tiles 2p, 2p+1): n0 + wc*WN + 32 p + 8 fq + 4 (j & 1) + t; odd tail tile: n0 + wc*WN + 16 (NJ-1) +
  // 4 fq + t. GEGLU (NJ = 8): output column (n0 >> 1) + wc*64 + 32 h + 8 fq + 4 p + t for h = j >> 2,
  // p = (j >> 1) & 1, with a = tile j even, g = j + 1; half h covers weight rows wc*128 + 64 h + [0, 64).
  // Bias values come through the scalar cache (s_load: lgkm, no vmcnt wait behind the in-flight DMAs).
  auto sbias = [&](int c0, auto nd_c, int (&dw)[4][2], uint2 (&out)[2]) {
    // nd dwords of bias from column c0; lane fq takes dwords dw[fq][0..1] for words 0 / 1
    constexpr int ND = decltype(nd_c)::value;
    cptr_u32 bp = (cptr_u32)(e.bias + c0);
    uint32_t sv[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) sv[k] = __builtin_amdgcn_readfirstlane(bp[k]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int d0 = dw[0][q], d1 = dw[1][q], d2 = dw[2][q], d3 = dw[3][q];
      out[q].x = fq == 0 ? sv[d0] : fq == 1 ? sv[d1] : fq == 2 ? sv[d2] : sv[d3];
      out[q].y = fq == 0 ? sv[d0 + 1] : fq == 1 ? sv[d1 + 1] : fq == 2 ? sv[d2 + 1] : sv[d3 + 1];
    }
  };
  auto epilogue_t = [&](int m0, int n0, auto hbc, auto hrc) {
    constexpr bool HB = decltype(hbc)::value, HR = decltype(hrc)::value;
    const int ncw = n0 + wc * WN;
    float2 rst[8];                    // LayerNorm (mean, rstd) of the lane's 8 rows
    if constexpr (LN) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        int row = m0 + wr * 128 + 16 * i + fr;
        row = row < M ? row : M - 1;
        rst[i] = *reinterpret_cast<const float2*>(e.rs + 2 * (long long)row);
      }
    }
    // v = LN-folded accumulator + bias; tile j's 4 columns start at column col
    auto finish = [&](int i, int j, int col, const float4& bb, const float4& cs) {
      const f32x4 v = acc[i][j];
      float v0 = v[0] * e.alpha, v1 = v[1] * e.alpha, v2 = v[2] * e.alpha, v3 = v[3] * e.alpha;
      if constexpr (LN) {
        const float mr = rst[i].x * rst[i].y, rs = rst[i].y;
        v0 = rs * v[0] - mr * cs.x;
        v1 = rs * v[1] - mr * cs.y;
        v2 = rs * v[2] - mr * cs.z;
        v3 = rs * v[3] - mr * cs.w;
      }
      (void)col;
      return float4{v0 + bb.x, v1 + bb.y, v2 + bb.z, v3 + bb.w};
    };
    auto colsum = [&](int col) {
      if constexpr (LN) {
        col = col < N ? col : N - 4;
        return *reinterpret_cast<const float4*>(e.cs + col);
      } else {
        return float4{0.f, 0.f, 0.f, 0.f};
      }
    };
    if constexpr (GG) {
      const int Nout = N >> 1;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c0h = ncw + 64 * h;          // this half's 64 weight rows
        float4 bv[4], cv[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int o = 8 * fq + 4 * ((jj >> 1) & 1);
          const int lw = (o >> 4) * 32 + 16 * (jj & 1) + (o & 15);   // weight row within the half
          bv[jj] = float4{0.f, 0.f, 0.f, 0.f};
          cv[jj] = colsum(c0h + lw);
          if constexpr (HB) {
            if (c0h + 64 > N) {
              int col = c0h + lw;
              col = col < N ? col : N - 4;
              bv[jj] = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
            }
          }
        }
        if constexpr (HB) {
          if (c0h + 64 <= N) {
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              int dw[4][2];
#pragma unroll
              for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                  const int o = 8 * f + 4 * pp;
                  dw[f][q] = ((o >> 4) * 32 + 16 * q + (o & 15)) >> 1;
                }
              uint2 w2[2];
              sbias(c0h, std::integral_constant<int, 32>{}, dw, w2);
              bv[2 * pp] = unpack4_bf16(w2[0]);
              bv[2 * pp + 1] = unpack4_bf16(w2[1]);
            }
          }
        }
        const int ocol = (n0 >> 1) + wc * 64 + 32 * h + 8 * fq;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = m0 + wr * 128 + 16 * i + fr;
          uint2 o2[2];
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            const float4 a = finish(i, 4 * h + 2 * pp, 0, bv[2 * pp], cv[2 * pp]);
            const float4 g = finish(i, 4 * h + 2 * pp + 1, 0, bv[2 * pp + 1], cv[2 * pp + 1]);
            const f32x2_t g01 = gelu_sig2(f32x2_t{g.x, g.y}), g23 = gelu_sig2(f32x2_t{g.z, g.w});
            const f32x2_t o01 = f32x2_t{a.x, a.y} * g01, o23 = f32x2_t{a.z, a.w} * g23;
            o2[pp] = pack4_bf16(o01.x, o01.y, o23.x, o23.y);
          }
          if (row < M && ocol < Nout)
            *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + ocol) =
                u32x4_t{o2[0].x, o2[0].y, o2[1].x, o2[1].y};
        }
      }
    } else {
#pragma unroll
      for (int p = 0; p < NP; ++p) {             // column-tile pairs: 16-B stores
        const int cp = ncw + 32 * p;             // the pair's 32 columns
        float4 bv[2], cv[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          bv[q] = float4{0.f, 0.f, 0.f, 0.f};
          cv[q] = colsum(cp + 8 * fq + 4 * q);
        }
        if constexpr (HB) {
          if (cp + 32 <= N) {
            int dw[4][2];
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
              for (int q = 0; q < 2; ++q) dw[f][q] = (8 * f + 4 * q) >> 1;
            uint2 w2[2];
            sbias(cp, std::integral_constant<int, 16>{}, dw, w2);
            bv[0] = unpack4_bf16(w2[0]);
            bv[1] = unpack4_bf16(w2[1]);
          } else {
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              int col = cp + 8 * fq + 4 * q;
              col = col < N ? col : N - 4;
              bv[q] = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + col));
            }
          }
        }
        const int col = cp + 8 * fq;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = m0 + wr * 128 + 16 * i + fr;
          uint4 rq = uint4{0u, 0u, 0u, 0u};
          if constexpr (HR) {
            const int rr = row < M ? row : M - 1, cc = col < N ? col : N - 8;
            rq = *reinterpret_cast<const uint4*>(e.R + (long long)rr * e.ldr + cc);
          }
          uint2 hv[2];
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            float4 v = finish(i, 2 * p + q, col, bv[q], cv[q]);
            if constexpr (HR) {
              const float4 r4 = unpack4_bf16(q ? uint2{rq.z, rq.w} : uint2{rq.x, rq.y});
              v.x += r4.x; v.y += r4.y; v.z += r4.z; v.w += r4.w;
            }
            hv[q] = pack4_bf16(v.x, v.y, v.z, v.w);
          }
          if (row < M && col < N)
            *reinterpret_cast<u32x4_t*>(e.C + (long long)row * e.ldc + col) =
                u32x4_t{hv[0].x, hv[0].y, hv[1].x, hv[1].y};
        }
      }
      if constexpr (NJ & 1) {                    // odd tail tile: 16 plain columns, 8-B stores
        constexpr int j = NJ - 1;
        const int col = ncw + 16 * (NJ - 1) + 4 * fq;
        float4 bv = float4{0.f, 0.f, 0.f, 0.f};
        const float4 cv = colsum(col);
        if constexpr (HB) {
          const int cc = col < N ? col : N - 4;
          bv = unpack4_bf16(*reinterpret_cast<const uint2*>(e.bias + cc));
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = m0 + wr * 128 + 16 * i + fr;
          float4 v = finish(i, j, col, bv, cv);
          if constexpr (HR) {
            const int rr = row < M ? row : M - 1, cc = col < N ? col : N - 4;
            const float4 r4 = unpack4_bf16(*reinterpret_cast<const uint2*>(e.R + (long long)rr * e.ldr + cc));
            v.x += r4.x; v.y += r4.y; v.z += r4.z; v.w += r4.w;
          }
          if (row < M && col < N)
            *reinterpret_cast<uint2*>(e.C + (long long)row * e.ldc + col) = pack4_bf16(v.x, v.y, v.z, v.w);
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
  dma_tile(0, 0);
  dma_tile(1, 1);
  mc::wait_vmcnt<8 + NJ>();
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
    pin(std::integral_constant<int, 8 * NJ>{}, std::integral_constant<int, 8 + NJ>{}, I0{});
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
    // reads and DMAs alternate in PROGRAM order (r0 d0 r1 d1 ...): a DMA writes LDS, so the scheduler
    // keeps it ordered against every ds_read -- issued as all-reads-then-all-DMAs, the pin below could
    // not be met and the compiler bunched the 16 reads and 16 DMAs ahead of the MFMAs
    read_dma(sb ^ 1, c0, fa0, fb0, sb, kd);
    mma(I4{}, I8{}, F_{}, fa1, fb1);
    pin(std::integral_constant<int, 4 * NJ>{}, std::integral_constant<int, 8 + NJ>{},
        std::integral_constant<int, 8 + NJ>{});
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

template <int NJ, bool GG, bool LN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_bf16_nt_w4_kernel(
    const u16* __restrict__ A, const u16* __restrict__ W, u16* __restrict__ C, const u16* __restrict__ bias,
    const u16* __restrict__ R, int M, int N, int K, long long lda, long long ldw, long long ldc, long long ldr,
    int epi, float alpha, int tiles_m, int tiles_n, int group_m, const float* rs, const float* cs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  mc::Epi e{C, bias, R, ldc, ldr, epi, alpha, rs, cs};
  w4::run<NJ, GG, LN>(A, lda, W, ldw, M, N, K, e, smem, tiles_m, tiles_n, group_m);
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

template <int NJ, bool GG, bool LN>
static void w4_go(int grid, const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N, int K,
                  long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha, int tiles_m,
                  int tiles_n, const float* rs, const float* cs, hipStream_t stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_nt_w4_kernel<NJ, GG, LN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, w4::Geo<NJ>::LDS);
    attr = true;
  }
  gemm_bf16_nt_w4_kernel<NJ, GG, LN><<<grid, w4::THREADS, w4::Geo<NJ>::LDS, stream>>>(
      (const u16*)A, (const u16*)W, (u16*)C, (const u16*)bias, (const u16*)R, M, N, K, lda, ldw, ldc, ldr, epi, alpha,
      tiles_m, tiles_n, g_w4_group, rs, cs);
}

// epi: 1 bias, 2 residual, 4 GEGLU, 8 LayerNorm fold (rs / cs as in cgs_gemm_bf16_lnfold). bn: tile width
// 256 or 160 (0: 160 when N % 160 == 0 and it gives fewer / whole rounds of tiles, else 256; GEGLU: 256).
CGS_EXPORT int cgs_gemm_bf16_w4(const void* A, const void* W, void* C, const void* bias, const void* R, int M, int N,
                                int K, long long lda, long long ldw, long long ldc, long long ldr, int epi, float alpha,
                                const float* rs, const float* cs, int bn, hipStream_t stream) {
  const bool gg = (epi & MC_EPI_GEGLU) != 0, ln = (epi & MC_EPI_LNFOLD) != 0;
  const int nout = gg ? N / 2 : N;
  if (gg) return (int)hipErrorInvalidValue;     // GEGLU form numerically wrong (see STATUS above)
  if (K % 64 || K < 128 || lda % 8 || ldw % 8 || ldc % 8 || nout % 8 || (gg && N % 32) ||
      ((epi & MC_EPI_RESIDUAL) && (gg || ln || ldr % 8)) || (epi & MC_EPI_F32OUT) ||
      ((uintptr_t)A | (uintptr_t)W | (uintptr_t)C | (uintptr_t)R) % 16 || ((uintptr_t)bias % 8) ||
      (ln && (!rs || !cs || ((uintptr_t)cs % 16) || ((uintptr_t)rs % 8))) || (bn != 0 && bn != 160 && bn != 256) ||
      (gg && bn == 160) || (long long)M * lda * 2 >= (1ll << 31) || (long long)N * ldw * 2 >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  if (M == 0 || N == 0) return 0;
  if (g_w4_group < 0) g_w4_group = getenv("CGS_W4_GROUP") ? atoi(getenv("CGS_W4_GROUP")) : 4;
  const int tiles_m = (M + w4::BM - 1) / w4::BM;
  const int cus = w4_num_cus();
  if (bn == 0) {   // fewest rounds of CUs x tile width (least tail waste); GEGLU stays 256 wide
    const long long r256 = ((long long)tiles_m * ((N + 255) / 256) + cus - 1) / cus * 256;
    const long long r160 = ((long long)tiles_m * ((N + 159) / 160) + cus - 1) / cus * 160;
    bn = (!gg && N % 160 == 0 && r160 < r256) ? 160 : 256;
  }
  const int tiles_n = (N + bn - 1) / bn;
  const long long T = (long long)tiles_m * tiles_n;
  const int grid = (int)(T < cus ? T : cus);
#define W4A grid, A, W, C, bias, R, M, N, K, lda, ldw, ldc, ldr, epi, alpha, tiles_m, tiles_n, rs, cs, stream
  if (gg) {
    if (ln) w4_go<8, true, true>(W4A);
    else w4_go<8, true, false>(W4A);
  } else if (bn == 160) {
    if (ln) w4_go<5, false, true>(W4A);
    else w4_go<5, false, false>(W4A);
  } else {
    if (ln) w4_go<8, false, true>(W4A);
    else w4_go<8, false, false>(W4A);
  }
#undef W4A
  return (int)hipGetLastError();
}
