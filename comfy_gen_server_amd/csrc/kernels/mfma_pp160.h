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

constexpr int BM = 256, BN = 160, BK = 64;
constexpr int THREADS = 512;
constexpr int A_BYTES = BM * 128;
constexpr int B_BYTES = BN * 128;
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int LDS = 3 * STAGE;     // 156 KiB
constexpr int EPI_PITCH = 176;     // bytes per staged output row (80 bf16 + pad, 16-B aligned)

// AL: loader with setup(slot, global_row) for slots 0..3 (tile rows slot*64 + (tid >> 3)) and
// src(slot, k0) -> this lane's 16-B source for K offset k0 (swizzled chunk already applied).
template <class AL>
__device__ __forceinline__ void tile(AL& al, const u16* __restrict__ W, long long ldw, int M, int N, int K, int m0,
                                     int n0, const mc::Epi& e, unsigned char* smem) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2;
  const int wm = wave & 3;
  const int nk = K / BK;

  const int lrow = tid >> 3;
  const int lch = tid & 7;
#pragma unroll
  for (int g = 0; g < 4; ++g) al.setup(g, m0 + g * 64 + lrow);
  const u16* bsrc[3];
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    const int r = g * 64 + lrow;
    int n = n0 + (r < BN ? r : BN - 1);
    n = n < N ? n : N - 1;
    bsrc[g] = W + (long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7));
  }
  auto stage = [&](int kt) {
    const int k0 = (kt < nk ? kt : nk - 1) * BK;   // past the end: reload the last tile into a dead slot
    unsigned char* base = smem + (kt % 3) * STAGE + wave * 1024;
#pragma unroll
    for (int g = 0; g < 4; ++g) mc::lds_dma16(al.src(g, k0), base + g * 8192);
    unsigned char* bb = base + A_BYTES;
    mc::lds_dma16((const void*)(bsrc[0] + k0), bb);
    mc::lds_dma16((const void*)(bsrc[1] + k0), bb + 8192);
    if (grp == 0) mc::lds_dma16((const void*)(bsrc[2] + k0), bb + 16384);   // B rows 128..159
  };
  auto wait_tile = [&]() {   // all but the 7 (group 0) / 6 (group 1) youngest DMAs retired
    if (grp == 0) mc::wait_vmcnt<7>();
    else mc::wait_vmcnt<6>();
  };

  f32x4 acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[4], bfr[5];
  auto read_frags = [&](const unsigned char* S, int kk) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + 16 * i + fr;
      const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
      af[i] = *reinterpret_cast<const bf16x8*>(S + r * 128 + 16 * c);
    }
    const unsigned char* SB = S + A_BYTES;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int r = grp * 80 + 16 * j + fr;
      const int c = (4 * kk + fq) ^ ((r >> 1) & 7);
      bfr[j] = *reinterpret_cast<const bf16x8*>(SB + r * 128 + 16 * c);
    }
  };
  auto mma = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  stage(0);
  stage(1);
  wait_tile();
  pp::barrier();
  if (grp == 1) pp::barrier();   // stagger: group 1 runs one segment behind group 0

  for (int kt = 0; kt < nk; ++kt) {
    const unsigned char* S = smem + (kt % 3) * STAGE;
    // phase 0: fragments k 0..31; DMA tile kt+2 into the slot tile kt-1 vacated
    read_frags(S, 0);
    stage(kt + 2);
    pp::wait_lgkm0();
    pp::barrier();
    mma();
    pp::barrier();
    // phase 1: fragments k 32..63; retire this wave's DMAs of tile kt+1
    read_frags(S, 1);
    wait_tile();
    pp::wait_lgkm0();
    pp::barrier();
    mma();
    pp::barrier();
  }
  if (grp == 0) pp::barrier();   // balance the stagger

  // ---- epilogue through LDS: 16x16 C layout col = lane & 15, row = 4 * (lane >> 4) + r
  mc::wait_vmcnt<0>();
  __syncthreads();
  unsigned char* region = smem + wave * (64 * EPI_PITCH);
  const int m_w = wm * 64, n_w = grp * 80;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int oc = 16 * j + fr;
    const int col = n0 + n_w + oc;
    const float bv = ((e.flags & MC_EPI_BIAS) && col < N) ? bf2f(e.bias[col]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * i + 4 * fq + r;
        *reinterpret_cast<u16*>(region + row * EPI_PITCH + 2 * oc) = f2bf(acc[i][j][r] * e.alpha + bv);
      }
  }
  for (int idx = lane; idx < 64 * 10; idx += 64) {
    const int rr = idx / 10, ch = idx - rr * 10;
    const int grow = m0 + m_w + rr;
    const int gcol = n0 + n_w + 8 * ch;
    s16x8 v = *reinterpret_cast<const s16x8*>(region + rr * EPI_PITCH + 16 * ch);
    if (grow < M && gcol < N) {
      if (e.flags & MC_EPI_RESIDUAL) {
        const s16x8 rv = *reinterpret_cast<const s16x8*>(e.R + (long long)grow * e.ldr + gcol);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((u16)v[t]) + bf2f((u16)rv[t]));
      }
      *reinterpret_cast<s16x8*>(e.C + (long long)grow * e.ldc + gcol) = v;
    }
  }
}

}  // namespace pq
