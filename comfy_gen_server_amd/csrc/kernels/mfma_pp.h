// Ping-pong MFMA main loop ("v5") for GEMM and implicit-GEMM conv on gfx950 (CDNA4).
//
// Block tile 256 x 256 x 64, 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns rows wr*128..+128 and
// cols wc*64..+64 = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs).
// The two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7; one of each per SIMD) run staggered by
// one s_barrier: while one group issues its 16-MFMA segment, its SIMD partner issues the next
// segment's fragment ds_reads and LDS-DMA loads -- the SIMD's MFMA pipe never waits for LDS or VMEM
// issue (cdna_hip_programming.md §5, the 256² 8-phase template, T3/T4/T5).
//
// K-tile (64 deep) = 4 phases, one per output quadrant of the wave (mq, nq) in the order
// (0,0) (0,1) (1,1) (1,0). Each K-tile is staged as four 16 KiB "parts" (128 rows x 128 B each):
//   A-part mq = tile rows {mq*64 + [0,64)} u {128 + mq*64 + [0,64)}   (group wr reads rows wr*64..+64)
//   B-part nq = tile cols {wc*64 + nq*32 + [0,32)}, wc = 0..3          (wave wc reads rows wc*32..+32)
// so a part is dead as soon as its quadrant's reads retire: A0, B0 after phase 1, B1 after phase 2,
// A1 after phase 3 (phase 4 reuses the B nq0 fragments kept in registers). Two 64 KiB buffers; while
// K-tile t (buffer t&1) is consumed, phase 1 DMAs A1(t+1) into the other buffer and phases 2-4 DMA
// A0/B0/B1(t+2) into the parts of buffer t&1 that died one phase earlier. Every part is issued 6
// phases before its first read (>= 1.3 us at full MFMA rate -- HBM/L2 latency hidden).
//
// Ordering rules (MI355X: LDS-DMA completion is visible to a ds_read only through the issuing wave's
// vmcnt + a barrier the reader passed; WAR needs the readers' lgkmcnt retired before a barrier):
//   * every load segment ends with lgkmcnt(0) BEFORE its barrier, so a part may be re-staged one
//     phase after its last read;
//   * the vmcnt(10) (5 younger parts x 2 DMAs in flight) is placed in the load segment of the phase
//     BEFORE the one that reads the part (one extra barrier covers the stagger).
// LDS rows are 128 B; 16-B chunk c of row r lives at chunk c ^ ((r >> 1) & 7) -- conflict-free for
// ds_read_b128 fragment reads; applied on the DMA source address (LDS DMA writes lane-linearly).
#pragma once
#include "common.h"
#include "mfma_core.h"   // Epi, wait_vmcnt, static_for, lds_dma16, MC_EPI_*

namespace pp {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int THREADS = 512;
constexpr int PART = 128 * 128;           // bytes per part
constexpr int BUF = 4 * PART;             // A0 A1 B0 B1
constexpr int LDS = 2 * BUF;              // 128 KiB
constexpr int P_A0 = 0, P_A1 = 1, P_B0 = 2, P_B1 = 3;

__device__ __forceinline__ void barrier() { __builtin_amdgcn_s_barrier(); }
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }   // lgkmcnt(0) only

// tile row of A-part mq, part-local row r (0..127)
__device__ __forceinline__ int a_row(int mq, int r) { return (r & 63) + ((r >> 6) << 7) + mq * 64; }
// tile col of B-part nq, part-local row r
__device__ __forceinline__ int b_col(int nq, int r) { return ((r >> 5) << 6) + nq * 32 + (r & 31); }

// AL: A loader, __device__ void setup(int slot, int row) for slot = mq*2 + round (row = global row,
// may be >= M) and __device__ const void* src(int slot, int k0) const (k0 multiple of 64).
template <class AL>
__device__ __forceinline__ void tile(AL& al, const u16* __restrict__ W, long long ldw, int M, int N, int K, int m0,
                                     int n0, const mc::Epi& e, unsigned char* smem) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int nk = K / BK;

  // ---- loader setup: thread t stages part-local rows (t >> 3) and 64 + (t >> 3), chunk t & 7
  const int lrow = tid >> 3;
  const int lch = tid & 7;
  if constexpr (mc::own_dma<AL>::value) al.tile(m0);
#pragma unroll
  for (int mq = 0; mq < 2; ++mq)
#pragma unroll
    for (int g = 0; g < 2; ++g) al.setup(mq * 2 + g, m0 + a_row(mq, g * 64 + lrow));
  const u16* bsrc[2][2];
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int r = g * 64 + lrow;
      int n = n0 + b_col(nq, r);
      n = n < N ? n : N - 1;
      bsrc[nq][g] = W + (long long)n * ldw + 8 * (lch ^ ((r >> 1) & 7));
    }
  // A-loader chunk swizzle is the same function of (r, lch); loaders apply it via src_chunk8().
  auto stage = [&](int part, int kt) {
    const int k0 = (kt < nk ? kt : nk - 1) * BK;   // past the end: reload the last tile into a dead part
    unsigned char* base = smem + (kt & 1) * BUF + part * PART + wave * 1024;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      if constexpr (mc::own_dma<AL>::value) {
        if (part == P_A0 || part == P_A1) al.dma((part == P_A0 ? 0 : 2) + g, k0, base + g * 8192);
        else mc::lds_dma16((const void*)(bsrc[part == P_B0 ? 0 : 1][g] + k0), base + g * 8192);
      } else {
        const void* src;
        if (part == P_A0) src = al.src(0 * 2 + g, k0);
        else if (part == P_A1) src = al.src(1 * 2 + g, k0);
        else if (part == P_B0) src = (const void*)(bsrc[0][g] + k0);
        else src = (const void*)(bsrc[1][g] + k0);
        mc::lds_dma16(src, base + g * 8192);
      }
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: row = base + 16*i + (lane & 15), chunk c = 4*kk + (lane >> 4)
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
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], b[j][kk], acc[mq * 4 + i][nq * 2 + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;

  // ---- prologue: A0 B0 B1 A1 of tile 0, A0 B0 B1 of tile 1 -> wait for A0(0), B0(0)
  stage(P_A0, 0);
  stage(P_B0, 0);
  stage(P_B1, 0);
  stage(P_A1, 0);
  stage(P_A0, 1);
  stage(P_B0, 1);
  stage(P_B1, 1);
  mc::wait_vmcnt<10>();
  barrier();
  if (wr == 1) barrier();   // stagger: group 1 runs one segment behind group 0

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    // phase 1 (mq0, nq0): read A0, B0; DMA A1(t+1); retire B1(t) for phase 2
    read_a(buf, 0);
    read_b(buf, 0, bf0);
    stage(P_A1, kt + 1);
    mc::wait_vmcnt<10>();
    wait_lgkm0();
    barrier();
    mma(I0{}, I0{}, bf0);
    barrier();
    // phase 2 (mq0, nq1): read B1; DMA A0(t+2); retire A1(t) for phase 3
    read_b(buf, 1, bf1);
    stage(P_A0, kt + 2);
    mc::wait_vmcnt<10>();
    wait_lgkm0();
    barrier();
    mma(I0{}, I1{}, bf1);
    barrier();
    // phase 3 (mq1, nq1): read A1; DMA B0(t+2)
    read_a(buf, 1);
    stage(P_B0, kt + 2);
    wait_lgkm0();
    barrier();
    mma(I1{}, I1{}, bf1);
    barrier();
    // phase 4 (mq1, nq0): no reads (B nq0 kept); DMA B1(t+2); retire A0(t+1), B0(t+1) for next phase 1
    stage(P_B1, kt + 2);
    mc::wait_vmcnt<10>();
    barrier();
    mma(I1{}, I0{}, bf0);
    barrier();
  }
  if (wr == 0) barrier();   // balance the stagger

  // ---- epilogue through LDS (16x16 C layout: col = lane & 15, row = 4 * (lane >> 4) + r)
  mc::wait_vmcnt<0>();      // clamped tail DMAs target LDS the epilogue reuses
  __syncthreads();
  const bool geglu = (e.flags & MC_EPI_GEGLU) != 0;
  const int OW = geglu ? 32 : 64;      // output cols of this wave
  const int CPR = OW / 8;
  const int pitch = OW * 2;
  unsigned char* region = smem + wave * (128 * 64 * 2);
  const int m_w = wr * 128, n_w = wc * 64;
  if (geglu) {
    // interleaved 16-row groups: MFMA col tile 2p holds 'a', 2p+1 the matching 'g'
    mc::static_for<0, 2>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      const int col_a = n0 + n_w + 32 * p + fr;
      float ba = 0.f, bg = 0.f;
      if ((e.flags & MC_EPI_BIAS) && n0 + n_w + 32 * p < N) { ba = bf2f(e.bias[col_a]); bg = bf2f(e.bias[col_a + 16]); }
      const int oc = 16 * p + fr;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fq + r;
          const float a = acc[i][2 * p][r] * e.alpha + ba;
          const float g = acc[i][2 * p + 1][r] * e.alpha + bg;
          *reinterpret_cast<u16*>(region + row * pitch + 16 * ((oc >> 3) ^ (row & (CPR - 1))) + 2 * (oc & 7)) =
              f2bf(a * gelu_sig(g));
        }
    });
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oc = 16 * j + fr;
      const int col = n0 + n_w + oc;
      const float bv = ((e.flags & MC_EPI_BIAS) && col < N) ? bf2f(e.bias[col]) : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fq + r;
          *reinterpret_cast<u16*>(region + row * pitch + 16 * ((oc >> 3) ^ (row & (CPR - 1))) + 2 * (oc & 7)) =
              f2bf(acc[i][j][r] * e.alpha + bv);
        }
    }
  }
  const int rows_per_it = 64 / CPR;
  const int gcol0 = geglu ? (n0 + n_w) / 2 : n0 + n_w;
  const int Nout = geglu ? N / 2 : N;
  const int ch = lane % CPR;
  for (int rr = lane / CPR; rr < 128; rr += rows_per_it) {
    const int grow = m0 + m_w + rr;
    const int gcol = gcol0 + 8 * ch;
    s16x8 v = *reinterpret_cast<const s16x8*>(region + rr * pitch + 16 * (ch ^ (rr & (CPR - 1))));
    if (grow < M && gcol < Nout) {
      if (e.flags & MC_EPI_RESIDUAL) {
        const s16x8 rv = *reinterpret_cast<const s16x8*>(e.R + (long long)grow * e.ldr + gcol);
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (short)f2bf(bf2f((u16)v[t]) + bf2f((u16)rv[t]));
      }
      *reinterpret_cast<s16x8*>(e.C + (long long)grow * e.ldc + gcol) = v;
    }
  }
}

// chunk swizzle for a loader row: part-local row r = g*64 + (tid >> 3), chunk tid & 7
__device__ __forceinline__ int src_chunk8(int g) {
  const int r = g * 64 + (threadIdx.x >> 3);
  return (threadIdx.x & 7) ^ ((r >> 1) & 7);
}

}  // namespace pp
