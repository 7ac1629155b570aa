// Flash attention forward for gfx950 (K02 self-attention, K03 short-KV cross-attention,
// K04 causal / key-padding masked CLIP attention). Reference semantics:
// comfy/ldm/modules/attention.py:88-383 (softmax(QK^T/sqrt(d))V with fp32 softmax accumulate).
//
// Design (CDNA4, wave64, MFMA 32x32x16 bf16):
//  * block = 4 waves, each wave owns 32 query rows (block = 128 queries) of one (batch, head);
//    a 1-D grid is XCD-remapped so the query blocks of one head share an XCD's L2 (K/V reuse).
//  * K/V tiles of 64 keys are staged through LDS (row-major, padded), register-staged one tile
//    ahead (issue global loads before the compute of the current tile, write LDS after barrier).
//  * "swapped" scores: S^T = K * Q^T so each lane holds 32 scores of ONE query -> the online
//    softmax (running max / sum / rescale) is lane-local except one xor-32 shuffle.
//  * output is accumulated transposed, O^T = V^T * P^T: the P^T accumulator registers ARE the
//    B operand of the next MFMA (no LDS round trip for P); V^T fragments come from
//    ds_read_b64_tr_b16 hardware-transposed LDS reads.
//  * exp2 with log2(e) folded into the score scale; fully-masked rows stay finite.
#include "common.h"

#define ATT_KV 64
#define ATT_WAVES 4
#define ATT_QB (32 * ATT_WAVES)

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// Additive fp32 score terms of the generic kernel (Swin-family window attention, K04): ``bias`` [H, Sq, Sk]
// (relative-position bias, shared by every batch entry) and ``mask`` [nW, Sq, Sk] for batch entry b taken at
// b % nW (shifted-window mask; -inf blocks a key). Both are added to the scaled scores before the softmax.
// ``hscale`` [H] (optional) multiplies head h's scores first (SwinV2's learned logit scale on cosine scores).
struct AttnBias {
  const float* bias;
  const float* mask;
  const float* hscale;
  int nW;
};

template <int DP, bool BIAS = false>
__global__ __launch_bounds__(256, (DP >= 160 ? 1 : 2)) void flash_fwd_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int B, int H, int Sq, int Sk, int D,
    long long qsb, long long qss, long long qsh, long long ksb, long long kss, long long ksh,
    long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float scale_log2, const signed char* __restrict__ key_mask, int causal, int nqb, float* __restrict__ lse,
    AttnBias ab = AttnBias{nullptr, nullptr, nullptr, 1}) {
  constexpr int KS = DP / 16;        // k-steps of the QK product
  constexpr int NDT = DP / 32;       // 32-wide d tiles of the output
  constexpr int LDW = DP + 8;        // padded LDS row (elements)
  constexpr int CH = DP / 8;         // 16-byte chunks per row
  constexpr int NCHUNK = ATT_KV * CH / 256;  // chunks per thread per tile (K and V each)
  static_assert((ATT_KV * CH) % 256 == 0, "tile must split evenly");

  __shared__ __attribute__((aligned(16))) u16 Ks[ATT_KV * LDW];
  __shared__ __attribute__((aligned(16))) u16 Vs[ATT_KV * LDW];

  const int nwg = gridDim.x;
  const int logical = xcd_remap(blockIdx.x, nwg);
  const int qb = logical % nqb;
  const int bh = logical / nqb;
  const int b = bh / H;
  const int h = bh % H;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int l32 = lane & 31;
  const int hf = lane >> 5;

  const u16* qbase = qp + b * qsb + h * qsh;
  const u16* kbase = kp + b * ksb + h * ksh;
  const u16* vbase = vp + b * vsb + h * vsh;
  u16* obase = op + b * osb + h * osh;

  const int q_row = qb * ATT_QB + wave * 32 + l32;   // this lane's query (for Q frag / softmax)
  const bool q_ok = q_row < Sq;

  // ---- Q fragments (B operand of S^T = K Q^T): lane holds Q[q_row][ks*16 + 8*hf + 0..7]
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    int d0 = ks * 16 + 8 * hf;
    if (q_ok && d0 < D) {
      s16x8 t = *reinterpret_cast<const s16x8*>(qbase + (long long)q_row * qss + d0);
      qf[ks] = __builtin_bit_cast(bf16x8, t);
    } else {
      qf[ks] = __builtin_bit_cast(bf16x8, s16x8{0, 0, 0, 0, 0, 0, 0, 0});
    }
  }

  f32x16 ot[NDT];
#pragma unroll
  for (int i = 0; i < NDT; ++i) ot[i] = f32x16{};
  float m_run = -INFINITY;
  float l_run = 0.f;

  if (BIAS && ab.hscale) scale_log2 *= ab.hscale[h];
  const int ntiles = (Sk + ATT_KV - 1) / ATT_KV;
  int tiles_end = ntiles;
  if (causal) {
    int last_q = min(Sq - 1, qb * ATT_QB + ATT_QB - 1);
    tiles_end = min(ntiles, last_q / ATT_KV + 1);
  }

  s16x8 kreg[NCHUNK], vreg[NCHUNK];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int c = 0; c < NCHUNK; ++c) {
      int idx = tid + c * 256;
      int key = idx / CH;
      int dch = idx % CH;
      int gk = t * ATT_KV + key;
      bool ok = gk < Sk && dch * 8 < D;
      s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
      kreg[c] = ok ? *reinterpret_cast<const s16x8*>(kbase + (long long)gk * kss + dch * 8) : zero;
      vreg[c] = ok ? *reinterpret_cast<const s16x8*>(vbase + (long long)gk * vss + dch * 8) : zero;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int c = 0; c < NCHUNK; ++c) {
      int idx = tid + c * 256;
      int key = idx / CH;
      int dch = idx % CH;
      *reinterpret_cast<s16x8*>(&Ks[key * LDW + dch * 8]) = kreg[c];
      *reinterpret_cast<s16x8*>(&Vs[key * LDW + dch * 8]) = vreg[c];
    }
  };

  if (tiles_end > 0) load_tile(0);
  for (int t = 0; t < tiles_end; ++t) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (t + 1 < tiles_end) load_tile(t + 1);

    // ---- S^T = K Q^T for two 32-key sub-tiles
    f32x16 s[2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        s16x8 a = *reinterpret_cast<const s16x8*>(&Ks[(kt * 32 + l32) * LDW + ks * 16 + 8 * hf]);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), qf[ks], s[kt], 0, 0, 0);
      }
    }
    // ---- masks + online softmax (lane = one query, 32 of the tile's 64 keys)
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int key = t * ATT_KV + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
        float v = s[kt][r] * scale_log2;
        bool valid = key < Sk;
        if (key_mask) valid = valid && key_mask[(long long)b * Sk + min(key, Sk - 1)] != 0;
        if (causal) valid = valid && key <= q_row;
        if (BIAS) {
          // LOG2E: the scores live in the exp2 domain
          const long long qk = (long long)min(q_row, Sq - 1) * Sk + min(key, Sk - 1);
          float add = ab.bias[(long long)h * Sq * Sk + qk];
          if (ab.mask) add += ab.mask[(long long)(b % ab.nW) * Sq * Sk + qk];
          v = fmaf(add, 1.4426950408889634f, v);
        }
        v = valid ? v : -INFINITY;
        s[kt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    float m_new = fmaxf(m_run, tmax);
    float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    float psum = 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = exp2f(s[kt][r] - m_use);
        s[kt][r] = p;
        psum += p;
      }
    l_run = l_run * alpha + psum;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[dt][r] *= alpha;

    // ---- O^T += V^T P^T ; P^T registers are the B operand directly
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)s[kt][8 * st + j];
        const int kb = kt * 32 + 16 * st;
        const int i16 = lane & 15;
        const int row0 = kb + 4 * hf + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
          bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)&Vs[row0 * LDW + col]);
          bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)&Vs[(row0 + 8) * LDW + col]);
          bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          ot[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, ot[dt], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: O[q][d] = O^T[d][q] / l
  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  // natural-log LSE of the scaled scores (ring attention merge): sum_k e^(s scale) = 2^m_run * l_tot
  if (lse && q_ok && hf == 0)
    lse[((long long)b * H + h) * Sq + q_row] = l_tot > 0.f ? (m_run + __log2f(l_tot)) * 0.69314718055994531f : -INFINITY;
  if (q_ok) {
    u16* orow = obase + (long long)q_row * oss;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        int d0 = dt * 32 + 8 * r4 + 4 * hf;
        if (d0 < D) {
          s16x4 w;
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = (short)f2bf(ot[dt][4 * r4 + j] * inv);
          *reinterpret_cast<s16x4*>(orow + d0) = w;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Fast path: D = 64, no mask / causal (SDXL / SD2 / Cascade self- and cross-attention).
//  * 8 waves x 32 query rows = 256-row Q block per workgroup (one WG per CU, 2 waves per SIMD);
//    K/V tiles of 64 keys in a 2-slot LDS ring, ONE barrier per tile.
//  * software pipeline inside each wave: QK^T of tile t+1 is issued in the same basic block as the
//    softmax of tile t (independent MFMA and VALU streams interleave), then PV of tile t.
//    K is staged two tiles ahead, V one tile ahead (register-staged: global loads issued at the
//    top of the tile, LDS writes after the compute — T14).
//  * K image: 128-B rows, 16-B chunk c stored at c ^ ((row>>1)&7) -> conflict-free ds_read_b128 of
//    the 32x32x16 A operand; V image: chunk c ^ (((row>>1)&1)<<2) -> conflict-free
//    ds_read_b64_tr_b16 of the transposed V^T operand.
//  * softmax: fma-folded scale (exp2 domain), v_max3 chains, permlane32 max exchange, deferred
//    rescale (only when a lane's running max grows by > 2^8 — bf16 keeps its relative precision),
//    only the last tile masks (keys >= Sk).
#define AF_THR 8.0f

__device__ __forceinline__ float af_xmax(float v) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// MSUM: the row sums come from the P.V MFMAs (an all-ones A operand into ``lsum``, see
// attn_fwd_d64_kernel) instead of 32 v_add_f32 per lane per tile; only the rescale touches lsum.
template <bool TAIL, bool MSUM = false>
__device__ __forceinline__ void af_softmax(f32x16 (&s)[2], bf16x8 (&pf)[4], f32x16 (&ot)[2], float& m_run,
                                           float& l_run, float c, int key0, int Sk, int hf,
                                           f32x16* lsum = nullptr) {
  if (TAIL) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int key = key0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
        s[kt][r] = key < Sk ? s[kt][r] : -INFINITY;
      }
  }
  float mx = fmaxf(s[0][0], s[0][1]);
#pragma unroll
  for (int i = 2; i < 32; i += 2) mx = fmaxf(fmaxf(mx, s[i >> 4][i & 15]), s[i >> 4][(i & 15) + 1]);
  mx = af_xmax(mx) * c;
  if (__any(mx > m_run + AF_THR)) {
    float m_new = fmaxf(m_run, mx);
    float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[dt][r] *= alpha;
    if constexpr (MSUM) {
#pragma unroll
      for (int r = 0; r < 16; ++r) (*lsum)[r] *= alpha;
    }
  }
  const float nm = -m_run;
  float ps = 0.f;
  // (v_pk_fma_f32 pairs for these exponent arguments measured 2-4 % SLOWER at SDXL levels 1 / 2,
  // profiles/r04/attn_pkfma_ab.log: scalar v_fma_f32 stays)
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][r], c, nm));
      if constexpr (!MSUM) ps += p;
      pf[kt * 2 + (r >> 3)][r & 7] = (__bf16)p;
    }
  if constexpr (!MSUM) l_run += ps;
}

// O epilogue of the D = 64 kernels (T21): lanes l and l + 32 hold the same query row as 8-B halves of
// each 16-B column group; one v_permlane32_swap per dword pairs them so every lane stores 16 B (4
// instead of 8 store instructions per lane, full 32-B runs per lane pair). Needs 16-B aligned rows (al16).
// Measured vs the 8-B form (profiles/r03/attn_t21_stores.log): level-2 self-attention +12 %, the
// short-KV cross-attention +14..16 %, level-1 self-attention neutral; outputs bitwise equal.
__device__ __forceinline__ void af_store_row64(u16* __restrict__ orow, const f32x16 (&ot)[2], float inv, int hf,
                                               bool ok) {
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int rp = 0; rp < 2; ++rp) {
      uint2 a = pack4_bf16(ot[dt][8 * rp] * inv, ot[dt][8 * rp + 1] * inv, ot[dt][8 * rp + 2] * inv,
                           ot[dt][8 * rp + 3] * inv);
      uint2 b = pack4_bf16(ot[dt][8 * rp + 4] * inv, ot[dt][8 * rp + 5] * inv, ot[dt][8 * rp + 6] * inv,
                           ot[dt][8 * rp + 7] * inv);
      auto rx = __builtin_amdgcn_permlane32_swap(a.x, b.x, false, false);
      auto ry = __builtin_amdgcn_permlane32_swap(a.y, b.y, false, false);
      if (ok) *reinterpret_cast<uint4*>(orow + dt * 32 + 16 * rp + 8 * hf) = uint4{rx[0], ry[0], rx[1], ry[1]};
    }
}

// Second K/V source (TWO): keys [0, sk1) come from the kernel's k / v, keys [sk1, Sk) from k / v here
// (same head stride). Stable Cascade's self-attention attends over cat([x, kv_mapped]) -- with two
// sources neither the concat nor a separate K / V projection of it is materialised.
struct KV2 {
  const u16* k;
  const u16* v;
  int sk1;
  long long ksb, kss, vsb, vss;
};

// A persistent form (one WG per CU walking the units, the next unit's K / V / Q streamed in under the last
// tiles of the current one) was built and measured in round 4: level 2 651 vs 632 TF/s (auto 663), level 1
// 792 vs 844 (246 VGPRs) -- the per-unit prologue is not where level 2 loses (profiles/r04/
// attn_persistent_ab_r04ak.log); a second version that also issued the next unit's first QK^T under the
// current unit's last softmax (no pipeline drain between units, 255 VGPRs) measured 663 vs 639-685 at
// level 2 and 843 vs 834-871 at level 1 (within the run-to-run spread of sequential timing,
// attn_persistent_v2_r04at.log); removed.
// NW = 8: 256-row Q block, one WG per CU. NW = 4: 128-row Q block, two WGs per CU -- twice the
// workgroups for the under-filled grids of small batches (batch-1 SDXL level 2: 160 -> 320).
// KS > 1 (key split, small grids): the grid is KS x (Q blocks x B x H); split s attends over its run of
// ceil(tiles / KS) 64-key tiles only and writes its normalised partial O to op + s * ospl and its
// log-sum-exp to lse + s * B * H * Sq; attn_ks_combine_kernel merges the KS partials. The host
// guarantees every split has at least one key.
template <int NW, bool TWO = false, bool PRIO = true, int KS = 1>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_fwd_d64_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int H, int Sq, int Sk, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
    long long ksh, long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float c, int nqb, float* __restrict__ lse = nullptr, KV2 kv2 = KV2{nullptr, nullptr, 0, 0, 0, 0, 0},
    long long ospl = 0) {
  __shared__ __attribute__((aligned(16))) u16 Ks[2][64 * 64];
  __shared__ __attribute__((aligned(16))) u16 Vs[2][64 * 64];

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = logical % nqb;
  int bh = logical / nqb;
  int k_lo = 0;
  if constexpr (KS > 1) {
    const int BH = (int)(gridDim.x / ((unsigned)nqb * KS));
    const int split = bh / BH;
    bh -= split * BH;
    const int tps = ((Sk + 63) / 64 + KS - 1) / KS;
    k_lo = split * tps * 64;
    Sk = min(Sk - k_lo, tps * 64);
    op += split * ospl;
    lse += (long long)split * BH * Sq;
  }
  const int b = bh / H, h = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hf = lane >> 5;

  const u16* qbase = qp + b * qsb + h * qsh;
  const u16* kbase = kp + b * ksb + h * ksh + (long long)k_lo * kss;
  const u16* vbase = vp + b * vsb + h * vsh + (long long)k_lo * vss;
  u16* obase = op + b * osb + h * osh;

  const int q_row = qb * (32 * NW) + wave * 32 + l32;
  const bool q_ok = q_row < Sq;
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    s16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q_ok) t = *reinterpret_cast<const s16x8*>(qbase + (long long)q_row * qss + ks * 16 + 8 * hf);
    qf[ks] = __builtin_bit_cast(bf16x8, t);
  }

  // staging: thread -> (key = tid>>3 + 64/LPT * i, chunk = tid&7) of a 64x64 tile, LPT keys per thread
  constexpr int LPT = 8 / NW;
  const int st_c = tid & 7;
  int k_woff[LPT], v_woff[LPT], st_key[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    st_key[i] = (tid >> 3) + i * (8 * NW);
    k_woff[i] = st_key[i] * 64 + 8 * (st_c ^ ((st_key[i] >> 1) & 7));
    v_woff[i] = st_key[i] * 64 + 8 * (st_c ^ (((st_key[i] >> 1) & 1) << 2));
  }
  const int n = (Sk + 63) >> 6;
  struct Stg { s16x8 v[LPT]; };
  // per-lane row offsets computed once; per tile only the uniform t * 64 * stride (scalar) is added
  // (keys past Sk read the last row: they are masked in the softmax)
  long long koff[LPT], voff[LPT];
#pragma unroll
  for (int i = 0; i < LPT; ++i) {
    koff[i] = (long long)st_key[i] * kss + st_c * 8;
    voff[i] = (long long)st_key[i] * vss + st_c * 8;
  }
  const long long kclamp = (long long)(Sk - 1) * kss + st_c * 8, vclamp = (long long)(Sk - 1) * vss + st_c * 8;
  auto gload = [&](const u16* base, long long ss, const long long (&off)[LPT], long long clampo, int t) -> Stg {
    Stg r;
    const long long tb = (long long)(t * 64) * ss;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const long long o = (t * 64 + st_key[i] < Sk) ? tb + off[i] : clampo;
      r.v[i] = *reinterpret_cast<const s16x8*>(base + o);
    }
    return r;
  };
  // two-source loads: key -> (source, row) per lane (keys past Sk read the last key: masked later)
  const u16* k2base = TWO ? kv2.k + b * kv2.ksb + h * ksh : nullptr;
  const u16* v2base = TWO ? kv2.v + b * kv2.vsb + h * vsh : nullptr;
  auto gload2 = [&](bool isk, int t) -> Stg {
    Stg r;
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int key = min(t * 64 + st_key[i], Sk - 1);
      const u16* p = key < kv2.sk1 ? (isk ? kbase + (long long)key * kss : vbase + (long long)key * vss)
                                   : (isk ? k2base + (long long)(key - kv2.sk1) * kv2.kss
                                          : v2base + (long long)(key - kv2.sk1) * kv2.vss);
      r.v[i] = *reinterpret_cast<const s16x8*>(p + st_c * 8);
    }
    return r;
  };
  auto ldk = [&](int t) -> Stg {
    if constexpr (TWO) return gload2(true, t);
    else return gload(kbase, kss, koff, kclamp, t);
  };
  auto ldv = [&](int t) -> Stg {
    if constexpr (TWO) return gload2(false, t);
    else return gload(vbase, vss, voff, vclamp, t);
  };
  auto lds_put = [&](u16* tile, const int (&off)[LPT], const Stg& x) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) *reinterpret_cast<s16x8*>(&tile[off[i]]) = x.v[i];
  };
  // QK^T A-operand read offsets (elements) for kt = 0/1, ks = 0..3
  auto k_roff = [&](int kt, int ks) {
    int key = kt * 32 + l32;
    return key * 64 + 8 * ((2 * ks + hf) ^ ((key >> 1) & 7));
  };
  auto qk = [&](const u16* Kt, f32x16 (&s)[2]) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 a = *reinterpret_cast<const s16x8*>(Kt + k_roff(kt, ks));
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), qf[ks], s[kt], 0, 0, 0);
      }
    }
  };
  const int i16 = lane & 15;
  // row sums on the matrix core: an all-ones A operand turns P into sum_k P[k][q] in every row of
  // lsum (bf16-rounded P, the same weights the numerator uses)
  const bf16x8 ones = {(__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f, (__bf16)1.f,
                       (__bf16)1.f};
  f32x16 lsum = f32x16{};
  auto pv = [&](const u16* Vt, const bf16x8 (&pf)[4], f32x16 (&ot)[2]) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        lsum = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ones, pf[kt * 2 + st], lsum, 0, 0, 0);
        const int row0 = kt * 32 + 16 * st + 4 * hf + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
          const int ch = col >> 3, half = (col >> 2) & 1;
          const int r1 = row0 + 8;
          const int o0 = row0 * 64 + 8 * (ch ^ (((row0 >> 1) & 1) << 2)) + 4 * half;
          const int o1 = r1 * 64 + 8 * (ch ^ (((r1 >> 1) & 1) << 2)) + 4 * half;
          bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vt + o0));
          bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vt + o1));
          bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          ot[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt * 2 + st], ot[dt], 0, 0, 0);
        }
      }
  };

  f32x16 ot[2] = {f32x16{}, f32x16{}};
  float m_run = -INFINITY, l_run = 0.f;
  bf16x8 pf[4];
  f32x16 sA[2], sB[2];

  // prologue: K(0) -> slot 0, K(1) -> slot 1, V(0) -> slot 0; S(0)
  {
    const Stg k0 = ldk(0);
    const Stg k1 = ldk(n > 1 ? 1 : 0);
    const Stg v0 = ldv(0);
    lds_put(Ks[0], k_woff, k0);
    lds_put(Ks[1], k_woff, k1);
    lds_put(Vs[0], v_woff, v0);
  }
  // two register stages: the K / V rows written to LDS at the end of tile t were loaded during tile
  // t - 1, so a global load has a whole tile of compute (not just the rest of its own tile) to land
  Stg kq[2], vq[2];
  kq[0] = ldk(min(2, n - 1));
  vq[0] = ldv(min(1, n - 1));
  __syncthreads();
  qk(Ks[0], sA);

  // steady state: iteration t consumes S(t) (in sCur), produces S(t+1) (in sNext); it loads
  // K(t+3) / V(t+2) into register set LD and writes K(t+2) / V(t+1) from set WR (= t & 1)
  auto body = [&](int t, f32x16 (&sCur)[2], f32x16 (&sNext)[2], auto ldc) {
    constexpr int LD = decltype(ldc)::value, WR = LD ^ 1;
    const int slot = t & 1;
    kq[LD] = ldk(min(t + 3, n - 1));
    vq[LD] = ldv(min(t + 2, n - 1));
    qk(Ks[slot ^ 1], sNext);
    af_softmax<false, true>(sCur, pf, ot, m_run, l_run, c, t * 64, Sk, hf, &lsum);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);   // the dependent P.V MFMAs ahead of the partner's VALU
    pv(Vs[slot], pf, ot);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    lds_put(Ks[slot], k_woff, kq[WR]);
    lds_put(Vs[slot ^ 1], v_woff, vq[WR]);
    __syncthreads();
  };
  using L1 = std::integral_constant<int, 1>;
  using L0 = std::integral_constant<int, 0>;
  int t = 0;
  for (; t + 2 < n; t += 2) {
    body(t, sA, sB, L1{});
    body(t + 1, sB, sA, L0{});
  }
  if (t + 1 < n) {   // one full iteration left before the last tile
    body(t, sA, sB, L1{});
    ++t;
    af_softmax<true, true>(sB, pf, ot, m_run, l_run, c, t * 64, Sk, hf, &lsum);
  } else {
    af_softmax<true, true>(sA, pf, ot, m_run, l_run, c, t * 64, Sk, hf, &lsum);
  }
  pv(Vs[t & 1], pf, ot);

  // epilogue: O[q][d] = O^T[d][q] / l (every row of lsum holds the full key sum of this lane's q)
  float l_tot = lsum[0];
  float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (lse && q_ok && hf == 0)
    lse[((long long)b * H + h) * Sq + q_row] = l_tot > 0.f ? (m_run + __log2f(l_tot)) * 0.69314718055994531f : -INFINITY;
  af_store_row64(obase + (long long)q_row * oss, ot, inv, hf, q_ok);
}

// ------------------------------------------------------------------------------------------------
// Short-KV path (K03): cross-attention against the text context, D = 64, Sk <= 128 keys
// (SDXL/SD2 77-token context, Cascade 4..85-token kv_mapper tokens). Every key fits in LDS at once,
// so there is no key loop and no online softmax: K and V are staged ONCE per workgroup (zero padded
// to NKT*32 keys, same swizzled images as the D=64 kernel), each wave computes S^T = K Q^T for its
// 32 queries over all NKT 32-key sub-tiles, takes the exact row max / sum in registers (one
// permlane32 exchange), and does O^T = V^T P^T. 4 waves x 32 queries = 128 queries per workgroup.
// The reference runs this shape through the same optimized_attention as self-attention
// (comfy/ldm/modules/attention.py:352-383); the general flash kernel would pay a full 64-key
// pipeline for 77 keys.
// QI > 1: each wave walks QI 32-query blocks (stride 128 queries) with the next block's Q rows loaded
// while the current one computes, so K / V are staged once per 128 * QI queries and the Q stream stays
// in flight: at QI = 1 a workgroup's life was one K/V + Q load latency for ~1 us of math (SDXL
// cross-attention ran at ~2.5 TB/s of its Q + O traffic).
// QI = 1, NKT <= 3 is built for 5 waves per SIMD (launch bounds: <= 102 registers instead of ~110, 4 -> 5 workgroups per
// CU): SDXL level-2 cross-attention 25.7 -> 24.4 us (profiles/r06/skv_lb_ab.log; 6 waves measured no better).
template <int NKT, bool PRIO = true, int QI = 1>
__global__ __launch_bounds__(256, (QI == 1 && NKT <= 3) ? 5 : 1) void attn_fwd_d64_shortkv_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int H, int Sq, int Sk, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
    long long ksh, long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float c, int nqb) {
  constexpr int NK = NKT * 32;
  __shared__ __attribute__((aligned(16))) u16 Ks[NK * 64];
  __shared__ __attribute__((aligned(16))) u16 Vs[NK * 64];

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = logical % nqb;
  const int bh = logical / nqb;
  const int b = bh / H, h = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hf = lane >> 5;

  const u16* qbase = qp + b * qsb + h * qsh;
  const u16* kbase = kp + b * ksb + h * ksh;
  const u16* vbase = vp + b * vsb + h * vsh;
  u16* obase = op + b * osb + h * osh;

  // stage all keys: thread -> (key, 16-B chunk); keys >= Sk are zero (masked below)
#pragma unroll
  for (int it = 0; it < NKT; ++it) {
    const int idx = it * 256 + tid;
    const int key = idx >> 3, ch = idx & 7;
    s16x8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (key < Sk) {
      kv = *reinterpret_cast<const s16x8*>(kbase + (long long)key * kss + ch * 8);
      vv = *reinterpret_cast<const s16x8*>(vbase + (long long)key * vss + ch * 8);
    }
    *reinterpret_cast<s16x8*>(&Ks[key * 64 + 8 * (ch ^ ((key >> 1) & 7))]) = kv;
    *reinterpret_cast<s16x8*>(&Vs[key * 64 + 8 * (ch ^ (((key >> 1) & 1) << 2))]) = vv;
  }

  auto loadq = [&](int q_row, bf16x8 (&qf)[4]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      s16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q_row < Sq) t = *reinterpret_cast<const s16x8*>(qbase + (long long)q_row * qss + ks * 16 + 8 * hf);
      qf[ks] = __builtin_bit_cast(bf16x8, t);
    }
  };
  const int row_base = qb * (128 * QI) + wave * 32 + l32;
  bf16x8 qf[4];
  loadq(row_base, qf);
  __syncthreads();

#pragma unroll 1
  for (int qi = 0; qi < QI; ++qi) {
    const int q_row = row_base + 128 * qi;
    bf16x8 qn[4];
    if (QI > 1 && qi + 1 < QI) loadq(q_row + 128, qn);   // next block's Q rows, in flight under this one
    f32x16 s[NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      s[kt] = f32x16{};
      const int key = kt * 32 + l32;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s16x8 a = *reinterpret_cast<const s16x8*>(&Ks[key * 64 + 8 * ((2 * ks + hf) ^ ((key >> 1) & 7))]);
        s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), qf[ks], s[kt], 0, 0, 0);
      }
    }
    // exact softmax over the whole key set (lane = one query, its half of the keys)
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hf;
        s[kt][r] = key < Sk ? s[kt][r] : -INFINITY;
        mx = fmaxf(mx, s[kt][r]);
      }
    mx = af_xmax(mx) * c;
    const float nm = -mx;
    float ps = 0.f;
    bf16x8 pf[2 * NKT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][r], c, nm));
        ps += p;
        pf[kt * 2 + (r >> 3)][r & 7] = (__bf16)p;
      }
    f32x16 ot[2] = {f32x16{}, f32x16{}};
    const int i16 = lane & 15;
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);   // P.V MFMAs ahead of co-resident waves' softmax VALU
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int row0 = kt * 32 + 16 * st + 4 * hf + (i16 >> 2);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
          const int ch = col >> 3, half = (col >> 2) & 1;
          const int r1 = row0 + 8;
          const int o0 = row0 * 64 + 8 * (ch ^ (((row0 >> 1) & 1) << 2)) + 4 * half;
          const int o1 = r1 * 64 + 8 * (ch ^ (((r1 >> 1) & 1) << 2)) + 4 * half;
          bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vs + o0));
          bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vs + o1));
          bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          ot[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt * 2 + st], ot[dt], 0, 0, 0);
        }
      }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    const float l_tot = ps + __shfl_xor(ps, 32, 64);
    const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    af_store_row64(obase + (long long)q_row * oss, ot, inv, hf, q_row < Sq);
    if constexpr (QI > 1) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) qf[ks] = qn[ks];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Wide-head path (K22): the KL-VAE mid-block attention, ONE head of D = 512 over H*W tokens
// (16 k tokens at 1024², comfy/ldm/modules/diffusionmodules/model.py:227-292). A 32-query O^T
// accumulator for D = 512 does not fit one wave (256 accumulator registers), so the head dim is
// split over the 4 waves of a workgroup: wave w owns d in [128w, 128w+128) of Q, of the output
// and of the V^T operand. Per 32-key tile each wave computes a PARTIAL S^T = K Q^T over its d
// slice (8 MFMA 32x32x16), the 4 partials are summed through LDS (every wave ends up with the
// full, identical scores), the online softmax runs redundantly in the 4 waves, and each wave does
// O^T[its 128 d] += V^T P^T (8 MFMA). K/V tiles (32 keys x 512 d) are register-prefetched one tile
// ahead into a single LDS buffer; K rows use a chunk ^ (key & 15) swizzle (conflict-free
// ds_read_b128 A fragments), V rows chunk ^ ((key & 3) << 2) (conflict-free ds_read_b64_tr_b16).
constexpr int WD_D = 512;
constexpr int WD_KT = 32;                      // keys per tile
constexpr int WD_CH = WD_D / 8;                // 16-B chunks per row

__global__ __launch_bounds__(256, 1) void attn_fwd_wide_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int H, int Sq, int Sk, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
    long long ksh, long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float c, int nqb) {
  __shared__ __attribute__((aligned(16))) u16 Ks[WD_KT * WD_D];
  __shared__ __attribute__((aligned(16))) u16 Vs[WD_KT * WD_D];
  __shared__ __attribute__((aligned(16))) float Sx[4][64][16];

  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qb = logical % nqb;
  const int bh = logical / nqb;
  const int b = bh / H, h = bh % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l32 = lane & 31, hf = lane >> 5, i16 = lane & 15;
  const int d0 = wave * 128;

  const u16* qbase = qp + b * qsb + h * qsh;
  const u16* kbase = kp + b * ksb + h * ksh;
  const u16* vbase = vp + b * vsb + h * vsh;
  u16* obase = op + b * osb + h * osh;

  const int q_row = qb * 32 + l32;
  const bool q_ok = q_row < Sq;
  bf16x8 qf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    s16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
    if (q_ok) t = *reinterpret_cast<const s16x8*>(qbase + (long long)q_row * qss + d0 + ks * 16 + 8 * hf);
    qf[ks] = __builtin_bit_cast(bf16x8, t);
  }

  const int ntiles = (Sk + WD_KT - 1) / WD_KT;
  s16x8 kr[8], vr[8];
  auto gload = [&](int t) {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int idx = it * 256 + tid;
      const int key = idx >> 6, ch = idx & 63;
      const int gk = t * WD_KT + key;
      s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
      kr[it] = gk < Sk ? *reinterpret_cast<const s16x8*>(kbase + (long long)gk * kss + ch * 8) : z;
      vr[it] = gk < Sk ? *reinterpret_cast<const s16x8*>(vbase + (long long)gk * vss + ch * 8) : z;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int idx = it * 256 + tid;
      const int key = idx >> 6, ch = idx & 63;
      *reinterpret_cast<s16x8*>(&Ks[key * WD_D + 8 * (ch ^ (key & 15))]) = kr[it];
      *reinterpret_cast<s16x8*>(&Vs[key * WD_D + 8 * (ch ^ ((key & 3) << 2))]) = vr[it];
    }
  };

  f32x16 ot[4] = {f32x16{}, f32x16{}, f32x16{}, f32x16{}};
  float m_run = -INFINITY, l_run = 0.f;
  gload(0);
  lstore();
  __syncthreads();
  for (int t = 0; t < ntiles; ++t) {
    if (t + 1 < ntiles) gload(t + 1);
    // partial S^T over this wave's 128-d slice
    f32x16 sp = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int ch = 16 * wave + 2 * ks + hf;
      s16x8 a = *reinterpret_cast<const s16x8*>(&Ks[l32 * WD_D + 8 * (ch ^ (l32 & 15))]);
      sp = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), qf[ks], sp, 0, 0, 0);
    }
#pragma unroll
    for (int r4 = 0; r4 < 4; ++r4)
      *reinterpret_cast<float4_t*>(&Sx[wave][lane][4 * r4]) = float4_t{sp[4 * r4], sp[4 * r4 + 1], sp[4 * r4 + 2],
                                                                      sp[4 * r4 + 3]};
    __syncthreads();
    f32x16 s = f32x16{};
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        float4_t v = *reinterpret_cast<const float4_t*>(&Sx[w][lane][4 * r4]);
        s[4 * r4] += v[0]; s[4 * r4 + 1] += v[1]; s[4 * r4 + 2] += v[2]; s[4 * r4 + 3] += v[3];
      }
    // online softmax (identical in the 4 waves)
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = t * WD_KT + (r & 3) + 8 * (r >> 2) + 4 * hf;
      s[r] = key < Sk ? s[r] : -INFINITY;
      mx = fmaxf(mx, s[r]);
    }
    mx = af_xmax(mx) * c;
    const float m_new = fmaxf(m_run, mx);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
    m_run = m_new;
    float ps = 0.f;
    bf16x8 pf[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], c, -m_use));
      ps += p;
      pf[r >> 3][r & 7] = (__bf16)p;
    }
    l_run = l_run * alpha + ps;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) ot[dt][r] *= alpha;
    // O^T[d slice] += V^T P^T
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int row0 = 16 * st + 4 * hf + (i16 >> 2);
      const int r1 = row0 + 8;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int col = d0 + dt * 32 + 16 * ((lane >> 4) & 1) + 4 * (i16 & 3);
        const int ch = col >> 3, half = (col >> 2) & 1;
        const int o0 = row0 * WD_D + 8 * (ch ^ ((row0 & 3) << 2)) + 4 * half;
        const int o1 = r1 * WD_D + 8 * (ch ^ ((r1 & 3) << 2)) + 4 * half;
        bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vs + o0));
        bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vs + o1));
        bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        ot[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[st], ot[dt], 0, 0, 0);
      }
    }
    __syncthreads();   // every wave is done with Ks / Vs / Sx of tile t
    if (t + 1 < ntiles) {
      lstore();
      __syncthreads();
    }
  }
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (q_ok) {
    u16* orow = obase + (long long)q_row * oss + d0;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        s16x4 w;
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (short)f2bf(ot[dt][4 * r4 + j] * inv);
        *reinterpret_cast<s16x4*>(orow + dt * 32 + 8 * r4 + 4 * hf) = w;
      }
  }
}

// ------------------------------------------------------------------------------------------------
// Wide-head path, materialised form (K22 v2). At one head of D = 512 the flash kernel above is
// bound by its K/V re-reads (32 queries per workgroup: 64 KB of K/V per 2 MFLOP), while the score
// matrix of one image (16 k x 16 k fp32 = 1 GiB) is small next to 288 GB of HBM. So the op layer
// runs, per image and query chunk: S = (scale log2e) Q K^T on the v7 GEMM with an fp32 epilogue
// (MC_EPI_F32OUT), P = softmax2(S) -> bf16 (below, one pass over S), O = P (V^T)^T on the v7 GEMM
// (split-K tail) with V^T from the transpose below. Two big MFMA GEMMs + two streaming passes.

// P[r, :] = 2^(S[r, :] - max) / sum, S already in log2 units. One workgroup per row, the row held
// in registers (NV float4 per thread: cols <= 1024 NV), cols % 4 == 0.
template <int NV>
__global__ __launch_bounds__(256) void softmax2_f32_bf16_kernel(const float* __restrict__ x, u16* __restrict__ y,
                                                                int cols, long long ldx, long long ldy) {
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* xr = x + (long long)blockIdx.x * ldx;
  u16* yr = y + (long long)blockIdx.x * ldy;
  float4 v[NV];
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 256 + tid) * 4;
    v[i] = c < cols ? *reinterpret_cast<const float4*>(xr + c) : float4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    mx = fmaxf(mx, fmaxf(fmaxf(v[i].x, v[i].y), fmaxf(v[i].z, v[i].w)));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i].x = __builtin_amdgcn_exp2f(v[i].x - mx);
    v[i].y = __builtin_amdgcn_exp2f(v[i].y - mx);
    v[i].z = __builtin_amdgcn_exp2f(v[i].z - mx);
    v[i].w = __builtin_amdgcn_exp2f(v[i].w - mx);
    s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) red[4 + wave] = s;
  __syncthreads();
  const float inv = 1.f / ((red[4] + red[5]) + (red[6] + red[7]));
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 256 + tid) * 4;
    if (c < cols) {
      uint2 w;
      w.x = (uint32_t)f2bf(v[i].x * inv) | ((uint32_t)f2bf(v[i].y * inv) << 16);
      w.y = (uint32_t)f2bf(v[i].z * inv) | ((uint32_t)f2bf(v[i].w * inv) << 16);
      *reinterpret_cast<uint2*>(yr + c) = w;
    }
  }
}

CGS_EXPORT int cgs_softmax2_f32_bf16(const float* x, void* y, long long rows, int cols, long long ldx, long long ldy,
                                     hipStream_t stream) {
  if (rows <= 0) return 0;
  if (cols <= 0 || cols % 4 || ldx % 4 || ldy % 4 || rows > 0x7fffffffLL || cols > 16384 ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(y) & 7))
    return (int)hipErrorInvalidValue;
  const unsigned g = (unsigned)rows;
  u16* yy = (u16*)y;
  if (cols <= 1024) softmax2_f32_bf16_kernel<1><<<g, 256, 0, stream>>>(x, yy, cols, ldx, ldy);
  else if (cols <= 2048) softmax2_f32_bf16_kernel<2><<<g, 256, 0, stream>>>(x, yy, cols, ldx, ldy);
  else if (cols <= 4096) softmax2_f32_bf16_kernel<4><<<g, 256, 0, stream>>>(x, yy, cols, ldx, ldy);
  else if (cols <= 8192) softmax2_f32_bf16_kernel<8><<<g, 256, 0, stream>>>(x, yy, cols, ldx, ldy);
  else softmax2_f32_bf16_kernel<16><<<g, 256, 0, stream>>>(x, yy, cols, ldx, ldy);
  return (int)hipGetLastError();
}

// y[c, r] = x[r, c] for a bf16 [rows, cols] matrix (row stride ldx) -> [cols, rows] (row stride ldy):
// 64 x 64 tiles through LDS, 16-B global loads and stores. rows, cols % 8 == 0.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const u16* __restrict__ x, u16* __restrict__ y, int rows,
                                                             int cols, long long ldx, long long ldy) {
  __shared__ u16 t[64][64 + 2];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tid = threadIdx.x, ch = tid & 7, rr = tid >> 3;   // 8 chunks of 8 elements x 32 rows
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int r = rr + 32 * it, gr = r0 + r, gc = c0 + 8 * ch;
    s16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (gr < rows && gc < cols) v = *reinterpret_cast<const s16x8*>(x + (long long)gr * ldx + gc);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[r][8 * ch + j] = (u16)v[j];
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = rr + 32 * it, gc = c0 + c, gr = r0 + 8 * ch;
    if (gc < cols && gr < rows) {
      s16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)t[8 * ch + j][c];
      *reinterpret_cast<s16x8*>(y + (long long)gc * ldy + gr) = v;
    }
  }
}

CGS_EXPORT int cgs_transpose_bf16(const void* x, void* y, int rows, int cols, long long ldx, long long ldy,
                                  hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return 0;
  if (rows % 8 || cols % 8 || ldx % 8 || ldy % 8 || ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15))
    return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  transpose_bf16_kernel<<<g, 256, 0, stream>>>((const u16*)x, (u16*)y, rows, cols, ldx, ldy);
  return (int)hipGetLastError();
}

static int g_attn_variant = 0;   // 0 auto, 1 generic kernel, 2 D=64 fast kernel (256-row Q blocks), 3 short-KV
                                 // kernel, 4 D=64 r2, 5 D=64 fast kernel with 128-row Q blocks
static int num_cus_attn() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t p;
    n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount : 256;
  }
  return n;
}
CGS_EXPORT void cgs_attn_set_variant(int v) { g_attn_variant = v; }
// s_setprio(1) around the P.V MFMAs of the D = 64 kernel (default on: +1.5 / +2.2 % at SDXL levels 1 / 2,
// profiles/r03/attn_setprio_pv.log); cgs_attn_set_prio(0) selects the 8-wave form without it (A/B)
static bool g_attn_prio = true;
CGS_EXPORT void cgs_attn_set_prio(int on) { g_attn_prio = on != 0; }

static int flash_attn_impl(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk, int D,
                           long long qsb, long long qss, long long qsh, long long ksb, long long kss, long long ksh,
                           long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
                           float scale, const void* key_mask, int causal, float* lse, hipStream_t stream) {
  if (D % 8) return (int)hipErrorInvalidValue;
  int nqb = (Sq + ATT_QB - 1) / ATT_QB;
  long long nwg = (long long)nqb * B * H;
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  float sl2 = scale * 1.4426950408889634f;
  const bool al16 = ((qss | kss | vss | oss | qsb | ksb | vsb | osb | qsh | ksh | vsh | osh) & 7) == 0 &&
                    ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) |
                      reinterpret_cast<uintptr_t>(v) | reinterpret_cast<uintptr_t>(o)) & 15) == 0;
  if (D == 64 && !key_mask && !causal && al16 && Sk > 0 && Sk <= 128 && !lse &&
      (g_attn_variant == 0 || g_attn_variant == 3)) {
    // QI 32-query blocks per wave (K / V staged once per 128 * QI queries): measured +4.5 % at SDXL level 1
    // (Sq = 4096), -2.6 % at level 2 (profiles/r04/shortkv_qi_ab_r04al.log) -> QI = 4 for Sq >= 2048 while
    // that leaves >= 2 workgroups per CU; CGS_SKV_QI=1|2|4 overrides (A/B)
    const long long blocks128 = (long long)((Sq + 127) / 128) * B * H;
    static const int qi_env = getenv("CGS_SKV_QI") ? atoi(getenv("CGS_SKV_QI")) : 0;
    int qi = 1;
    if (qi_env == 1 || qi_env == 2 || qi_env == 4) qi = qi_env;
    else if (Sq >= 2048 && blocks128 / 4 >= 2 * num_cus_attn()) qi = 4;
    const int nqb3 = (Sq + 128 * qi - 1) / (128 * qi);
    const long long nwg3 = (long long)nqb3 * B * H;
    if (nwg3 > 0x7fffffff) return (int)hipErrorInvalidValue;
#define SKV_GO(NKT, QIV)                                                                                             \
  do {                                                                                                              \
    if (g_attn_prio)                                                                                                \
      attn_fwd_d64_shortkv_kernel<NKT, true, QIV><<<dim3((unsigned)nwg3), 256, 0, stream>>>(                        \
          (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss,   \
          vsh, osb, oss, osh, sl2, nqb3);                                                                           \
    else                                                                                                            \
      attn_fwd_d64_shortkv_kernel<NKT, false, QIV><<<dim3((unsigned)nwg3), 256, 0, stream>>>(                       \
          (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss,   \
          vsh, osb, oss, osh, sl2, nqb3);                                                                           \
  } while (0)
#define SKV_LAUNCH(NKT)                                                                                              \
  do {                                                                                                              \
    if (qi == 4) SKV_GO(NKT, 4);                                                                                    \
    else if (qi == 2) SKV_GO(NKT, 2);                                                                               \
    else SKV_GO(NKT, 1);                                                                                            \
  } while (0)
    if (Sk <= 32) SKV_LAUNCH(1);
    else if (Sk <= 64) SKV_LAUNCH(2);
    else if (Sk <= 96) SKV_LAUNCH(3);
    else SKV_LAUNCH(4);
#undef SKV_GO
#undef SKV_LAUNCH
    return (int)hipGetLastError();
  }
  if (g_attn_variant == 3) return (int)hipErrorInvalidValue;
  if (D == WD_D) {
    if (key_mask || causal || !al16 || Sk <= 0 || lse) return (int)hipErrorInvalidValue;
    const int nqb4 = (Sq + 31) / 32;
    const long long nwg4 = (long long)nqb4 * B * H;
    if (nwg4 > 0x7fffffff) return (int)hipErrorInvalidValue;
    attn_fwd_wide_kernel<<<dim3((unsigned)nwg4), 256, 0, stream>>>(
        (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh,
        osb, oss, osh, sl2, nqb4);
    return (int)hipGetLastError();
  }
  if (D == 64 && !key_mask && !causal && al16 && g_attn_variant != 1 && Sk > 0) {
    // 256-row Q blocks (8 waves) unless that leaves the grid under one round of the CUs and the
    // 128-row form (4 waves, two WGs per CU) is asked for (variant 5) or auto-picked (variant 0)
    const long long nwg256 = (long long)((Sq + 255) / 256) * B * H;
    const bool small = g_attn_variant == 5 || (g_attn_variant == 0 && nwg256 < num_cus_attn());
    const int rows = small ? 128 : 256;
    int nqb2 = (Sq + rows - 1) / rows;
    long long nwg2 = (long long)nqb2 * B * H;
    if (nwg2 > 0x7fffffff) return (int)hipErrorInvalidValue;
    if (small)
      attn_fwd_d64_kernel<4><<<dim3((unsigned)nwg2), 256, 0, stream>>>(
          (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh,
          osb, oss, osh, sl2, nqb2, lse);
    else if (!g_attn_prio)
      attn_fwd_d64_kernel<8, false, false><<<dim3((unsigned)nwg2), 512, 0, stream>>>(
          (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh,
          osb, oss, osh, sl2, nqb2, lse);
    else
      attn_fwd_d64_kernel<8><<<dim3((unsigned)nwg2), 512, 0, stream>>>(
          (const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, H, Sq, Sk, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh,
          osb, oss, osh, sl2, nqb2, lse);
    return (int)hipGetLastError();
  }
  if (g_attn_variant == 2) return (int)hipErrorInvalidValue;
  dim3 grid((unsigned)nwg);
#define ATT_LAUNCH(DPV)                                                                                         \
  flash_fwd_kernel<DPV><<<grid, 256, 0, stream>>>((const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, B, H, Sq, \
                                                   Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss,  \
                                                   osh, sl2, (const signed char*)key_mask, causal, nqb, lse)
  if (D <= 32) ATT_LAUNCH(32);
  else if (D <= 64) ATT_LAUNCH(64);
  else if (D <= 96) ATT_LAUNCH(96);
  else if (D <= 128) ATT_LAUNCH(128);
  else if (D <= 160) ATT_LAUNCH(160);
  else return (int)hipErrorInvalidValue;
#undef ATT_LAUNCH
  return (int)hipGetLastError();
}

// Per-call kernel choice for the op-layer autotuner (variant as in cgs_attn_set_variant; the process
// setting is restored before returning).
CGS_EXPORT int cgs_flash_attn_fwd_v(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                    int D, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
                                    long long ksh, long long vsb, long long vss, long long vsh, long long osb,
                                    long long oss, long long osh, float scale, int variant, hipStream_t stream) {
  const int saved = g_attn_variant;
  g_attn_variant = variant;
  const int rc = flash_attn_impl(q, k, v, o, B, H, Sq, Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss, osh,
                                 scale, nullptr, 0, nullptr, stream);
  g_attn_variant = saved;
  return rc;
}

// Merge of the KS key-split partials: O = sum_s exp(lse_s - L) O_s with L = log sum_s exp(lse_s) (every
// partial is already normalised by its own row sum). One thread per 8 channels of one (b, q, h) row.
template <int KS>
__global__ __launch_bounds__(256) void attn_ks_combine_kernel(const u16* __restrict__ part, const float* __restrict__ lse,
                                                              u16* __restrict__ o, int B, int H, int Sq,
                                                              long long ospl, long long osb, long long oss,
                                                              long long osh) {
  const long long total = (long long)B * Sq * H * 8;
  const long long lspl = (long long)B * H * Sq;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c8 = (int)(i & 7);
    const long long r = i >> 3;                  // (b, q, h) row, h fastest
    const int h = (int)(r % H);
    const long long bq = r / H;
    const int q = (int)(bq % Sq);
    const int b = (int)(bq / Sq);
    float l[KS], mx = -INFINITY;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      l[s] = lse[s * lspl + ((long long)b * H + h) * Sq + q];
      mx = fmaxf(mx, l[s]);
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, wsum = 0.f;
    const long long po = ((long long)b * Sq + q) * H * 64 + h * 64 + c8 * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float w = mx == -INFINITY ? 0.f : __expf(l[s] - mx);
      wsum += w;
      const s16x8 v = *reinterpret_cast<const s16x8*>(part + s * ospl + po);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_fmaf(w, cvt_in<CGS_BF16>((u16)v[j]), acc[j]);
    }
    const float inv = wsum > 0.f ? 1.f / wsum : 0.f;
    s16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = (short)cvt_out<CGS_BF16>(acc[j] * inv);
    *reinterpret_cast<s16x8*>(o + (long long)b * osb + (long long)q * oss + (long long)h * osh + c8 * 8) = out;
  }
}

// D = 64 self-attention with the keys split KS ways (2 or 4) for under-filled grids (batch-1 SDXL: 160-320
// workgroups of 256 query rows on 256 CUs): KS x the workgroups, then one merge pass. ws_o: KS * B * Sq * H * 64
// bf16, ws_lse: KS * B * H * Sq floats. 256-row Q blocks (8 waves).
CGS_EXPORT int cgs_flash_attn_fwd_ks(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                     long long qsb, long long qss, long long ksb, long long kss, long long vsb,
                                     long long vss, long long osb, long long oss, float scale, int KS, void* ws_o,
                                     void* ws_lse, hipStream_t stream) {
  if ((KS != 2 && KS != 4) || B <= 0 || H <= 0 || Sq <= 0 || Sk <= 0 || !ws_o || !ws_lse) return (int)hipErrorInvalidValue;
  const bool al16 = ((qss | qsb | kss | ksb | vss | vsb | oss | osb) & 7) == 0 &&
                    ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k) | reinterpret_cast<uintptr_t>(v) |
                      reinterpret_cast<uintptr_t>(o) | reinterpret_cast<uintptr_t>(ws_o)) & 15) == 0;
  const int tiles = (Sk + 63) / 64;
  const int tps = (tiles + KS - 1) / KS;
  if (!al16 || (long long)(KS - 1) * tps * 64 >= Sk) return (int)hipErrorInvalidValue;   // every split has keys
  const int nqb = (Sq + 255) / 256;
  const long long nwg = (long long)nqb * B * H * KS;
  const long long ospl = (long long)B * Sq * H * 64;
  if (nwg > 0x7fffffff || ospl * KS > 0x7fffffffffffll) return (int)hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const long long wsb = (long long)Sq * H * 64, wss = (long long)H * 64;
#define CGS_KS_GO(KV)                                                                                              \
  attn_fwd_d64_kernel<8, false, true, KV><<<dim3((unsigned)nwg), 512, 0, stream>>>(                                \
      (const u16*)q, (const u16*)k, (const u16*)v, (u16*)ws_o, H, Sq, Sk, qsb, qss, 64, ksb, kss, 64, vsb, vss, 64,   \
      wsb, wss, 64, sl2, nqb, (float*)ws_lse, KV2{nullptr, nullptr, 0, 0, 0, 0, 0}, ospl)
  if (KS == 2) CGS_KS_GO(2); else CGS_KS_GO(4);
#undef CGS_KS_GO
  const long long thr = (long long)B * Sq * H * 8;
  long long nb = (thr + 255) / 256;
  const int blocks = (int)(nb > 16384 ? 16384 : nb);
  if (KS == 2)
    attn_ks_combine_kernel<2><<<blocks, 256, 0, stream>>>((const u16*)ws_o, (const float*)ws_lse, (u16*)o, B, H, Sq,
                                                          ospl, osb, oss, 64);
  else
    attn_ks_combine_kernel<4><<<blocks, 256, 0, stream>>>((const u16*)ws_o, (const float*)ws_lse, (u16*)o, B, H, Sq,
                                                          ospl, osb, oss, 64);
  return (int)hipGetLastError();
}

static int g_kv2_rows = 0;   // Q rows per workgroup of the two-source kernel: 0 auto, 128, 256 (A/B switch)
CGS_EXPORT void cgs_attn_set_kv2_rows(int r) { g_kv2_rows = r == 128 || r == 256 ? r : 0; }

// D = 64 attention over the key concat of two K / V sources (see KV2): keys [0, Sk1) from k1 / v1 ([B, Sk1]
// rows), keys [Sk1, Sk1 + Sk2) from k2 / v2. Head stride D in every source; no mask.
CGS_EXPORT int cgs_flash_attn_fwd_kv2(const void* q, const void* k1, const void* v1, const void* k2, const void* v2,
                                      void* o, int B, int H, int Sq, int Sk1, int Sk2, long long qsb, long long qss,
                                      long long k1sb, long long k1ss, long long v1sb, long long v1ss, long long k2sb,
                                      long long k2ss, long long v2sb, long long v2ss, long long osb, long long oss,
                                      float scale, hipStream_t stream) {
  const int Sk = Sk1 + Sk2;
  const bool al16 = ((qss | qsb | k1sb | k1ss | v1sb | v1ss | k2sb | k2ss | v2sb | v2ss | osb | oss) & 7) == 0 &&
                    ((reinterpret_cast<uintptr_t>(q) | reinterpret_cast<uintptr_t>(k1) | reinterpret_cast<uintptr_t>(v1) |
                      reinterpret_cast<uintptr_t>(k2) | reinterpret_cast<uintptr_t>(v2) | reinterpret_cast<uintptr_t>(o)) &
                     15) == 0;
  if (!al16 || Sk1 <= 0 || Sk2 <= 0 || Sq <= 0 || B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const long long nwg256 = (long long)((Sq + 255) / 256) * B * H;
  // 128-row blocks only for tiny grids: at Cascade batch 1 (B x H = 64 / 40, 576 / 1024 queries: 192 / 160
  // workgroups of 256 rows) the 256-row form measured 13-16 % faster than the 128-row one it used to pick
  // below one round of CUs (profiles/r05/attn_kv2_rows.md)
  const bool small = g_kv2_rows == 128 || (g_kv2_rows == 0 && nwg256 * 4 < num_cus_attn());
  const int rows = small ? 128 : 256;
  const int nqb2 = (Sq + rows - 1) / rows;
  const long long nwg2 = (long long)nqb2 * B * H;
  if (nwg2 > 0x7fffffff) return (int)hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const KV2 kv2{(const u16*)k2, (const u16*)v2, Sk1, k2sb, k2ss, v2sb, v2ss};
  if (small)
    attn_fwd_d64_kernel<4, true><<<dim3((unsigned)nwg2), 256, 0, stream>>>(
        (const u16*)q, (const u16*)k1, (const u16*)v1, (u16*)o, H, Sq, Sk, qsb, qss, 64, k1sb, k1ss, 64, v1sb, v1ss, 64,
        osb, oss, 64, sl2, nqb2, nullptr, kv2);
  else
    attn_fwd_d64_kernel<8, true><<<dim3((unsigned)nwg2), 512, 0, stream>>>(
        (const u16*)q, (const u16*)k1, (const u16*)v1, (u16*)o, H, Sq, Sk, qsb, qss, 64, k1sb, k1ss, 64, v1sb, v1ss, 64,
        osb, oss, 64, sl2, nqb2, nullptr, kv2);
  return (int)hipGetLastError();
}

// Generic flash kernel with additive fp32 score terms (AttnBias): bias [H, Sq, Sk] contiguous, mask
// [nW, Sq, Sk] contiguous or null (batch entry b uses mask b % nW), per-head score multiplier hscale [H] or
// null. D <= 160, D % 8 == 0.
CGS_EXPORT int cgs_flash_attn_fwd_bias(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq,
                                       int Sk, int D, long long qsb, long long qss, long long qsh, long long ksb,
                                       long long kss, long long ksh, long long vsb, long long vss, long long vsh,
                                       long long osb, long long oss, long long osh, float scale, const float* bias,
                                       const float* mask, int nW, const float* hscale, hipStream_t stream) {
  if (D % 8 || D > 160 || !bias || nW <= 0 || B <= 0 || H <= 0 || Sq <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  const int nqb = (Sq + ATT_QB - 1) / ATT_QB;
  const long long nwg = (long long)nqb * B * H;
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  const float sl2 = scale * 1.4426950408889634f;
  const AttnBias ab{bias, mask, hscale, nW};
  dim3 grid((unsigned)nwg);
#define ATTB_LAUNCH(DPV)                                                                                          \
  flash_fwd_kernel<DPV, true><<<grid, 256, 0, stream>>>((const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, B, H, \
                                                        Sq, Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, \
                                                        oss, osh, sl2, nullptr, 0, nqb, nullptr, ab)
  if (D <= 32) ATTB_LAUNCH(32);
  else if (D <= 64) ATTB_LAUNCH(64);
  else if (D <= 96) ATTB_LAUNCH(96);
  else if (D <= 128) ATTB_LAUNCH(128);
  else ATTB_LAUNCH(160);
#undef ATTB_LAUNCH
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                  int D, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
                                  long long ksh, long long vsb, long long vss, long long vsh, long long osb,
                                  long long oss, long long osh, float scale, const void* key_mask, int causal,
                                  hipStream_t stream) {
  return flash_attn_impl(q, k, v, o, B, H, Sq, Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss, osh, scale,
                         key_mask, causal, nullptr, stream);
}

// Same, plus the per-(b, h, query) natural-log LSE of the scaled scores (fp32 [B, H, Sq]) for
// merging partial results over K/V blocks (ring attention, parallel/sp.py). D = 64 or the generic kernel.
CGS_EXPORT int cgs_flash_attn_fwd_lse(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H,
                                      int Sq, int Sk, int D, long long qsb, long long qss, long long qsh, long long ksb,
                                      long long kss, long long ksh, long long vsb, long long vss, long long vsh,
                                      long long osb, long long oss, long long osh, float scale, hipStream_t stream) {
  if (!lse) return (int)hipErrorInvalidValue;
  return flash_attn_impl(q, k, v, o, B, H, Sq, Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss, osh, scale,
                         nullptr, 0, lse, stream);
}
