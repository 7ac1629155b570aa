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

template <int DP>
__global__ __launch_bounds__(256, (DP >= 160 ? 1 : 2)) void flash_fwd_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int B, int H, int Sq, int Sk, int D,
    long long qsb, long long qss, long long qsh, long long ksb, long long kss, long long ksh,
    long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float scale_log2, const signed char* __restrict__ key_mask, int causal, int nqb) {
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

CGS_EXPORT int cgs_flash_attn_fwd(const void* q, const void* k, const void* v, void* o, int B, int H, int Sq, int Sk,
                                  int D, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
                                  long long ksh, long long vsb, long long vss, long long vsh, long long osb,
                                  long long oss, long long osh, float scale, const void* key_mask, int causal,
                                  hipStream_t stream) {
  if (D % 8) return (int)hipErrorInvalidValue;
  int nqb = (Sq + ATT_QB - 1) / ATT_QB;
  long long nwg = (long long)nqb * B * H;
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  float sl2 = scale * 1.4426950408889634f;
  dim3 grid((unsigned)nwg);
#define ATT_LAUNCH(DPV)                                                                                         \
  flash_fwd_kernel<DPV><<<grid, 256, 0, stream>>>((const u16*)q, (const u16*)k, (const u16*)v, (u16*)o, B, H, Sq, \
                                                   Sk, D, qsb, qss, qsh, ksb, kss, ksh, vsb, vss, vsh, osb, oss,  \
                                                   osh, sl2, (const signed char*)key_mask, causal, nqb)
  if (D <= 32) ATT_LAUNCH(32);
  else if (D <= 64) ATT_LAUNCH(64);
  else if (D <= 96) ATT_LAUNCH(96);
  else if (D <= 128) ATT_LAUNCH(128);
  else if (D <= 160) ATT_LAUNCH(160);
  else return (int)hipErrorInvalidValue;
#undef ATT_LAUNCH
  return (int)hipGetLastError();
}
