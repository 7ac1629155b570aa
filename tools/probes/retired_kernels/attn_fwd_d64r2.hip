// Retired from libcgs_kernels.so in round 5 (never auto-dispatched; measured slower than
// attn_fwd_d64_kernel, see the note below). Kept for reference only: it is not built. It relied on
// the helpers of csrc/kernels/attention.hip (K/V staging ring, softmax pieces) at the time of removal.
// ------------------------------------------------------------------------------------------------
// D = 64, two 32-row query blocks per wave ("r2"): 4 waves x 64 rows = 256-row Q block per WG,
// one wave per SIMD with the whole 512-entry register file. Every K fragment read from LDS feeds
// the QK^T MFMAs of BOTH row blocks and every V^T fragment both PV MFMAs, so LDS traffic per FLOP is
// half that of attn_fwd_d64_kernel (there 8 waves x 32 rows each re-read the full K/V tile: LDS
// bandwidth, not MFMA, bounds it at ~32 flop/B). Same K/V images, staging ring and software pipeline
// (QK^T of tile t+1 interleaved with the softmax of tile t inside each wave).
// Measured (kbench, B=16 SDXL shapes): 779 vs 867 TF/s at Sq=Sk=4096 and 546 vs 641 at 1024 — the
// halved LDS traffic does not pay for one wave per SIMD (253 VGPR + 224 AGPR): with no second wave
// to switch to, ds_read / global latency is exposed. Kept as the explicit variant 4, not auto.
__global__ __launch_bounds__(256, 1) void attn_fwd_d64r2_kernel(
    const u16* __restrict__ qp, const u16* __restrict__ kp, const u16* __restrict__ vp, u16* __restrict__ op,
    int H, int Sq, int Sk, long long qsb, long long qss, long long qsh, long long ksb, long long kss,
    long long ksh, long long vsb, long long vss, long long vsh, long long osb, long long oss, long long osh,
    float c, int nqb) {
  __shared__ __attribute__((aligned(16))) u16 Ks[2][64 * 64];
  __shared__ __attribute__((aligned(16))) u16 Vs[2][64 * 64];

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

  int q_row[2];
  bf16x8 qf[2][4];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    q_row[r] = qb * 256 + wave * 64 + r * 32 + l32;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      s16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q_row[r] < Sq) t = *reinterpret_cast<const s16x8*>(qbase + (long long)q_row[r] * qss + ks * 16 + 8 * hf);
      qf[r][ks] = __builtin_bit_cast(bf16x8, t);
    }
  }

  // staging: 256 threads x 2 chunks cover a 64-key x 64-d tile (keys tid>>3 and 32 + tid>>3)
  const int st_c = tid & 7;
  int k_woff[2], v_woff[2], st_key[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    st_key[i] = (tid >> 3) + 32 * i;
    k_woff[i] = st_key[i] * 64 + 8 * (st_c ^ ((st_key[i] >> 1) & 7));
    v_woff[i] = st_key[i] * 64 + 8 * (st_c ^ (((st_key[i] >> 1) & 1) << 2));
  }
  const int n = (Sk + 63) >> 6;
  auto gload = [&](const u16* base, long long ss, int t, int i) -> s16x8 {
    int key = t * 64 + st_key[i];
    key = key < Sk ? key : Sk - 1;   // clamp: tail rows are masked in the softmax
    return *reinterpret_cast<const s16x8*>(base + (long long)key * ss + st_c * 8);
  };
  auto k_roff = [&](int kt, int ks) {
    int key = kt * 32 + l32;
    return key * 64 + 8 * ((2 * ks + hf) ^ ((key >> 1) & 7));
  };
  auto qk = [&](const u16* Kt, f32x16 (&s)[2][2]) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[0][kt] = f32x16{};
      s[1][kt] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const s16x8*>(Kt + k_roff(kt, ks)));
        s[0][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[0][ks], s[0][kt], 0, 0, 0);
        s[1][kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[1][ks], s[1][kt], 0, 0, 0);
      }
    }
  };
  const int i16 = lane & 15;
  f32x16 ot[2][2] = {{f32x16{}, f32x16{}}, {f32x16{}, f32x16{}}};
  bf16x8 pf[2][4];
  auto pv = [&](const u16* Vt) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
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
          bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vt + o0));
          bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(Vt + o1));
          bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          ot[0][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[0][kt * 2 + st], ot[0][dt], 0, 0, 0);
          ot[1][dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[1][kt * 2 + st], ot[1][dt], 0, 0, 0);
        }
      }
  };

  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};
  f32x16 sA[2][2], sB[2][2];
  {
    s16x8 k0a = gload(kbase, kss, 0, 0), k0b = gload(kbase, kss, 0, 1);
    s16x8 k1a = gload(kbase, kss, n > 1 ? 1 : 0, 0), k1b = gload(kbase, kss, n > 1 ? 1 : 0, 1);
    s16x8 v0a = gload(vbase, vss, 0, 0), v0b = gload(vbase, vss, 0, 1);
    *reinterpret_cast<s16x8*>(&Ks[0][k_woff[0]]) = k0a;
    *reinterpret_cast<s16x8*>(&Ks[0][k_woff[1]]) = k0b;
    *reinterpret_cast<s16x8*>(&Ks[1][k_woff[0]]) = k1a;
    *reinterpret_cast<s16x8*>(&Ks[1][k_woff[1]]) = k1b;
    *reinterpret_cast<s16x8*>(&Vs[0][v_woff[0]]) = v0a;
    *reinterpret_cast<s16x8*>(&Vs[0][v_woff[1]]) = v0b;
  }
  __syncthreads();
  qk(Ks[0], sA);

  auto body = [&](int t, f32x16 (&sCur)[2][2], f32x16 (&sNext)[2][2]) {
    const int slot = t & 1;
    const int tk = min(t + 2, n - 1);
    s16x8 kna = gload(kbase, kss, tk, 0), knb = gload(kbase, kss, tk, 1);
    s16x8 vna = gload(vbase, vss, t + 1, 0), vnb = gload(vbase, vss, t + 1, 1);
    qk(Ks[slot ^ 1], sNext);
    af_softmax<false>(sCur[0], pf[0], ot[0], m_run[0], l_run[0], c, t * 64, Sk, hf);
    af_softmax<false>(sCur[1], pf[1], ot[1], m_run[1], l_run[1], c, t * 64, Sk, hf);
    pv(Vs[slot]);
    *reinterpret_cast<s16x8*>(&Ks[slot][k_woff[0]]) = kna;
    *reinterpret_cast<s16x8*>(&Ks[slot][k_woff[1]]) = knb;
    *reinterpret_cast<s16x8*>(&Vs[slot ^ 1][v_woff[0]]) = vna;
    *reinterpret_cast<s16x8*>(&Vs[slot ^ 1][v_woff[1]]) = vnb;
    __syncthreads();
  };
  int t = 0;
  for (; t + 2 < n; t += 2) {
    body(t, sA, sB);
    body(t + 1, sB, sA);
  }
  if (t + 1 < n) {
    body(t, sA, sB);
    ++t;
    af_softmax<true>(sB[0], pf[0], ot[0], m_run[0], l_run[0], c, t * 64, Sk, hf);
    af_softmax<true>(sB[1], pf[1], ot[1], m_run[1], l_run[1], c, t * 64, Sk, hf);
  } else {
    af_softmax<true>(sA[0], pf[0], ot[0], m_run[0], l_run[0], c, t * 64, Sk, hf);
    af_softmax<true>(sA[1], pf[1], ot[1], m_run[1], l_run[1], c, t * 64, Sk, hf);
  }
  pv(Vs[t & 1]);

#pragma unroll
  for (int r = 0; r < 2; ++r) {
    float l_tot = l_run[r] + __shfl_xor(l_run[r], 32, 64);
    float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
    if (q_row[r] < Sq) {
      u16* orow = obase + (long long)q_row[r] * oss;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          s16x4 w;
#pragma unroll
          for (int j = 0; j < 4; ++j) w[j] = (short)f2bf(ot[r][dt][4 * r4 + j] * inv);
          *reinterpret_cast<s16x4*>(orow + dt * 32 + 8 * r4 + 4 * hf) = w;
        }
    }
  }
}

