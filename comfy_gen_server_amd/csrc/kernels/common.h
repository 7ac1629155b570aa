// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of comfy_gen_server_amd.
// Wave = 64 lanes. bf16 is handled as raw ushort with explicit RNE conversion so the kernels
// never depend on host-side bf16 types.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#define CGS_EXPORT extern "C" __attribute__((visibility("default")))

typedef unsigned short bf16_t;
typedef uint16_t u16;
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

enum CgsDType { CGS_F32 = 0, CGS_BF16 = 1, CGS_F16 = 2 };

__device__ __forceinline__ float bf2f(u16 v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// fp32 -> bf16, round-to-nearest-even, NaN kept NaN: the gfx950 conversion instruction (v_cvt_pk_bf16_f32),
// one VALU op and no branch (the integer RNE sequence with its inf / NaN branch was ~8 ops + an exec-mask
// branch per element: most of the VALU of the elementwise kernels)
__device__ __forceinline__ u16 f2bf(float f) {
  return __builtin_bit_cast(u16, (__bf16)f);
}

__device__ __forceinline__ float h2f(u16 v) {
  return __half2float(__ushort_as_half(v));
}

__device__ __forceinline__ u16 f2h(float f) {
  return __half_as_ushort(__float2half(f));
}

template <int DT>
__device__ __forceinline__ float ld_act(const u16* p) {
  if constexpr (DT == CGS_BF16) return bf2f(*p);
  else return h2f(*p);
}

template <int DT>
__device__ __forceinline__ float cvt_in(u16 v) {
  if constexpr (DT == CGS_BF16) return bf2f(v);
  else return h2f(v);
}

template <int DT>
__device__ __forceinline__ u16 cvt_out(float f) {
  if constexpr (DT == CGS_BF16) return f2bf(f);
  else return f2h(f);
}

// 4 floats -> 4 bf16 (hardware v_cvt_pk_bf16_f32: round-to-nearest-even, NaN kept) as one 8-B word
__device__ __forceinline__ uint2 pack4_bf16(float a, float b, float c, float d) {
  bf16x4 v = {(__bf16)a, (__bf16)b, (__bf16)c, (__bf16)d};
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ float4 unpack4_bf16(uint2 w) {
  return float4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                __uint_as_float(w.y & 0xffff0000u)};
}

// x * sigmoid(x) with the hardware reciprocal (v_rcp_f32, 1 ulp) instead of an IEEE division (~10 VALU ops:
// div_scale x2, rcp, fma chain, div_fmas, div_fixup): far below the bf16 / fp16 output ulp
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

__device__ __forceinline__ float gelu_f(float x) {  // exact erf GELU (torch default)
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

// erf-GELU with Abramowitz-Stegun 7.1.26 for erf (|err| <= 1.5e-7, far below the bf16 output ulp):
// ~15 VALU ops and few live temporaries, for register-tight GEMM epilogues.
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __frcp_rn(1.0f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erf_abs = 1.0f - poly * __expf(-z * z);
  const float erf_v = x < 0.0f ? -erf_abs : erf_abs;
  return 0.5f * x * (1.0f + erf_v);
}

// Two GELUs at once: the same A&S 7.1.26 erf as gelu_fast, written on float2 so the polynomial,
// the scalings and the final product issue as packed fp32 ops (v_pk_fma_f32 / v_pk_mul_f32: two
// lanes' worth of work per instruction); only rcp and exp stay per element. Used by the GEGLU GEMM
// epilogue, where the gate math is a visible fraction of a short-K tile.
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t gelu_fast2(f32x2_t x) {
  const f32x2_t z = f32x2_t{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const f32x2_t d = z * 0.3275911f + 1.0f;
  const f32x2_t t = f32x2_t{__frcp_rn(d.x), __frcp_rn(d.y)};
  f32x2_t poly = t * 1.061405429f + (-1.453152027f);
  poly = poly * t + 1.421413741f;
  poly = poly * t + (-0.284496736f);
  poly = poly * t + 0.254829592f;
  poly = poly * t;
  const f32x2_t zz = z * z;
  const f32x2_t e = f32x2_t{__expf(-zz.x), __expf(-zz.y)};
  const f32x2_t erf_abs = 1.0f - poly * e;
  const f32x2_t erf_v = f32x2_t{__builtin_copysignf(erf_abs.x, x.x), __builtin_copysignf(erf_abs.y, x.y)};
  return (x * 0.5f) * (erf_v + 1.0f);
}

// GELU as x * sigmoid(p(x)) with p an odd quintic fitted minimax to the erf GELU on [-9, 9]
// (x clamped to [-8, 8] inside p, where p is monotone): |GELU - exact| <= 2.6e-5 absolute over all
// of fp32 -- far below the bf16 output ulp -- at one v_exp_f32 + one v_rcp_f32 + 6 plain VALU ops
// per element (the A&S form above costs 2 transcendentals + ~13 ops). C* = -coefficient * log2(e).
constexpr float kGeluC0 = -2.301121339e+00f, kGeluC1 = -1.067757240e-01f, kGeluC2 = 1.014263055e-03f;
__device__ __forceinline__ float gelu_sig(float x) {
  const float xc = __builtin_amdgcn_fmed3f(x, -8.0f, 8.0f);
  const float x2 = xc * xc;
  const float q = __builtin_fmaf(x2, __builtin_fmaf(x2, kGeluC2, kGeluC1), kGeluC0);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(xc * q));
}
__device__ __forceinline__ f32x2_t gelu_sig2(f32x2_t x) {
  const f32x2_t xc = f32x2_t{__builtin_amdgcn_fmed3f(x.x, -8.0f, 8.0f), __builtin_amdgcn_fmed3f(x.y, -8.0f, 8.0f)};
  const f32x2_t x2 = xc * xc;
  const f32x2_t q = (x2 * kGeluC2 + kGeluC1) * x2 + kGeluC0;
  const f32x2_t t = xc * q;
  const f32x2_t d = f32x2_t{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + 1.0f;
  return x * f32x2_t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Sum over the 16 lanes of a DPP row (lane bits 0-3), the total in every lane of the row: two
// quad_perm swaps, then row_half_mirror / row_mirror pair the 4- and 8-lane partial sums.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective block remap (MI355X: 8 XCDs with private L2; blocks are dealt round-robin).
// Consecutive logical tiles land on the same XCD so they share L2 panels.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  int q = nwg / nx, r = nwg % nx;
  int x = bid % nx, i = bid / nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Grouped tile order on top of xcd_remap: logical tile index -> (tm, tn), walking `gm_max` tile
// rows at a time, so the ~32 tiles an XCD runs together form a gm x (32/gm) block that shares A
// row-panels and B col-panels in that XCD's L2 instead of streaming 32 distinct B panels.
__device__ __forceinline__ void grouped_tile(int logical, int tiles_m, int tiles_n, int gm_max, int& tm, int& tn) {
  if (gm_max <= 1) {
    tm = logical / tiles_n;
    tn = logical % tiles_n;
    return;
  }
  const int group = gm_max * tiles_n;
  const int gid = logical / group;
  const int first = gid * gm_max;
  const int gm = (tiles_m - first) < gm_max ? (tiles_m - first) : gm_max;
  const int in = logical - gid * group;
  tm = first + in % gm;
  tn = in / gm;
}
