// Counter-based device RNG for the sampling loop (SURVEY §2.4 K18, §2.3 "torchsde -> device Brownian").
//
// Every random number is a pure function of (seed, GLOBAL image index, stream, element index):
//   key     = image_key(seed, index)                    (splitmix64 mix, one Philox key per image)
//   counter = (element_group lo, hi, stream lo, stream hi)
//   Philox4x32-10 -> 4 uint32 -> 2 Box-Muller pairs -> 4 N(0,1) floats for elements 4g..4g+3.
// So noise never depends on how a batch is split over data-parallel ranks (a DP run equals the
// one-GPU run of the whole batch), on the device, or on launch geometry. `stream` is the sampler
// step for ancestral/SDE noise; Brownian-tree nodes use a disjoint stream domain (bit 63 set).
//
// The same math is mirrored bit-for-bit in sampling/rng.py (torch int64 ops) for the CPU path
// and as the numerics oracle. Reference behaviour being replaced: torch.randn_like per step
// (comfy/k_diffusion/sampling.py:60-61) and torchsde.BrownianTree on the CPU (:64-123).
#include "common.h"

namespace {

constexpr uint32_t PH_M0 = 0xD2511F53u, PH_M1 = 0xCD9E8D57u;
constexpr uint32_t PH_W0 = 0x9E3779B9u, PH_W1 = 0xBB67AE85u;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t image_key(uint64_t seed, uint64_t index) {
  return mix64(mix64(seed) ^ (index * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull));
}

__device__ __forceinline__ void philox10(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                                         uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(PH_M0, c0), lo0 = PH_M0 * c0;
    const uint32_t hi1 = __umulhi(PH_M1, c2), lo1 = PH_M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += PH_W0; k1 += PH_W1;
  }
}

// 24-bit uniform strictly inside (0, 1): exact in fp32, identical on host and device.
__device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// 4 normals for element group g of the image with key `key` on `stream`.
__device__ __forceinline__ float4 normal4(uint64_t key, uint64_t g, uint64_t stream) {
  uint32_t c0 = (uint32_t)g, c1 = (uint32_t)(g >> 32), c2 = (uint32_t)stream, c3 = (uint32_t)(stream >> 32);
  philox10(c0, c1, c2, c3, (uint32_t)key, (uint32_t)(key >> 32));
  const float r0 = sqrtf(-2.0f * logf(u01(c0))), t0 = 6.2831853f * u01(c1);
  const float r1 = sqrtf(-2.0f * logf(u01(c2))), t1 = 6.2831853f * u01(c3);
  return float4{r0 * cosf(t0), r0 * sinf(t0), r1 * cosf(t1), r1 * sinf(t1)};
}

__device__ __forceinline__ float f4_get(const float4& v, int j) {
  return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w;
}

inline int rng_blocks(long long work) {
  long long b = (work + 255) / 256;
  return (int)(b < 16384 ? (b < 1 ? 1 : b) : 16384);
}

// ------------------------------------------------------------------ N(0,1) fill, [B, n] fp32 / bf16
template <bool BF16>
__global__ void philox_randn_kernel(void* __restrict__ out, int B, long long n, uint64_t seed, long long index0,
                                    uint64_t stream, const long long* __restrict__ dev_step, float scale,
                                    const long long* __restrict__ dev_key) {
  const long long groups = (n + 3) >> 2;
  if (dev_step) stream += (uint64_t)(*dev_step);
  if (dev_key) {              // (seed, index0) from device memory: a captured sampler run serves any seed
    seed = (uint64_t)dev_key[0];
    index0 = dev_key[1];
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)B * groups;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / groups);
    const long long g = i - (long long)b * groups;
    const float4 z = normal4(image_key(seed, (uint64_t)(index0 + b)), (uint64_t)g, stream);
    const long long base = (long long)b * n + g * 4;
    const int cnt = (int)((n - g * 4) < 4 ? (n - g * 4) : 4);
    if (!BF16) {
      float* o = (float*)out + base;
      if (cnt == 4 && (base & 3) == 0) {
        *reinterpret_cast<float4*>(o) = float4{z.x * scale, z.y * scale, z.z * scale, z.w * scale};
      } else {
        for (int j = 0; j < cnt; ++j) o[j] = f4_get(z, j) * scale;
      }
    } else {
      u16* o = (u16*)out + base;
      for (int j = 0; j < cnt; ++j) o[j] = f2bf(f4_get(z, j) * scale);
    }
  }
}

// ------------------------------------------------------------------ Euler-ancestral with in-register noise
//  d = (x - den)/sigma ; x += d*(sigma_down - sigma) ; x += N(seed, image, step) * s_up     (fp32, in place)
// Bit-identical to cgs_euler_step(noise = philox_randn(stream=step)) — the noise tensor never exists.
__global__ void euler_anc_philox_kernel(float* __restrict__ x, const float* __restrict__ den, int B, long long n,
                                        float inv_sigma, float dt, float s_up, uint64_t seed, long long index0,
                                        uint64_t stream, const long long* __restrict__ dev_key) {
  const long long groups = n >> 2;  // host guarantees n % 4 == 0
  if (dev_key) {
    seed = (uint64_t)dev_key[0];
    index0 = dev_key[1];
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)B * groups;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / groups);
    const long long g = i - (long long)b * groups;
    float4 xv = reinterpret_cast<float4*>(x)[i];
    const float4 dv = reinterpret_cast<const float4*>(den)[i];
    xv.x = fmaf((xv.x - dv.x) * inv_sigma, dt, xv.x);
    xv.y = fmaf((xv.y - dv.y) * inv_sigma, dt, xv.y);
    xv.z = fmaf((xv.z - dv.z) * inv_sigma, dt, xv.z);
    xv.w = fmaf((xv.w - dv.w) * inv_sigma, dt, xv.w);
    if (s_up > 0.0f) {
      const float4 z = normal4(image_key(seed, (uint64_t)(index0 + b)), (uint64_t)g, stream);
      xv.x = fmaf(z.x, s_up, xv.x);
      xv.y = fmaf(z.y, s_up, xv.y);
      xv.z = fmaf(z.z, s_up, xv.z);
      xv.w = fmaf(z.w, s_up, xv.w);
    }
    reinterpret_cast<float4*>(x)[i] = xv;
  }
}

// ------------------------------------------------------------------ virtual Brownian tree increment
// W on [t0, t1]: W(t1) - W(t0) = N(node 0) * sqrt(t1 - t0); each dyadic midpoint is drawn from the
// Brownian bridge, N(node (depth, idx)) * sqrt((b - a) / 4) around the mean of its endpoints, until
// the interval is below `tol` (or max_depth); then linear interpolation. The path through the tree
// depends only on t, so it is walked in double (host-identical branching) while the values are fp32.
__device__ __forceinline__ uint64_t tree_stream(int depth, uint64_t idx) {
  return (1ull << 63) | ((uint64_t)depth << 40) | idx;
}

__device__ float4 tree_value(uint64_t key, uint64_t g, double t, double t0, double t1, double tol, int max_depth) {
  if (t <= t0) return float4{0.f, 0.f, 0.f, 0.f};
  const float4 w1n = normal4(key, g, tree_stream(0, 0));
  const float s1 = (float)sqrt(t1 - t0);
  float4 wa = {0.f, 0.f, 0.f, 0.f};
  float4 wb = {w1n.x * s1, w1n.y * s1, w1n.z * s1, w1n.w * s1};
  double a = t0, b = t1;
  uint64_t idx = 0;
  int depth = 0;
  while ((b - a) > tol && depth < max_depth) {
    const double m = 0.5 * (a + b);
    const float sd = (float)sqrt((b - a) / 4.0);
    const float4 z = normal4(key, g, tree_stream(depth + 1, idx));
    const float4 wm = {0.5f * (wa.x + wb.x) + z.x * sd, 0.5f * (wa.y + wb.y) + z.y * sd,
                       0.5f * (wa.z + wb.z) + z.z * sd, 0.5f * (wa.w + wb.w) + z.w * sd};
    if (t <= m) { b = m; wb = wm; idx = 2 * idx; }
    else { a = m; wa = wm; idx = 2 * idx + 1; }
    ++depth;
  }
  const float f = (b > a) ? (float)((t - a) / (b - a)) : 0.0f;
  return float4{wa.x + (wb.x - wa.x) * f, wa.y + (wb.y - wa.y) * f, wa.z + (wb.z - wa.z) * f,
                wa.w + (wb.w - wa.w) * f};
}

__global__ void brownian_increment_kernel(float* __restrict__ out, int B, long long n, uint64_t seed, long long index0,
                                          double t0, double t1, double ta, double tb, double tol, int max_depth,
                                          float scale, const long long* __restrict__ dev_key) {
  const long long groups = n >> 2;
  if (dev_key) {
    seed = (uint64_t)dev_key[0];
    index0 = dev_key[1];
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)B * groups;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / groups);
    const long long g = i - (long long)b * groups;
    const uint64_t key = image_key(seed, (uint64_t)(index0 + b));
    const float4 wb = tree_value(key, (uint64_t)g, tb, t0, t1, tol, max_depth);
    const float4 wa = tree_value(key, (uint64_t)g, ta, t0, t1, tol, max_depth);
    reinterpret_cast<float4*>(out)[i] =
        float4{(wb.x - wa.x) * scale, (wb.y - wa.y) * scale, (wb.z - wa.z) * scale, (wb.w - wa.w) * scale};
  }
}


// ------------------------------------------------------------------ device-parameterised sampler step (K16)
// One kernel = CFG combine + Euler / Euler-ancestral update + in-register noise, with every per-step
// scalar read from device memory, so one captured hipGraph serves every step of every job:
//   params[step * stride + 0..3] = sigma, sigma_down, sigma_up, s_noise   (host-built table per job)
//   meta[0] = step, meta[1] = seed, meta[2] = global index of image 0     (meta[0] advanced in-graph)
//   den = u + (c - u) * cfg  (u == nullptr: den = c) ; x += (x - den)/sigma * (sigma_down - sigma)
//   if sigma_up > 0: x += N(seed, image, stream = step) * sigma_up * s_noise ; den_out = den (optional)
__global__ void sampler_step_dev_kernel(float* __restrict__ x, const float* __restrict__ c, const float* __restrict__ u,
                                        float* __restrict__ den_out, int B, long long n, float cfg,
                                        const float* __restrict__ params, int stride,
                                        const long long* __restrict__ meta) {
  const long long step = meta[0];
  const uint64_t seed = (uint64_t)meta[1];
  const long long index0 = meta[2];
  const float* pr = params + step * stride;
  const float sigma = pr[0], sdown = pr[1], sup = pr[2] * pr[3];
  const float inv_sigma = 1.0f / sigma, dt = sdown - sigma;
  const long long groups = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < (long long)B * groups;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / groups);
    const long long g = i - (long long)b * groups;
    float4 xv = reinterpret_cast<float4*>(x)[i];
    float4 dv = reinterpret_cast<const float4*>(c)[i];
    if (u) {
      const float4 uv = reinterpret_cast<const float4*>(u)[i];
      dv.x = uv.x + (dv.x - uv.x) * cfg;
      dv.y = uv.y + (dv.y - uv.y) * cfg;
      dv.z = uv.z + (dv.z - uv.z) * cfg;
      dv.w = uv.w + (dv.w - uv.w) * cfg;
    }
    if (den_out) reinterpret_cast<float4*>(den_out)[i] = dv;
    xv.x = fmaf((xv.x - dv.x) * inv_sigma, dt, xv.x);
    xv.y = fmaf((xv.y - dv.y) * inv_sigma, dt, xv.y);
    xv.z = fmaf((xv.z - dv.z) * inv_sigma, dt, xv.z);
    xv.w = fmaf((xv.w - dv.w) * inv_sigma, dt, xv.w);
    if (sup > 0.0f) {
      const float4 z = normal4(image_key(seed, (uint64_t)(index0 + b)), (uint64_t)g, (uint64_t)step);
      xv.x = fmaf(z.x, sup, xv.x);
      xv.y = fmaf(z.y, sup, xv.y);
      xv.z = fmaf(z.z, sup, xv.z);
      xv.w = fmaf(z.w, sup, xv.w);
    }
    reinterpret_cast<float4*>(x)[i] = xv;
  }
}

// out[0..B) = params[step * stride + col] (the per-image sigma vector the model is called with)
__global__ void step_param_kernel(float* __restrict__ out, int B, const float* __restrict__ params, int stride, int col,
                                  const long long* __restrict__ meta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) out[i] = params[meta[0] * stride + col];
}

__global__ void step_advance_kernel(long long* meta) {
  if (blockIdx.x == 0 && threadIdx.x == 0) meta[0] += 1;
}
}  // namespace

CGS_EXPORT int cgs_philox_randn(void* out, int B, long long n, unsigned long long seed, long long index0,
                                unsigned long long stream, const void* dev_step, float scale, int dtype,
                                const void* dev_key, hipStream_t s) {
  if (B <= 0 || n <= 0) return 0;
  const int blocks = rng_blocks((long long)B * ((n + 3) / 4));
  if (dtype == CGS_F32)
    philox_randn_kernel<false><<<blocks, 256, 0, s>>>(out, B, n, seed, index0, stream, (const long long*)dev_step,
                                                      scale, (const long long*)dev_key);
  else if (dtype == CGS_BF16)
    philox_randn_kernel<true><<<blocks, 256, 0, s>>>(out, B, n, seed, index0, stream, (const long long*)dev_step,
                                                     scale, (const long long*)dev_key);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_euler_ancestral_philox(void* x, const void* den, int B, long long n, float sigma, float sigma_down,
                                          float sigma_up, unsigned long long seed, long long index0,
                                          unsigned long long stream, const void* dev_key, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  euler_anc_philox_kernel<<<rng_blocks((long long)B * (n / 4)), 256, 0, s>>>(
      (float*)x, (const float*)den, B, n, 1.0f / sigma, sigma_down - sigma, sigma_up, seed, index0, stream,
      (const long long*)dev_key);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_brownian_increment(void* out, int B, long long n, unsigned long long seed, long long index0,
                                      double t0, double t1, double ta, double tb, double tol, int max_depth,
                                      float scale, const void* dev_key, hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  brownian_increment_kernel<<<rng_blocks((long long)B * (n / 4)), 256, 0, s>>>(
      (float*)out, B, n, seed, index0, t0, t1, ta, tb, tol, max_depth, scale, (const long long*)dev_key);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_sampler_step_dev(void* x, const void* cond_den, const void* uncond_den, void* den_out, int B,
                                    long long n, float cfg, const void* params, int stride, const void* meta,
                                    hipStream_t s) {
  if (n % 4) return (int)hipErrorInvalidValue;
  sampler_step_dev_kernel<<<rng_blocks((long long)B * (n / 4)), 256, 0, s>>>(
      (float*)x, (const float*)cond_den, (const float*)uncond_den, (float*)den_out, B, n, cfg, (const float*)params,
      stride, (const long long*)meta);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_step_param(void* out, int B, const void* params, int stride, int col, const void* meta,
                              hipStream_t s) {
  step_param_kernel<<<(B + 63) / 64, 64, 0, s>>>((float*)out, B, (const float*)params, stride, col,
                                                 (const long long*)meta);
  return (int)hipGetLastError();
}

CGS_EXPORT int cgs_step_advance(void* meta, hipStream_t s) {
  step_advance_kernel<<<1, 64, 0, s>>>((long long*)meta);
  return (int)hipGetLastError();
}
