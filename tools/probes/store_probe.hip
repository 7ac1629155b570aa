// Store-pattern probe for the GEMM epilogue (gfx950): how fast can one CU write a 256 x 256 bf16
// output tile (128 KiB) with 8 waves, by store shape?  Build: hipcc --offload-arch=gfx950 -O3.
//   P1: dwordx4, one instruction = 16 rows x 64 B   (v7 register epilogue today)
//   P2: dwordx4, one instruction =  8 rows x 128 B  (full 128-B lines)
//   P3: dwordx2, one instruction = 16 rows x 32 B   (round-1 8-B stores)
// Persistent grid (one workgroup per CU walking tiles) and one-tile-per-workgroup grid.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

template <int P>
__device__ __forceinline__ void store_tile(unsigned short* C, int ldc, int m0, int n0, unsigned seed) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;
  unsigned short* base = C + (long long)(m0 + wr * 128) * ldc + n0 + wc * 64;
  if constexpr (P == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq) {
        const int row = 16 * i + fr, col = nq * 32 + 8 * fq;
        *reinterpret_cast<u32x4*>(base + (long long)row * ldc + col) = u32x4{seed + i, seed ^ lane, (unsigned)nq, (unsigned)row};
      }
  } else if constexpr (P == 2) {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int row = 8 * t + (lane >> 3), col = 8 * (lane & 7);
      *reinterpret_cast<u32x4*>(base + (long long)row * ldc + col) = u32x4{seed + t, seed ^ lane, (unsigned)t, (unsigned)row};
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = 16 * i + fr, col = nq * 32 + 8 * fq + 4 * j;
          *reinterpret_cast<u32x2*>(base + (long long)row * ldc + col) = u32x2{seed + i, seed ^ lane};
        }
  }
}

template <int P, bool PERSIST>
__global__ __launch_bounds__(512) void probe(unsigned short* C, int M, int N, unsigned seed) {
  const int tn = N / 256, T = (M / 256) * tn;
  if (PERSIST) {
    for (int u = blockIdx.x; u < T; u += gridDim.x) store_tile<P>(C, N, (u / tn) * 256, (u % tn) * 256, seed);
  } else {
    const int u = blockIdx.x;
    store_tile<P>(C, N, (u / tn) * 256, (u % tn) * 256, seed);
  }
}

template <int P, bool PERSIST>
float run(unsigned short* C, int M, int N, int cus, int iters) {
  const int T = (M / 256) * (N / 256);
  const int grid = PERSIST ? cus : T;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) probe<P, PERSIST><<<grid, 512>>>(C, M, N, w);
  hipEventRecord(a);
  for (int it = 0; it < iters; ++it) probe<P, PERSIST><<<grid, 512>>>(C, M, N, it);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

// few active CUs: per-CU store rate when the chip's write bandwidth is not the limit
template <int P>
float run_few(unsigned short* C, int M, int N, int grid, int tiles_per_wg, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int Mx = 256 * ((grid * tiles_per_wg + N / 256 - 1) / (N / 256));
  for (int w = 0; w < 3; ++w) probe<P, true><<<grid, 512>>>(C, Mx, N, w);
  hipEventRecord(a);
  for (int it = 0; it < iters; ++it) probe<P, true><<<grid, 512>>>(C, Mx, N, it);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main(int argc, char** argv) {
  {
    const int N = 4096;
    unsigned short* C = nullptr;
    if (hipMalloc(&C, (size_t)65536 * N * 2) != hipSuccess) return 1;
    for (int g : {8, 32, 64, 128, 256}) {
      const int tpw = 8;
      const int Mx = 256 * ((g * tpw + N / 256 - 1) / (N / 256));
      const int T = (Mx / 256) * (N / 256);
      const float t1 = run_few<1>(C, Mx, N, g, tpw, 50), t2 = run_few<2>(C, Mx, N, g, tpw, 50);
      const double per_wg = (double)T / g;
      printf("active WGs %3d: P1 %6.2f us/tile (%5.1f GB/s per CU)  P2 %6.2f us/tile (%5.1f GB/s per CU)\n", g,
             t1 * 1e3 / per_wg, 131072.0 / (t1 * 1e-3 / per_wg) / 1e9, t2 * 1e3 / per_wg,
             131072.0 / (t2 * 1e-3 / per_wg) / 1e9);
    }
    hipFree(C);
  }
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 50;
  const int shapes[][2] = {{16384, 4096}, {65536, 2560}, {16384, 1280}, {65536, 640}};
  for (auto& s : shapes) {
    const int M = s[0], N = s[1];
    unsigned short* C = nullptr;
    if (hipMalloc(&C, (size_t)M * N * 2) != hipSuccess) return 1;
    const double bytes = (double)M * N * 2;
    const int T = (M / 256) * (N / 256);
    float t[6];
    t[0] = run<1, true>(C, M, N, cus, iters);
    t[1] = run<2, true>(C, M, N, cus, iters);
    t[2] = run<3, true>(C, M, N, cus, iters);
    t[3] = run<1, false>(C, M, N, cus, iters);
    t[4] = run<2, false>(C, M, N, cus, iters);
    t[5] = run<3, false>(C, M, N, cus, iters);
    const char* names[6] = {"P1 persist", "P2 persist", "P3 persist", "P1 grid", "P2 grid", "P3 grid"};
    for (int i = 0; i < 6; ++i)
      printf("M=%d N=%d tiles=%d %-11s %8.1f us  %6.2f TB/s  %6.2f us/tile/CU\n", M, N, T, names[i], t[i] * 1e3,
             bytes / (t[i] * 1e-3) / 1e12, t[i] * 1e3 / ((double)T / cus));
    hipFree(C);
  }
  return 0;
}
