// Host -> HBM upload of checkpoint bytes ("direct H2D into a pre-allocated HBM arena").
//
// The safetensors data section is mmap'ed (csrc/runtime/safetensors.cpp); this streams it into one
// device allocation through two pinned staging buffers: while the DMA engine copies chunk i on
// `stream`, host threads fault in + memcpy chunk i+1 into the other buffer. A chunk's buffer is
// reused only after the event recorded behind its copy has completed. Pageable memcpy in HIP would
// stage through a driver buffer one chunk at a time with no overlap.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#define CGS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

void parallel_memcpy(char* dst, const char* src, size_t n, int threads) {
  if (threads <= 1 || n < (8u << 20)) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<std::thread> pool;
  const size_t part = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    size_t a = (size_t)t * part, b = std::min(n, a + part);
    if (a >= b) break;
    pool.emplace_back([=] { std::memcpy(dst + a, src + a, b - a); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

// Copies `nbytes` from host `src` (any pageable memory, e.g. an mmap) to device `dst`.
// chunk: staging chunk size in bytes (0 -> 64 MiB); threads: host memcpy threads (0 -> 4).
// Synchronous with respect to the caller: returns after the last chunk has landed.
CGS_EXPORT int cgs_h2d_upload(const void* src, void* dst, long long nbytes, long long chunk, int threads,
                              hipStream_t stream) {
  if (nbytes <= 0) return 0;
  if (!src || !dst) return (int)hipErrorInvalidValue;
  const size_t C = chunk > 0 ? (size_t)chunk : (size_t)64 << 20;
  const int T = threads > 0 ? threads : 4;
  char* stage[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t err = hipSuccess;
  for (int i = 0; i < 2 && err == hipSuccess; ++i) {
    err = hipHostMalloc((void**)&stage[i], std::min(C, (size_t)nbytes), hipHostMallocDefault);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  }
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  bool pending[2] = {false, false};
  size_t off = 0;
  int k = 0;
  while (err == hipSuccess && off < (size_t)nbytes) {
    const size_t n = std::min(C, (size_t)nbytes - off);
    if (pending[k]) {
      err = hipEventSynchronize(ev[k]);
      if (err != hipSuccess) break;
    }
    parallel_memcpy(stage[k], s + off, n, T);
    err = hipMemcpyAsync(d + off, stage[k], n, hipMemcpyHostToDevice, stream);
    if (err == hipSuccess) err = hipEventRecord(ev[k], stream);
    pending[k] = true;
    off += n;
    k ^= 1;
  }
  for (int i = 0; i < 2; ++i) {
    if (pending[i] && ev[i]) {
      hipError_t e = hipEventSynchronize(ev[i]);
      if (err == hipSuccess) err = e;
    }
    if (ev[i]) hipEventDestroy(ev[i]);
    if (stage[i]) hipHostFree(stage[i]);
  }
  return (int)err;
}

// Ends a stream capture that an exception left open (sampling/run_graph.py failure path): a capture
// invalidated by an unsupported call can survive the framework's own end-capture attempt, and every
// later HIP call in the process then fails with "operation not permitted when stream is capturing".
// Returns 1 if a capture was ended, 0 if the stream was not capturing, < 0 on error.
CGS_EXPORT int cgs_abort_stream_capture(hipStream_t stream) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess) return -1;
  if (st == hipStreamCaptureStatusNone) return 0;
  hipGraph_t g = nullptr;
  (void)hipStreamEndCapture(stream, &g);
  if (g) (void)hipGraphDestroy(g);
  (void)hipGetLastError();
  return 1;
}
