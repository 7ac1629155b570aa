// BLAKE3 content hash (portable C++; tree-parallel over std::async for large inputs).
//
// Replaces the Rust `blake3` wheel the reference imports for IS_CHANGED hashing
// (reference nodes.py:9, :586-600, :1895-1909) and the proto WorkflowFile.blake3_hash field.
// The tree is hashed recursively (left subtree = largest power-of-two number of whole chunks),
// so the two halves of a large input can run on different cores; the digest equals the
// sequential BLAKE3 definition.
#include "runtime.h"

#include <cstring>
#include <fcntl.h>
#include <future>
#include <stdexcept>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace cgs {
namespace {

constexpr uint32_t IV[8] = {0x6A09E667u, 0xBB67AE85u, 0x3C6EF372u, 0xA54FF53Au,
                            0x510E527Fu, 0x9B05688Cu, 0x1F83D9ABu, 0x5BE0CD19u};
constexpr int PERM[16] = {2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8};
constexpr uint32_t CHUNK_START = 1, CHUNK_END = 2, PARENT = 4, ROOT = 8;
constexpr size_t BLOCK = 64, CHUNK = 1024;
constexpr size_t PAR_THRESHOLD = size_t(1) << 22;  // subtrees >= 4 MiB split across threads

inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

inline void g(uint32_t* s, int a, int b, int c, int d, uint32_t mx, uint32_t my) {
  s[a] = s[a] + s[b] + mx; s[d] = rotr(s[d] ^ s[a], 16);
  s[c] = s[c] + s[d];      s[b] = rotr(s[b] ^ s[c], 12);
  s[a] = s[a] + s[b] + my; s[d] = rotr(s[d] ^ s[a], 8);
  s[c] = s[c] + s[d];      s[b] = rotr(s[b] ^ s[c], 7);
}

void compress(const uint32_t cv[8], const uint32_t block[16], uint64_t counter, uint32_t block_len,
              uint32_t flags, uint32_t out[16]) {
  uint32_t s[16] = {cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7],
                    IV[0], IV[1], IV[2], IV[3], uint32_t(counter), uint32_t(counter >> 32), block_len, flags};
  uint32_t m[16];
  std::memcpy(m, block, sizeof(m));
  for (int r = 0; r < 7; ++r) {
    g(s, 0, 4, 8, 12, m[0], m[1]);   g(s, 1, 5, 9, 13, m[2], m[3]);
    g(s, 2, 6, 10, 14, m[4], m[5]);  g(s, 3, 7, 11, 15, m[6], m[7]);
    g(s, 0, 5, 10, 15, m[8], m[9]);  g(s, 1, 6, 11, 12, m[10], m[11]);
    g(s, 2, 7, 8, 13, m[12], m[13]); g(s, 3, 4, 9, 14, m[14], m[15]);
    if (r < 6) {
      uint32_t t[16];
      for (int i = 0; i < 16; ++i) t[i] = m[PERM[i]];
      std::memcpy(m, t, sizeof(m));
    }
  }
  for (int i = 0; i < 8; ++i) { out[i] = s[i] ^ s[i + 8]; out[i + 8] = s[i + 8] ^ cv[i]; }
}

inline void load_block(const uint8_t* p, size_t n, uint32_t w[16]) {
  uint8_t buf[BLOCK] = {0};
  if (n) std::memcpy(buf, p, n);
  for (int i = 0; i < 16; ++i)
    w[i] = uint32_t(buf[4 * i]) | uint32_t(buf[4 * i + 1]) << 8 | uint32_t(buf[4 * i + 2]) << 16 |
           uint32_t(buf[4 * i + 3]) << 24;
}

// A node whose final compression is deferred so the caller picks chaining value vs. root output.
struct Output {
  uint32_t cv[8];
  uint32_t block[16];
  uint64_t counter;
  uint32_t block_len;
  uint32_t flags;
  void chaining_value(uint32_t out[8]) const {
    uint32_t o[16];
    compress(cv, block, counter, block_len, flags, o);
    std::memcpy(out, o, 32);
  }
  void root_bytes(uint8_t* out, size_t n) const {
    uint64_t ctr = 0;
    while (n) {
      uint32_t o[16];
      compress(cv, block, ctr++, block_len, flags | ROOT, o);
      for (int i = 0; i < 16 && n; ++i)
        for (int b = 0; b < 4 && n; ++b, --n) *out++ = uint8_t(o[i] >> (8 * b));
    }
  }
};

Output chunk_output(const uint8_t* p, size_t len, uint64_t chunk_counter) {
  uint32_t cv[8];
  std::memcpy(cv, IV, 32);
  size_t nblocks = len == 0 ? 1 : (len + BLOCK - 1) / BLOCK;
  uint32_t w[16];
  for (size_t b = 0; b + 1 < nblocks; ++b) {
    load_block(p + b * BLOCK, BLOCK, w);
    uint32_t o[16];
    compress(cv, w, chunk_counter, BLOCK, b == 0 ? CHUNK_START : 0, o);
    std::memcpy(cv, o, 32);
  }
  size_t last = (nblocks - 1) * BLOCK;
  Output out;
  std::memcpy(out.cv, cv, 32);
  load_block(p + last, len - last, out.block);
  out.counter = chunk_counter;
  out.block_len = uint32_t(len - last);
  out.flags = CHUNK_END | (nblocks == 1 ? CHUNK_START : 0);
  return out;
}

Output parent_output(const uint32_t l[8], const uint32_t r[8]) {
  Output out;
  std::memcpy(out.cv, IV, 32);
  std::memcpy(out.block, l, 32);
  std::memcpy(out.block + 8, r, 32);
  out.counter = 0;
  out.block_len = BLOCK;
  out.flags = PARENT;
  return out;
}

inline size_t left_len(size_t len) {
  size_t full = (len - 1) / CHUNK;
  size_t p = 1;
  while (p * 2 <= full) p *= 2;
  return p * CHUNK;
}

Output subtree(const uint8_t* p, size_t len, uint64_t chunk_counter, int depth) {
  if (len <= CHUNK) return chunk_output(p, len, chunk_counter);
  size_t ll = left_len(len);
  uint32_t lcv[8], rcv[8];
  if (len >= PAR_THRESHOLD && depth < 4) {
    auto fut = std::async(std::launch::async, [=] { return subtree(p, ll, chunk_counter, depth + 1); });
    subtree(p + ll, len - ll, chunk_counter + ll / CHUNK, depth + 1).chaining_value(rcv);
    fut.get().chaining_value(lcv);
  } else {
    subtree(p, ll, chunk_counter, depth + 1).chaining_value(lcv);
    subtree(p + ll, len - ll, chunk_counter + ll / CHUNK, depth + 1).chaining_value(rcv);
  }
  return parent_output(lcv, rcv);
}

std::string to_hex(const uint8_t* d, size_t n) {
  static const char* hx = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) { s[2 * i] = hx[d[i] >> 4]; s[2 * i + 1] = hx[d[i] & 15]; }
  return s;
}

}  // namespace

std::string blake3_hex(const uint8_t* data, size_t len, size_t out_len) {
  std::vector<uint8_t> out(out_len);
  subtree(data, len, 0, 0).root_bytes(out.data(), out_len);
  return to_hex(out.data(), out_len);
}

std::string blake3_file_hex(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("blake3: cannot open " + path);
  struct stat st;
  if (fstat(fd, &st) != 0) { ::close(fd); throw std::runtime_error("blake3: stat failed " + path); }
  size_t n = size_t(st.st_size);
  if (n == 0) { ::close(fd); return blake3_hex(nullptr, 0); }
  void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) throw std::runtime_error("blake3: mmap failed " + path);
  madvise(m, n, MADV_SEQUENTIAL);
  std::string h = blake3_hex(static_cast<const uint8_t*>(m), n);
  munmap(m, n);
  return h;
}

}  // namespace cgs
