// Threaded stress driver for the C++ host runtime, built with sanitizers on the CPU
// (`build_native.py --sanitize=address,undefined` / `--sanitize=thread`).
//
// Exercises every multithreaded path of csrc/runtime: safetensors copy_many (a thread pool
// page-faulting an mmap into caller buffers), tree-parallel BLAKE3 over a > 4 MiB input, and the
// shared BPE cache hit from many threads at once. Checks results against single-threaded
// recomputation and exits non-zero on any mismatch; the sanitizer runtime aborts on any memory /
// UB / data-race report.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "../runtime.h"

using namespace cgs;

static int fail(const char* what) {
  std::fprintf(stderr, "stress: FAILED %s\n", what);
  return 1;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
  // ---- safetensors: write 6 tensors (one > the 8 MiB copy slice), read back with a thread pool
  std::vector<SaveItem> items;
  for (int t = 0; t < 6; ++t) {
    SaveItem it;
    it.name = "t" + std::to_string(t);
    it.dtype = "F32";
    const int64_t n = t == 0 ? (int64_t(3) << 20) : 1000 + 37 * t;   // 12 MiB for t0
    it.shape = {n};
    it.bytes.resize(size_t(n) * 4);
    for (int64_t i = 0; i < n; ++i) {
      const float v = float(i % 1013) * 0.5f + float(t);
      std::memcpy(&it.bytes[size_t(i) * 4], &v, 4);
    }
    items.push_back(std::move(it));
  }
  const std::string path = dir + "/cgs_stress.safetensors";
  save_safetensors(path, items, {{"format", "pt"}, {"note", "stress \"quoted\""}});
  for (int round = 0; round < 4; ++round) {
    SafeTensors st(path);
    std::vector<std::vector<uint8_t>> bufs(items.size());
    std::vector<std::pair<std::string, uint8_t*>> dst;
    for (size_t i = 0; i < items.size(); ++i) {
      bufs[i].resize(items[i].bytes.size());
      dst.emplace_back(items[i].name, bufs[i].data());
    }
    st.copy_many(dst, threads);
    for (size_t i = 0; i < items.size(); ++i)
      if (std::memcmp(bufs[i].data(), items[i].bytes.data(), bufs[i].size()) != 0) return fail("copy_many bytes");
    if (st.metadata().at("note") != "stress \"quoted\"") return fail("metadata round trip");
  }
  // ---- BLAKE3: tree-parallel hash of 20 MiB from several threads at once == serial result
  std::vector<uint8_t> blob(size_t(20) << 20);
  for (size_t i = 0; i < blob.size(); ++i) blob[i] = uint8_t((i * 2654435761u) >> 13);
  const std::string ref = blake3_hex(blob.data(), blob.size());
  std::atomic<int> bad{0};
  {
    std::vector<std::thread> pool;
    for (int t = 0; t < 4; ++t)
      pool.emplace_back([&] {
        if (blake3_hex(blob.data(), blob.size()) != ref) bad++;
      });
    for (auto& th : pool) th.join();
  }
  if (bad) return fail("blake3 concurrent");
  if (blake3_hex(nullptr, 0) != "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262")
    return fail("blake3 empty vector");
  // ---- BPE: shared cache under concurrent encode_word
  std::vector<std::string> merges = {"#version", "l o", "lo w</w>", "e r", "n e", "ne w</w>", "w e"};
  std::vector<std::string> vocab;
  for (const char* s : {"l", "o", "w", "e", "r", "n", "l</w>", "o</w>", "w</w>", "e</w>", "r</w>", "n</w>", "lo",
                        "low</w>", "er", "ne", "new</w>", "we"})
    vocab.push_back(s);
  BPE bpe(merges, vocab);
  const std::vector<std::string> words = {"low", "lower", "new", "newer", "wer", "olw", "renew", "lowlow"};
  std::vector<std::vector<int>> ref_ids;
  for (const auto& w : words) ref_ids.push_back(BPE(merges, vocab).encode_word(w));
  {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, t] {
        for (int r = 0; r < 200; ++r) {
          const size_t k = size_t(t + r) % words.size();
          if (bpe.encode_word(words[k]) != ref_ids[k]) bad++;
        }
      });
    for (auto& th : pool) th.join();
  }
  if (bad) return fail("bpe concurrent");
  // ---- weight-arena allocator: concurrent alloc/free, blocks never overlap, all coalesce back
  {
    Arena arena(256ull << 20);
    std::mutex mu;
    std::vector<std::pair<int64_t, uint64_t>> live;
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&, t] {
        uint64_t state = 0x9E3779B97F4A7C15ull * (t + 1);
        std::vector<int64_t> mine;
        for (int r = 0; r < 2000; ++r) {
          state ^= state << 13; state ^= state >> 7; state ^= state << 17;
          if (!mine.empty() && (state & 3) == 0) {
            if (!arena.free((uint64_t)mine.back())) bad++;
            mine.pop_back();
          } else {
            const uint64_t n = 1 + state % (1u << 20);
            const int64_t off = arena.alloc(n);
            if (off >= 0) mine.push_back(off);
          }
        }
        for (int64_t off : mine)
          if (!arena.free((uint64_t)off)) bad++;
      });
    for (auto& th : pool) th.join();
    const ArenaStats st = arena.stats();
    if (st.used != 0 || st.free_blocks != 1 || st.live_blocks != 0) bad++;
  }
  if (bad) return fail("arena concurrent");
  std::remove(path.c_str());
  std::printf("stress ok (%d threads)\n", threads);
  return 0;
}
