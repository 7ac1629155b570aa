// Shared declarations for the C++ host runtime (_cgs_runtime).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace cgs {

// ---- HBM weight-arena offset allocator (arena.cpp)
struct ArenaStats {
  uint64_t capacity = 0, used = 0, peak = 0, largest_free = 0;
  size_t free_blocks = 0, live_blocks = 0;
};

class Arena {
 public:
  explicit Arena(uint64_t capacity, uint64_t align = 256);
  int64_t alloc(uint64_t bytes);      // byte offset, or -1 when no free block fits
  bool free(uint64_t off);            // false for an offset that is not a live block
  ArenaStats stats() const;
  uint64_t align() const { return align_; }

 private:
  void insert_free(uint64_t off, uint64_t size);
  void erase_free(uint64_t off, uint64_t size);
  uint64_t cap_, align_;
  uint64_t in_use_ = 0, peak_ = 0;
  std::map<uint64_t, uint64_t> by_off_;        // free: offset -> size
  std::multimap<uint64_t, uint64_t> by_size_;  // free: size -> offset
  std::map<uint64_t, uint64_t> used_;          // live: offset -> size
  mutable std::mutex mu_;
};

// ---- BLAKE3 (blake3.cpp)
std::string blake3_hex(const uint8_t* data, size_t len, size_t out_len = 32);
std::string blake3_file_hex(const std::string& path);

// ---- safetensors (safetensors.cpp)
struct TensorInfo {
  std::string dtype;
  std::vector<int64_t> shape;
  uint64_t begin = 0, end = 0;  // byte offsets relative to the data section
};

class MappedFile {
 public:
  explicit MappedFile(const std::string& path);
  ~MappedFile();
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  uint8_t* data() const { return base_; }
  size_t size() const { return size_; }

 private:
  uint8_t* base_ = nullptr;
  size_t size_ = 0;
};

class SafeTensors {
 public:
  explicit SafeTensors(const std::string& path);
  const std::vector<std::string>& keys() const { return order_; }
  const TensorInfo& info(const std::string& name) const;
  uint8_t* tensor_ptr(const std::string& name) const;
  const std::map<std::string, std::string>& metadata() const { return meta_; }
  std::shared_ptr<MappedFile> file() const { return file_; }
  // The tensor data section (everything after the header) as one span of the mapping.
  uint8_t* data_section() const { return file_->data() + data_off_; }
  size_t data_section_size() const { return file_->size() - data_off_; }
  // Copy tensors into caller-provided host buffers with a thread pool: page faults of a cold
  // mmap are the load bottleneck, parallel touch keeps the page cache / NVMe queue full.
  void copy_many(const std::vector<std::pair<std::string, uint8_t*>>& dst, int threads) const;

 private:
  std::shared_ptr<MappedFile> file_;
  uint64_t data_off_ = 0;
  std::vector<std::string> order_;
  std::map<std::string, TensorInfo> tensors_;
  std::map<std::string, std::string> meta_;
};

struct SaveItem {
  std::string name, dtype;
  std::vector<int64_t> shape;
  std::string bytes;
};
void save_safetensors(const std::string& path, const std::vector<SaveItem>& items,
                      const std::map<std::string, std::string>& metadata);
std::string json_escape(const std::string& s);

// ---- CLIP byte-level BPE (bpe.cpp)
class BPE {
 public:
  BPE(const std::vector<std::string>& merges, const std::vector<std::string>& vocab);
  std::vector<int> encode_word(const std::string& utf8_word);
  size_t vocab_size() const { return encoder_.size(); }

 private:
  std::vector<int> bpe(const std::string& word) const;
  std::unordered_map<std::string, int> encoder_;
  std::unordered_map<std::string, int> ranks_;  // "a b" -> rank
  std::unordered_map<std::string, std::vector<int>> cache_;
  std::mutex mu_;
};

}  // namespace cgs
