// Offset allocator of the HBM weight arena (C27; SURVEY §7.1 runtime/ "HBM arena"): one device slab
// per GPU holds every resident model's weights; this class decides where. Best fit over a free
// list kept in two indexes (by offset for O(log n) coalescing with both neighbours on free, by size
// for O(log n) best-fit search), every block aligned (default 256 B: one MFMA-friendly, 16-B-vector
// and LDS-DMA-aligned origin). Thread-safe; knows nothing about the device (the slab is a torch
// tensor on the Python side), so it is unit-tested on the CPU and under the sanitizer builds.
#include "runtime.h"

#include <stdexcept>

namespace cgs {

Arena::Arena(uint64_t capacity, uint64_t align) : cap_(capacity), align_(align ? align : 256) {
  if (align_ & (align_ - 1)) throw std::invalid_argument("arena alignment must be a power of two");
  cap_ -= cap_ % align_;
  if (cap_) insert_free(0, cap_);
}

void Arena::insert_free(uint64_t off, uint64_t size) {
  by_off_[off] = size;
  by_size_.emplace(size, off);
}

void Arena::erase_free(uint64_t off, uint64_t size) {
  by_off_.erase(off);
  auto range = by_size_.equal_range(size);
  for (auto it = range.first; it != range.second; ++it)
    if (it->second == off) {
      by_size_.erase(it);
      return;
    }
}

int64_t Arena::alloc(uint64_t bytes) {
  std::lock_guard<std::mutex> g(mu_);
  const uint64_t need = ((bytes ? bytes : 1) + align_ - 1) / align_ * align_;
  auto it = by_size_.lower_bound(need);            // smallest free block that fits
  if (it == by_size_.end()) return -1;
  const uint64_t size = it->first, off = it->second;
  erase_free(off, size);
  if (size > need) insert_free(off + need, size - need);
  used_[off] = need;
  in_use_ += need;
  peak_ = std::max(peak_, in_use_);
  return (int64_t)off;
}

bool Arena::free(uint64_t off) {
  std::lock_guard<std::mutex> g(mu_);
  auto u = used_.find(off);
  if (u == used_.end()) return false;
  uint64_t start = off, size = u->second;
  used_.erase(u);
  in_use_ -= size;
  auto next = by_off_.lower_bound(start);
  if (next != by_off_.end() && next->first == start + size) {      // merge with the right neighbour
    const uint64_t ns = next->second;
    erase_free(next->first, ns);
    size += ns;
  }
  auto prev = by_off_.lower_bound(start);
  if (prev != by_off_.begin()) {                                   // merge with the left neighbour
    --prev;
    if (prev->first + prev->second == start) {
      const uint64_t po = prev->first, ps = prev->second;
      erase_free(po, ps);
      start = po;
      size += ps;
    }
  }
  insert_free(start, size);
  return true;
}

ArenaStats Arena::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  ArenaStats s;
  s.capacity = cap_;
  s.used = in_use_;
  s.peak = peak_;
  s.free_blocks = by_off_.size();
  s.live_blocks = used_.size();
  s.largest_free = by_size_.empty() ? 0 : by_size_.rbegin()->first;
  return s;
}

}  // namespace cgs
