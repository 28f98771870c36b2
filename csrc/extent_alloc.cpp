// First-fit extent allocator of the HBM arena (host-only code; see extent_alloc.h).
#include "extent_alloc.h"

#include <algorithm>
#include <iterator>

namespace dfs {

ExtentAllocator::ExtentAllocator(uint64_t capacity) : cap_(capacity) {
  if (capacity) free_[0] = capacity;
}

int64_t ExtentAllocator::alloc(uint64_t bytes) {
  if (bytes == 0) bytes = 256;
  for (auto it = free_.begin(); it != free_.end(); ++it) {
    if (it->second >= bytes) {
      uint64_t off = it->first, len = it->second;
      free_.erase(it);
      if (len > bytes) free_[off + bytes] = len - bytes;
      used_ += bytes;
      return static_cast<int64_t>(off);
    }
  }
  return -1;
}

void ExtentAllocator::free(uint64_t off, uint64_t bytes) {
  if (bytes == 0) bytes = 256;
  used_ -= bytes;
  auto next = free_.lower_bound(off);
  if (next != free_.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      bytes += prev->second;
      free_.erase(prev);
    }
  }
  next = free_.lower_bound(off);
  if (next != free_.end() && off + bytes == next->first) {
    bytes += next->second;
    free_.erase(next);
  }
  free_[off] = bytes;
}

uint64_t ExtentAllocator::largest_free() const {
  uint64_t m = 0;
  for (auto& kv : free_) m = std::max(m, kv.second);
  return m;
}

}  // namespace dfs
