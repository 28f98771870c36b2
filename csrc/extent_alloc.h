// HBM arena allocator of the chunk store (host-side bookkeeping only, no HIP).
#pragma once
#include <cstdint>
#include <map>

namespace dfs {

// First-fit extent allocator over [0, capacity) with coalescing.
class ExtentAllocator {
 public:
  explicit ExtentAllocator(uint64_t capacity = 0);
  int64_t alloc(uint64_t bytes);  // -1 when no fit
  void free(uint64_t off, uint64_t bytes);
  uint64_t used() const { return used_; }
  uint64_t capacity() const { return cap_; }
  uint64_t largest_free() const;

 private:
  uint64_t cap_, used_ = 0;
  std::map<uint64_t, uint64_t> free_;  // off -> len
};

}  // namespace dfs
