// GF(2^8) arithmetic and the Reed-Solomon coding matrix, bit-compatible with the
// reference's `reed-solomon-erasure` galois_8 codec (field poly 0x11D, generator 2,
// Vandermonde matrix made systematic by the inverse of its top k x k block;
// reference usage: dfs/common/src/erasure.rs:7-59).
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace dfs::gf {

struct Tables {
  uint8_t log[256];
  uint8_t exp[512];
};
const Tables& tables();

inline uint8_t mul(uint8_t a, uint8_t b) {
  if (!a || !b) return 0;
  const auto& t = tables();
  return t.exp[t.log[a] + t.log[b]];
}
uint8_t inv(uint8_t a);
uint8_t pow(uint8_t a, unsigned n);

using Matrix = std::vector<std::vector<uint8_t>>;
Matrix identity(int n);
Matrix multiply(const Matrix& a, const Matrix& b);
Matrix invert(Matrix m);  // throws std::runtime_error if singular
// (k+m) x k systematic encoding matrix.
Matrix rs_matrix(int k, int m);
// Rows of the decode matrix that rebuild `wanted` shard indices from the k shards listed
// in `present` (ascending, size k).
Matrix rs_decode_rows(int k, int m, const std::vector<int>& present, const std::vector<int>& wanted);

// CPU codec: out[r] = sum_c mat[r][c] * in[c] over len bytes (split-table multiply).
void matmul_cpu(const Matrix& mat, const uint8_t* const* in, uint8_t* const* out, size_t len);

}  // namespace dfs::gf
