#include "gf256.h"

#include <cstring>

namespace dfs::gf {

namespace {
Tables build() {
  Tables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(x);
    t.log[x] = static_cast<uint8_t>(i);
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
  t.log[0] = 0;  // never used for zero operands
  return t;
}
}  // namespace

const Tables& tables() {
  static const Tables t = build();
  return t;
}

uint8_t inv(uint8_t a) {
  if (!a) throw std::runtime_error("gf: inverse of zero");
  const auto& t = tables();
  return t.exp[255 - t.log[a]];
}

uint8_t pow(uint8_t a, unsigned n) {
  if (n == 0) return 1;
  if (a == 0) return 0;
  const auto& t = tables();
  return t.exp[(t.log[a] * static_cast<unsigned long>(n)) % 255];
}

Matrix identity(int n) {
  Matrix m(n, std::vector<uint8_t>(n, 0));
  for (int i = 0; i < n; ++i) m[i][i] = 1;
  return m;
}

Matrix multiply(const Matrix& a, const Matrix& b) {
  size_t r = a.size(), inner = b.size(), c = b.empty() ? 0 : b[0].size();
  Matrix out(r, std::vector<uint8_t>(c, 0));
  for (size_t i = 0; i < r; ++i)
    for (size_t j = 0; j < c; ++j) {
      uint8_t acc = 0;
      for (size_t k = 0; k < inner; ++k) acc ^= mul(a[i][k], b[k][j]);
      out[i][j] = acc;
    }
  return out;
}

Matrix invert(Matrix m) {
  int n = static_cast<int>(m.size());
  Matrix r = identity(n);
  for (int col = 0; col < n; ++col) {
    int piv = col;
    while (piv < n && m[piv][col] == 0) ++piv;
    if (piv == n) throw std::runtime_error("gf: singular matrix");
    std::swap(m[piv], m[col]);
    std::swap(r[piv], r[col]);
    uint8_t s = inv(m[col][col]);
    for (int j = 0; j < n; ++j) {
      m[col][j] = mul(m[col][j], s);
      r[col][j] = mul(r[col][j], s);
    }
    for (int row = 0; row < n; ++row) {
      if (row == col || m[row][col] == 0) continue;
      uint8_t f = m[row][col];
      for (int j = 0; j < n; ++j) {
        m[row][j] ^= mul(f, m[col][j]);
        r[row][j] ^= mul(f, r[col][j]);
      }
    }
  }
  return r;
}

Matrix rs_matrix(int k, int m) {
  if (k <= 0 || m <= 0 || k + m > 256) throw std::runtime_error("rs: bad shard counts");
  int total = k + m;
  Matrix vm(total, std::vector<uint8_t>(k));
  for (int r = 0; r < total; ++r)
    for (int c = 0; c < k; ++c) vm[r][c] = pow(static_cast<uint8_t>(r), c);
  Matrix top(vm.begin(), vm.begin() + k);
  return multiply(vm, invert(top));
}

Matrix rs_decode_rows(int k, int m, const std::vector<int>& present,
                      const std::vector<int>& wanted) {
  if (static_cast<int>(present.size()) != k) throw std::runtime_error("rs: need k shards");
  Matrix enc = rs_matrix(k, m);
  Matrix sub;
  for (int idx : present) sub.push_back(enc.at(idx));
  Matrix dec = invert(sub);  // data = dec * present
  Matrix rows;
  for (int w : wanted) {
    if (w < k) {
      rows.push_back(dec[w]);
    } else {  // parity row re-encoded from reconstructed data
      Matrix one{enc.at(w)};
      rows.push_back(multiply(one, dec)[0]);
    }
  }
  return rows;
}

void matmul_cpu(const Matrix& mat, const uint8_t* const* in, uint8_t* const* out, size_t len) {
  size_t rows = mat.size();
  size_t k = rows ? mat[0].size() : 0;
  // Per-coefficient 256-entry multiply tables; process in 4 KiB blocks for cache reuse.
  std::vector<uint8_t> mt(rows * k * 256);
  for (size_t r = 0; r < rows; ++r)
    for (size_t c = 0; c < k; ++c)
      for (int v = 0; v < 256; ++v) mt[(r * k + c) * 256 + v] = mul(mat[r][c], static_cast<uint8_t>(v));
  constexpr size_t kBlock = 4096;
  for (size_t base = 0; base < len; base += kBlock) {
    size_t n = len - base < kBlock ? len - base : kBlock;
    for (size_t r = 0; r < rows; ++r) {
      uint8_t* o = out[r] + base;
      std::memset(o, 0, n);
      for (size_t c = 0; c < k; ++c) {
        const uint8_t* t = &mt[(r * k + c) * 256];
        const uint8_t* src = in[c] + base;
        if (mat[r][c] == 0) continue;
        if (mat[r][c] == 1) {
          for (size_t i = 0; i < n; ++i) o[i] ^= src[i];
        } else {
          for (size_t i = 0; i < n; ++i) o[i] ^= t[src[i]];
        }
      }
    }
  }
}

}  // namespace dfs::gf
