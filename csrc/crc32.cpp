// Host CRC-32/IEEE engine. See crc32.h. Bit-compatible with crc32fast / zlib.
#include "crc32.h"

#include <cpuid.h>
#include <immintrin.h>

#include <cstring>
#include <mutex>

namespace dfs {

namespace {

CrcTables build_tables() {
  CrcTables t;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : (c >> 1);
    t.slice16[0][i] = c;
  }
  for (int k = 1; k < 16; ++k)
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t prev = t.slice16[k - 1][i];
      t.slice16[k][i] = (prev >> 8) ^ t.slice16[0][prev & 0xff];
    }
  return t;
}

inline uint32_t load_le32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// Raw register update with slicing-by-16 (register already inverted by caller).
uint32_t update_sliced(uint32_t c, const uint8_t* p, size_t n) {
  const auto& T = crc_tables().slice16;
  while (n >= 16) {
    uint32_t w0 = load_le32(p) ^ c, w1 = load_le32(p + 4), w2 = load_le32(p + 8),
             w3 = load_le32(p + 12);
    c = T[15][w0 & 0xff] ^ T[14][(w0 >> 8) & 0xff] ^ T[13][(w0 >> 16) & 0xff] ^
        T[12][w0 >> 24] ^ T[11][w1 & 0xff] ^ T[10][(w1 >> 8) & 0xff] ^
        T[9][(w1 >> 16) & 0xff] ^ T[8][w1 >> 24] ^ T[7][w2 & 0xff] ^ T[6][(w2 >> 8) & 0xff] ^
        T[5][(w2 >> 16) & 0xff] ^ T[4][w2 >> 24] ^ T[3][w3 & 0xff] ^ T[2][(w3 >> 8) & 0xff] ^
        T[1][(w3 >> 16) & 0xff] ^ T[0][w3 >> 24];
    p += 16;
    n -= 16;
  }
  while (n--) c = T[0][(c ^ *p++) & 0xff] ^ (c >> 8);
  return c;
}

// Carry-less multiply folding (4x128-bit lanes) for the reflected IEEE polynomial.
// Constants are x^(k) mod P in bit-reflected form: fold-by-512, fold-by-128, 64->32 and
// Barrett (P', mu). Requires n >= 64 and n % 16 == 0. Operates on the raw register.
__attribute__((target("pclmul,sse4.1"))) uint32_t update_clmul(uint32_t c, const uint8_t* p,
                                                                size_t n) {
  const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596LL, 0x0154442bd4LL);
  const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
  const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124LL);
  const __m128i poly = _mm_set_epi64x(0x01f7011641LL, 0x01db710641LL);
  const __m128i* q = reinterpret_cast<const __m128i*>(p);
  __m128i x1 = _mm_loadu_si128(q + 0), x2 = _mm_loadu_si128(q + 1),
          x3 = _mm_loadu_si128(q + 2), x4 = _mm_loadu_si128(q + 3);
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128(static_cast<int>(c)));
  q += 4;
  n -= 64;
  while (n >= 64) {
    __m128i x5 = _mm_clmulepi64_si128(x1, k1k2, 0x00);
    __m128i x6 = _mm_clmulepi64_si128(x2, k1k2, 0x00);
    __m128i x7 = _mm_clmulepi64_si128(x3, k1k2, 0x00);
    __m128i x8 = _mm_clmulepi64_si128(x4, k1k2, 0x00);
    x1 = _mm_clmulepi64_si128(x1, k1k2, 0x11);
    x2 = _mm_clmulepi64_si128(x2, k1k2, 0x11);
    x3 = _mm_clmulepi64_si128(x3, k1k2, 0x11);
    x4 = _mm_clmulepi64_si128(x4, k1k2, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128(q + 0));
    x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128(q + 1));
    x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128(q + 2));
    x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128(q + 3));
    q += 4;
    n -= 64;
  }
#define FOLD128(acc, next)                                                            \
  _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(acc, k3k4, 0x11),                 \
                              _mm_clmulepi64_si128(acc, k3k4, 0x00)),                \
                next)
  x1 = FOLD128(x1, x2);
  x1 = FOLD128(x1, x3);
  x1 = FOLD128(x1, x4);
  while (n >= 16) {
    x1 = FOLD128(x1, _mm_loadu_si128(q));
    ++q;
    n -= 16;
  }
  // 128 -> 64
  __m128i x = _mm_clmulepi64_si128(x1, k3k4, 0x10);
  const __m128i mask32 = _mm_setr_epi32(~0, 0, ~0, 0);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x);
  // 64 -> 32
  x = _mm_srli_si128(x1, 4);
  x1 = _mm_and_si128(x1, mask32);
  x1 = _mm_clmulepi64_si128(x1, k5k0, 0x00);
  x1 = _mm_xor_si128(x1, x);
  // Barrett reduction
  x = _mm_and_si128(x1, mask32);
  x = _mm_clmulepi64_si128(x, poly, 0x10);
  x = _mm_and_si128(x, mask32);
  x = _mm_clmulepi64_si128(x, poly, 0x00);
  x1 = _mm_xor_si128(x1, x);
  return static_cast<uint32_t>(_mm_extract_epi32(x1, 1));
#undef FOLD128
}

bool detect_pclmul() {
  unsigned a, b, c, d;
  if (!__get_cpuid(1, &a, &b, &c, &d)) return false;
  return (c & bit_PCLMUL) && (c & bit_SSE4_1);
}

struct Pow2Ops {
  Gf2Mat m[64];
  Pow2Ops() {
    // operator for one zero *bit*, then square up to one byte.
    Gf2Mat bit;
    bit.col[0] = kCrcPoly;
    for (int i = 1; i < 32; ++i) bit.col[i] = 1u << (i - 1);
    Gf2Mat two = gf2_mul(bit, bit), four = gf2_mul(two, two);
    m[0] = gf2_mul(four, four);
    for (int b = 1; b < 64; ++b) m[b] = gf2_mul(m[b - 1], m[b - 1]);
  }
};

}  // namespace

const CrcTables& crc_tables() {
  static const CrcTables t = build_tables();
  return t;
}

bool cpu_has_pclmul() {
  static const bool v = detect_pclmul();
  return v;
}

uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
  uint32_t c = ~crc;
  if (n >= 64 && cpu_has_pclmul()) {
    size_t bulk = n & ~size_t(15);
    c = update_clmul(c, p, bulk);
    p += bulk;
    n -= bulk;
  }
  c = update_sliced(c, p, n);
  return ~c;
}

size_t num_slices(size_t n) { return (n + kSliceBytes - 1) / kSliceBytes; }

void crc32_slices(const uint8_t* p, size_t n, uint32_t* out) {
  size_t s = 0;
  for (size_t off = 0; off < n; off += kSliceBytes, ++s) {
    size_t len = n - off < kSliceBytes ? n - off : kSliceBytes;
    out[s] = crc32(p + off, len);
  }
}

uint32_t gf2_apply(const Gf2Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1) r ^= m.col[i];
  return r;
}

Gf2Mat gf2_mul(const Gf2Mat& a, const Gf2Mat& b) {
  Gf2Mat r;
  for (int i = 0; i < 32; ++i) r.col[i] = gf2_apply(a, b.col[i]);
  return r;
}

const Gf2Mat& shift_pow2_bytes(int b) {
  static const Pow2Ops ops;
  return ops.m[b];
}

uint32_t crc_shift(uint32_t v, uint64_t nbytes) {
  for (int b = 0; nbytes && v; ++b, nbytes >>= 1)
    if (nbytes & 1) v = gf2_apply(shift_pow2_bytes(b), v);
  return v;
}

Gf2Mat shift_matrix(uint64_t nbytes) {
  Gf2Mat r;
  for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
  for (int b = 0; nbytes; ++b, nbytes >>= 1)
    if (nbytes & 1) r = gf2_mul(shift_pow2_bytes(b), r);
  return r;
}

uint32_t crc_init_term(uint64_t nbytes) { return crc_shift(0xFFFFFFFFu, nbytes) ^ 0xFFFFFFFFu; }

uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  // crc(A||B) = shift(crc_a, |B|) ^ crc_b  (init/xorout terms cancel in this form)
  return crc_shift(crc_a, len_b) ^ crc_b;
}

void shift_table(uint64_t nbytes, uint32_t out[4][256]) {
  Gf2Mat m = shift_matrix(nbytes);
  for (int j = 0; j < 4; ++j)
    for (uint32_t v = 0; v < 256; ++v) out[j][v] = gf2_apply(m, v << (8 * j));
}

uint32_t crc32_from_slices(const uint32_t* sc, size_t n) {
  if (n == 0) return 0;
  static uint32_t t512[4][256];
  static std::once_flag once;
  std::call_once(once, [] { shift_table(kSliceBytes, t512); });
  size_t s = num_slices(n);
  size_t full = (n % kSliceBytes) ? s - 1 : s;
  // raw register of the full-slice prefix via Horner over the 512-byte shift
  uint32_t r = 0;
  const uint32_t s512 = crc_init_term(kSliceBytes);
  for (size_t i = 0; i < full; ++i) r = apply_shift_table(t512, r) ^ (sc[i] ^ s512);
  if (full != s) {
    size_t tail = n - full * kSliceBytes;
    r = crc_shift(r, tail) ^ (sc[s - 1] ^ crc_init_term(tail));
  }
  return r ^ crc_init_term(n);
}

}  // namespace dfs
