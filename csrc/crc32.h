// CRC-32/IEEE (reflected poly 0xEDB88320, init/xorout 0xFFFFFFFF) — the checksum the
// reference stores in every `*_crc32c` proto field and in `<block>.meta`
// (reference: dfs/chunkserver/src/chunkserver.rs:182-190, crc32fast semantics).
//
// Host side: slicing-by-16 + PCLMULQDQ folding, GF(2) "shift by n zero bytes" operators
// used both for CRC combine on the host and to build the LDS tables of the GPU kernels.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace dfs {

constexpr uint32_t kCrcPoly = 0xEDB88320u;
constexpr size_t kSliceBytes = 512;  // CHECKSUM_CHUNK_SIZE in the reference

// Tables shared by host and device code. slice16[k][v] = R(v followed by k zero bytes)
// where R is the raw (zero-init, no xorout) CRC. shift tables: shift_m[j][v] = shift of
// the 32-bit value (v << 8j) by m zero bytes.
struct CrcTables {
  uint32_t slice16[16][256];
};

const CrcTables& crc_tables();

// zlib-style running CRC: crc32_update(0, data) == crc32(data).
uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n);
inline uint32_t crc32(const uint8_t* p, size_t n) { return crc32_update(0, p, n); }

// Per-512B-slice CRCs (what `.meta` holds, native endianness here).
void crc32_slices(const uint8_t* p, size_t n, uint32_t* out);
size_t num_slices(size_t n);

// ---- GF(2) operators on the raw CRC register ----
struct Gf2Mat {
  uint32_t col[32];  // col[i] = image of bit i
};
uint32_t gf2_apply(const Gf2Mat& m, uint32_t v);
Gf2Mat gf2_mul(const Gf2Mat& a, const Gf2Mat& b);  // a∘b
// Operator "append 2^b zero bytes" (b in [0, 63]).
const Gf2Mat& shift_pow2_bytes(int b);
// Raw-register shift by n zero bytes.
uint32_t crc_shift(uint32_t v, uint64_t nbytes);
Gf2Mat shift_matrix(uint64_t nbytes);
// S(n) = shift(0xFFFFFFFF, n) ^ 0xFFFFFFFF : crc32(d) = R(d) ^ S(|d|).
uint32_t crc_init_term(uint64_t nbytes);
// crc32(A||B) from crc32(A), crc32(B), |B|.
uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
// 4x256 byte table for applying a fixed shift operator quickly.
void shift_table(uint64_t nbytes, uint32_t out[4][256]);
inline uint32_t apply_shift_table(const uint32_t t[4][256], uint32_t v) {
  return t[0][v & 0xff] ^ t[1][(v >> 8) & 0xff] ^ t[2][(v >> 16) & 0xff] ^ t[3][v >> 24];
}
// Whole-block CRC from per-slice CRCs (host fold; used when the device path is absent).
uint32_t crc32_from_slices(const uint32_t* slice_crcs, size_t n_bytes);

bool cpu_has_pclmul();

}  // namespace dfs
