// CDNA4 kernels for the chunk data path. Design notes:
//  * 64-lane waves: 8 lanes x 64 B cover one 512 B slice, so a wave checksums 8 slices
//    (4 KiB) and a 256-thread workgroup a 16 KiB tile. Each lane runs a slicing-by-16
//    chain over its 64 B (16 independent LDS lookups per 16 B, state carried between
//    chunks), then the wave combines lane/slice partials with a butterfly over
//    __shfl_xor and "shift by 2^k bytes" byte tables — all tables live in LDS (48 KiB).
//  * Whole-block CRC (K2) comes out of the same pass: slices are combined into a tile
//    value, and each tile is shifted to its final position with GF(2) matrices applied
//    lane-parallel (lane i owns column i, 5 xor-shuffles), so the host only XORs
//    `grid` partials. Leading zero slices do not change a raw CRC, which lets the tiling
//    be aligned at the block END (virtual front padding) without any inverse operator.
//  * Grid = min(tiles, 1024) with a grid-stride loop: the LDS table fill (48 KiB from
//    L2) is paid once per workgroup, not per tile.
#include "gpu_kernels.h"

#include <atomic>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crc32.h"
#include "gf256.h"

namespace dfs {

namespace {

__device__ __forceinline__ uint32_t tab4(const uint32_t (*t)[256], uint32_t v) {
  return t[0][v & 0xff] ^ t[1][(v >> 8) & 0xff] ^ t[2][(v >> 16) & 0xff] ^ t[3][v >> 24];
}

__device__ __forceinline__ uint32_t chunk16(const uint32_t (*T)[256], uint32_t c, uint4 w) {
  uint32_t w0 = w.x ^ c;
  return T[15][w0 & 0xff] ^ T[14][(w0 >> 8) & 0xff] ^ T[13][(w0 >> 16) & 0xff] ^
         T[12][w0 >> 24] ^ T[11][w.y & 0xff] ^ T[10][(w.y >> 8) & 0xff] ^
         T[9][(w.y >> 16) & 0xff] ^ T[8][w.y >> 24] ^ T[7][w.z & 0xff] ^
         T[6][(w.z >> 8) & 0xff] ^ T[5][(w.z >> 16) & 0xff] ^ T[4][w.z >> 24] ^
         T[3][w.w & 0xff] ^ T[2][(w.w >> 8) & 0xff] ^ T[1][(w.w >> 16) & 0xff] ^ T[0][w.w >> 24];
}

// Value of lane `lane ^ m` without LDS traffic: DPP for m <= 8 (xor 4 = half-row mirror of
// the xor-3 quad permutation; xor 8 = rotate the 16-lane row by 8, either direction), the
// CDNA4 permlane swaps for 16 and 32 (swapping v with itself leaves the even half-rows /
// half-waves in r[0] and the odd ones in r[1]).
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t x) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), kCtrl, 0xF, 0xF, false));
}

template <int m>
__device__ __forceinline__ uint32_t xchg(uint32_t v, int lane) {
  if constexpr (m == 1) return dpp_mov<0xB1>(v);  // quad_perm [1,0,3,2]
  else if constexpr (m == 2) return dpp_mov<0x4E>(v);  // quad_perm [2,3,0,1]
  else if constexpr (m == 4) return dpp_mov<0x141>(dpp_mov<0x1B>(v));  // quad_perm [3,2,1,0], then half-row mirror
  else if constexpr (m == 8) return dpp_mov<0x128>(v);  // row_ror:8
  else if constexpr (m == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane & 16) ? r[0] : r[1];
  } else {
    static_assert(m == 32, "xchg: 1, 2, 4, 8, 16 or 32");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane & 32) ? r[0] : r[1];
  }
}

// Butterfly step: lanes with (lane & m) == 0 hold the earlier bytes.
template <int m>
__device__ __forceinline__ uint32_t combine(uint32_t r, int lane, const uint32_t (*t)[256]) {
  uint32_t p = xchg<m>(r, lane);
  bool right = lane & m;
  uint32_t left = right ? p : r;
  uint32_t rgt = right ? r : p;
  return tab4(t, left) ^ rgt;
}

// XOR all-reduce steps inside the wave without LDS traffic (ds_bpermute plus its address
// arithmetic is what __shfl_xor compiles to). Applied smallest group first: xr4 / xr8 pair
// lanes by mirroring a half-row / row (DPP), which equals the xor-4 / xor-8 partner's value
// once the quads / 8-lane groups are already uniform; xr16 / xr32 use the CDNA4 permlane
// swaps (a swap of v with itself leaves the two halves' values in the two results).
template <int kCtrl>
__device__ __forceinline__ uint32_t xr_dpp(uint32_t v) {
  return v ^ static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), kCtrl, 0xF, 0xF, false));
}
__device__ __forceinline__ uint32_t xr1(uint32_t v) { return xr_dpp<0xB1>(v); }   // quad_perm [1,0,3,2]
__device__ __forceinline__ uint32_t xr2(uint32_t v) { return xr_dpp<0x4E>(v); }   // quad_perm [2,3,0,1]
__device__ __forceinline__ uint32_t xr4(uint32_t v) { return xr_dpp<0x141>(v); }  // row_half_mirror
__device__ __forceinline__ uint32_t xr8(uint32_t v) { return xr_dpp<0x140>(v); }  // row_mirror
__device__ __forceinline__ uint32_t xr16(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return r[0] ^ r[1];
}
__device__ __forceinline__ uint32_t xr32(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return r[0] ^ r[1];
}

// Lane-parallel GF(2) matrix apply: v uniform across the wave, lanes 0..31 own columns.
__device__ __forceinline__ uint32_t mat_apply(const uint32_t* col, uint32_t v, int lane) {
  int i = lane & 31;
  uint32_t x = ((v >> i) & 1u) ? col[i] : 0u;
  return xr16(xr8(xr4(xr2(xr1(x)))));
}

__device__ __forceinline__ void load_tables(const DevCrcTables* __restrict__ gt, DevCrcTables* lt) {
  const uint4* src = reinterpret_cast<const uint4*>(gt);
  uint4* dst = reinterpret_cast<uint4*>(lt);
  constexpr int n16 = sizeof(DevCrcTables) / 16;
  for (int i = threadIdx.x; i < n16; i += kCrcWgThreads) dst[i] = src[i];
}

// One 512 B slice per 8 lanes: lane `sl` hashes bytes [sl*64, sl*64+64), then the three
// butterflies leave the slice CRC (raw, before the init term) in lane sl == 0.
__device__ __forceinline__ uint32_t slice_crc(const DevCrcTables& lt, const uint8_t* slice, int sl, int lane,
                                              bool valid) {
  uint32_t r = 0;
  if (valid) {
    const uint4* p = reinterpret_cast<const uint4*>(slice + sl * 64);
    uint4 c0 = p[0], c1 = p[1], c2 = p[2], c3 = p[3];
    r = chunk16(lt.slice16, 0, c0);
    r = chunk16(lt.slice16, r, c1);
    r = chunk16(lt.slice16, r, c2);
    r = chunk16(lt.slice16, r, c3);
  }
  r = combine<1>(r, lane, lt.sh64);
  r = combine<2>(r, lane, lt.sh128);
  return combine<4>(r, lane, lt.sh256);
}

// ---------------------------------------------------------------------------------------
// Matrix-core chunk CRC. The raw CRC of a 64-byte chunk is a GF(2)-linear map of its 512
// bits: R(chunk) = XOR over set bits (byte b, bit p) of V[b][p], V[b][p] = R(e_{b,p}).
// That is a 32 x 512 binary matrix times the chunk's bit vector — an integer GEMM whose
// result only needs its parity. One v_mfma_i32_32x32x32_i8 multiplies A (32 CRC bits x 32
// K-bits of the basis) by B (32 K-bits x 32 chunks); 16 of them cover the 512 bits of 32
// chunks (2 KiB), two passes the wave's 4 KiB.
//  * B (data): lane (n = l&31, h = l>>5) loads bytes [32h, 32h+32) of chunk n. K-step s
//    uses dword s>>1 and bit planes 4(s&1)..4(s&1)+3: fragment dword q is the dword ANDed
//    with 0x01010101 << p (one VALU op; the planes are not shifted down).
//  * A (basis, in 64 VGPRs for the whole kernel): element (s, h, j) is 2^(7-p) where bit i
//    of V[byte][p] is set, so every product of a set data bit is 2^7 (mod 2^8) and bit 7 of
//    the int32 accumulator is the parity — the GF(2) sum — for any K order, as long as A
//    and B agree on it (the host builds A in upload_crc_tables with the same mapping).
//  * D: lane (n, h) holds CRC bits i = (r&3) + 8(r>>2) + 4h of chunk n in register r; the
//    two half-waves OR their 16 bits together with one shuffle.
// 64 LDS table lookups per lane per 64 B become 32 MFMAs per 4 KiB per wave.
using i32x4 = __attribute__((ext_vector_type(4))) int;
using i32x16 = __attribute__((ext_vector_type(16))) int;

__device__ __forceinline__ void load_basis(const i32x4* __restrict__ basis, int lane, i32x4 (&A)[16]) {
#pragma unroll
  for (int s = 0; s < 16; ++s) A[s] = basis[s * 64 + lane];
}

// The 64 B this lane feeds to the two MFMA passes over the wave's 8 slices starting at slice
// i0 (two halves of chunk n in pass 0 and pass 1); slices outside [lo, hi) read as zeros.
struct WaveData {
  uint4 v[4];
};

__device__ __forceinline__ WaveData load_wave(const uint8_t* __restrict__ data, int64_t i0, int64_t lo, int64_t hi,
                                              int lane) {
  const int n = lane & 31, h = lane >> 5;
  WaveData d;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = it * 32 + n;
    const int64_t i = i0 + (c >> 3);
    d.v[2 * it] = d.v[2 * it + 1] = make_uint4(0, 0, 0, 0);
    if (i >= lo && i < hi) {
      // streamed once: non-temporal, so checksum passes do not evict hot lines from L2
      using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
      const u32x4* p = reinterpret_cast<const u32x4*>(data + static_cast<uint64_t>(i) * 512 + (c & 7) * 64 + h * 32);
      u32x4 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
      d.v[2 * it] = make_uint4(x[0], x[1], x[2], x[3]);
      d.v[2 * it + 1] = make_uint4(y[0], y[1], y[2], y[3]);
    }
  }
  return d;
}

// Ring form of load_wave for the pipelined kernels: the loads are unconditional (slices
// outside [lo, hi) read slice lo instead; requires lo < hi) and the consumer zeroes the
// CHUNK CRCs of those slices (one select per lane instead of 16 on the data; the raw CRC of
// zeros is zero, so it is the same as zeroed data). A conditional load into a zeroed
// register is a VALU write to a register the ring may still have a load pending on, and the
// compiler resolves that with a vmcnt(0) that drains the whole ring.
__device__ __forceinline__ WaveData load_wave_ring(const uint8_t* __restrict__ data, int64_t i0, int64_t lo,
                                                   int64_t hi, int lane) {
  const int n = lane & 31, h = lane >> 5;
  WaveData d;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = it * 32 + n;
    int64_t i = i0 + (c >> 3);
    i = (i >= lo && i < hi) ? i : lo;
    using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
    const u32x4* p = reinterpret_cast<const u32x4*>(data + static_cast<uint64_t>(i) * 512 + (c & 7) * 64 + h * 32);
    u32x4 x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
    d.v[2 * it] = make_uint4(x[0], x[1], x[2], x[3]);
    d.v[2 * it + 1] = make_uint4(y[0], y[1], y[2], y[3]);
  }
  return d;
}

// Raw CRC of the 64-byte chunk `lane` of the wave's 4 KiB (wave-wide: all 64 lanes together).
// Every product in the accumulators is 0 or +-2^7, so an accumulator's low byte is 0x80 or 0
// (its parity, nothing below): three byte permutes gather the low bytes of four accumulators
// into one dword (acc[4k + q] -> byte k), four such dwords shifted by q land in distinct bits,
// and the half-waves interleave by 4. The basis rows are laid out so that this gather IS the
// CRC bit order (row R of the MFMA carries CRC bit R ^ 7, see upload_crc_tables): 17 VALU
// per pass instead of one extract-and-insert pair per accumulator.
__device__ __forceinline__ uint32_t wave_chunk_crcs(const i32x4 (&A)[16], const WaveData& d, int lane) {
  const int h = lane >> 5;
  uint32_t mine = 0;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const uint4 w0 = d.v[2 * it], w1 = d.v[2 * it + 1];
    const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    i32x16 acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const uint32_t x = w[s >> 1];
      const uint32_t m = 0x01010101u << (4 * (s & 1));
      i32x4 b;
      b.x = static_cast<int>(x & m);
      b.y = static_cast<int>(x & (m << 1));
      b.z = static_cast<int>(x & (m << 2));
      b.w = static_cast<int>(x & (m << 3));
      acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], b, acc, 0, 0, 0);
    }
    uint32_t part = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = __builtin_amdgcn_perm(static_cast<uint32_t>(acc[4 + q]), static_cast<uint32_t>(acc[q]), 0x0c0c0400u);
      const uint32_t hi = __builtin_amdgcn_perm(static_cast<uint32_t>(acc[12 + q]), static_cast<uint32_t>(acc[8 + q]),
                                                0x0c0c0400u);
      part |= __builtin_amdgcn_perm(hi, lo, 0x05040100u) >> q;  // bit 7 + 8k - q: acc[4k + q]
    }
    part >>= 4 * h;
    part = xr32(part);  // the half-waves' bits are disjoint: XOR = OR
    if (it == h) mine = part;  // lane L keeps chunk L: it comes out of pass L >> 5
  }
  return mine;
}

// The same chunk CRCs on the FP4 matrix cores. v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1
// operands (unit block scales) takes 64 K per instruction at the cycles of the i8 32x32x32, so a
// 64 B chunk is 8 instructions instead of 16 and the basis 32 VGPRs instead of 64:
//  * B: one data dword x gives the whole 32-element fragment: x & 0x11111111 (each nibble 0 or
//    0b0001 = 0.5), x & 0x22222222 (0 or 1.0), x & 0x44444444 (0 or 2.0) and
//    (x >> 1) & 0x44444444 (bit 3 of each nibble; 0 or 2.0; bit 3 itself is the sign).
//  * A: 2.0 / 1.0 / 0.5 / 0.5 where the basis bit is set, so every product of two set bits is
//    exactly 1.0 and the f32 accumulator counts them (at most 512 per pass: exact).
//  * The accumulators start at 65536 = 2^16: in [2^16, 2^17) one ulp is 2^-7, so the count's
//    bit 0 — the parity — is bit 7 of the float's encoding and bits 0..6 are 0. The low byte is
//    0x80 or 0, exactly what the i8 form's gather expects.
using i32x8 = __attribute__((ext_vector_type(8))) int;
using f32x16 = __attribute__((ext_vector_type(16))) float;

__device__ __forceinline__ uint32_t wave_chunk_crcs_fp4(const i32x4 (&A)[8], const WaveData& d, int lane) {
  const int h = lane >> 5;
  uint32_t mine = 0;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const uint4 w0 = d.v[2 * it], w1 = d.v[2 * it + 1];
    const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 65536.0f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const uint32_t x = w[s];
      const i32x8 b = {static_cast<int>(x & 0x11111111u), static_cast<int>(x & 0x22222222u),
                       static_cast<int>(x & 0x44444444u), static_cast<int>((x >> 1) & 0x44444444u), 0, 0, 0, 0};
      const i32x8 a = {A[s].x, A[s].y, A[s].z, A[s].w, 0, 0, 0, 0};
      acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, acc, 4, 4, 0, 127, 0, 127);
    }
    uint32_t part = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(acc[4 + q]), __float_as_uint(acc[q]), 0x0c0c0400u);
      const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(acc[12 + q]), __float_as_uint(acc[8 + q]), 0x0c0c0400u);
      part |= __builtin_amdgcn_perm(hi, lo, 0x05040100u) >> q;
    }
    part >>= 4 * h;
    part = xr32(part);
    if (it == h) mine = part;
  }
  return mine;
}

// The basis of either form in VGPRs, loaded from the uploaded image (kernels that keep no LDS copy).
template <bool kFp4>
struct ChunkBasis {
  static constexpr int kFrags = kFp4 ? 8 : 16;
  i32x4 A[kFrags];
  __device__ __forceinline__ void load(const DevCrcTables* __restrict__ gt, int lane) {
    const i32x4* p = reinterpret_cast<const i32x4*>(reinterpret_cast<const uint8_t*>(gt + 1) +
                                                    (kFp4 ? kCrcBasisFp4Offset : 0));
#pragma unroll
    for (int s = 0; s < kFrags; ++s) A[s] = p[s * 64 + lane];
  }
  __device__ __forceinline__ uint32_t crcs(const WaveData& d, int lane) const {
    if constexpr (kFp4) return wave_chunk_crcs_fp4(A, d, lane);
    else return wave_chunk_crcs(A, d, lane);
  }
};

// Chunk CRCs -> slice CRC in one lookup round: lane sl of a slice's 8-lane group moves its
// chunk CRC past the 64 * (7 - sl) bytes that follow the chunk in the slice (one tab4 into
// its own shift table; sl == 7 needs none) and three xor-shuffles fold the group, since the
// raw CRC of a concatenation is the XOR of the shifted parts. Every lane of the group ends
// with the slice CRC. (The butterfly it replaces did three dependent tab4 rounds — 12 LDS
// lookups per lane, the kernels' only bank conflicts — for the same result.)
template <class L>
__device__ __forceinline__ uint32_t slice_from_chunks(const L& lt, uint32_t r, int lane) {
  const int sl = lane & 7;
  uint32_t v = sl < 7 ? tab4(lt.cs[sl], r) : r;
  return xr4(xr2(xr1(v)));
}

// LDS images of the matrix-core kernels: only the GF(2) shift tables they look up (the
// slicing-by-16 tables of the table kernels are not needed: short tail slices go through
// the MFMA path front-padded with zeros). `cs` comes from the chunk-shift tables stored
// behind the MFMA basis, the tile part is the suffix of DevCrcTables from sh512 on.
struct MfmaSliceLds {  // K1b, fused K3: chunk -> slice combine (28 KiB)
  uint32_t cs[7][4][256];
};
struct MfmaTileLds {  // K1/K2/K3: + slice -> sub-tile combine and the tile shifts (48 KiB)
  uint32_t cs[7][4][256];
  uint32_t sh512[4][256], sh1k[4][256], sh2k[4][256];
  uint32_t sh4k[4][256];
  uint32_t tile_pow2[32][32];
};
static_assert(sizeof(MfmaSliceLds) == kCrcChunkShiftBytes, "chunk-shift image");
static_assert(sizeof(MfmaTileLds) - sizeof(MfmaSliceLds) == sizeof(DevCrcTables) - offsetof(DevCrcTables, sh512),
              "LDS image layout");

template <int kThreads = kCrcWgThreads>
__device__ __forceinline__ void copy16(const void* __restrict__ from, void* to, int bytes) {
  const uint4* src = reinterpret_cast<const uint4*>(from);
  uint4* dst = reinterpret_cast<uint4*>(to);
  const int n16 = bytes / 16;
#pragma unroll 4
  for (int i = threadIdx.x; i < n16; i += kThreads) dst[i] = src[i];
}

// The same copy by LDS-DMA (global_load_lds_dwordx4: each wave instruction moves 1 KiB straight
// into LDS, no VGPRs, no wait before the next one), so a kernel's whole LDS image is in flight at
// once instead of one register round trip per pass. The destination of one instruction is
// wave-uniform base + 16 x lane, which a linear copy is. bytes % 16 == 0; completes at the next
// __syncthreads() (its vmcnt(0)).
template <int kThreads>
__device__ __forceinline__ void dma16(const void* __restrict__ from, void* to, int bytes) {
  using LdsPtr = __attribute__((address_space(3))) void*;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(from);
  uint8_t* dst = reinterpret_cast<uint8_t*>(to);
  for (int base = wave * 1024; base < bytes; base += kThreads * 16)
    if (base + lane * 16 < bytes)
      __builtin_amdgcn_global_load_lds(src + base + lane * 16, (LdsPtr)(dst + base), 16, 0, 0);
}

template <class L, int kThreads = kCrcWgThreads>
__device__ __forceinline__ void load_lds_image(const DevCrcTables* __restrict__ gt, L* lt) {
  const uint8_t* cs = reinterpret_cast<const uint8_t*>(gt + 1) + kCrcBasisBytes;
  copy16<kThreads>(cs, lt, kCrcChunkShiftBytes);
  if constexpr (sizeof(L) > kCrcChunkShiftBytes)
    copy16<kThreads>(&gt->sh512, reinterpret_cast<uint8_t*>(lt) + kCrcChunkShiftBytes,
                     static_cast<int>(sizeof(L)) - kCrcChunkShiftBytes);
}

// The short tail slice (len < 512 bytes at `base`) as slice 0 of a wave's 4 KiB, front-padded
// with zeros to 512 B (the raw CRC ignores leading zeros); every other slice reads as zeros.
// Byte loads: it runs once per block.
__device__ __forceinline__ WaveData load_tail_wave(const uint8_t* __restrict__ base, uint32_t len, int lane) {
  const int n = lane & 31, h = lane >> 5;
  WaveData d;
#pragma unroll
  for (int k = 0; k < 4; ++k) d.v[k] = make_uint4(0, 0, 0, 0);
  if (n < 8) {
    const int pad = 512 - static_cast<int>(len);
    uint32_t w[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t v = 0;
      for (int b = 0; b < 4; ++b) {
        const int pos = n * 64 + h * 32 + q * 4 + b;
        v |= (pos >= pad ? static_cast<uint32_t>(base[pos - pad]) : 0u) << (8 * b);
      }
      w[q] = v;
    }
    d.v[0] = make_uint4(w[0], w[1], w[2], w[3]);
    d.v[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
  return d;
}

// Short slice of `len` bytes, front-padded with zeros to 512 B (wave-wide call, lanes 0..7 work).
__device__ __forceinline__ uint32_t tail_crc(const DevCrcTables& lt, const uint8_t* base, uint32_t len, int lane) {
  const int sw = lane >> 3, sl = lane & 7;
  const uint32_t pad = 512u - len;
  uint32_t r = 0;
  if (sw == 0) {
    uint32_t words[16];
    for (int q = 0; q < 16; ++q) {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) {
        uint32_t pos = sl * 64 + q * 4 + b;
        uint32_t byte = pos >= pad ? base[pos - pad] : 0u;
        w |= byte << (8 * b);
      }
      words[q] = w;
    }
    for (int q = 0; q < 4; ++q)
      r = chunk16(lt.slice16, r, make_uint4(words[4 * q], words[4 * q + 1], words[4 * q + 2], words[4 * q + 3]));
  }
  r = combine<1>(r, lane, lt.sh64);
  r = combine<2>(r, lane, lt.sh128);
  return combine<4>(r, lane, lt.sh256);
}

// Contiguous, balanced tile runs: workgroup b owns [b*T/G, (b+1)*T/G), so every workgroup
// gets floor or ceil of T/G tiles. (A ceil-sized split gave 64 MiB = 4096 tiles over 768
// workgroups as 683 runs of 6 — some CUs 18 tiles, others 12 — and left 85 slots idle.)
__device__ __forceinline__ uint64_t tile_run_begin(uint64_t ntiles, uint64_t b) {
  return b * ntiles / gridDim.x;
}

// LDS slicing-by-16 implementation (DFS_CRC_MFMA=0; the A/B baseline of crc_bench).
__global__ __launch_bounds__(kCrcWgThreads) void crc_slices_kernel(CrcLaunch a,
                                                                   const DevCrcTables* __restrict__ gt) {
  __shared__ DevCrcTables lt;
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t wg_bad;
  load_tables(gt, &lt);
  if (threadIdx.x == 0) wg_bad = 0xFFFFFFFFu;
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int sw = lane >> 3;   // slice within wave
  const int sl = lane & 7;    // 64 B sub-chunk within slice
  uint32_t acc = 0;
  uint32_t bad = 0xFFFFFFFFu;

  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    int64_t v = static_cast<int64_t>(t * kSlicesPerTile + wave * 8 + sw);
    int64_t i = static_cast<int64_t>(a.slice_lo) + v - static_cast<int64_t>(a.vfront);
    bool valid = i >= static_cast<int64_t>(a.slice_lo) && i < static_cast<int64_t>(a.slice_hi);
    uint32_t r = slice_crc(lt, a.data + (valid ? static_cast<uint64_t>(i) * 512 : 0), sl, lane, valid);
    if (valid && sl == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.full_init);
      if (a.meta_out) a.meta_out[i] = be;
      if (a.meta_host) a.meta_host[i] = be;
      if (a.meta_expect && a.meta_expect[i] != be) bad = min(bad, static_cast<uint32_t>(i));
    }
    if (a.part_crc) {
      r = combine<8>(r, lane, lt.sh512);
      r = combine<16>(r, lane, lt.sh1k);
      r = combine<32>(r, lane, lt.sh2k);
      if (lane == 0) wsum[wave] = r;
      __syncthreads();
      if (wave == 0) {
        uint32_t tv = wsum[0];
        tv = tab4(lt.sh4k, tv) ^ wsum[1];
        tv = tab4(lt.sh4k, tv) ^ wsum[2];
        tv = tab4(lt.sh4k, tv) ^ wsum[3];
        uint64_t e = a.ntiles - 1 - t;  // tiles that follow this one
        for (int b = 0; e; ++b, e >>= 1)
          if (e & 1) tv = mat_apply(lt.tile_pow2[b], tv, lane);
        acc ^= tv;
      }
      __syncthreads();
    }
  }

  // Short tail slice: front-pad the window with zeros (raw CRC is invariant to them).
  if (a.has_tail && blockIdx.x == 0 && wave == 0) {
    uint32_t r = tail_crc(lt, a.data + a.s_full * 512, a.tail_len, lane);
    if (lane == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.tail_init);
      if (a.meta_out) a.meta_out[a.s_full] = be;
      if (a.meta_host) a.meta_host[a.s_full] = be;
      if (a.meta_expect && a.meta_expect[a.s_full] != be) bad = min(bad, static_cast<uint32_t>(a.s_full));
    }
  }

  if (a.part_bad && bad != 0xFFFFFFFFu) atomicMin(&wg_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.part_crc) a.part_crc[blockIdx.x] = acc;
    if (a.part_bad) a.part_bad[blockIdx.x] = wg_bad;
  }
}

// ---------------------------------------------------------------------------------------
// K1b: batched scrub over many blocks in one launch (see ScrubLaunch).
__global__ __launch_bounds__(kCrcWgThreads) void crc_scrub_kernel(ScrubLaunch a, const DevCrcTables* __restrict__ gt) {
  __shared__ DevCrcTables lt;
  load_tables(gt, &lt);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int sw = lane >> 3, sl = lane & 7;
  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    // last block whose tile range starts at or before t (workgroup-uniform)
    uint32_t lo = 0, hi = a.nblocks;
    while (hi - lo > 1) {
      uint32_t mid = (lo + hi) >> 1;
      if (a.blocks[mid].tile_start <= t) lo = mid;
      else hi = mid;
    }
    const ScrubBlock& b = a.blocks[lo];
    uint64_t i = (t - b.tile_start) * kSlicesPerTile + wave * 8 + sw;
    bool valid = i < b.s_full;
    uint32_t r = slice_crc(lt, b.data + (valid ? i * 512 : 0), sl, lane, valid);
    if (valid && sl == 0 && b.meta[i] != __builtin_bswap32(r ^ a.full_init))
      atomicMin(&a.bad[lo], static_cast<uint32_t>(i));
  }
  // short tail slices: one wave per block
  const int waves = kCrcWgThreads / 64;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * waves + wave; k < a.nblocks;
       k += static_cast<uint64_t>(gridDim.x) * waves) {
    const ScrubBlock& b = a.blocks[k];
    if (!b.tail_len) continue;
    uint32_t r = tail_crc(lt, b.data + b.s_full * 512, b.tail_len, lane);
    if (lane == 0 && b.meta[b.s_full] != __builtin_bswap32(r ^ b.tail_init))
      atomicMin(&a.bad[k], static_cast<uint32_t>(b.s_full));
  }
}

// ---------------------------------------------------------------------------------------
// K1/K2/K3 on the matrix cores (default). Each workgroup owns a CONTIGUOUS run of 16 KiB
// tiles; each wave owns one 4 KiB sub-tile per tile and runs its own Horner accumulator for
// the whole-block CRC (consecutive sub-tiles of a wave are exactly one tile apart, so one
// lane-parallel GF(2) shift per tile) — no barrier inside the tile loop. The next tile's
// data is loaded while the current one is on the matrix cores, and the first tile's loads
// are issued before the LDS table fill, so a 1 MiB block costs one memory round trip.
// 3 waves/SIMD (168 VGPRs: the 64-VGPR basis + double-buffered data, no spills) x 4 SIMDs =
// 3 workgroups per CU, which their 32 KiB LDS images allow; the grid is sized to exactly one
// resident round (kMaxGridCrc = 3 x 256 CUs), so no second, partly empty round.
__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void crc_tile_mfma_kernel(CrcLaunch a,
                                                                      const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaTileLds lt;
  __shared__ uint32_t wacc[4];
  __shared__ uint32_t wg_bad;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(a.ntiles, blockIdx.x), t_end = tile_run_begin(a.ntiles, blockIdx.x + 1);
  const int64_t lo = static_cast<int64_t>(a.slice_lo), hi = static_cast<int64_t>(a.slice_hi);
  auto first_slice = [&](uint64_t t) {
    return lo + static_cast<int64_t>(t * kSlicesPerTile + wave * 8) - static_cast<int64_t>(a.vfront);
  };
  WaveData cur;
  if (t_begin < t_end) cur = load_wave(a.data, first_slice(t_begin), lo, hi, lane);
  i32x4 A[16];
  load_basis(reinterpret_cast<const i32x4*>(gt + 1), lane, A);
  load_lds_image(gt, &lt);
  if (threadIdx.x == 0) wg_bad = 0xFFFFFFFFu;
  __syncthreads();

  uint32_t acc = 0;
  uint32_t bad = 0xFFFFFFFFu;
  for (uint64_t t = t_begin; t < t_end; ++t) {
    WaveData nxt;
    if (t + 1 < t_end) nxt = load_wave(a.data, first_slice(t + 1), lo, hi, lane);
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, cur, lane), lane);
    const int64_t i = first_slice(t) + sw;
    if (i >= lo && i < hi && sl == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.full_init);
      if (a.meta_out) a.meta_out[i] = be;
      if (a.meta_expect && a.meta_expect[i] != be) bad = min(bad, static_cast<uint32_t>(i));
    }
    if (a.part_crc) {
      r = combine<8>(r, lane, lt.sh512);
      r = combine<16>(r, lane, lt.sh1k);
      r = combine<32>(r, lane, lt.sh2k);  // wave-uniform: the 4 KiB sub-tile's raw CRC
      acc = mat_apply(lt.tile_pow2[0], acc, lane) ^ r;
    }
    if (t + 1 < t_end) cur = nxt;
  }

  if (a.has_tail && blockIdx.x == 0 && wave == 0) {
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, load_tail_wave(a.data + a.s_full * 512, a.tail_len, lane),
                                                       lane), lane);
    if (lane == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.tail_init);
      if (a.meta_out) a.meta_out[a.s_full] = be;
      if (a.meta_expect && a.meta_expect[a.s_full] != be) bad = min(bad, static_cast<uint32_t>(a.s_full));
    }
  }
  if (a.part_crc) {
    // place this wave's accumulator in the block: (3 - wave) sub-tiles of its last tile
    // and (ntiles - t_end) whole tiles follow it
    for (int k = wave; k < 3; ++k) acc = tab4(lt.sh4k, acc);
    uint64_t e = t_begin < t_end ? a.ntiles - t_end : 0;
    for (int b = 0; e; ++b, e >>= 1)
      if (e & 1) acc = mat_apply(lt.tile_pow2[b], acc, lane);
    if (lane == 0) wacc[wave] = acc;
  }
  if (a.part_bad && bad != 0xFFFFFFFFu) atomicMin(&wg_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.part_crc) a.part_crc[blockIdx.x] = wacc[0] ^ wacc[1] ^ wacc[2] ^ wacc[3];
    if (a.part_bad) a.part_bad[blockIdx.x] = wg_bad;
  }
}

// K1/K2 with one workgroup per CU: kGroups groups of 4 waves share one LDS image and one
// LDS copy of the MFMA basis. Each group is a "virtual workgroup" of the kernel above (its own
// balanced tile run, partial word and verdict: part_crc/part_bad are indexed by
// blockIdx.x * kGroups + group, so the host sees the same `grid` words). The per-tile combine
// is two dependent table rounds instead of five: every lane of a slice group moves its slice
// CRC to the end of the wave's 4 KiB with one lookup in its own shift table (ss[sw], the
// slice-level twin of slice_from_chunks) and three xor-shuffles fold the sub-tile; the Horner
// step is one lookup in the 16 KiB shift table (all lanes the same value: an LDS broadcast)
// instead of a lane-parallel matrix apply with five shuffles. The image (68 KiB) only fits
// one workgroup per CU, which is what this kernel is.
struct MfmaWideLds {
  uint32_t cs[7][4][256];  // chunk -> slice (64 B * (7 - sl))
  uint32_t ss[7][4][256];  // slice -> sub-tile (512 B * (7 - sw))
  uint32_t sh16k[4][256];  // one tile
  uint32_t sh4k[4][256];   // one sub-tile (epilogue)
  uint32_t tile_pow2[32][32];
};
static_assert(offsetof(MfmaWideLds, sh4k) == kCrcChunkShiftBytes + kCrcWideExtraBytes, "wide image: contiguous head");
static_assert(sizeof(MfmaWideLds) - offsetof(MfmaWideLds, sh4k) == sizeof(DevCrcTables) - offsetof(DevCrcTables, sh4k),
              "wide image: DevCrcTables tail");

// kWrite: the K1/K2 write form (slice words out, whole-block partials, nothing to verify),
// with those checks resolved at compile time so the loop body has no uniform branches.
// kFp4: the chunk CRCs on the FP4 matrix cores (wave_chunk_crcs_fp4), else i8.
template <int kGroups, bool kWrite, bool kFp4 = false>
__global__ __launch_bounds__(kCrcWgThreads * kGroups) __attribute__((amdgpu_waves_per_eu(kGroups, kGroups)))
void crc_tile_wide_kernel(CrcLaunch a, const DevCrcTables* __restrict__ gt) {
  constexpr int kThreads = kCrcWgThreads * kGroups;
  constexpr int kFrags = kFp4 ? 8 : 16;  // A fragments per lane
  __shared__ __attribute__((aligned(16))) MfmaWideLds lt;
  __shared__ i32x4 lbasis[kFrags * 64];
  __shared__ uint32_t wacc[4 * kGroups];
  __shared__ uint32_t wg_bad[kGroups];
  const int lane = threadIdx.x & 63, gw = threadIdx.x >> 6, wave = gw & 3, grp = gw >> 2, sw = lane >> 3,
            sl = lane & 7;
  const uint64_t vb = static_cast<uint64_t>(blockIdx.x) * kGroups + grp, vg = static_cast<uint64_t>(gridDim.x) * kGroups;
  const uint64_t t_begin = vb * a.ntiles / vg, t_end = (vb + 1) * a.ntiles / vg;
  const int64_t lo = static_cast<int64_t>(a.slice_lo), hi = static_cast<int64_t>(a.slice_hi);
  auto first_slice = [&](uint64_t t) {
    return lo + static_cast<int64_t>(t * kSlicesPerTile + wave * 8) - static_cast<int64_t>(a.vfront);
  };
  // unconditional loads (load_wave_ring: out-of-block slices re-read slice lo, and their chunk
  // CRCs are zeroed below), so no exec-masked branches around the loads in the loop
  WaveData cur;
  const uint8_t* img = reinterpret_cast<const uint8_t*>(gt + 1);
  if constexpr (kFp4) {
    // the LDS image and basis by LDS-DMA, all in flight together with the first tile's loads
    dma16<kThreads>(img + kCrcBasisFp4Offset, lbasis, kCrcBasisFp4Bytes);
    dma16<kThreads>(img + kCrcBasisBytes, &lt, kCrcChunkShiftBytes + kCrcWideExtraBytes);
    dma16<kThreads>(&gt->sh4k, &lt.sh4k, static_cast<int>(sizeof(DevCrcTables) - offsetof(DevCrcTables, sh4k)));
    if (t_begin < t_end) cur = load_wave_ring(a.data, first_slice(t_begin), lo, hi, lane);
  } else {
    if (t_begin < t_end) cur = load_wave_ring(a.data, first_slice(t_begin), lo, hi, lane);
    copy16<kThreads>(img, lbasis, kCrcBasisBytes);
    copy16<kThreads>(img + kCrcBasisBytes, &lt, kCrcChunkShiftBytes + kCrcWideExtraBytes);
    copy16<kThreads>(&gt->sh4k, &lt.sh4k, static_cast<int>(sizeof(DevCrcTables) - offsetof(DevCrcTables, sh4k)));
  }
  if (threadIdx.x < kGroups) wg_bad[threadIdx.x] = 0xFFFFFFFFu;
  __syncthreads();
  i32x4 A[kFrags];
#pragma unroll
  for (int s = 0; s < kFrags; ++s) A[s] = lbasis[s * 64 + lane];
  auto chunk_crcs = [&](const WaveData& d) {
    if constexpr (kFp4) return wave_chunk_crcs_fp4(A, d, lane);
    else return wave_chunk_crcs(A, d, lane);
  };

  uint32_t acc = 0;
  uint32_t bad = 0xFFFFFFFFu;
  // tile t's combine (table lookups and shuffles: a latency chain) is issued after tile t+1's
  // matrix-core work, so each wave has independent MFMAs to issue while its lookups are out
  auto finish = [&](uint32_t c, uint64_t t) {
    const int64_t i = first_slice(t) + sw;
    const bool valid = i >= lo && i < hi;
    uint32_t r = slice_from_chunks(lt, valid ? c : 0u, lane);
    if (valid && sl == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.full_init);
      if (kWrite || a.meta_out) a.meta_out[i] = be;
      if (!kWrite && a.meta_expect && a.meta_expect[i] != be) bad = min(bad, static_cast<uint32_t>(i));
    }
    if (kWrite || a.part_crc) {
      uint32_t v = sw < 7 ? tab4(lt.ss[sw], r) : r;
      v = xr32(xr16(xr8(v)));  // wave-uniform: the 4 KiB sub-tile's raw CRC
      acc = tab4(lt.sh16k, acc) ^ v;
    }
  };
  uint32_t cprev = 0;
  for (uint64_t t = t_begin; t < t_end; ++t) {
    WaveData nxt;
    if (t + 1 < t_end) nxt = load_wave_ring(a.data, first_slice(t + 1), lo, hi, lane);
    const uint32_t c = chunk_crcs(cur);
    if (t > t_begin) finish(cprev, t - 1);
    cprev = c;
    if (t + 1 < t_end) cur = nxt;
  }
  if (t_begin < t_end) finish(cprev, t_end - 1);

  if (a.has_tail && vb == 0 && wave == 0) {
    uint32_t r = slice_from_chunks(lt, chunk_crcs(load_tail_wave(a.data + a.s_full * 512, a.tail_len, lane)), lane);
    if (lane == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.tail_init);
      if (a.meta_out) a.meta_out[a.s_full] = be;
      if (a.meta_expect && a.meta_expect[a.s_full] != be) bad = min(bad, static_cast<uint32_t>(a.s_full));
    }
  }
  if (a.part_crc) {
    for (int k = wave; k < 3; ++k) acc = tab4(lt.sh4k, acc);
    uint64_t e = t_begin < t_end ? a.ntiles - t_end : 0;
    for (int b = 0; e; ++b, e >>= 1)
      if (e & 1) acc = mat_apply(lt.tile_pow2[b], acc, lane);
    if (lane == 0) wacc[gw] = acc;
  }
  if (a.part_bad && bad != 0xFFFFFFFFu) atomicMin(&wg_bad[grp], bad);
  __syncthreads();
  if (threadIdx.x < kGroups) {
    const int g = threadIdx.x;
    const uint64_t v = static_cast<uint64_t>(blockIdx.x) * kGroups + g;
    if (a.part_crc) a.part_crc[v] = wacc[4 * g] ^ wacc[4 * g + 1] ^ wacc[4 * g + 2] ^ wacc[4 * g + 3];
    if (a.part_bad) a.part_bad[v] = wg_bad[g];
  }
}

// K3 fused: verify AND deliver a read in one pass over HBM. The data the MFMA chunk CRC
// already holds in registers is stored straight to the reader's buffer — host memory that
// the store registered (the client's shared-memory slot), so the stores cross PCIe from the
// CUs — instead of a verify kernel followed by an SDMA copy that reads the same bytes from
// HBM again, plus a second small copy for the verdict. Only bytes inside [off, off + len)
// are stored; the verdict per workgroup goes to host-visible memory too, so one kernel and
// one stream sync make the whole read. The host guarantees (out - off) % 16 == 0.
// Bytes of lane segment `q` (0..7, dwords of the lane's 32 B) of iteration `it`.
__device__ __forceinline__ uint32_t seg_dword(const WaveData& d, int it, int q) {
  const uint4 v = d.v[2 * it + (q >> 2)];
  const int k = q & 3;
  return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}

__device__ __forceinline__ void store_wave(const ReadCopyLaunch& a, int64_t i0, const WaveData& d, int lane) {
  const int n = lane & 31, h = lane >> 5;
  const int64_t lo = static_cast<int64_t>(a.c.slice_lo), hi = static_cast<int64_t>(a.c.slice_hi);
  const uint64_t end = a.off + a.len;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = it * 32 + n;
    const int64_t i = i0 + (c >> 3);
    if (i < lo || i >= hi) continue;
    const uint64_t pos = static_cast<uint64_t>(i) * 512 + (c & 7) * 64 + h * 32;
    if (pos >= a.off && pos + 32 <= end) {
      uint4* dst = reinterpret_cast<uint4*>(a.out + (pos - a.off));
      dst[0] = d.v[2 * it];
      dst[1] = d.v[2 * it + 1];
    } else if (pos + 32 > a.off && pos < end) {  // the range's first / last 32 B
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint32_t w = seg_dword(d, it, q);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint64_t p = pos + 4 * q + b;
          if (p >= a.off && p < end) a.out[p - a.off] = static_cast<uint8_t>(w >> (8 * b));
        }
      }
    }
  }
}

__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void crc_read_copy_kernel(
    ReadCopyLaunch a, const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaSliceLds lt;
  __shared__ uint32_t wg_bad;
  const CrcLaunch& c = a.c;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(c.ntiles, blockIdx.x), t_end = tile_run_begin(c.ntiles, blockIdx.x + 1);
  const int64_t lo = static_cast<int64_t>(c.slice_lo), hi = static_cast<int64_t>(c.slice_hi);
  auto first_slice = [&](uint64_t t) { return lo + static_cast<int64_t>(t * kSlicesPerTile + wave * 8); };
  WaveData cur;
  if (t_begin < t_end) cur = load_wave(c.data, first_slice(t_begin), lo, hi, lane);
  i32x4 A[16];
  load_basis(reinterpret_cast<const i32x4*>(gt + 1), lane, A);
  load_lds_image(gt, &lt);
  if (threadIdx.x == 0) wg_bad = 0xFFFFFFFFu;
  __syncthreads();

  uint32_t bad = 0xFFFFFFFFu;
  for (uint64_t t = t_begin; t < t_end; ++t) {
    WaveData nxt;
    if (t + 1 < t_end) nxt = load_wave(c.data, first_slice(t + 1), lo, hi, lane);
    const int64_t i0 = first_slice(t);
    store_wave(a, i0, cur, lane);
    const uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, cur, lane), lane);
    const int64_t i = i0 + sw;
    if (i >= lo && i < hi && sl == 0 && c.meta_expect[i] != __builtin_bswap32(r ^ c.full_init))
      bad = min(bad, static_cast<uint32_t>(i));
    if (t + 1 < t_end) cur = nxt;
  }

  if (c.has_tail && blockIdx.x == 0 && wave == 0) {
    const uint8_t* base = c.data + c.s_full * 512;
    const uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, load_tail_wave(base, c.tail_len, lane), lane), lane);
    if (lane == 0 && c.meta_expect[c.s_full] != __builtin_bswap32(r ^ c.tail_init))
      bad = min(bad, static_cast<uint32_t>(c.s_full));
    const uint64_t p0 = c.s_full * 512, end = a.off + a.len;
    for (uint32_t k = lane; k < c.tail_len; k += 64) {
      const uint64_t p = p0 + k;
      if (p >= a.off && p < end) a.out[p - a.off] = base[k];
    }
  }
  if (bad != 0xFFFFFFFFu) atomicMin(&wg_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) a.part_bad[blockIdx.x] = wg_bad;
}

// K1/K2 fused with the host-to-device copy of a write (the mirror of crc_read_copy_kernel):
// the waves load the block straight from the writer's registered host slot over PCIe, store
// it into the HBM extent, checksum the registers they already hold on the matrix cores, and
// write the .meta image both next to the block in HBM and into host-visible memory together
// with the whole-block partials — one kernel and one stream sync instead of an SDMA copy,
// the checksum kernel and two device-to-host copies (the .meta image and the partials).
__device__ __forceinline__ void store_wave_dst(uint8_t* __restrict__ dst, int64_t i0, int64_t lo, int64_t hi,
                                               const WaveData& d, int lane) {
  const int n = lane & 31, h = lane >> 5;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = it * 32 + n;
    const int64_t i = i0 + (c >> 3);
    if (i < lo || i >= hi) continue;
    uint4* p = reinterpret_cast<uint4*>(dst + static_cast<uint64_t>(i) * 512 + (c & 7) * 64 + h * 32);
    p[0] = d.v[2 * it];
    p[1] = d.v[2 * it + 1];
  }
}

__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void crc_write_copy_kernel(
    WriteCopyLaunch a, const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaTileLds lt;
  __shared__ uint32_t wacc[4];
  const CrcLaunch& c = a.c;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(c.ntiles, blockIdx.x), t_end = tile_run_begin(c.ntiles, blockIdx.x + 1);
  const int64_t lo = static_cast<int64_t>(c.slice_lo), hi = static_cast<int64_t>(c.slice_hi);
  auto first_slice = [&](uint64_t t) {
    return lo + static_cast<int64_t>(t * kSlicesPerTile + wave * 8) - static_cast<int64_t>(c.vfront);
  };
  WaveData cur;
  if (t_begin < t_end) cur = load_wave(c.data, first_slice(t_begin), lo, hi, lane);  // PCIe latency first
  i32x4 A[16];
  load_basis(reinterpret_cast<const i32x4*>(gt + 1), lane, A);
  load_lds_image(gt, &lt);
  __syncthreads();

  uint32_t acc = 0;
  for (uint64_t t = t_begin; t < t_end; ++t) {
    WaveData nxt;
    if (t + 1 < t_end) nxt = load_wave(c.data, first_slice(t + 1), lo, hi, lane);
    const int64_t i0 = first_slice(t);
    store_wave_dst(a.dst, i0, lo, hi, cur, lane);
    if (a.dst_host) store_wave_dst(a.dst_host, i0, lo, hi, cur, lane);
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, cur, lane), lane);
    const int64_t i = i0 + sw;
    if (i >= lo && i < hi && sl == 0) {
      const uint32_t be = __builtin_bswap32(r ^ c.full_init);
      c.meta_out[i] = be;
      a.meta_host[i] = be;
    }
    r = combine<8>(r, lane, lt.sh512);
    r = combine<16>(r, lane, lt.sh1k);
    r = combine<32>(r, lane, lt.sh2k);
    acc = mat_apply(lt.tile_pow2[0], acc, lane) ^ r;
    if (t + 1 < t_end) cur = nxt;
  }

  if (c.has_tail && blockIdx.x == 0 && wave == 0) {
    const uint8_t* base = c.data + c.s_full * 512;
    const uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, load_tail_wave(base, c.tail_len, lane), lane), lane);
    if (lane == 0) {
      const uint32_t be = __builtin_bswap32(r ^ c.tail_init);
      c.meta_out[c.s_full] = be;
      a.meta_host[c.s_full] = be;
    }
    uint8_t* out = a.dst + c.s_full * 512;
    uint8_t* hout = a.dst_host ? a.dst_host + c.s_full * 512 : nullptr;
    for (uint32_t k = lane; k < c.tail_len; k += 64) {
      out[k] = base[k];
      if (hout) hout[k] = base[k];
    }
  }
  for (int k = wave; k < 3; ++k) acc = tab4(lt.sh4k, acc);
  uint64_t e = t_begin < t_end ? c.ntiles - t_end : 0;
  for (int b = 0; e; ++b, e >>= 1)
    if (e & 1) acc = mat_apply(lt.tile_pow2[b], acc, lane);
  if (lane == 0) wacc[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) c.part_crc[blockIdx.x] = wacc[0] ^ wacc[1] ^ wacc[2] ^ wacc[3];
}

// K1b on the matrix cores: contiguous tile runs per workgroup, so the tile -> block lookup is
// one binary search per workgroup and then a forward walk, and the next tile's data (and its
// block) are fetched while the current tile computes.
__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(3, 3))) void crc_scrub_mfma_kernel(ScrubLaunch a,
                                                                       const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaSliceLds lt;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(a.ntiles, blockIdx.x), t_end = tile_run_begin(a.ntiles, blockIdx.x + 1);
  uint32_t blk = 0;
  if (t_begin < t_end) {
    uint32_t l = 0, h = a.nblocks;
    while (h - l > 1) {
      uint32_t mid = (l + h) >> 1;
      if (a.blocks[mid].tile_start <= t_begin) l = mid;
      else h = mid;
    }
    blk = l;
  }
  auto advance = [&](uint64_t t, uint32_t b) {
    while (b + 1 < a.nblocks && a.blocks[b + 1].tile_start <= t) ++b;
    return b;
  };
  auto first_slice = [&](uint64_t t, uint32_t b) {
    return static_cast<int64_t>((t - a.blocks[b].tile_start) * kSlicesPerTile + wave * 8);
  };
  WaveData cur;
  if (t_begin < t_end)
    cur = load_wave(a.blocks[blk].data, first_slice(t_begin, blk), 0, static_cast<int64_t>(a.blocks[blk].s_full), lane);
  i32x4 A[16];
  load_basis(reinterpret_cast<const i32x4*>(gt + 1), lane, A);
  load_lds_image(gt, &lt);
  __syncthreads();
  for (uint64_t t = t_begin; t < t_end; ++t) {
    WaveData nxt;
    uint32_t nb = blk;
    if (t + 1 < t_end) {
      nb = advance(t + 1, blk);
      nxt = load_wave(a.blocks[nb].data, first_slice(t + 1, nb), 0, static_cast<int64_t>(a.blocks[nb].s_full), lane);
    }
    const ScrubBlock& b = a.blocks[blk];
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, cur, lane), lane);
    const int64_t i = first_slice(t, blk) + sw;
    if (sl == 0 && i < static_cast<int64_t>(b.s_full) && b.meta[i] != __builtin_bswap32(r ^ a.full_init))
      atomicMin(&a.bad[blk], static_cast<uint32_t>(i));
    if (t + 1 < t_end) {
      cur = nxt;
      blk = nb;
    }
  }
  const int waves = kCrcWgThreads / 64;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * waves + wave; k < a.nblocks;
       k += static_cast<uint64_t>(gridDim.x) * waves) {
    const ScrubBlock& b = a.blocks[k];
    if (!b.tail_len) continue;
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, load_tail_wave(b.data + b.s_full * 512, b.tail_len, lane),
                                                       lane), lane);
    if (lane == 0 && b.meta[b.s_full] != __builtin_bswap32(r ^ b.tail_init))
      atomicMin(&a.bad[k], static_cast<uint32_t>(b.s_full));
  }
}



// ---------------------------------------------------------------------------------------
// Deep-ring variants of the two MFMA kernels (R = 3..4 buffers: crc_ring_buffers() for the
// scrub, crc_tile_ring_buffers() for K1/K2/K3, see gpu_kernels.h for the defaults; deeper
// rings spill at the 256-VGPR budget of 2 waves/SIMD).
// The kernels stream every byte once, so what bounds them is the data in flight per CU, not
// the matrix cores (32 MFMAs per 4 KiB per wave ≈ 9.8 TB/s at full rate): the kernels above
// keep one tile in flight per wave at 3 waves/SIMD. Here each wave keeps R-1 tiles in flight
// in a register ring (16 VGPRs per buffer) at 2 waves/SIMD (grid 512 = one resident round).
// For the compiler to wait with a counted vmcnt(N) instead of draining the ring:
//  * the ring loads are unconditional (tiles past the run re-read its last tile, slices
//    outside the block read slice lo and their chunk CRCs are zeroed), and the loop
//    runs whole groups of R tiles with the remainder (already loaded) after it;
//  * nothing else in the loop is a global load whose result is used: the expected .meta word
//    of a lane's slice is loaded with its data, and the scrub's block table is read through
//    the constant address space (scalar loads; the table is read-only for the launch, and
//    the atomics on `bad` would otherwise make the compiler treat it as clobbered).
template <int R>
struct Ring {
  WaveData b[R];
  uint32_t expect[R];
};

template <int R>
__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
void crc_tile_ring_kernel(CrcLaunch a, const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaTileLds lt;
  __shared__ uint32_t wacc[4];
  __shared__ uint32_t wg_bad;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(a.ntiles, blockIdx.x), t_end = tile_run_begin(a.ntiles, blockIdx.x + 1);
  const int64_t lo = static_cast<int64_t>(a.slice_lo), hi = static_cast<int64_t>(a.slice_hi);
  auto first_slice = [&](uint64_t t) {
    return lo + static_cast<int64_t>(t * kSlicesPerTile + wave * 8) - static_cast<int64_t>(a.vfront);
  };
  Ring<R> ring;
  auto load = [&](int slot, uint64_t t) {
    t = t < t_end ? t : t_end - 1;
    const int64_t i0 = first_slice(t), i = i0 + sw;
    ring.b[slot] = load_wave_ring(a.data, i0, lo, hi, lane);
    ring.expect[slot] = a.meta_expect ? a.meta_expect[(i >= lo && i < hi) ? i : lo] : 0u;
  };
  const bool work = t_begin < t_end;  // workgroup-uniform
  if (work) {
#pragma unroll
    for (int k = 0; k < R - 1; ++k) load(k, t_begin + k);
  }
  i32x4 A[16];
  load_basis(reinterpret_cast<const i32x4*>(gt + 1), lane, A);
  load_lds_image(gt, &lt);
  if (threadIdx.x == 0) wg_bad = 0xFFFFFFFFu;
  __syncthreads();

  uint32_t acc = 0;
  uint32_t bad = 0xFFFFFFFFu;
  auto step = [&](int slot, uint64_t t) {
    const int64_t i = first_slice(t) + sw;
    const bool valid = i >= lo && i < hi;
    const uint32_t c = wave_chunk_crcs(A, ring.b[slot], lane);
    uint32_t r = slice_from_chunks(lt, valid ? c : 0u, lane);
    if (valid && sl == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.full_init);
      if (a.meta_out) a.meta_out[i] = be;
      if (a.meta_expect && ring.expect[slot] != be) bad = min(bad, static_cast<uint32_t>(i));
    }
    if (a.part_crc) {
      r = combine<8>(r, lane, lt.sh512);
      r = combine<16>(r, lane, lt.sh1k);
      r = combine<32>(r, lane, lt.sh2k);  // wave-uniform: the 4 KiB sub-tile's raw CRC
      acc = mat_apply(lt.tile_pow2[0], acc, lane) ^ r;
    }
  };
  uint64_t t0 = t_begin;
  if (work) {
    for (; t0 + R <= t_end; t0 += R) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        load((k + R - 1) % R, t0 + k + R - 1);
        step(k, t0 + k);
      }
    }
#pragma unroll
    for (int k = 0; k < R - 1; ++k)
      if (t0 + k < t_end) step(k, t0 + k);  // loaded by the last group (or the prologue)
  }

  if (a.has_tail && blockIdx.x == 0 && wave == 0) {
    uint32_t r = slice_from_chunks(lt, wave_chunk_crcs(A, load_tail_wave(a.data + a.s_full * 512, a.tail_len, lane),
                                                       lane), lane);
    if (lane == 0) {
      uint32_t be = __builtin_bswap32(r ^ a.tail_init);
      if (a.meta_out) a.meta_out[a.s_full] = be;
      if (a.meta_expect && a.meta_expect[a.s_full] != be) bad = min(bad, static_cast<uint32_t>(a.s_full));
    }
  }
  if (a.part_crc) {
    for (int k = wave; k < 3; ++k) acc = tab4(lt.sh4k, acc);
    uint64_t e = work ? a.ntiles - t_end : 0;
    for (int b = 0; e; ++b, e >>= 1)
      if (e & 1) acc = mat_apply(lt.tile_pow2[b], acc, lane);
    if (lane == 0) wacc[wave] = acc;
  }
  if (a.part_bad && bad != 0xFFFFFFFFu) atomicMin(&wg_bad, bad);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.part_crc) a.part_crc[blockIdx.x] = wacc[0] ^ wacc[1] ^ wacc[2] ^ wacc[3];
    if (a.part_bad) a.part_bad[blockIdx.x] = wg_bad;
  }
}

using ConstScrubBlock = const __attribute__((address_space(4))) ScrubBlock;

template <int R, bool kFp4 = false>
__global__ __launch_bounds__(kCrcWgThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
void crc_scrub_ring_kernel(ScrubLaunch a, const DevCrcTables* __restrict__ gt) {
  __shared__ MfmaSliceLds lt;
  ConstScrubBlock* blocks = (ConstScrubBlock*)a.blocks;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, sw = lane >> 3, sl = lane & 7;
  const uint64_t t_begin = tile_run_begin(a.ntiles, blockIdx.x), t_end = tile_run_begin(a.ntiles, blockIdx.x + 1);
  const bool work = t_begin < t_end;  // workgroup-uniform
  uint32_t blk = 0;
  if (work) {
    uint32_t l = 0, h = a.nblocks;
    while (h - l > 1) {
      uint32_t mid = (l + h) >> 1;
      if (blocks[mid].tile_start <= t_begin) l = mid;
      else h = mid;
    }
    blk = l;
  }
  auto advance = [&](uint64_t t, uint32_t b) {
    while (b + 1 < a.nblocks && blocks[b + 1].tile_start <= t) ++b;
    return b;
  };
  Ring<R> ring;
  uint32_t lblk = blk;  // block of the next tile to load (non-decreasing: clamped tiles are too)
  auto load = [&](int slot, uint64_t t) {
    t = t < t_end ? t : t_end - 1;
    lblk = advance(t, lblk);
    const uint8_t* data = blocks[lblk].data;
    const uint32_t* meta = blocks[lblk].meta;
    const int64_t i0 = static_cast<int64_t>((t - blocks[lblk].tile_start) * kSlicesPerTile + wave * 8);
    const int64_t hi = static_cast<int64_t>(blocks[lblk].s_full);
    ring.b[slot] = load_wave_ring(data, i0, 0, hi, lane);
    ring.expect[slot] = meta[i0 + sw < hi ? i0 + sw : 0];
  };
  if (work) {
#pragma unroll
    for (int k = 0; k < R - 1; ++k) load(k, t_begin + k);
  }
  ChunkBasis<kFp4> basis;
  basis.load(gt, lane);
  load_lds_image(gt, &lt);
  __syncthreads();
  auto step = [&](int slot, uint64_t t) {
    blk = advance(t, blk);
    const int64_t i0 = static_cast<int64_t>((t - blocks[blk].tile_start) * kSlicesPerTile + wave * 8);
    const int64_t hi = static_cast<int64_t>(blocks[blk].s_full);
    // slices past the block end are never compared, so their (re-read) data needs no masking
    uint32_t r = slice_from_chunks(lt, basis.crcs(ring.b[slot], lane), lane);
    const int64_t i = i0 + sw;
    if (sl == 0 && i < hi && ring.expect[slot] != __builtin_bswap32(r ^ a.full_init))
      atomicMin(&a.bad[blk], static_cast<uint32_t>(i));
  };
  if (work) {
    uint64_t t0 = t_begin;
    for (; t0 + R <= t_end; t0 += R) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        load((k + R - 1) % R, t0 + k + R - 1);
        step(k, t0 + k);
      }
    }
#pragma unroll
    for (int k = 0; k < R - 1; ++k)
      if (t0 + k < t_end) step(k, t0 + k);
  }
  const int waves = kCrcWgThreads / 64;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * waves + wave; k < a.nblocks;
       k += static_cast<uint64_t>(gridDim.x) * waves) {
    ConstScrubBlock& b = blocks[k];
    if (!b.tail_len) continue;
    uint32_t r = slice_from_chunks(lt, basis.crcs(load_tail_wave(b.data + b.s_full * 512, b.tail_len, lane), lane), lane);
    if (lane == 0 && b.meta[b.s_full] != __builtin_bswap32(r ^ b.tail_init))
      atomicMin(&a.bad[k], static_cast<uint32_t>(b.s_full));
  }
}

// ---------------------------------------------------------------------------------------
// Roofline probe for the benches: a plain streaming read of n bytes (16 B per lane, four
// loads in flight per lane, non-temporal like the CRC kernels) XOR-folded into one word per
// workgroup. Its TB/s on the same box is what "fraction of achievable HBM" divides by.
__global__ __launch_bounds__(256) void stream_read_kernel(const uint4* __restrict__ p, uint64_t nvec, uint32_t* out) {
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  uint32_t x = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  uint64_t i = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x;
  for (; i + 3 * stride < nvec; i += 4 * stride) {
    u32x4 a = __builtin_nontemporal_load(q + i), b = __builtin_nontemporal_load(q + i + stride);
    u32x4 c = __builtin_nontemporal_load(q + i + 2 * stride), d = __builtin_nontemporal_load(q + i + 3 * stride);
    a ^= b ^ c ^ d;
    x ^= a[0] ^ a[1] ^ a[2] ^ a[3];
  }
  for (; i < nvec; i += stride) {
    u32x4 a = __builtin_nontemporal_load(q + i);
    x ^= a[0] ^ a[1] ^ a[2] ^ a[3];
  }
  for (int m = 32; m; m >>= 1) x ^= __shfl_xor(x, m);
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = x;
}

// ---------------------------------------------------------------------------------------
// GF(2^8) shard matrix multiply (K4 encode / K5 reconstruct): out[r] = XOR_c mat[r][c] * in[c].
// Branch-free split-nibble form (ISA-L style): c * x = T_lo[x & 15] ^ T_hi[x >> 4], with the
// two 16-byte tables per coefficient looked up four bytes at a time by v_perm_b32 (a byte
// shuffle over an 8-byte table pair; bit 3 of the nibble picks the half through v_bfi_b32).
// Per input dword the nibble selectors are prepared once and reused for every output row;
// the tables of one (row, input) pair are wave-uniform and sit in scalar registers. No LDS,
// no data-dependent branches: ~8 VALU ops per input byte for RS(6,3), far under the VALU
// rate needed to keep up with HBM.
struct NibbleSel {
  uint32_t lo7, lo_m, hi7, hi_m;
};

__device__ __forceinline__ NibbleSel nibble_sel(uint32_t x) {
  NibbleSel n;
  n.lo7 = x & 0x07070707u;
  n.hi7 = (x >> 4) & 0x07070707u;
  // bit 3 of each nibble -> 0x00 / 0xFF per byte (perm selector 12 = 0x00, 13 = 0xFF)
  n.lo_m = __builtin_amdgcn_perm(0u, 0u, ((x >> 3) & 0x01010101u) | 0x0C0C0C0Cu);
  n.hi_m = __builtin_amdgcn_perm(0u, 0u, ((x >> 7) & 0x01010101u) | 0x0C0C0C0Cu);
  return n;
}

// t[0..3]: low-nibble table bytes 0..15, t[4..7]: high-nibble table.
__device__ __forceinline__ uint32_t gf_mul4(const uint32_t* __restrict__ t, const NibbleSel& n) {
  uint32_t a = __builtin_amdgcn_perm(t[1], t[0], n.lo7), b = __builtin_amdgcn_perm(t[3], t[2], n.lo7);
  uint32_t c = __builtin_amdgcn_perm(t[5], t[4], n.hi7), d = __builtin_amdgcn_perm(t[7], t[6], n.hi7);
  return ((a & ~n.lo_m) | (b & n.lo_m)) ^ ((c & ~n.hi_m) | (d & n.hi_m));
}

constexpr int kGfRowBlock = 4;

__global__ __launch_bounds__(256) void gf256_matmul_kernel(GfLaunch a) {
  const uint64_t nvec = (a.len + 15) / 16;
  for (uint64_t vi = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; vi < nvec;
       vi += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    for (int r0 = 0; r0 < a.rows; r0 += kGfRowBlock) {
      uint32_t acc[kGfRowBlock][4] = {};
      for (int c = 0; c < a.k; ++c) {
        const uint4 w = reinterpret_cast<const uint4*>(a.in[c])[vi];
        const NibbleSel ns[4] = {nibble_sel(w.x), nibble_sel(w.y), nibble_sel(w.z), nibble_sel(w.w)};
#pragma unroll
        for (int rr = 0; rr < kGfRowBlock; ++rr) {
          const int r = r0 + rr;
          if (r >= a.rows) break;
          const uint32_t* t = a.tables + (r * a.k + c) * 8;  // uniform: scalar loads
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[rr][q] ^= gf_mul4(t, ns[q]);
        }
      }
      for (int rr = 0; rr < kGfRowBlock; ++rr) {
        int r = r0 + rr;
        if (r >= a.rows) break;
        reinterpret_cast<uint4*>(a.out[r])[vi] = make_uint4(acc[rr][0], acc[rr][1], acc[rr][2], acc[rr][3]);
      }
    }
  }
}

}  // namespace

// Raw CRC (zero init, no xorout) of a 64-byte message whose only set bit is bit p of byte b.
static uint32_t chunk_basis_crc(int b, int p) {
  uint32_t r = 0;
  for (int i = 0; i < 64; ++i) {
    r ^= i == b ? (1u << p) : 0u;
    for (int k = 0; k < 8; ++k) r = (r >> 1) ^ ((r & 1u) ? kCrcPoly : 0u);
  }
  return r;
}

static std::atomic<int> g_crc_mfma{-1};

bool crc_mfma_enabled() {
  int v = g_crc_mfma.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("DFS_CRC_MFMA");
    v = (e && e[0] == '0') ? 0 : 1;
    g_crc_mfma.store(v);
  }
  return v == 1;
}

void set_crc_mfma(bool on) { g_crc_mfma.store(on ? 1 : 0); }

static std::atomic<int> g_crc_ring{0}, g_crc_tile_ring{0};

static int ring_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  int v = e ? std::atoi(e) : dflt;
  return v < 2 ? 2 : (v > 4 ? 4 : v);
}

int crc_ring_buffers() {
  int v = g_crc_ring.load(std::memory_order_relaxed);
  if (v == 0) g_crc_ring.store(v = ring_env("DFS_CRC_RING", kCrcRingDefault));
  return v;
}

int crc_tile_ring_buffers() {
  int v = g_crc_tile_ring.load(std::memory_order_relaxed);
  if (v == 0) g_crc_tile_ring.store(v = ring_env("DFS_CRC_TILE_RING", kCrcTileRingDefault));
  return v;
}

void set_crc_ring(int scrub_buffers, int tile_buffers) {
  g_crc_ring.store(scrub_buffers < 2 ? 2 : (scrub_buffers > 4 ? 4 : scrub_buffers));
  g_crc_tile_ring.store(tile_buffers < 2 ? 2 : (tile_buffers > 4 ? 4 : tile_buffers));
}

// Ring depth of a K1/K2/K3 launch over `ntiles` tiles: a deep ring only pays once workgroups
// have several tiles each (below kCrcRingMinTiles its longer prologue costs ~0.3 us per
// launch, e.g. on 1 MiB blocks).
// Size-based K1/K2 dispatch: below DFS_CRC_LDS_MAX_MIB (default 16 MiB) the LDS-table kernel
// wins (its per-workgroup setup is smaller: 1 MiB 6.02 vs 6.47 us, 8 MiB 7.39 vs 8.89 us in
// profiles/archive/r2_crc4/crc_default.json); from 64 MiB up the matrix-core kernel is 1.3-1.9x faster.
static std::atomic<int64_t> g_lds_max_mib{-1};

void set_crc_lds_max_mib(int mib) { g_lds_max_mib.store(mib < 0 ? 0 : mib); }

static uint64_t lds_max_tiles() {
  int64_t mib = g_lds_max_mib.load(std::memory_order_relaxed);
  if (mib < 0) {
    const char* e = std::getenv("DFS_CRC_LDS_MAX_MIB");
    long v = e ? std::atol(e) : kCrcLdsMaxMibDefault;
    g_lds_max_mib.store(mib = v > 0 ? v : 0);
  }
  return static_cast<uint64_t>(mib) * (1ull << 20) / (kSlicesPerTile * 512ull);
}

static int ring_for(uint64_t ntiles) {
  if (!crc_mfma_enabled() || ntiles < lds_max_tiles()) return 0;
  return ntiles >= kCrcRingMinTiles ? crc_tile_ring_buffers() : 2;
}

// One resident round: 3 workgroups per CU at 3 waves/SIMD (R = 2), 2 at 2 waves/SIMD.
static uint64_t crc_grid_cap(int ring) { return ring > 2 ? 2 * 256 : kMaxGridCrc; }

// K1/K2 as crc_tile_wide_kernel (one workgroup of G x 4 waves per CU): 0 = off, 1 = G = 3
// (3 waves/SIMD), 2 = G = 2 (2 waves/SIMD). DFS_CRC_WIDE overrides the default.
// Why G = 2 can win although it halves the waves: the loop is matrix-pipe + VALU bound, so a
// tile-iteration of a group costs ~G units on a CU, and a block of T tiles takes
// ceil(T / (256 G)) iterations: 64 MiB = 4096 tiles is 6 x 3 = 18 units at G = 3 (runs of 5 or
// 6: the CUs with 6 set the time) but 8 x 2 = 16 at G = 2 (every run exactly 8); every
// power-of-two size divides evenly at G = 2.
static std::atomic<int> g_crc_wide{-1};

void set_crc_wide(int mode) { g_crc_wide.store(mode <= 0 ? 0 : (mode >= 2 ? 2 : 1)); }

int crc_wide_mode() {
  int v = g_crc_wide.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("DFS_CRC_WIDE");
    v = e ? std::atoi(e) : kCrcWideDefault;
    g_crc_wide.store(v = v <= 0 ? 0 : (v >= 2 ? 2 : 1));
  }
  return v;
}

static int crc_wide_groups() { return crc_wide_mode() == 2 ? 2 : kMaxGridCrc / 256; }

static std::atomic<int> g_crc_fp4{-1};

void set_crc_fp4(bool on) { g_crc_fp4.store(on ? 1 : 0); }

bool crc_fp4_enabled() {
  int v = g_crc_fp4.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = std::getenv("DFS_CRC_FP4");
    g_crc_fp4.store(v = (e ? std::atoi(e) : kCrcFp4Default) ? 1 : 0);
  }
  return v != 0;
}

DevCrcTables* upload_crc_tables(hipStream_t s) {
  static_assert(sizeof(DevCrcTables) % 16 == 0, "table image must be uint4-copyable");
  std::vector<uint8_t> host(sizeof(DevCrcTables));
  auto* t = reinterpret_cast<DevCrcTables*>(host.data());
  std::memcpy(t->slice16, crc_tables().slice16, sizeof(t->slice16));
  shift_table(64, t->sh64);
  shift_table(128, t->sh128);
  shift_table(256, t->sh256);
  shift_table(512, t->sh512);
  shift_table(1024, t->sh1k);
  shift_table(2048, t->sh2k);
  shift_table(4096, t->sh4k);
  for (int b = 0; b < 32; ++b) {
    const Gf2Mat& m = shift_pow2_bytes(14 + b);  // 16 KiB * 2^b
    std::memcpy(t->tile_pow2[b], m.col, sizeof(m.col));
  }
  // MFMA basis right behind the LDS image (never copied to LDS): fragment [s][lane] of A,
  // element j = byte j of the 16 B: CRC bit i = lane & 31 of V[32h + 4(s>>1) + (j&3)][4(s&1) + (j>>2)],
  // scaled by 2^(7-p) (see wave_chunk_crcs)
  host.resize(sizeof(DevCrcTables) + kCrcBasisFp4Offset + kCrcBasisFp4Bytes);
  static_assert(kCrcBasisFp4Offset == kCrcBasisBytes + kCrcChunkShiftBytes + kCrcWideExtraBytes, "image order");
  // chunk-shift tables behind the basis: cs[sl] moves a 64 B chunk's CRC past 64 * (7 - sl) bytes;
  // then ss[sw] (a slice's CRC past 512 * (7 - sw) bytes) and the 16 KiB tile shift
  auto* cs = reinterpret_cast<uint32_t(*)[4][256]>(host.data() + sizeof(DevCrcTables) + kCrcBasisBytes);
  for (int sl = 0; sl < 7; ++sl) shift_table(64 * (7 - sl), cs[sl]);
  for (int sw = 0; sw < 7; ++sw) shift_table(512 * (7 - sw), cs[7 + sw]);
  shift_table(16384, cs[14]);
  int8_t* basis = reinterpret_cast<int8_t*>(host.data() + sizeof(DevCrcTables));
  for (int st = 0; st < 16; ++st)
    for (int lane = 0; lane < 64; ++lane)
      for (int j = 0; j < 16; ++j) {
        // row R = lane & 31 of A carries CRC bit R ^ 7 (the order wave_chunk_crcs gathers in)
        const int h = lane >> 5, bit = (lane & 31) ^ 7;
        const int byte = 32 * h + 4 * (st >> 1) + (j & 3), p = 4 * (st & 1) + (j >> 2);
        const uint32_t v = chunk_basis_crc(byte, p);
        basis[(st * 64 + lane) * 16 + j] = ((v >> bit) & 1u) ? static_cast<int8_t>(static_cast<uint8_t>(1u << (7 - p))) : 0;
      }
  // FP4 basis (wave_chunk_crcs_fp4): fragment [s][lane], dword r, nibble q is the element that
  // B takes from bit 4(q & 1) + r of byte (q >> 1) of data dword s of the lane's 32 B half;
  // value 2.0 / 1.0 / 0.5 / 0.5 (e2m1 0b0100 / 0b0010 / 0b0001) for planes r = 0..3 where
  // the basis bit is set, so the product with B's 0.5 / 1.0 / 2.0 / 2.0 is 1.0
  uint8_t* b4 = host.data() + sizeof(DevCrcTables) + kCrcBasisFp4Offset;
  std::memset(b4, 0, kCrcBasisFp4Bytes);
  static const uint8_t kFp4Code[4] = {0x4, 0x2, 0x1, 0x1};
  for (int st = 0; st < 8; ++st)
    for (int lane = 0; lane < 64; ++lane)
      for (int r = 0; r < 4; ++r)
        for (int q = 0; q < 8; ++q) {
          const int h = lane >> 5, bit = (lane & 31) ^ 7;
          const uint32_t v = chunk_basis_crc(32 * h + 4 * st + (q >> 1), 4 * (q & 1) + r);
          if ((v >> bit) & 1u) b4[(st * 64 + lane) * 16 + 4 * r + (q >> 1)] |= kFp4Code[r] << (4 * (q & 1));
        }
  t = reinterpret_cast<DevCrcTables*>(host.data());
  DevCrcTables* d = nullptr;
  if (hipMalloc(&d, host.size()) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  return d;
}


int crc_grid_for(uint64_t ntiles, uint32_t has_tail) {
  // small blocks: at least `per` tiles per workgroup, so the per-workgroup fixed cost (the
  // 16 KiB basis per wave and the LDS image, both from L2) is amortised over more data
  static const uint64_t per = [] {
    const char* e = std::getenv("DFS_CRC_MIN_TILES_PER_WG");
    long v = e ? std::atol(e) : 1;
    return static_cast<uint64_t>(v > 0 ? v : 1);
  }();
  uint64_t g = (ntiles + per - 1) / per;
  const int ring = ring_for(ntiles);
  uint64_t cap = crc_grid_cap(ring);
  const uint64_t G = crc_wide_groups();
  if (ring == 2 && crc_wide_mode()) cap = 256 * G;  // one resident round of the wide kernel
  g = g < cap ? g : cap;
  // the wide kernel runs G virtual workgroups per launched one (empty runs leave a zero
  // partial and no verdict)
  if (ring == 2 && crc_wide_mode() && g) g = (g + G - 1) / G * G;
  if (g == 0 && has_tail) g = 1;
  return static_cast<int>(g);
}

bool crc_meta_host_ok(uint64_t ntiles) { return ring_for(ntiles) == 0; }

hipError_t launch_crc(const CrcLaunch& a, const DevCrcTables* t, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  if (a.meta_host && ring_for(a.ntiles) != 0) return hipErrorInvalidValue;  // only the LDS kernel mirrors it
  switch (ring_for(a.ntiles)) {
    case 0: hipLaunchKernelGGL(crc_slices_kernel, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t); break;
    case 2:
      if (crc_wide_mode() && grid % crc_wide_groups() == 0) {
        const int G = crc_wide_groups();
        const dim3 g(grid / G), b(kCrcWgThreads * G);
        const bool w = a.meta_out && !a.meta_expect && a.part_crc;
        constexpr int G3 = kMaxGridCrc / 256;
        const int v = (G == 2 ? 0 : 4) | (w ? 2 : 0) | (crc_fp4_enabled() ? 1 : 0);
        switch (v) {
          case 0: hipLaunchKernelGGL((crc_tile_wide_kernel<2, false, false>), g, b, 0, s, a, t); break;
          case 1: hipLaunchKernelGGL((crc_tile_wide_kernel<2, false, true>), g, b, 0, s, a, t); break;
          case 2: hipLaunchKernelGGL((crc_tile_wide_kernel<2, true, false>), g, b, 0, s, a, t); break;
          case 3: hipLaunchKernelGGL((crc_tile_wide_kernel<2, true, true>), g, b, 0, s, a, t); break;
          case 4: hipLaunchKernelGGL((crc_tile_wide_kernel<G3, false, false>), g, b, 0, s, a, t); break;
          case 5: hipLaunchKernelGGL((crc_tile_wide_kernel<G3, false, true>), g, b, 0, s, a, t); break;
          case 6: hipLaunchKernelGGL((crc_tile_wide_kernel<G3, true, false>), g, b, 0, s, a, t); break;
          default: hipLaunchKernelGGL((crc_tile_wide_kernel<G3, true, true>), g, b, 0, s, a, t); break;
        }
      } else {
        hipLaunchKernelGGL(crc_tile_mfma_kernel, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t);
      }
      break;
    case 3: hipLaunchKernelGGL(crc_tile_ring_kernel<3>, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t); break;
    default: hipLaunchKernelGGL(crc_tile_ring_kernel<4>, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t); break;
  }
  return hipGetLastError();
}

hipError_t launch_read_copy(const ReadCopyLaunch& a, const DevCrcTables* t, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  if (grid > kMaxGridCrc) return hipErrorInvalidValue;  // part_bad holds kMaxGridCrc words
  hipLaunchKernelGGL(crc_read_copy_kernel, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t);
  return hipGetLastError();
}

hipError_t launch_write_copy(const WriteCopyLaunch& a, const DevCrcTables* t, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  // part_crc holds kMaxGridCrc words; the plan must be a whole block (K1/K2, no verify)
  if (grid > kMaxGridCrc || a.c.slice_lo != 0 || a.c.slice_hi != a.c.s_full || !a.c.meta_out || !a.meta_host ||
      !a.c.part_crc || !a.dst ||
      (reinterpret_cast<uintptr_t>(a.c.data) | reinterpret_cast<uintptr_t>(a.dst) | reinterpret_cast<uintptr_t>(a.dst_host)) % 16)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(crc_write_copy_kernel, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t);
  return hipGetLastError();
}

hipError_t launch_scrub(const ScrubLaunch& a, const DevCrcTables* t, hipStream_t s) {
  if (a.nblocks == 0) return hipSuccess;
  const int ring = crc_mfma_enabled() ? crc_ring_buffers() : 0;
  const uint64_t cap = ring ? crc_grid_cap(ring) : 2048;
  uint64_t g = a.ntiles < cap ? a.ntiles : cap;
  uint64_t tail_waves = (a.nblocks + 3) / 4;
  if (g < tail_waves) g = tail_waves < cap ? tail_waves : cap;
  if (g == 0) g = 1;
  const dim3 grid(static_cast<unsigned>(g));
  switch (ring) {
    case 0: hipLaunchKernelGGL(crc_scrub_kernel, grid, dim3(kCrcWgThreads), 0, s, a, t); break;
    case 2: hipLaunchKernelGGL(crc_scrub_mfma_kernel, grid, dim3(kCrcWgThreads), 0, s, a, t); break;
    case 3:
      if (crc_fp4_enabled()) hipLaunchKernelGGL((crc_scrub_ring_kernel<3, true>), grid, dim3(kCrcWgThreads), 0, s, a, t);
      else hipLaunchKernelGGL((crc_scrub_ring_kernel<3, false>), grid, dim3(kCrcWgThreads), 0, s, a, t);
      break;
    default:
      if (crc_fp4_enabled()) hipLaunchKernelGGL((crc_scrub_ring_kernel<4, true>), grid, dim3(kCrcWgThreads), 0, s, a, t);
      else hipLaunchKernelGGL((crc_scrub_ring_kernel<4, false>), grid, dim3(kCrcWgThreads), 0, s, a, t);
      break;
  }
  return hipGetLastError();
}

hipError_t launch_stream_read(const uint8_t* d, uint64_t n, uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(stream_read_kernel, dim3(kStreamReadGrid), dim3(256), 0, s, reinterpret_cast<const uint4*>(d), n / 16,
                     out);
  return hipGetLastError();
}

void gf_nibble_tables(const uint8_t* mat, int rows, int k, uint32_t* out) {
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < k; ++c) {
      uint8_t coef = mat[r * k + c];
      uint8_t lo[16], hi[16];
      for (int v = 0; v < 16; ++v) {
        lo[v] = gf::mul(coef, static_cast<uint8_t>(v));
        hi[v] = gf::mul(coef, static_cast<uint8_t>(v << 4));
      }
      uint32_t* t = out + (r * k + c) * 8;
      std::memcpy(t, lo, 16);
      std::memcpy(t + 4, hi, 16);
    }
}

hipError_t launch_gf_matmul(const GfLaunch& a, hipStream_t s) {
  if (a.len == 0 || a.rows == 0) return hipSuccess;
  uint64_t nvec = (a.len + 15) / 16;
  uint64_t blocks = (nvec + 255) / 256;
  int grid = static_cast<int>(blocks < 2048 ? blocks : 2048);
  hipLaunchKernelGGL(gf256_matmul_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace dfs
