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

// Butterfly step: lanes with (lane & m) == 0 hold the earlier bytes.
__device__ __forceinline__ uint32_t combine(uint32_t r, int m, int lane, const uint32_t (*t)[256]) {
  uint32_t p = __shfl_xor(r, m);
  bool right = lane & m;
  uint32_t left = right ? p : r;
  uint32_t rgt = right ? r : p;
  return tab4(t, left) ^ rgt;
}

// Lane-parallel GF(2) matrix apply: v uniform across the wave, lanes 0..31 own columns.
__device__ __forceinline__ uint32_t mat_apply(const uint32_t* col, uint32_t v, int lane) {
  int i = lane & 31;
  uint32_t x = ((v >> i) & 1u) ? col[i] : 0u;
  x ^= __shfl_xor(x, 16);
  x ^= __shfl_xor(x, 8);
  x ^= __shfl_xor(x, 4);
  x ^= __shfl_xor(x, 2);
  x ^= __shfl_xor(x, 1);
  return x;
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
  r = combine(r, 1, lane, lt.sh64);
  r = combine(r, 2, lane, lt.sh128);
  return combine(r, 4, lane, lt.sh256);
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
  r = combine(r, 1, lane, lt.sh64);
  r = combine(r, 2, lane, lt.sh128);
  return combine(r, 4, lane, lt.sh256);
}

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
      if (a.meta_expect && a.meta_expect[i] != be) bad = min(bad, static_cast<uint32_t>(i));
    }
    if (a.part_crc) {
      r = combine(r, 8, lane, lt.sh512);
      r = combine(r, 16, lane, lt.sh1k);
      r = combine(r, 32, lane, lt.sh2k);
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
// GF(2^8) shard matrix multiply: out[r] = XOR_c mat[r][c] * in[c]. Each lane owns 16 B of
// every shard; logs of the input bytes are looked up once and reused by every output row.
constexpr int kGfRowBlock = 4;

__global__ __launch_bounds__(256) void gf256_matmul_kernel(GfLaunch a) {
  __shared__ uint8_t s_log[256];
  __shared__ uint8_t s_exp[512];
  __shared__ uint8_t s_clog[kMaxShards * kMaxShards];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) s_log[i] = a.gf_tables[i];
  for (int i = threadIdx.x; i < 512; i += blockDim.x) s_exp[i] = a.gf_tables[256 + i];
  __syncthreads();
  for (int i = threadIdx.x; i < a.rows * a.k; i += blockDim.x) s_clog[i] = s_log[a.mat[i]];
  __syncthreads();

  const uint64_t nvec = (a.len + 15) / 16;
  for (uint64_t vi = blockIdx.x * static_cast<uint64_t>(blockDim.x) + threadIdx.x; vi < nvec;
       vi += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    for (int r0 = 0; r0 < a.rows; r0 += kGfRowBlock) {
      uint32_t acc[kGfRowBlock][4] = {};
      for (int c = 0; c < a.k; ++c) {
        uint4 w = reinterpret_cast<const uint4*>(a.in[c])[vi];
        uint32_t words[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            uint32_t byte = (words[q] >> (8 * b)) & 0xff;
            if (!byte) continue;
            uint32_t lb = s_log[byte];
#pragma unroll
            for (int rr = 0; rr < kGfRowBlock; ++rr) {
              int r = r0 + rr;
              if (r >= a.rows) break;
              uint8_t coef = a.mat[r * a.k + c];
              if (!coef) continue;
              acc[rr][q] ^= static_cast<uint32_t>(s_exp[lb + s_clog[r * a.k + c]]) << (8 * b);
            }
          }
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
  DevCrcTables* d = nullptr;
  if (hipMalloc(&d, sizeof(DevCrcTables)) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, host.data(), sizeof(DevCrcTables), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  return d;
}

const uint8_t* upload_gf_tables(hipStream_t s) {
  const auto& t = gf::tables();
  std::vector<uint8_t> host(768);
  std::memcpy(host.data(), t.log, 256);
  std::memcpy(host.data() + 256, t.exp, 512);
  uint8_t* d = nullptr;
  if (hipMalloc(&d, host.size()) != hipSuccess) return nullptr;
  if (hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    (void)hipFree(d);
    return nullptr;
  }
  return d;
}

int crc_grid_for(uint64_t ntiles, uint32_t has_tail) {
  uint64_t g = ntiles < static_cast<uint64_t>(kMaxGridCrc) ? ntiles : kMaxGridCrc;
  if (g == 0 && has_tail) g = 1;
  return static_cast<int>(g);
}

hipError_t launch_crc(const CrcLaunch& a, const DevCrcTables* t, int grid, hipStream_t s) {
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(crc_slices_kernel, dim3(grid), dim3(kCrcWgThreads), 0, s, a, t);
  return hipGetLastError();
}

hipError_t launch_scrub(const ScrubLaunch& a, const DevCrcTables* t, hipStream_t s) {
  if (a.nblocks == 0) return hipSuccess;
  uint64_t g = a.ntiles < 2048 ? a.ntiles : 2048;
  uint64_t tail_waves = (a.nblocks + 3) / 4;
  if (g < tail_waves) g = tail_waves < 2048 ? tail_waves : 2048;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(crc_scrub_kernel, dim3(static_cast<unsigned>(g)), dim3(kCrcWgThreads), 0, s, a, t);
  return hipGetLastError();
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
