// CDNA4 (gfx950) kernels for the chunk data path.
//   K1/K2  crc_slices_kernel  : per-512B-slice CRC32 (big-endian .meta image) fused with the
//                               whole-block CRC (shift-combine tree, per-workgroup partials).
//   K3     same kernel in range/verify mode: recompute only touched slices and compare with
//          the HBM-resident .meta image (reference verify_partial_read, chunkserver.rs:296-351).
//   K1b    crc_scrub_kernel: one launch verifies every resident block against its .meta.
//   K4/K5  gf256_matmul_kernel: GF(2^8) matrix x shards (Reed-Solomon encode / reconstruct;
//          reference erasure.rs:7-49).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dfs {

constexpr int kCrcWgThreads = 256;
constexpr int kSlicesPerTile = 32;  // 4 waves x 8 slices x 512 B = 16 KiB per tile
constexpr int kMaxGridCrc = 768;  // 3 resident workgroups x 256 CUs (see crc_tile_mfma_kernel)
constexpr int kMaxShards = 32;
constexpr int kCrcBasisBytes = 16 * 64 * 16;  // MFMA basis (A fragments), stored after DevCrcTables
constexpr int kCrcChunkShiftBytes = 7 * 4 * 256 * 4;  // chunk -> slice shift tables, stored after the basis
// behind those: slice -> 4 KiB sub-tile shift tables (7) and the 16 KiB tile shift (wide kernel)
constexpr int kCrcWideExtraBytes = 8 * 4 * 256 * 4;
// behind those: the basis of the FP4 matrix-core form (8 A fragments of 16 B per lane)
constexpr int kCrcBasisFp4Bytes = 8 * 64 * 16;
constexpr int kCrcBasisFp4Offset = kCrcBasisBytes + kCrcChunkShiftBytes + kCrcWideExtraBytes;  // after DevCrcTables

struct DevCrcTables {
  uint32_t slice16[16][256];
  uint32_t sh64[4][256], sh128[4][256], sh256[4][256];  // lane combine inside a slice
  uint32_t sh512[4][256], sh1k[4][256], sh2k[4][256];   // slice combine inside a wave
  uint32_t sh4k[4][256];                                 // wave combine inside a workgroup
  uint32_t tile_pow2[32][32];                            // GF(2) matrices: 16 KiB * 2^b
};

struct CrcLaunch {
  const uint8_t* data;
  uint64_t n;
  uint64_t s_full;      // number of full 512 B slices in the block
  uint64_t slice_lo;    // first full slice processed
  uint64_t slice_hi;    // one past last full slice processed
  uint64_t vfront;      // virtual leading zero slices (aligns block combine to tiles)
  uint64_t ntiles;      // virtual tiles covering [slice_lo - vfront, slice_hi)
  uint32_t full_init;   // S(512)
  uint32_t has_tail;    // process the short tail slice (index s_full)
  uint32_t tail_len;
  uint32_t tail_init;   // S(tail_len)
  uint32_t* meta_out;             // BE CRC per slice (nullable)
  const uint32_t* meta_expect;    // BE CRC per slice to verify against (nullable)
  uint32_t* part_crc;             // [grid] raw shifted partials for whole-block CRC (nullable)
  uint32_t* part_bad;             // [grid] min mismatching slice index, 0xFFFFFFFF = none
  // device view of host-visible memory that receives a copy of meta_out (nullable; honoured
  // only by the LDS kernel, see crc_meta_host_ok): the .meta image needs no readback copy
  uint32_t* meta_host;
};

// K1b: one launch verifies many resident blocks against their HBM .meta images. Blocks are
// laid out on a global tile axis (tile_start = prefix sum of ceil(s_full / 32)); each
// workgroup finds its block by binary search, so every tile of every block is one
// grid-stride step and the LDS table fill is paid once per workgroup per launch.
struct ScrubBlock {
  const uint8_t* data;
  const uint32_t* meta;  // BE CRC per slice (HBM-resident .meta image)
  uint64_t s_full;
  uint64_t tile_start;
  uint32_t tail_len;
  uint32_t tail_init;
};

struct ScrubLaunch {
  const ScrubBlock* blocks;  // device, sorted by tile_start
  uint32_t nblocks;
  uint64_t ntiles;
  uint32_t full_init;
  uint32_t* bad;  // [nblocks] min mismatching slice index, pre-set to 0xFFFFFFFF
};

struct GfLaunch {
  const uint8_t* in[kMaxShards];
  uint8_t* out[kMaxShards];
  uint64_t len;   // bytes per shard (buffers padded to 16 B)
  int k;          // inputs
  int rows;       // outputs
  const uint32_t* tables;  // device: [rows][k] x 8 dwords, split-nibble product tables (gf_nibble_tables)
};
// Host: split-nibble tables of a rows x k coefficient matrix (poly 0x11D): per (r, c) the
// 16 products of the low nibble, then the 16 of the high nibble, 32 bytes.
void gf_nibble_tables(const uint8_t* mat, int rows, int k, uint32_t* out);

// Upload tables once per device (LDS image followed by the MFMA basis). Returns device pointer.
// K1/K2/K1b use the matrix-core chunk CRC unless DFS_CRC_MFMA=0 (the LDS slicing-by-16 path).
bool crc_mfma_enabled();
void set_crc_mfma(bool on);  // benchmarks / tests: pick the K1 implementation
// K1/K2 blocks below this many MiB run the LDS-table kernel even with the matrix-core path
// enabled (size-based dispatch; DFS_CRC_LDS_MAX_MIB, 0 = always the matrix cores).
constexpr int kCrcLdsMaxMibDefault = 16;
void set_crc_lds_max_mib(int mib);
DevCrcTables* upload_crc_tables(hipStream_t s);
int crc_grid_for(uint64_t ntiles, uint32_t has_tail);
// Tile buffers per wave in the MFMA kernels' register ring (2..4; 2 = the 3-waves/SIMD
// kernels, 3..4 = the deep-ring kernels at 2 waves/SIMD). Measured (profiles/archive/r2_crc3): the
// K1b scrub gains ~19 % from 3 buffers; K1/K2 does not (its per-tile combine work, not load
// latency, is what the third wave hides), so it keeps 2. DFS_CRC_RING / DFS_CRC_TILE_RING
// override, set_crc_ring is the benches' A/B switch; K1/K2/K3 launches below
// kCrcRingMinTiles tiles (32 MiB) always use 2. Grid caps follow, never above kMaxGridCrc.
constexpr int kCrcRingDefault = 3;
constexpr int kCrcTileRingDefault = 2;
int crc_ring_buffers();       // K1b scrub
int crc_tile_ring_buffers();  // K1/K2/K3
void set_crc_ring(int scrub_buffers, int tile_buffers);
constexpr uint64_t kCrcRingMinTiles = 2048;
// K1/K2 on matrix cores with one 12-wave workgroup per CU (shared LDS image + MFMA basis, and
// a two-lookup combine per tile) from kCrcWideMinTiles tiles up; 0 = three 4-wave workgroups
// per CU everywhere. DFS_CRC_WIDE overrides, set_crc_wide is the benches' A/B switch.
constexpr int kCrcWideDefault = 1;
int crc_wide_mode();
void set_crc_wide(int mode);
// The wide K1/K2 kernel's chunk CRC on the FP4 matrix cores (v_mfma_scale_f32_32x32x64_f8f6f4:
// 64 input bits per row per instruction at the cycles of the i8 form's 32) instead of i8.
// DFS_CRC_FP4 overrides, set_crc_fp4 is the benches' A/B switch.
constexpr int kCrcFp4Default = 1;
bool crc_fp4_enabled();
void set_crc_fp4(bool on);

// Benches: streaming read of n bytes (n % 16 == 0) on kStreamReadGrid x 256 threads; `out`
// holds 4 x kStreamReadGrid words.
constexpr int kStreamReadGrid = 2048;
hipError_t launch_stream_read(const uint8_t* d, uint64_t n, uint32_t* out, hipStream_t s);

hipError_t launch_crc(const CrcLaunch& a, const DevCrcTables* t, int grid, hipStream_t s);

// K3 fused verify + copy of a range read (crc_read_copy_kernel): `c` is the range plan
// (meta_expect set, part_* unused), `out` a device-visible pointer (registered host memory)
// that receives [off, off + len) with (out - off) % 16 == 0, `part_bad` [grid] device-visible
// words (min mismatching slice per workgroup, 0xFFFFFFFF = none). grid <= kMaxGridCrc.
struct ReadCopyLaunch {
  CrcLaunch c;
  uint8_t* out;
  uint64_t off, len;
  uint32_t* part_bad;
};
hipError_t launch_read_copy(const ReadCopyLaunch& a, const DevCrcTables* t, int grid, hipStream_t s);

// K1/K2 fused with a write's host-to-device copy (crc_write_copy_kernel): `c` is a whole-block
// plan whose `data` is the device-visible view of registered host memory, `meta_out` the HBM
// .meta image and `part_crc` [grid] device-visible host words (whole-block partials);
// `dst` the HBM extent, `meta_host` a device-visible host copy of the .meta image. The data
// and dst must be 16 B aligned. grid <= kMaxGridCrc.
struct WriteCopyLaunch {
  CrcLaunch c;
  uint8_t* dst;
  uint32_t* meta_host;
  // optional second copy of the bytes into device-visible host memory (16 B aligned): a
  // pulled replica that the journal appends from the host, with no device-to-host copy
  uint8_t* dst_host = nullptr;
};
// True when launch_crc runs a block of `ntiles` tiles on the kernel that honours
// CrcLaunch::meta_host (the LDS kernel, below the MFMA size threshold).
bool crc_meta_host_ok(uint64_t ntiles);
hipError_t launch_write_copy(const WriteCopyLaunch& a, const DevCrcTables* t, int grid, hipStream_t s);
hipError_t launch_gf_matmul(const GfLaunch& a, hipStream_t s);
hipError_t launch_scrub(const ScrubLaunch& a, const DevCrcTables* t, hipStream_t s);

}  // namespace dfs
