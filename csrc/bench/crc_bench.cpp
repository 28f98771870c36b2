// Kernel-only microbenchmark of the checksum kernels on device-resident data (no H2D):
// K1+K2 (per-slice .meta + whole-block CRC) at several block sizes, and the K1b batched
// scrub over 1 GiB of 1 MiB blocks — each with the matrix-core chunk CRC (MFMA) and with
// the LDS slicing-by-16 tables, every result checked against the host CRC.
//
//   build/native/crc_bench [--iters N] [--mib TOTAL]     -> JSON on stdout
//   build/native/crc_bench --single MIB [--iters N] -> the production K1/K2 dispatch at one size
//   build/native/crc_bench --sweep                        -> K1/K2 grid x register-ring sweep at
//                                                            8 / 64 / 256 MiB, plus the streaming
//                                                            read at those sizes (JSON)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "crc32.h"
#include "gf256.h"
#include "gpu_kernels.h"

using namespace dfs;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

struct Run {
  double us;
  bool ok;
};

static Run bench_block(const uint8_t* d, uint64_t n, const DevCrcTables* t, uint32_t* dmeta, uint32_t* dpart,
                       hipStream_t s, int iters, const std::vector<uint8_t>& host, int grid_override = 0) {
  CrcLaunch a{};
  a.data = d;
  a.n = n;
  a.s_full = n / kSliceBytes;
  a.slice_lo = 0;
  a.slice_hi = a.s_full;
  a.vfront = (kSlicesPerTile - a.s_full % kSlicesPerTile) % kSlicesPerTile;
  a.ntiles = (a.s_full + a.vfront) / kSlicesPerTile;
  a.full_init = crc_init_term(kSliceBytes);
  a.meta_out = dmeta;
  a.part_crc = dpart;
  int grid = grid_override > 0 ? grid_override : crc_grid_for(a.ntiles, 0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(launch_crc(a, t, grid, s));  // warm-up + correctness
  std::vector<uint32_t> part(grid), meta(a.s_full);
  CK(hipMemcpyAsync(part.data(), dpart, grid * 4, hipMemcpyDeviceToHost, s));
  CK(hipMemcpyAsync(meta.data(), dmeta, a.s_full * 4, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  uint32_t r = 0;
  for (uint32_t v : part) r ^= v;
  r ^= crc_init_term(n);
  bool ok = r == crc32(host.data(), n);
  std::vector<uint32_t> ref(a.s_full);
  crc32_slices(host.data(), n, ref.data());
  for (uint64_t i = 0; ok && i < a.s_full; ++i) ok = __builtin_bswap32(meta[i]) == ref[i];
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) CK(launch_crc(a, t, grid, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return {1e3 * ms / iters, ok};
}

int main(int argc, char** argv) {
  int iters = 50;
  uint64_t total_mib = 1024;
  bool sweep = false;
  bool wide_ab = false;  // --wide-ab: K1/K2 on the matrix cores, 3 x 4-wave vs 1 x 12-wave workgroups per CU
  bool fp4_ab = false;   // --fp4-ab: the wide kernel's chunk CRCs on i8 vs FP4 matrix cores, 3 and 2 groups
  uint64_t single_mib = 0;  // --single MIB: only the production K1/K2 dispatch at that size (PMC runs)
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--mib" && i + 1 < argc) total_mib = std::strtoull(argv[++i], nullptr, 10);
    else if (a == "--sweep") sweep = true;
    else if (a == "--wide-ab") wide_ab = true;
    else if (a == "--fp4-ab") fp4_ab = true;
    else if (a == "--single" && i + 1 < argc) single_mib = std::strtoull(argv[++i], nullptr, 10);
  }
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const uint64_t total = total_mib << 20;
  std::vector<uint8_t> host(total);
  std::mt19937_64 rng(42);
  for (uint64_t i = 0; i < total; i += 8) {
    uint64_t v = rng();
    std::memcpy(host.data() + i, &v, 8);
  }
  uint8_t* d = nullptr;
  uint32_t *dmeta = nullptr, *dpart = nullptr;
  CK(hipMalloc(&d, total));
  CK(hipMalloc(&dmeta, (total / kSliceBytes + 64) * 4));
  CK(hipMalloc(&dpart, kMaxGridCrc * 4));
  CK(hipMemcpy(d, host.data(), total, hipMemcpyHostToDevice));
  DevCrcTables* t = upload_crc_tables(s);
  if (!t) return 3;
  // roofline probe: a plain streaming read of the whole buffer on this box
  double stream_gbps = 0;
  {
    uint32_t* dout = nullptr;
    CK(hipMalloc(&dout, 4 * kStreamReadGrid * 4));
    CK(launch_stream_read(d, total, dout, s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int it = std::max(3, iters / 10);
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < it; ++i) CK(launch_stream_read(d, total, dout, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    stream_gbps = total / (1e3 * ms / it) / 1e3;
    (void)hipFree(dout);
  }
  if (single_mib) {
    const uint64_t n = std::min<uint64_t>(single_mib << 20, total);
    Run r = bench_block(d, n, t, dmeta, dpart, s, iters, host);
    std::printf("{\"bytes\": %llu, \"us\": %.2f, \"GBps\": %.1f, \"ok\": %s}\n", static_cast<unsigned long long>(n), r.us,
                n / r.us / 1e3, r.ok ? "true" : "false");
    return r.ok ? 0 : 1;
  }
  if (fp4_ab) {
    // plus a streaming read of the same bytes, so each size has its own like-for-like roofline
    std::printf("{\"stream_read_GBps\": %.1f, \"k1k2\": [", stream_gbps);
    set_crc_mfma(true);
    set_crc_lds_max_mib(0);
    uint32_t* dout = nullptr;
    CK(hipMalloc(&dout, 4 * kStreamReadGrid * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    bool f = true;
    for (uint64_t mib : std::vector<uint64_t>{1, 8, 16, 32, 64, 128, 256, 1024}) {
      const uint64_t n = mib << 20;
      if (n > total) continue;
      const int it = n >= (256ull << 20) ? std::max(3, iters / 10) : iters;
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < it; ++i) CK(launch_stream_read(d, n, dout, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double stream_us = 1e3 * ms / it;
      for (int rep = 0; rep < 2; ++rep)
        for (int w : {1, 2})
          for (int fp4 : {0, 1}) {
            set_crc_wide(w);
            set_crc_fp4(fp4 != 0);
            Run r = bench_block(d, n, t, dmeta, dpart, s, it, host);
            std::printf("%s\n  {\"bytes\": %llu, \"wide\": %d, \"fp4\": %d, \"rep\": %d, \"us\": %.2f, \"GBps\": %.1f, "
                        "\"of_stream\": %.3f, \"stream_same_size_us\": %.2f, \"of_stream_same_size\": %.3f, \"ok\": %s}",
                        f ? "" : ",", static_cast<unsigned long long>(n), w, fp4, rep, r.us, n / r.us / 1e3,
                        n / r.us / 1e3 / stream_gbps, stream_us, stream_us / r.us, r.ok ? "true" : "false");
            f = false;
          }
    }
    std::printf("\n]}\n");
    (void)hipFree(dout);
    return 0;
  }
  if (wide_ab) {
    std::printf("{\"stream_read_GBps\": %.1f, \"k1k2\": [", stream_gbps);
    set_crc_mfma(true);
    set_crc_lds_max_mib(0);
    bool f = true;
    for (uint64_t mib : std::vector<uint64_t>{1, 8, 16, 32, 64, 128, 256, 1024}) {
      const uint64_t n = mib << 20;
      if (n > total) continue;
      for (int rep = 0; rep < 2; ++rep)
        for (int w : {0, 1, 2}) {
          set_crc_wide(w);
          Run r = bench_block(d, n, t, dmeta, dpart, s, n >= (256ull << 20) ? std::max(3, iters / 10) : iters, host);
          std::printf("%s\n  {\"bytes\": %llu, \"wide\": %d, \"rep\": %d, \"us\": %.2f, \"GBps\": %.1f, \"of_stream\": %.3f, "
                      "\"ok\": %s}", f ? "" : ",", static_cast<unsigned long long>(n), w, rep, r.us, n / r.us / 1e3,
                      n / r.us / 1e3 / stream_gbps, r.ok ? "true" : "false");
          f = false;
        }
    }
    std::printf("\n]}\n");
    return 0;
  }
  if (sweep) {
    // where the 64 MiB K1/K2 time goes: per-workgroup fixed cost (grid) vs load latency (ring)
    std::printf("{\"stream_read_1GiB_GBps\": %.1f, \"stream\": [", stream_gbps);
    bool f = true;
    for (uint64_t n : std::vector<uint64_t>{8ull << 20, 64ull << 20, 256ull << 20}) {
      uint32_t* dout = nullptr;
      CK(hipMalloc(&dout, 4 * kStreamReadGrid * 4));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(launch_stream_read(d, n, dout, s));
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; ++i) CK(launch_stream_read(d, n, dout, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = 1e3 * ms / iters;
      std::printf("%s{\"bytes\": %llu, \"us\": %.2f, \"GBps\": %.1f}", f ? "" : ", ",
                  static_cast<unsigned long long>(n), us, n / us / 1e3);
      f = false;
      (void)hipFree(dout);
    }
    std::printf("], \"k1k2\": [");
    f = true;
    set_crc_mfma(true);
    set_crc_lds_max_mib(0);
    for (uint64_t n : std::vector<uint64_t>{8ull << 20, 64ull << 20, 256ull << 20}) {
      for (int ring : {2, 3, 4}) {
        set_crc_ring(crc_ring_buffers(), ring);
        for (int grid : {128, 256, 384, 512, 640, 768}) {
          if (ring > 2 && grid > 512) continue;
          // the kernel choice follows ring_for(ntiles): below kCrcRingMinTiles it is the R = 2 kernel
          Run r = bench_block(d, n, t, dmeta, dpart, s, iters, host, grid);
          std::printf("%s\n  {\"bytes\": %llu, \"ring\": %d, \"grid\": %d, \"us\": %.2f, \"GBps\": %.1f, \"ok\": %s}",
                      f ? "" : ",", static_cast<unsigned long long>(n), ring, grid, r.us, n / r.us / 1e3,
                      r.ok ? "true" : "false");
          f = false;
        }
      }
    }
    std::printf("\n]}\n");
    return 0;
  }
  std::printf("{\"iters\": %d, \"scrub_ring_buffers\": %d, \"tile_ring_buffers\": %d, \"stream_read_GBps\": %.1f, "
              "\"k1k2\": [", iters, crc_ring_buffers(), crc_tile_ring_buffers(), stream_gbps);
  bool first = true;
  for (uint64_t n : std::vector<uint64_t>{4096, 65536, 1ull << 20, 8ull << 20, 64ull << 20, total}) {
    if (n > total) continue;
    for (int mf = 2; mf >= 0; --mf) {  // 2: the production size-based dispatch
      set_crc_mfma(mf >= 1);
      set_crc_lds_max_mib(mf == 2 ? kCrcLdsMaxMibDefault : 0);
      Run r = bench_block(d, n, t, dmeta, dpart, s, n >= (256ull << 20) ? std::max(3, iters / 10) : iters, host);
      std::printf("%s\n  {\"bytes\": %llu, \"impl\": \"%s\", \"us\": %.2f, \"GBps\": %.1f, \"of_stream\": %.3f, \"ok\": %s}",
                  first ? "" : ",", static_cast<unsigned long long>(n),
                  mf == 2 ? "dispatch" : (mf ? "mfma" : "lds_tables"), r.us, n / r.us / 1e3,
                  n / r.us / 1e3 / stream_gbps, r.ok ? "true" : "false");
      first = false;
    }
    set_crc_lds_max_mib(kCrcLdsMaxMibDefault);
  }
  std::printf("\n], \"scrub\": [");
  // K1b over total bytes as 1 MiB blocks (meta images from the K1 pass above)
  const uint64_t bs = 1 << 20, nb = total / bs;
  std::vector<uint32_t> metas(total / kSliceBytes);
  crc32_slices(host.data(), total, metas.data());
  for (auto& v : metas) v = __builtin_bswap32(v);
  CK(hipMemcpy(dmeta, metas.data(), metas.size() * 4, hipMemcpyHostToDevice));
  std::vector<ScrubBlock> blocks(nb);
  for (uint64_t b = 0; b < nb; ++b) {
    blocks[b].data = d + b * bs;
    blocks[b].meta = dmeta + b * (bs / kSliceBytes);
    blocks[b].s_full = bs / kSliceBytes;
    blocks[b].tile_start = b * (bs / kSliceBytes / kSlicesPerTile);
    blocks[b].tail_len = 0;
    blocks[b].tail_init = 0;
  }
  ScrubBlock* dblocks = nullptr;
  uint32_t* dbad = nullptr;
  CK(hipMalloc(&dblocks, nb * sizeof(ScrubBlock)));
  CK(hipMalloc(&dbad, nb * 4));
  CK(hipMemcpy(dblocks, blocks.data(), nb * sizeof(ScrubBlock), hipMemcpyHostToDevice));
  ScrubLaunch sl{};
  sl.blocks = dblocks;
  sl.nblocks = static_cast<uint32_t>(nb);
  sl.ntiles = nb * (bs / kSliceBytes / kSlicesPerTile);
  sl.full_init = crc_init_term(kSliceBytes);
  sl.bad = dbad;
  first = true;
  const bool fp4_saved = crc_fp4_enabled();
  for (int mf = 2; mf >= 0; --mf) {  // 2: matrix cores, FP4 form; 1: i8 form; 0: LDS tables
    set_crc_mfma(mf >= 1);
    set_crc_fp4(mf == 2);
    CK(hipMemset(dbad, 0xFF, nb * 4));
    CK(launch_scrub(sl, t, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> bad(nb);
    CK(hipMemcpy(bad.data(), dbad, nb * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    for (uint32_t v : bad) ok = ok && v == 0xFFFFFFFFu;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int it = std::max(3, iters / 10);
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < it; ++i) CK(launch_scrub(sl, t, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    double us = 1e3 * ms / it;
    std::printf("%s\n  {\"bytes\": %llu, \"blocks\": %llu, \"impl\": \"%s\", \"us\": %.1f, \"GBps\": %.1f, "
                "\"of_stream\": %.3f, \"ok\": %s}",
                first ? "" : ",", static_cast<unsigned long long>(total), static_cast<unsigned long long>(nb),
                mf == 2 ? "mfma_fp4" : (mf ? "mfma" : "lds_tables"), us, total / us / 1e3, total / us / 1e3 / stream_gbps,
                ok ? "true" : "false");
    first = false;
  }
  set_crc_fp4(fp4_saved);
  std::printf("\n], \"rs\": [");
  // K4: RS(k,m) parity of k shards of `shard` bytes, device-resident (kernel only)
  first = true;
  for (auto km : std::vector<std::pair<int, int>>{{6, 3}, {4, 2}, {10, 4}}) {
    const int k = km.first, m = km.second;
    const uint64_t shard = std::min<uint64_t>(16ull << 20, total / (k + m)) & ~uint64_t(255);
    CK(hipMemcpy(d, host.data(), (k + m) * shard, hipMemcpyHostToDevice));  // earlier outputs overwrote inputs
    std::vector<uint8_t> mat(static_cast<size_t>(m) * k);
    for (int r = 0; r < m; ++r)
      for (int c = 0; c < k; ++c) mat[r * k + c] = static_cast<uint8_t>(1 + ((r * 7 + c * 13) % 255));
    std::vector<uint32_t> htab(static_cast<size_t>(m) * k * 8);
    gf_nibble_tables(mat.data(), m, k, htab.data());
    uint32_t* dtab = nullptr;
    CK(hipMalloc(&dtab, htab.size() * 4));
    CK(hipMemcpy(dtab, htab.data(), htab.size() * 4, hipMemcpyHostToDevice));
    GfLaunch g{};
    g.k = k;
    g.rows = m;
    g.len = shard;
    g.tables = dtab;
    for (int c = 0; c < k; ++c) g.in[c] = d + c * shard;
    for (int r = 0; r < m; ++r) g.out[r] = d + (k + r) * shard;
    CK(launch_gf_matmul(g, s));  // warm-up + spot check of one output byte per row
    CK(hipStreamSynchronize(s));
    bool ok = true;
    for (int r = 0; r < m && ok; ++r) {
      uint8_t got = 0;
      CK(hipMemcpy(&got, g.out[r] + 12345, 1, hipMemcpyDeviceToHost));
      uint8_t want = 0;
      for (int c = 0; c < k; ++c) want ^= dfs::gf::mul(mat[r * k + c], host[c * shard + 12345]);
      ok = got == want;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < 20; ++i) CK(launch_gf_matmul(g, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    double us = 1e3 * ms / 20;
    std::printf("%s\n  {\"k\": %d, \"m\": %d, \"shard_bytes\": %llu, \"us\": %.1f, \"input_GBps\": %.1f, "
                "\"hbm_GBps\": %.1f, \"ok\": %s}",
                first ? "" : ",", k, m, static_cast<unsigned long long>(shard), us, k * shard / us / 1e3,
                (k + m) * shard / us / 1e3, ok ? "true" : "false");
    first = false;
    (void)hipFree(dtab);
  }
  std::printf("\n]}\n");
  return 0;
}
