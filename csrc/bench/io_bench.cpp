// io_bench — native ChunkServer I/O + kernel microbenchmark (C45).
//
// Reference: dfs/chunkserver/benches/io_bench.rs (criterion: write+fsync and read of
// 4 KiB / 64 KiB / 1 MiB, plus a 4 KiB partial read at offset 32 KiB of a 64 KiB file).
// Same cases against the HBM chunk store, in both durability modes, plus the data-plane
// kernels the reference runs on the CPU: CRC-32 slice checksums (GPU vs PCLMUL CPU),
// batched scrub, and Reed-Solomon RS(6,3) encode (GPU vs CPU). Run under
// `rocprofv3 --kernel-trace --stats` to get per-kernel device time.
//
//   io_bench [--device N] [--dir PATH] [--iters N] [--no-fsync] [--staged] [--rs-only]   -> one JSON object
//   io_bench --disk-sweep [--dir PATH]   -> aggregate 1 MiB write+fdatasync bandwidth of the
//            storage directory at 1..240 concurrent writers, buffered and O_DIRECT (what bounds
//            nvme-sync replication when every GPU of a node writes RF replicas to one volume)
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "trace.h"
#include "chunk_store.h"
#include "disk_gate.h"
#include "crc32.h"
#include "gf256.h"
#include "journal.h"
#include "md5_mb.h"

using namespace dfs;
using Clock = std::chrono::steady_clock;

static double secs(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

struct Lat {
  std::vector<double> v;
  void add(double s) { v.push_back(s); }
  double pct(double p) {
    if (v.empty()) return 0;
    std::vector<double> s = v;
    std::sort(s.begin(), s.end());
    return s[std::min(s.size() - 1, static_cast<size_t>(p * s.size()))];
  }
  double mean() const {
    double t = 0;
    for (double x : v) t += x;
    return v.empty() ? 0 : t / v.size();
  }
};

static std::vector<uint8_t> random_bytes(size_t n, uint32_t seed) {
  std::vector<uint8_t> b(n);
  std::mt19937_64 g(seed);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t x = g();
    std::memcpy(&b[i], &x, 8);
  }
  for (; i < n; ++i) b[i] = static_cast<uint8_t>(g());
  return b;
}

static void emit_case(bool& first, const char* name, size_t size, Lat& l) {
  std::printf("%s\n    \"%s_%zu\": {\"mean_us\": %.2f, \"p50_us\": %.2f, \"p99_us\": %.2f, \"MBps\": %.1f}",
              first ? "" : ",", name, size, l.mean() * 1e6, l.pct(0.5) * 1e6, l.pct(0.99) * 1e6,
              l.mean() > 0 ? size / l.mean() / (1 << 20) : 0.0);
  first = false;
}

// T threads each write `per` 1 MiB files (+ an 8 KiB sidecar like the .meta) with fdatasync.
static void disk_case(const std::string& dir, int threads, int per, bool direct, int gate_slots, bool first) {
  std::filesystem::create_directories(dir);
  DiskGate gate(dir, gate_slots);
  const size_t n = 1 << 20, meta = 8192;
  std::vector<Lat> lat(threads);
  std::vector<std::thread> ts;
  std::atomic<int> errors{0};
  auto t0 = Clock::now();
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      void* buf = nullptr;
      if (posix_memalign(&buf, 4096, n) != 0) { ++errors; return; }
      std::memset(buf, t + 1, n);
      for (int i = 0; i < per; ++i) {
        std::string f = dir + "/t" + std::to_string(t) + "_" + std::to_string(i);
        auto a = Clock::now();
        DiskGate::Slot slot = gate.acquire();
        int fd = ::open(f.c_str(), O_CREAT | O_WRONLY | O_TRUNC | (direct ? O_DIRECT : 0), 0644);
        int fm = ::open((f + ".meta").c_str(), O_CREAT | O_WRONLY | O_TRUNC | (direct ? O_DIRECT : 0), 0644);
        if (fd < 0 || fm < 0 || ::pwrite(fd, buf, n, 0) != static_cast<ssize_t>(n) ||
            ::pwrite(fm, buf, meta, 0) != static_cast<ssize_t>(meta) || ::fdatasync(fd) != 0 || ::fdatasync(fm) != 0)
          ++errors;
        if (fd >= 0) ::close(fd);
        if (fm >= 0) ::close(fm);
        slot.release();
        lat[t].add(secs(a, Clock::now()));
      }
      std::free(buf);
    });
  for (auto& th : ts) th.join();
  double el = secs(t0, Clock::now());
  Lat all;
  for (auto& l : lat) all.v.insert(all.v.end(), l.v.begin(), l.v.end());
  std::printf("%s\n    {\"threads\": %d, \"direct\": %s, \"gate\": %d, \"files\": %d, \"GBps\": %.2f, \"p50_ms\": %.3f, \"p99_ms\": %.3f, \"errors\": %d}",
              first ? "" : ",", threads, direct ? "true" : "false", gate_slots, threads * per,
              double(threads) * per * n / el / 1e9, all.pct(0.5) * 1e3, all.pct(0.99) * 1e3, errors.load());
  std::fflush(stdout);
  std::filesystem::remove_all(dir);
}

// Journal variant of disk_case: T threads append 1 MiB records (+ a 4 KiB header/.meta
// frame) to ONE preallocated, already-written segment at reserved offsets; a record is
// durable once a group fdatasync that started after its pwrite completed. mode 0: buffered
// appends, 1: O_DIRECT appends, 2: O_DIRECT|O_DSYNC per append (no group commit).
static void journal_case(const std::string& dir, int threads, int per, int mode, bool first, bool falloc = false,
                         int syncers = 1) {
  std::filesystem::create_directories(dir);
  const size_t n = 1 << 20, hdr = 4096, rec = n + hdr;
  const uint64_t total = uint64_t(threads) * per * rec;
  std::string f = dir + "/journal.seg";
  int fd = ::open(f.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0644);
  if (falloc) {  // unwritten extents: every first write converts them (a metadata change per flush)
    (void)::fallocate(fd, 0, 0, static_cast<off_t>(total));
    ::fsync(fd);
    ::close(fd);
  } else {  // preallocate by writing: later appends overwrite written extents (no metadata change)
    std::vector<uint8_t> z(8 << 20, 0);
    for (uint64_t off = 0; off < total; off += z.size())
      if (::pwrite(fd, z.data(), std::min<uint64_t>(z.size(), total - off), off) < 0) break;
    ::fsync(fd);
    ::close(fd);
  }
  int flags = O_RDWR | (mode >= 1 ? O_DIRECT : 0) | (mode == 2 ? O_DSYNC : 0);
  fd = ::open(f.c_str(), flags);
  std::atomic<uint64_t> tail{0};
  std::mutex mu;
  std::condition_variable cv;
  uint64_t issued = 0, done = 0, rounds = 0, syncing = 0;
  int running = 0;
  // group commit with up to `syncers` rounds in flight: a writer whose ticket no running
  // round covers starts its own (BlockJournal::commit's pipelined mode)
  auto group_sync = [&]() {
    std::unique_lock<std::mutex> lk(mu);
    uint64_t ticket = ++issued;
    while (done < ticket) {
      if (syncing >= ticket || running >= syncers) { cv.wait(lk); continue; }
      ++running;
      uint64_t covers = issued;
      syncing = covers;
      lk.unlock();
      ::fdatasync(fd);
      lk.lock();
      --running;
      done = std::max(done, covers);
      ++rounds;
      cv.notify_all();
    }
  };
  std::vector<Lat> lat(threads);
  std::vector<std::thread> ts;
  std::atomic<int> errors{0};
  auto t0 = Clock::now();
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t] {
      void* buf = nullptr;
      if (posix_memalign(&buf, 4096, rec) != 0) { ++errors; return; }
      std::memset(buf, t + 1, rec);
      for (int i = 0; i < per; ++i) {
        auto a = Clock::now();
        uint64_t off = tail.fetch_add(rec);
        if (::pwrite(fd, buf, rec, off) != static_cast<ssize_t>(rec)) ++errors;
        if (mode != 2) group_sync();
        lat[t].add(secs(a, Clock::now()));
      }
      std::free(buf);
    });
  for (auto& th : ts) th.join();
  double el = secs(t0, Clock::now());
  ::close(fd);
  Lat all;
  for (auto& l : lat) all.v.insert(all.v.end(), l.v.begin(), l.v.end());
  static const char* names[] = {"buffered", "direct", "direct_dsync"};
  std::printf("%s\n    {\"journal\": \"%s%s\", \"syncers\": %d, \"threads\": %d, \"records\": %d, \"GBps\": %.2f, \"p50_ms\": %.3f, \"p99_ms\": %.3f, \"sync_rounds\": %llu, \"errors\": %d}",
              first ? "" : ",", names[mode], falloc ? "_fallocated" : "", syncers, threads, threads * per, double(threads) * per * n / el / 1e9,
              all.pct(0.5) * 1e3, all.pct(0.99) * 1e3, static_cast<unsigned long long>(rounds), errors.load());
  std::fflush(stdout);
  std::filesystem::remove_all(dir);
}

// K journals on one volume (K chunkservers of a node), `per_journal` writers each appending
// 1 MiB records to their journal's pre-written segment. Flush policy:
//   0 per-journal group commit (each journal's leader fdatasyncs its own file),
//   1 node-wide combining, fdatasync: one leader at a time flushes every journal with
//     completed-but-unflushed records (one round covers all K),
//   2 node-wide combining, syncfs: one leader syncfs()es the filesystem per round.
// Threads stand in for processes: flush costs are the kernel's and the device's either way.
static void multi_journal_case(const std::string& dir, int K, int per_journal, int per, int mode, bool first) {
  std::filesystem::create_directories(dir);
  const size_t n = 1 << 20, hdr = 4096, rec = n + hdr;
  const uint64_t total = uint64_t(per_journal) * per * rec;
  std::vector<int> fds(K);
  for (int k = 0; k < K; ++k) {
    std::string f = dir + "/j" + std::to_string(k) + ".seg";
    int fd = ::open(f.c_str(), O_CREAT | O_RDWR | O_TRUNC, 0644);
    std::vector<uint8_t> z(8 << 20, 0);
    for (uint64_t off = 0; off < total; off += z.size())
      if (::pwrite(fd, z.data(), std::min<uint64_t>(z.size(), total - off), off) < 0) break;
    ::fsync(fd);
    fds[k] = fd;
  }
  std::vector<std::atomic<uint64_t>> tails(K);
  for (auto& t : tails) t = 0;
  // per-journal state (mode 0) or one node-wide state (modes 1, 2): ticket counters
  struct G {
    std::mutex mu;
    std::condition_variable cv;
    uint64_t issued = 0, done = 0;
    bool running = false;
  };
  std::vector<G> gs(mode == 0 ? K : 1);
  std::vector<std::atomic<bool>> dirty(K);
  for (auto& d : dirty) d = false;
  std::atomic<uint64_t> rounds{0};
  auto sync_for = [&](int k) {
    G& g = gs[mode == 0 ? k : 0];
    std::unique_lock<std::mutex> lk(g.mu);
    uint64_t ticket = ++g.issued;
    while (g.done < ticket) {
      if (g.running) {
        g.cv.wait(lk);
        continue;
      }
      g.running = true;
      uint64_t covers = g.issued;
      lk.unlock();
      if (mode == 0) {
        ::fdatasync(fds[k]);
      } else if (mode == 1) {
        for (int j = 0; j < K; ++j)
          if (dirty[j].exchange(false)) ::fdatasync(fds[j]);
      } else {
        ::syncfs(fds[0]);
      }
      lk.lock();
      g.running = false;
      g.done = covers;
      rounds++;
      g.cv.notify_all();
    }
  };
  std::vector<Lat> lat(K * per_journal);
  std::vector<std::thread> ts;
  std::atomic<int> errors{0};
  auto t0 = Clock::now();
  for (int k = 0; k < K; ++k)
    for (int w = 0; w < per_journal; ++w)
      ts.emplace_back([&, k, w] {
        std::vector<uint8_t> buf(rec, static_cast<uint8_t>(k * 16 + w + 1));
        for (int i = 0; i < per; ++i) {
          auto a = Clock::now();
          uint64_t off = tails[k].fetch_add(rec);
          if (::pwrite(fds[k], buf.data(), rec, off) != static_cast<ssize_t>(rec)) ++errors;
          dirty[k] = true;
          sync_for(k);
          lat[k * per_journal + w].add(secs(a, Clock::now()));
        }
      });
  for (auto& th : ts) th.join();
  double el = secs(t0, Clock::now());
  for (int fd : fds) ::close(fd);
  Lat all;
  for (auto& l : lat) all.v.insert(all.v.end(), l.v.begin(), l.v.end());
  static const char* names[] = {"per_journal_fdatasync", "node_wide_fdatasync", "node_wide_syncfs"};
  std::printf("%s\n    {\"journals\": %d, \"writers_per_journal\": %d, \"flush\": \"%s\", \"records\": %d, \"GBps\": %.2f, "
              "\"p50_ms\": %.3f, \"p99_ms\": %.3f, \"flush_rounds\": %llu, \"errors\": %d}",
              first ? "" : ",", K, per_journal, names[mode], K * per_journal * per,
              double(K) * per_journal * per * n / el / 1e9, all.pct(0.5) * 1e3, all.pct(0.99) * 1e3,
              static_cast<unsigned long long>(rounds.load()), errors.load());
  std::fflush(stdout);
  std::filesystem::remove_all(dir);
}

// PCIe roofline of the bench path: `threads` concurrent 1 MiB transfers
// host <-> HBM, (a) plain hipMemcpyAsync from pinned memory on one stream per thread (the
// copy engines' rate) and (b) the store's fused kernels (crc_write_copy_kernel: load over
// PCIe + checksum + store into HBM; crc_read_copy_kernel: verify + store over PCIe) from
// registered host memory, as the fast path drives them for co-located clients.
static void pcie_roofline(int device, int threads, int per, size_t n) {
  (void)hipSetDevice(device);
  StoreConfig cfg;
  cfg.storage_dir = "/tmp/io_bench_roofline";
  cfg.device = device;
  cfg.hbm_capacity = 16ull << 30;
  cfg.durability = Durability::HbmAck;
  cfg.sync_writes = false;
  cfg.lanes = std::max(8, threads);
  double h2d = 0, d2h = 0, wr = 0, rd = 0;
  uint64_t fused_w = 0, fused_r = 0;
  {
    ChunkStore store(cfg);
    store.debug_pause_spill(true);  // store only: no NVMe spill competing for the host
    // the writers' buffers as the fast path has them: ordinary pages, registered with the
    // store (hipHostRegister) so the fused kernels reach them over PCIe
    std::vector<uint8_t*> host(threads), dev(threads);
    std::vector<hipStream_t> st(threads);
    for (int t = 0; t < threads; ++t) {
      host[t] = static_cast<uint8_t*>(std::aligned_alloc(4096, (n + 4095) & ~size_t(4095)));
      for (size_t i = 0; i < n; ++i) host[t][i] = static_cast<uint8_t>(i * 131 + t);
      store.register_host(host[t], n);
      (void)hipMalloc(reinterpret_cast<void**>(&dev[t]), n);
      (void)hipStreamCreateWithFlags(&st[t], hipStreamNonBlocking);
    }
    auto run = [&](auto&& body) {
      std::vector<std::thread> ts;
      auto t0 = Clock::now();
      for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
          for (int i = 0; i < per; ++i) body(t);
        });
      for (auto& th : ts) th.join();
      return double(threads) * per * n / secs(t0, Clock::now()) / 1e9;
    };
    auto h2d_one = [&](int t) {
      (void)hipMemcpyAsync(dev[t], host[t], n, hipMemcpyHostToDevice, st[t]);
      (void)hipStreamSynchronize(st[t]);
    };
    auto d2h_one = [&](int t) {
      (void)hipMemcpyAsync(host[t], dev[t], n, hipMemcpyDeviceToHost, st[t]);
      (void)hipStreamSynchronize(st[t]);
    };
    run(h2d_one);  // warm-up
    h2d = run(h2d_one);
    d2h = run(d2h_one);
    for (int t = 0; t < threads; ++t)  // d2h overwrote them with the device's (random) bytes
      for (size_t i = 0; i < n; ++i) host[t][i] = static_cast<uint8_t>(i * 131 + t);
    std::vector<uint32_t> crcs(threads);
    for (int t = 0; t < threads; ++t) crcs[t] = crc32(host[t], n);
    std::atomic<int> seq{0};
    auto write_one = [&](int t) {
      std::string id = "r" + std::to_string(seq.fetch_add(1));
      if (!store.write(id, host[t], n, crcs[t]).ok) std::fprintf(stderr, "roofline write failed\n");
    };
    run(write_one);  // warm-up, and the blocks the reads use
    wr = run(write_one);
    std::atomic<int> rs{0};
    rd = run([&](int t) {
      std::string id = "r" + std::to_string(rs.fetch_add(1) % (threads * per));
      ReadResult r = store.read_into(id, 0, n, host[t]);
      if (r.status != ReadStatus::Ok) std::fprintf(stderr, "roofline read failed\n");
    });
    StoreStats ss = store.stats();
    fused_w = ss.fused_writes;
    fused_r = ss.fused_reads;
    for (int t = 0; t < threads; ++t) {
      store.unregister_host(host[t]);
      std::free(host[t]);
      (void)hipFree(dev[t]);
      (void)hipStreamDestroy(st[t]);
    }
    store.debug_pause_spill(false);
  }
  std::filesystem::remove_all("/tmp/io_bench_roofline");
  std::printf("{\"pcie_roofline\": {\"threads\": %d, \"bytes\": %zu, \"per_thread\": %d, \"memcpy_h2d_GBps\": %.2f, "
              "\"memcpy_d2h_GBps\": %.2f, \"store_write_fused_GBps\": %.2f, \"store_read_fused_GBps\": %.2f, "
              "\"write_vs_h2d\": %.3f, \"read_vs_d2h\": %.3f, \"fused_writes\": %llu, \"fused_reads\": %llu}}\n",
              threads, n, per, h2d, d2h, wr, rd, h2d > 0 ? wr / h2d : 0.0, d2h > 0 ? rd / d2h : 0.0,
              static_cast<unsigned long long>(fused_w), static_cast<unsigned long long>(fused_r));
}

// --md5: the ETag hash of a 1 MiB write, OpenSSL on one core against the multi-buffer engine
// (md5_mb.cpp): one message alone (latency), and `conc` messages in flight at once, each
// submitter starting its next as soon as its last returns (the benchmark's 10 writers).
static void md5_bench(int conc, int per) {
  const size_t n = 1 << 20;
  std::vector<std::vector<uint8_t>> bufs(conc, std::vector<uint8_t>(n));
  std::mt19937 rng(5);
  for (auto& b : bufs)
    for (auto& x : b) x = static_cast<uint8_t>(rng());
  auto timed = [&](auto&& fn) {
    auto t0 = Clock::now();
    fn();
    return secs(t0, Clock::now());
  };
  // engine: nullptr = OpenSSL on each submitting thread
  auto run = [&](Md5MultiBuffer* mb, double* one_ms, double* p50, double* cpu_cores) {
    double best = 1e9;
    for (int i = 0; i < 10; ++i)
      best = std::min(best, timed([&] {
        if (mb) (void)mb->submit(bufs[0].data(), n).get();
        else (void)md5_hex_scalar(bufs[0].data(), n);
      }));
    *one_ms = 1e3 * best;
    std::vector<double> lat;
    std::mutex mu;
    struct timespec c0, c1;
    ::clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c0);
    const double wall = timed([&] {
      std::vector<std::thread> ts;
      for (int t = 0; t < conc; ++t)
        ts.emplace_back([&, t] {
          std::vector<double> mine;
          for (int i = 0; i < per; ++i) {
            auto a = Clock::now();
            if (mb) (void)mb->submit(bufs[t].data(), n).get();
            else (void)md5_hex_scalar(bufs[t].data(), n);
            mine.push_back(secs(a, Clock::now()));
          }
          std::lock_guard<std::mutex> g(mu);
          lat.insert(lat.end(), mine.begin(), mine.end());
        });
      for (auto& t : ts) t.join();
    });
    ::clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c1);
    std::sort(lat.begin(), lat.end());
    *p50 = 1e3 * lat[lat.size() / 2];
    *cpu_cores = ((c1.tv_sec - c0.tv_sec) + 1e-9 * (c1.tv_nsec - c0.tv_nsec)) / wall;
    return conc * per * 1.0 / wall;  // MiB/s
  };
  std::printf("{\"md5\": {\"avx512\": %s, \"concurrent\": %d, \"engines\": [", Md5MultiBuffer::available() ? "true" : "false",
              conc);
  struct E {
    const char* name;
    Md5MultiBuffer::Kind kind;
    int lanes;
  };
  bool first = true;
  for (const E& e : {E{"openssl", Md5MultiBuffer::Kind::None, 0}, E{"scalar-x1", Md5MultiBuffer::Kind::Scalar, 1},
                     E{"scalar-x2", Md5MultiBuffer::Kind::Scalar, 2}, E{"scalar-x3", Md5MultiBuffer::Kind::Scalar, 3},
                     E{"avx512-x16", Md5MultiBuffer::Kind::Avx512, 16}}) {
    if (e.kind == Md5MultiBuffer::Kind::Avx512 && !Md5MultiBuffer::available()) continue;
    std::unique_ptr<Md5MultiBuffer> mb;
    if (e.kind != Md5MultiBuffer::Kind::None) {
      const int lanes = e.kind == Md5MultiBuffer::Kind::Avx512 ? Md5MultiBuffer::kLanes : e.lanes;
      mb = std::make_unique<Md5MultiBuffer>((conc + lanes - 1) / lanes, e.kind, e.lanes);
    }
    double one = 0, p50 = 0, cores = 0;
    const double rate = run(mb.get(), &one, &p50, &cores);
    std::printf("%s\n  {\"engine\": \"%s\", \"one_mib_ms\": %.3f, \"mib_s\": %.0f, \"p50_ms\": %.3f, \"cpu_cores\": %.2f}",
                first ? "" : ",", e.name, one, rate, p50, cores);
    first = false;
  }
  std::printf("\n]}}\n");
}

// --roofline: what the volume gives a chunkserver's journal right now — T writers appending
// 1 MiB block records (header + .meta image + data) to a BlockJournal like the store's
// (8 parts, 256 MiB segments, written out once before the timed appends), each record
// group-committed before the next. bench.py runs it on every rank at once after its timed
// region, so each rank's share of the node's volume is recorded next to its throughput.
static void roofline(const std::string& dir, int threads, int per) {
  std::filesystem::remove_all(dir);
  const uint64_t n = 1 << 20, S = num_slices(n);
  double secs_total = 0, mbps = 0;
  std::vector<double> lat;
  {
    JournalConfig c;
    c.dir = dir;
    c.max_segs = static_cast<int>((uint64_t(threads) * per * (n + 12288)) / (c.seg_bytes * 9 / 10)) + 2;
    BlockJournal j(c);
    (void)j.recover();
    for (int i = 0; i < 6000 && j.stats().parts_unready; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    std::vector<uint8_t> meta(4 * S, 0);
    std::mutex mu;
    auto t0 = Clock::now();
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([&, t] {
        std::vector<uint8_t> buf(n, static_cast<uint8_t>(t + 1));
        std::vector<double> mine;
        for (int i = 0; i < per; ++i) {
          auto a = Clock::now();
          JournalRec r;
          std::string err;
          if (!j.reserve(n, S, &r, &err) || !j.write(r, 0, buf.data(), n) ||
              !j.finish(&r, "roof-" + std::to_string(t) + "-" + std::to_string(i), n, 0, meta.data(), S) ||
              !j.commit(r))
            break;
          mine.push_back(secs(a, Clock::now()));
        }
        std::lock_guard<std::mutex> g(mu);
        lat.insert(lat.end(), mine.begin(), mine.end());
      });
    for (auto& t : ts) t.join();
    secs_total = secs(t0, Clock::now());
    mbps = lat.size() * (n / 1048576.0) / std::max(1e-9, secs_total);
  }
  std::filesystem::remove_all(dir);
  std::sort(lat.begin(), lat.end());
  auto pct = [&](double p) { return lat.empty() ? 0.0 : 1e3 * lat[std::min(lat.size() - 1, size_t(lat.size() * p))]; };
  std::printf("{\"roofline_mb_s\": %.1f, \"threads\": %d, \"records\": %zu, \"seconds\": %.3f, \"p50_ms\": %.3f, "
              "\"p99_ms\": %.3f}\n", mbps, threads, lat.size(), secs_total, pct(0.5), pct(0.99));
}

int main(int argc, char** argv) {
  dfs::trace_init();  // before any thread: roctx's first range calls setenv (trace.h)
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--md5") {
      int conc = 10, per = 20;
      for (int j = 1; j + 1 < argc; ++j) {
        if (std::string(argv[j]) == "--conc") conc = std::atoi(argv[j + 1]);
        if (std::string(argv[j]) == "--per") per = std::atoi(argv[j + 1]);
      }
      md5_bench(std::max(1, conc), std::max(1, per));
      return 0;
    }
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--roofline") {
      std::string dir = "/tmp/io_bench_roofline";
      int threads = 10, per = 30;
      for (int j = 1; j + 1 < argc; ++j) {
        if (std::string(argv[j]) == "--dir") dir = argv[j + 1];
        if (std::string(argv[j]) == "--threads") threads = std::atoi(argv[j + 1]);
        if (std::string(argv[j]) == "--per") per = std::atoi(argv[j + 1]);
      }
      roofline(dir, std::max(1, threads), std::max(1, per));
      return 0;
    }
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--multi-journal") {
      std::string dir = "/tmp/io_bench_mj";
      for (int j = 1; j + 1 < argc; ++j)
        if (std::string(argv[j]) == "--dir") dir = argv[j + 1];
      std::printf("{\"multi_journal\": [");
      bool first = true;
      for (int K : {1, 3, 7})
        for (int mode = 0; mode < 3; ++mode) {
          if (K == 1 && mode == 1) continue;  // same as per-journal
          multi_journal_case(dir, K, K == 1 ? 21 : 3, K == 1 ? 12 : (K == 3 ? 28 : 12), mode, first);
          first = false;
        }
      std::printf("\n]}\n");
      return 0;
    }
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--pcie-roofline") {
      int threads = 10, per = 200;
      size_t n = 1 << 20;
      for (int j = 1; j + 1 < argc; ++j) {
        if (std::string(argv[j]) == "--threads") threads = std::atoi(argv[j + 1]);
        if (std::string(argv[j]) == "--per") per = std::atoi(argv[j + 1]);
        if (std::string(argv[j]) == "--bytes") n = std::strtoull(argv[j + 1], nullptr, 10);
      }
      pcie_roofline(0, threads, per, n);
      return 0;
    }
  int device = 0, iters = 50;
  bool fsync = true;
  bool zero_copy = true;
  bool rs_only = false;  // only the RS(6,3) end-to-end case (pipeline tuning sweeps)
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--journal-sweep") {
      std::string dir = "/tmp/io_bench_journal";
      for (int j = 1; j + 1 < argc; ++j)
        if (std::string(argv[j]) == "--dir") dir = argv[j + 1];
      std::printf("{\"journal_sweep\": [");
      bool first = true;
      for (int t : {1, 10, 30, 70}) {
        disk_case(dir + "_files", t, std::max(8, 2400 / t / 4), false, 0, first);
        first = false;
        for (int mode = 0; mode < 3; ++mode) journal_case(dir, t, std::max(8, 2400 / t / 4), mode, false);
        journal_case(dir, t, std::max(8, 2400 / t / 4), 0, false, true);
        journal_case(dir, t, std::max(8, 2400 / t / 4), 0, false, false, 4);  // pipelined rounds
        journal_case(dir, t, std::max(8, 2400 / t / 4), 0, false, true, 4);
      }
      std::printf("\n]}\n");
      return 0;
    }
  for (int i = 1; i < argc; ++i)
    if (std::string(argv[i]) == "--disk-sweep") {
      std::string dir = "/tmp/io_bench_disk";
      for (int j = 1; j + 1 < argc; ++j)
        if (std::string(argv[j]) == "--dir") dir = argv[j + 1];
      std::printf("{\"disk_sweep\": [");
      bool first = true;
      for (int j = 1; j + 1 < argc; ++j)  // --cases "threads:gate[:direct],..." in this order
        if (std::string(argv[j]) == "--cases") {
          std::string c = argv[j + 1];
          size_t p = 0;
          while (p < c.size()) {
            size_t e = c.find(',', p);
            if (e == std::string::npos) e = c.size();
            int t = 0, g = 0, d = 0;  // threads:gate[:direct]
            if (std::sscanf(c.substr(p, e - p).c_str(), "%d:%d:%d", &t, &g, &d) >= 2 && t > 0) {
              disk_case(dir, t, std::max(4, 2400 / t / 4), d != 0, g, first);
              first = false;
            }
            p = e + 1;
          }
          std::printf("\n]}\n");
          return 0;
        }
      for (int direct = 0; direct < 2; ++direct)
        for (int t : {1, 10, 30, 60, 120, 240}) {
          disk_case(dir, t, std::max(4, 2400 / t / 4), direct != 0, 0, first);
          first = false;
        }
      // the same overload behind the node-wide gate (what ChunkStore does)
      for (int g : {8, 16, 24, 32})
        for (int t : {60, 240}) disk_case(dir, t, std::max(4, 2400 / t / 4), false, g, false);
      std::printf("\n]}\n");
      return 0;
    }
  std::string dir = "/tmp/io_bench_store";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--device" && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (a == "--dir" && i + 1 < argc) dir = argv[++i];
    else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
    else if (a == "--no-fsync") fsync = false;
    else if (a == "--staged") zero_copy = false;
    else if (a == "--rs-only") rs_only = true;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) device = -1;
  std::filesystem::remove_all(dir);

  // zero_copy: the client buffers are registered with the store the way the fast path
  // registers a client's shared-memory arena (one DMA per copy); --staged: pinned bounce
  if (rs_only) std::printf("{\n  \"device\": %d, \"rs_only\": true,\n", device);
  if (!rs_only) {
  std::printf("{\n  \"device\": %d, \"iters\": %d, \"fsync\": %s, \"zero_copy\": %s,\n  \"store\": {", device,
              iters, fsync ? "true" : "false", zero_copy ? "true" : "false");
  bool first = true;
  const size_t sizes[] = {4096, 65536, 1 << 20, 64u << 20};
  for (int mode = 0; mode < 2; ++mode) {
    StoreConfig cfg;
    cfg.storage_dir = dir + (mode == 0 ? "/nvme" : "/hbm");
    cfg.device = device;
    cfg.hbm_capacity = device >= 0 ? (8ull << 30) : 0;
    cfg.durability = mode == 0 ? Durability::NvmeSync : Durability::HbmAck;
    cfg.sync_writes = fsync;
    ChunkStore store(cfg);
    const char* tag = mode == 0 ? "write_nvme_sync" : "write_hbm_ack";
    for (size_t sz : sizes) {
      int n = sz >= (64u << 20) ? std::max(3, iters / 10) : iters;
      auto data = random_bytes(sz, static_cast<uint32_t>(sz + mode));
      uint32_t crc = crc32(data.data(), sz);
      Lat w, r, pr;
      std::vector<uint8_t> out(sz);
      bool reg = zero_copy && store.register_host(data.data(), sz) && store.register_host(out.data(), sz);
      for (int i = 0; i < n; ++i) {
        std::string id = std::string("b") + std::to_string(mode) + "_" + std::to_string(sz) + "_" + std::to_string(i);
        auto t0 = Clock::now();
        WriteResult wr = store.write(id, data.data(), sz, crc);
        auto t1 = Clock::now();
        if (!wr.ok) {
          std::fprintf(stderr, "write failed: %s\n", wr.error.c_str());
          return 1;
        }
        w.add(secs(t0, t1));
        t0 = Clock::now();
        ReadResult rr = store.read_into(id, 0, sz, out.data());
        t1 = Clock::now();
        if (rr.status != ReadStatus::Ok || std::memcmp(out.data(), data.data(), sz) != 0) {
          std::fprintf(stderr, "read mismatch (%s)\n", rr.error.c_str());
          return 1;
        }
        r.add(secs(t0, t1));
        if (sz >= 65536) {
          t0 = Clock::now();
          rr = store.read_into(id, 32768, 4096, out.data());
          t1 = Clock::now();
          if (rr.status != ReadStatus::Ok || std::memcmp(out.data(), data.data() + 32768, 4096) != 0) {
            std::fprintf(stderr, "partial read mismatch\n");
            return 1;
          }
          pr.add(secs(t0, t1));
        }
      }
      if (reg) {
        store.unregister_host(data.data());
        store.unregister_host(out.data());
      }
      emit_case(first, tag, sz, w);
      emit_case(first, mode == 0 ? "read_after_nvme_sync" : "read_after_hbm_ack", sz, r);
      if (sz >= 65536) emit_case(first, mode == 0 ? "partial4k_nvme" : "partial4k_hbm", sz, pr);
    }
    store.flush();
    if (mode == 0) {
      auto t0 = Clock::now();
      auto bad = store.scrub();
      auto t1 = Clock::now();
      StoreStats st = store.stats();
      std::printf(",\n    \"scrub\": {\"blocks\": %llu, \"bytes\": %llu, \"seconds\": %.4f, \"GBps\": %.2f, \"bad\": %zu}",
                  static_cast<unsigned long long>(st.blocks), static_cast<unsigned long long>(st.bytes),
                  secs(t0, t1), st.bytes / std::max(1e-9, secs(t0, t1)) / 1e9, bad.size());
    }
  }
  std::printf("\n  },\n");

  // ---- K1b: batched scrub of HBM-resident blocks (kernel path only; no disk re-read)
  if (device >= 0) {
    StoreConfig cfg;
    cfg.storage_dir = dir + "/scrub";
    cfg.device = device;
    cfg.hbm_capacity = 2ull << 30;
    cfg.durability = Durability::HbmAck;
    cfg.sync_writes = false;
    ChunkStore s(cfg);
    const int nb = 1024;
    auto data = random_bytes((1 << 20) + 100, 11);
    std::vector<std::string> ids;
    for (int i = 0; i < nb; ++i) {
      size_t sz = (i % 4 == 3) ? (1 << 20) + 100 : (1 << 20);  // every 4th block has a short tail slice
      std::string id = "s" + std::to_string(i);
      if (!s.stage(id, data.data(), sz, crc32(data.data(), sz)).ok) return 1;
      ids.push_back(id);
    }
    s.scrub_resident(ids);  // warm-up (allocations, code object)
    auto t0 = Clock::now();
    auto bad = s.scrub_resident(ids);
    auto t1 = Clock::now();
    double bytes = nb * double(1 << 20) + (nb / 4) * 100.0;
    std::printf("  \"scrub_hbm_1024x1MiB\": {\"seconds\": %.6f, \"GBps\": %.1f, \"bad\": %zu},\n", secs(t0, t1),
                bytes / secs(t0, t1) / 1e9, bad.size());
  }

  // ---- CRC: GPU (H2D + K1/K2) vs CPU PCLMUL, 256 MiB
  {
    const size_t n = 256u << 20;
    auto data = random_bytes(n, 7);
    auto t0 = Clock::now();
    uint32_t cpu = crc32(data.data(), n);
    auto t1 = Clock::now();
    double cpu_s = secs(t0, t1);
    double gpu_s = 0;
    uint32_t gpu = cpu;
    if (device >= 0) {
      StoreConfig cfg;
      cfg.storage_dir = dir + "/crc";
      cfg.device = device;
      cfg.hbm_capacity = 1ull << 30;
      ChunkStore s(cfg);
      std::vector<uint32_t> sl;
      s.gpu_crc(data.data(), 1 << 20, &sl);  // warm-up (tables, lanes)
      t0 = Clock::now();
      gpu = s.gpu_crc(data.data(), n, &sl);
      t1 = Clock::now();
      gpu_s = secs(t0, t1);
    }
    std::printf("  \"crc32_256MiB\": {\"cpu_GBps\": %.2f, \"gpu_incl_h2d_GBps\": %.2f, \"match\": %s},\n",
                n / cpu_s / 1e9, gpu_s > 0 ? n / gpu_s / 1e9 : 0.0, cpu == gpu ? "true" : "false");
  }

  }  // !rs_only

  // ---- RS(6,3) encode of 6 x 16 MiB shards: GPU vs CPU
  {
    const int k = 6, m = 3;
    const size_t len = 16u << 20;
    gf::Matrix full = gf::rs_matrix(k, m);
    gf::Matrix parity(full.begin() + k, full.end());
    std::vector<std::vector<uint8_t>> in(k), out_c(m, std::vector<uint8_t>(len)), out_g(m, std::vector<uint8_t>(len));
    std::vector<const uint8_t*> ip;
    std::vector<uint8_t*> oc, og;
    for (int i = 0; i < k; ++i) {
      in[i] = random_bytes(len, 100 + i);
      ip.push_back(in[i].data());
    }
    for (int i = 0; i < m; ++i) {
      oc.push_back(out_c[i].data());
      og.push_back(out_g[i].data());
    }
    auto t0 = Clock::now();
    gf::matmul_cpu(parity, ip.data(), oc.data(), len);
    auto t1 = Clock::now();
    double cpu_s = secs(t0, t1), gpu_s = 0;
    bool match = true;
    if (device >= 0) {
      StoreConfig cfg;
      cfg.storage_dir = dir + "/rs";
      cfg.device = device;
      cfg.hbm_capacity = 1ull << 30;
      ChunkStore s(cfg);
      if (zero_copy) {  // shards in registered memory, as a client's shm slot is
        for (auto* p : ip) s.register_host(p, len);
        for (auto* p : og) s.register_host(p, len);
      }
      s.gf_matmul_gpu(parity, ip, og, 4096);  // warm-up
      gpu_s = 1e9;
      for (int rep = 0; rep < 3; ++rep) {
        t0 = Clock::now();
        s.gf_matmul_gpu(parity, ip, og, len);
        t1 = Clock::now();
        gpu_s = std::min(gpu_s, secs(t0, t1));
      }
      for (int i = 0; i < m; ++i) match = match && out_c[i] == out_g[i];
    }
    std::printf("  \"rs63_encode_96MiB\": {\"cpu_GBps\": %.2f, \"gpu_incl_copies_GBps\": %.2f, \"match\": %s}\n}\n",
                k * len / cpu_s / 1e9, gpu_s > 0 ? k * len / gpu_s / 1e9 : 0.0, match ? "true" : "false");
  }
  std::filesystem::remove_all(dir);
  return 0;
}
