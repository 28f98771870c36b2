// ChunkStore implementation. See chunk_store.h for the design.
#include "chunk_store.h"
#include "thread_name.h"
#include "trace.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <future>
#include <stdexcept>
#include <unordered_map>

#include "crc32.h"
#include "gf256.h"

namespace dfs {

// ---------------------------------------------------------------- group commit
// The block stays resident in HBM (or is re-read on a miss): once its bytes are on the
// device, the host page-cache copy is dead weight that the kernel would otherwise have to
// reclaim in our writers' context under memory pressure. Drop it.
static void drop_cached(int fd) {
#ifdef POSIX_FADV_DONTNEED
  if (fd >= 0) (void)::posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
#endif
}

GroupSync::GroupSync(const std::string& dir, Mode mode) : mode_(mode) {
  fd_ = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
}

GroupSync::~GroupSync() {
  if (fd_ >= 0) ::close(fd_);
}

bool GroupSync::sync() {
  if (fd_ < 0) return false;
  std::unique_lock<std::mutex> lk(mu_);
  uint64_t ticket = ++issued_;
  while (done_ < ticket) {
    if (running_) {
      cv_.wait(lk);
      continue;
    }
    // lead a round: it covers every ticket issued before the flush starts
    running_ = true;
    uint64_t covers = issued_;
    lk.unlock();
    bool ok = (mode_ == Mode::FileSystem ? ::syncfs(fd_) : ::fsync(fd_)) == 0;
    lk.lock();
    running_ = false;
    if (!ok) failed_.emplace_back(done_ + 1, covers);
    done_ = covers;
    rounds_++;
    cv_.notify_all();
  }
  for (const auto& f : failed_)
    if (ticket >= f.first && ticket <= f.second) return false;
  return true;
}


namespace {

// the journal's clock (steady_clock since its epoch, ns): compared with last_append_ns()
uint64_t mono_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
          .count());
}

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

std::string errno_str(const std::string& what) { return what + ": " + std::strerror(errno); }

#define HIP_OK(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                                                   " at " #expr);                             \
  } while (0)

bool write_all(int fd, const uint8_t* p, uint64_t n, uint64_t off) {
  while (n) {
    ssize_t w = ::pwrite(fd, p, n, static_cast<off_t>(off));
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= static_cast<uint64_t>(w);
    off += static_cast<uint64_t>(w);
  }
  return true;
}

// DFS_ODIRECT=1 (A/B, off by default): a fresh block's data file is written with O_DIRECT
// straight from the caller's page-aligned buffer (the client's registered shm slot), so the
// bytes skip the page cache (no 1 MiB memcpy into it, no eviction afterwards); the sub-4 KiB
// tail, if any, is written buffered after clearing O_DIRECT on the descriptor.
bool odirect_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("DFS_ODIRECT");
    return e && e[0] == '1';
  }();
  return v;
}

// `off` and `p` 4 KiB aligned; a sub-4 KiB tail clears O_DIRECT (the last write of a file).
// If the kernel refuses the direct write of these pages (EINVAL / EFAULT: memory it cannot
// pin for DMA), the descriptor drops O_DIRECT and the range is written buffered.
bool write_direct(int fd, const uint8_t* p, uint64_t n, uint64_t off = 0) {
  auto buffered = [&](uint64_t from) {
    const int fl = ::fcntl(fd, F_GETFL);
    if (fl < 0 || ::fcntl(fd, F_SETFL, fl & ~O_DIRECT) != 0) return false;
    return write_all(fd, p + from, n - from, off + from);
  };
  const uint64_t na = n & ~uint64_t(4095);
  if (na && !write_all(fd, p, na, off)) {
    if (errno != EINVAL && errno != EFAULT) return false;
    return buffered(0);
  }
  return na == n || buffered(na);
}

bool read_all(int fd, uint8_t* p, uint64_t n, uint64_t off) {
  while (n) {
    ssize_t r = ::pread(fd, p, n, static_cast<off_t>(off));
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    if (r == 0) return false;
    p += r;
    n -= static_cast<uint64_t>(r);
    off += static_cast<uint64_t>(r);
  }
  return true;
}

bool file_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

int64_t file_size(const std::string& p) {
  struct stat st;
  if (::stat(p.c_str(), &st) != 0) return -1;
  return st.st_size;
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}

bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

void mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur.push_back(path[i]);
    if (path[i] == '/' || i + 1 == path.size()) ::mkdir(cur.c_str(), 0755);
  }
}

}  // namespace

// ---------------------------------------------------------------- ChunkStore
ChunkStore::ChunkStore(StoreConfig cfg) : cfg_(std::move(cfg)) {
  mkdirs(cfg_.storage_dir);
  if (!cfg_.cold_dir.empty()) mkdirs(cfg_.cold_dir);
  // Opt-in (DFS_GROUP_SYNC=1): a syncfs() round wins on devices where each flush is
  // expensive and many writers are in flight; on overlay filesystems it flushes far more
  // than our two files, so the per-file fdatasync pair stays the default.
  const char* gs = std::getenv("DFS_GROUP_SYNC");
  if (cfg_.sync_writes && gs && std::string(gs) == "1") gsync_ = std::make_unique<GroupSync>(cfg_.storage_dir);
  const char* ds = std::getenv("DFS_DIR_SYNC");  // 0: A/B runs only (renames not made durable)
  if (cfg_.sync_writes && !(ds && std::string(ds) == "0")) {
    // renames into place are durable only once the directory is flushed (the reference
    // writes final names directly and sync_all()s the file, chunkserver.rs:192-209)
    dsync_hot_ = std::make_unique<GroupSync>(cfg_.storage_dir, GroupSync::Mode::Directory);
    if (!cfg_.cold_dir.empty())
      dsync_cold_ = std::make_unique<GroupSync>(cfg_.cold_dir, GroupSync::Mode::Directory);
  }
  if (cfg_.sync_writes)
    gate_ = std::make_unique<DiskGate>(cfg_.storage_dir,
                                       cfg_.disk_inflight < 0 ? disk_inflight_default() : cfg_.disk_inflight);
  if (gpu()) {
    HIP_OK(hipSetDevice(cfg_.device));
    // how host threads wait for the device (every staging / read waits on an event):
    // DFS_HIP_SYNC=spin (busy-wait), yield, block (sleep until the completion interrupt);
    // unset = the runtime's default. Must precede the device's first use in the process.
    if (const char* hs = std::getenv("DFS_HIP_SYNC")) {
      const std::string m = hs;
      const unsigned f = m == "spin" ? hipDeviceScheduleSpin : m == "yield" ? hipDeviceScheduleYield
                         : m == "block" ? hipDeviceScheduleBlockingSync : hipDeviceScheduleAuto;
      if (hipSetDeviceFlags(f) != hipSuccess) {
        (void)hipGetLastError();
        std::fprintf(stderr, "[store] DFS_HIP_SYNC=%s ignored: the device was already in use\n", hs);
      }
    }
    uint64_t cap = cfg_.hbm_capacity;
    if (cap == 0) {
      size_t fr = 0, tot = 0;
      HIP_OK(hipMemGetInfo(&fr, &tot));
      cap = std::min<uint64_t>(fr / 2, 64ull << 30);
    }
    cap = align_up(cap, 1 << 20);
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&arena_), cap));
    alloc_ = ExtentAllocator(cap);
    int nl = std::max(2, cfg_.lanes);  // gf_matmul_gpu pipelines over two lanes
    for (int i = 0; i < nl; ++i) {
      auto l = std::make_unique<Lane>();
      HIP_OK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
      for (int b = 0; b < 2; ++b) {
        HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&l->pinned[b]), kChunk, hipHostMallocDefault));
        HIP_OK(hipEventCreateWithFlags(&l->ev[b], hipEventDisableTiming));
      }
      HIP_OK(hipMalloc(reinterpret_cast<void**>(&l->dscratch), 2 * kMaxGridCrc * sizeof(uint32_t)));
      ensure_hscratch(l.get(), 64 << 10);
      free_lanes_.push_back(l.get());
      lanes_.push_back(std::move(l));
    }
    dtables_ = upload_crc_tables(lanes_[0]->stream);
    if (!dtables_) throw std::runtime_error("failed to upload GPU tables");
    pull_pool_ = std::make_shared<PinnedPool>();
    if (hipMalloc(reinterpret_cast<void**>(&pull_parts_dev_), kMaxGridCrc * sizeof(uint32_t)) != hipSuccess) {
      (void)hipGetLastError();
      pull_parts_dev_ = nullptr;  // no receiver pull: the transport's senders copy
    }
    st_.hbm_capacity = cap;
    if (cfg_.durability == Durability::HbmAck)
      for (int i = 0; i < std::max(1, cfg_.spill_threads); ++i) spillers_.emplace_back([this] { spill_worker(); });
  }
  int jmode = cfg_.journal;
  if (jmode < 0) jmode = env_int("DFS_JOURNAL", 1);
  if (jmode > 0 && cfg_.sync_writes && cfg_.durability == Durability::NvmeSync) {
    // DFS_JOURNAL_EXPORT: store (default: the journal is the block's home; reference-format
    // files are exported at a bounded rate while the volume has headroom), never (no export
    // except on request), idle (round 4: everything materialized once the writers pause)
    const char* em = std::getenv("DFS_JOURNAL_EXPORT");
    const std::string emode = em && *em ? em : "store";
    store_mode_ = emode != "idle";
    export_ = emode != "never";
    export_bps_ = env_int("DFS_EXPORT_MBPS", 256) * 1e6;
    // while acked writes are arriving (an append in the last 50 ms) the exporter runs at this
    // rate in batches of at most 8 MiB, so its per-file flushes and directory flush never
    // land on the writers as a 64-file burst; at full rate again once they pause
    export_busy_bps_ = env_int("DFS_EXPORT_BUSY_MBPS", 64) * 1e6;
    uint64_t vol_total = 0;
    {
      struct statvfs sv;
      if (::statvfs(cfg_.storage_dir.c_str(), &sv) == 0) vol_total = static_cast<uint64_t>(sv.f_blocks) * sv.f_frsize;
    }
    // export doubles a block's footprint until its segment recycles: only while the volume
    // keeps this much free (default 25 % of it, at least 8 GiB)
    export_headroom_ = static_cast<uint64_t>(env_int("DFS_EXPORT_HEADROOM_MB", 0)) << 20;
    if (export_headroom_ == 0) export_headroom_ = std::max<uint64_t>(8ull << 30, vol_total / 4);
    JournalConfig jc;
    jc.dir = cfg_.storage_dir + "/.journal";
    jc.seg_bytes = static_cast<uint64_t>(env_int("DFS_JOURNAL_SEG_MB", 256)) << 20;
    jc.grow = store_mode_;
    jc.max_segs = env_int("DFS_JOURNAL_SEGS", store_mode_ ? 0 : 16);
    jc.reserve_bytes = static_cast<uint64_t>(env_int("DFS_JOURNAL_RESERVE_MB", 0)) << 20;
    if (jc.reserve_bytes == 0) jc.reserve_bytes = std::max<uint64_t>(2ull << 30, vol_total / 50);
    jc.direct = env_int("DFS_JOURNAL_DIRECT", 0) != 0;
    jc.early_wb_bytes = static_cast<uint64_t>(env_int("DFS_JOURNAL_EARLY_WB_KB", 0)) << 10;
    jc.spares = env_int("DFS_JOURNAL_SPARES", store_mode_ ? 4 : 2);
    jc.spares_low = env_int("DFS_JOURNAL_SPARES_LOW", 2);
    jc.zero_fill = env_int("DFS_JOURNAL_ZERO_FILL", 1) != 0;
    jc.idle_fill_ms = env_int("DFS_JOURNAL_IDLE_FILL_MS", 20);
    jc.syncers = env_int("DFS_JOURNAL_SYNCERS", 1);
    jc.parts = env_int("DFS_JOURNAL_PARTS", 8);
    jc.full_timeout_s = env_int("DFS_JOURNAL_FULL_TIMEOUT_S", 120);
    jc.sync_delay_us = env_int("DFS_JOURNAL_SYNC_DELAY_US", 0);
    jc.sync = cfg_.sync_writes;
    mat_pressure_ = env_int("DFS_JOURNAL_PRESSURE_PCT", 70) / 100.0;
    journal_bypass_ = env_int("DFS_JOURNAL_BYPASS", 1) != 0;  // 0: writers wait for the materializer
    journal_gate_ = env_int("DFS_JOURNAL_GATE", 0) != 0;
    // 500 ms: the pauses of a running benchmark (barriers, device syncs, a warm-up's end) are
    // shorter, so a batch and its syncfs do not land on the first timed writes (with 100 ms,
    // 256 blocks were materialized there and the driver's run lost 15-25 %: r4o, r4y)
    mat_idle_ns_ = static_cast<uint64_t>(env_int("DFS_JOURNAL_IDLE_MS", 500)) * 1000000ull;
    journal_ = std::make_unique<BlockJournal>(jc);
    replay_journal();
  }
  scan_dirs();
  if (journal_) materializer_ = std::thread([this] {
    name_thread("jr-export");
    materializer_loop();
  });
}

ChunkStore::~ChunkStore() {
  if (materializer_.joinable()) {
    {  // round-4 mode: a clean stop writes every journal record out (one pass; what fails
       // stays in the journal and is replayed); store mode: the journal is the home, the
       // exporter just stops
      std::lock_guard<std::mutex> g(mu_);
      mat_stop_ = true;
      mat_paused_ = false;
    }
    mat_cv_.notify_all();
    materializer_.join();
    bool drained;
    {
      std::lock_guard<std::mutex> g(mu_);
      drained = mat_q_.empty() && mat_errors_ == 0;
    }
    if (store_mode_) {
      journal_->mark_sealed_now();  // the next start trusts these records
      journal_->retire_ready();     // and finds no dead segment (the active one is sealed now)
    }
    else if (drained && !journal_->stats().failed) journal_->retire_all();
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : spillers_) t.join();
  if (gpu()) {
    (void)hipSetDevice(cfg_.device);
    for (auto& l : lanes_) {
      (void)hipStreamSynchronize(l->stream);
      for (int b = 0; b < 2; ++b) {
        (void)hipHostFree(l->pinned[b]);
        (void)hipEventDestroy(l->ev[b]);
      }
      (void)hipFree(l->dscratch);
      if (l->hscratch) (void)hipHostFree(l->hscratch);
      (void)hipStreamDestroy(l->stream);
    }
    if (arena_) (void)hipFree(arena_);
    if (dtables_) (void)hipFree(dtables_);
    if (pull_parts_dev_) (void)hipFree(pull_parts_dev_);
  }
}

std::string ChunkStore::data_path(const std::string& id, bool cold) const {
  return (cold ? cfg_.cold_dir : cfg_.storage_dir) + "/" + id;
}
std::string ChunkStore::meta_path(const std::string& id, bool cold) const {
  return data_path(id, cold) + ".meta";
}

void ChunkStore::scan_dirs() {
  auto scan = [&](const std::string& dir, bool cold) {
    if (dir.empty()) return;
    DIR* d = ::opendir(dir.c_str());
    if (!d) return;
    while (dirent* e = ::readdir(d)) {
      std::string name = e->d_name;
      if (ends_with(name, ".tmp")) {  // a write that crashed before its rename
        ::unlink((dir + "/" + name).c_str());
        continue;
      }
      // dot names: the journal directory, quarantined files (block ids never start with '.')
      if (name.empty() || name[0] == '.' || ends_with(name, ".meta")) continue;
      if (index_.count(name)) continue;  // replayed from the journal, its home
      int64_t sz = file_size(dir + "/" + name);
      if (sz < 0) continue;
      // a data file is a block only with its complete .meta beside it: anything else is a
      // write torn by a crash, set aside instead of being reported as a present block
      int64_t msz = file_size(dir + "/" + name + ".meta");
      if (msz != static_cast<int64_t>(num_slices(static_cast<uint64_t>(sz)) * 4)) {
        ::rename((dir + "/" + name).c_str(), (dir + "/.quarantine-" + name).c_str());
        if (msz >= 0) ::rename((dir + "/" + name + ".meta").c_str(), (dir + "/.quarantine-" + name + ".meta").c_str());
        continue;
      }
      Block& b = index_[name];
      b.size = static_cast<uint64_t>(sz);
      b.on_disk = true;
      b.cold = cold;
    }
    ::closedir(d);
  };
  std::lock_guard<std::mutex> g(mu_);
  scan(cfg_.storage_dir, false);
  scan(cfg_.cold_dir, true);
}

uint64_t ChunkStore::alloc_bytes(uint64_t n) const {
  return align_up(std::max<uint64_t>(n, 1), 256) + align_up(std::max<uint64_t>(num_slices(n) * 4, 4), 256);
}

void ChunkStore::touch_locked(const std::string& id, Block& b) {
  if (b.in_lru) lru_.erase(b.lru);
  lru_.push_front(id);
  b.lru = lru_.begin();
  b.in_lru = true;
}

void ChunkStore::lru_remove_locked(Block& b) {
  if (b.in_lru) lru_.erase(b.lru);
  b.in_lru = false;
}

void ChunkStore::free_extent_locked(Block& b) {
  if (b.dev_off >= 0) {
    alloc_.free(static_cast<uint64_t>(b.dev_off), b.dev_bytes);
    b.dev_off = -1;
    b.dev_bytes = 0;
  }
}

int64_t ChunkStore::alloc_locked(std::unique_lock<std::mutex>& lk, uint64_t bytes) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(30);
  for (;;) {
    int64_t off = alloc_.alloc(bytes);
    if (off >= 0) return off;
    bool evicted = false, any_dirty = false;
    for (auto it = lru_.rbegin(); it != lru_.rend(); ++it) {
      Block& b = index_[*it];
      if (b.dirty) any_dirty = true;
      if (b.pins == 0 && !b.dirty && (b.on_disk || b.jrec.seg) && b.dev_off >= 0) {
        free_extent_locked(b);
        lru_remove_locked(b);
        ++st_.evictions;
        evicted = true;
        break;
      }
    }
    if (evicted) continue;
    if (std::chrono::steady_clock::now() > deadline) return -1;
    if (!any_dirty && lru_.empty()) return -1;
    cv_.wait_for(lk, std::chrono::milliseconds(50));
  }
}

ChunkStore::Lane* ChunkStore::acquire_lane() {
  std::unique_lock<std::mutex> lk(lane_mu_);
  if (free_lanes_.empty()) {  // every stream context busy: count the wait (lane_waits / lane_wait_ns)
    const auto t0 = std::chrono::steady_clock::now();
    lane_cv_.wait(lk, [&] { return !free_lanes_.empty(); });
    lane_waits_++;
    lane_wait_ns_ += static_cast<uint64_t>(
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
  }
  Lane* l = free_lanes_.back();
  free_lanes_.pop_back();
  return l;
}

void ChunkStore::release_lane(Lane* l) {
  {
    std::lock_guard<std::mutex> g(lane_mu_);
    free_lanes_.push_back(l);
  }
  lane_cv_.notify_one();
}

void ChunkStore::ensure_hscratch(Lane* l, uint64_t bytes) {
  bytes = align_up(bytes + 2 * kMaxGridCrc * sizeof(uint32_t), 4096);
  if (l->hscratch_cap >= bytes) return;
  if (l->hscratch) HIP_OK(hipHostFree(l->hscratch));
  HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&l->hscratch), bytes, hipHostMallocDefault));
  l->hscratch_cap = bytes;
  if (hipHostGetDevicePointer(&l->hscratch_dev, l->hscratch, 0) != hipSuccess) {
    (void)hipGetLastError();
    l->hscratch_dev = nullptr;
  }
}

// Enqueue the CRC kernel on the lane stream and the D2H of its partials into hscratch
// (partials at [0, 2*kMaxGridCrc) u32). Returns the grid used (0 = nothing launched).
namespace {
struct CrcPlan {
  CrcLaunch a{};
  int grid = 0;
};
CrcPlan plan_crc(const uint8_t* d, uint64_t n, uint32_t* meta_out, const uint32_t* meta_expect, bool want_block,
                 uint64_t byte_lo, uint64_t byte_hi) {
  CrcPlan p;
  CrcLaunch& a = p.a;
  a.data = d;
  a.n = n;
  a.s_full = n / kSliceBytes;
  a.tail_len = static_cast<uint32_t>(n % kSliceBytes);
  a.full_init = crc_init_term(kSliceBytes);
  a.tail_init = a.tail_len ? crc_init_term(a.tail_len) : 0;
  a.meta_out = meta_out;
  a.meta_expect = meta_expect;
  if (n == 0) return p;
  if (want_block) {
    a.slice_lo = 0;
    a.slice_hi = a.s_full;
    a.vfront = (kSlicesPerTile - a.s_full % kSlicesPerTile) % kSlicesPerTile;
    a.ntiles = (a.s_full + a.vfront) / kSlicesPerTile;
    a.has_tail = a.tail_len ? 1 : 0;
  } else {
    uint64_t first = byte_lo / kSliceBytes;
    uint64_t last = (byte_hi - 1) / kSliceBytes;
    a.slice_lo = first;
    a.slice_hi = std::min<uint64_t>(last + 1, a.s_full);
    a.vfront = 0;
    a.ntiles = a.slice_hi > a.slice_lo ? (a.slice_hi - a.slice_lo + kSlicesPerTile - 1) / kSlicesPerTile : 0;
    if (a.slice_hi < a.slice_lo) a.slice_hi = a.slice_lo;
    a.has_tail = (a.tail_len && last >= a.s_full) ? 1 : 0;
  }
  p.grid = crc_grid_for(a.ntiles, a.has_tail);
  return p;
}
}  // namespace

bool ChunkStore::run_crc(Lane* l, const uint8_t* dptr, uint64_t n, uint32_t* meta_out, const uint32_t* meta_expect,
                         bool want_block, uint64_t byte_lo, uint64_t byte_hi, CrcOut* out, std::string* err,
                         uint8_t* hmeta, bool* meta_done) {
  // Synchronous helper used by paths that do not need to overlap anything else.
  if (meta_done) *meta_done = false;
  CrcPlan p = plan_crc(dptr, n, meta_out, meta_expect, want_block, byte_lo, byte_hi);
  if (p.grid == 0) {
    out->block_crc = 0;
    out->bad_slice = -1;
    return true;
  }
  // With a device view of the lane's pinned scratch, the kernel writes its partials (and, on
  // the LDS kernel, the .meta image) straight into host memory: no readback copies, each of
  // which costs a copy-engine round trip of ~20-30 us whatever its size (profiles/r5_final).
  const bool want_host_meta = meta_out && crc_meta_host_ok(p.a.ntiles) && (hmeta || (want_block && p.a.has_tail));
  // no destination of the caller's: the image goes after the partials (only its tail word is
  // read); sized before any pointer into the scratch is taken (a caller's hmeta already is)
  if (want_host_meta && !hmeta) ensure_hscratch(l, (p.a.s_full + 1) * 4 + 16);
  auto* hp = reinterpret_cast<uint32_t*>(l->hscratch);
  auto* hdev = static_cast<uint8_t*>(l->hscratch_dev);
  const bool direct = hdev != nullptr;
  const bool host_meta = direct && want_host_meta;
  uint32_t* tail_host = nullptr;  // where the tail slice's BE CRC lands on the host
  if (host_meta) {
    uint8_t* dst = hmeta ? hmeta : l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
    p.a.meta_host = reinterpret_cast<uint32_t*>(hdev + (dst - l->hscratch));
    tail_host = reinterpret_cast<uint32_t*>(dst) + p.a.s_full;
  }
  if (direct) {
    p.a.part_crc = want_block ? reinterpret_cast<uint32_t*>(hdev) : nullptr;
    p.a.part_bad = meta_expect ? reinterpret_cast<uint32_t*>(hdev) + kMaxGridCrc : nullptr;
  } else {
    p.a.part_crc = want_block ? l->dscratch : nullptr;
    p.a.part_bad = meta_expect ? l->dscratch + kMaxGridCrc : nullptr;
  }
  hipError_t e = launch_crc(p.a, dtables_, p.grid, l->stream);
  launches_++;
  if (e != hipSuccess) {
    *err = std::string("crc kernel launch: ") + hipGetErrorString(e);
    return false;
  }
  uint64_t tail_meta_off = 2 * kMaxGridCrc;
  if (!direct)
    HIP_OK(hipMemcpyAsync(hp, l->dscratch, 2 * kMaxGridCrc * sizeof(uint32_t), hipMemcpyDeviceToHost, l->stream));
  if (want_block && p.a.has_tail && meta_out && !host_meta)
    HIP_OK(hipMemcpyAsync(hp + tail_meta_off, meta_out + p.a.s_full, 4, hipMemcpyDeviceToHost, l->stream));
  HIP_OK(hipStreamSynchronize(l->stream));
  if (host_meta && hmeta && meta_done) *meta_done = true;
  out->bad_slice = -1;
  if (meta_expect) {
    uint32_t bad = 0xFFFFFFFFu;
    for (int g = 0; g < p.grid; ++g) bad = std::min(bad, hp[kMaxGridCrc + g]);
    if (bad != 0xFFFFFFFFu) out->bad_slice = bad;
  }
  if (want_block) {
    uint32_t r = 0;
    for (int g = 0; g < p.grid; ++g) r ^= hp[g];
    if (p.a.has_tail) {
      uint32_t tail_crc = __builtin_bswap32(host_meta ? *tail_host : hp[tail_meta_off]);
      r = crc_shift(r, p.a.tail_len) ^ (tail_crc ^ p.a.tail_init);
    }
    out->block_crc = r ^ crc_init_term(n);
  }
  return true;
}

// The writer's bytes sit in registered host memory: one kernel copies them into the HBM
// extent while it checksums them, and leaves the .meta image and the whole-block partials in
// the lane's pinned scratch (crc_write_copy_kernel) — no SDMA copy, no readback copies.
bool ChunkStore::write_copy(Lane* l, const uint8_t* src_dev, uint8_t* dst, uint64_t n, uint32_t* dmeta,
                            uint8_t* hmeta, CrcOut* out, std::string* err) {
  CrcPlan p = plan_crc(src_dev, n, dmeta, nullptr, true, 0, n);
  auto* hp = reinterpret_cast<uint32_t*>(l->hscratch);
  WriteCopyLaunch w;
  w.c = p.a;
  w.c.part_crc = static_cast<uint32_t*>(l->hscratch_dev);
  w.dst = dst;
  w.meta_host = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(l->hscratch_dev) + (hmeta - l->hscratch));
  hipError_t e = launch_write_copy(w, dtables_, p.grid, l->stream);
  launches_++;
  if (e != hipSuccess) {
    *err = std::string("write-copy kernel launch: ") + hipGetErrorString(e);
    return false;
  }
  HIP_OK(hipStreamSynchronize(l->stream));
  fused_writes_++;
  uint32_t r = 0;
  for (int g = 0; g < p.grid; ++g) r ^= hp[g];
  if (p.a.has_tail) {
    const uint32_t tail_crc = __builtin_bswap32(reinterpret_cast<const uint32_t*>(hmeta)[p.a.s_full]);
    r = crc_shift(r, p.a.tail_len) ^ (tail_crc ^ p.a.tail_init);
  }
  out->block_crc = r ^ crc_init_term(n);
  out->bad_slice = -1;
  return true;
}

// hscratch layout of a sliced stage: [0, 16 + S*4) after the standard partial words holds
// the host .meta image (as in stage_impl), then kMaxGridCrc partial words per slice.
static uint64_t sliced_partials_off(uint64_t S) {
  return (2 * kMaxGridCrc * sizeof(uint32_t) + 16 + S * 4 + 63) / 64 * 64;
}

bool ChunkStore::stage_slices_begin(const uint8_t* data, uint64_t n, uint64_t slice, SliceStage* ss,
                                    std::string* err) {
  if (!gpu() || n == 0 || slice == 0 || slice % kSliceBytes != 0 || !crc_mfma_enabled()) return false;
  const uint8_t* src_dev = device_view(data, n);
  if (!src_dev || reinterpret_cast<uintptr_t>(src_dev) % 16 != 0) return false;
  HIP_OK(hipSetDevice(cfg_.device));
  ss->ext = reserve(n);
  if (ss->ext.off < 0) {
    *err = "HBM arena full";
    return false;
  }
  ss->n = n;
  ss->slice = slice;
  Lane* l = acquire_lane();
  ss->lane = l;
  const uint64_t S = num_slices(n), nsl = (n + slice - 1) / slice;
  ensure_hscratch(l, sliced_partials_off(S) + nsl * kMaxGridCrc * sizeof(uint32_t));
  if (!l->hscratch_dev) {
    release_lane(l);
    release(ss->ext);
    ss->lane = nullptr;
    return false;
  }
  auto* dmeta = reinterpret_cast<uint32_t*>(ss->ext.ptr + align_up(n, 256));
  auto* hdev = static_cast<uint8_t*>(l->hscratch_dev);
  auto* meta_host_dev = reinterpret_cast<uint32_t*>(hdev + 2 * kMaxGridCrc * sizeof(uint32_t) + 16);
  auto* parts_dev = reinterpret_cast<uint32_t*>(hdev + sliced_partials_off(S));
  for (uint64_t k = 0; k < nsl; ++k) {
    const uint64_t off = k * slice, len = std::min(slice, n - off);
    CrcPlan p = plan_crc(src_dev + off, len, dmeta + off / kSliceBytes, nullptr, true, 0, len);
    WriteCopyLaunch w;
    w.c = p.a;
    w.c.part_crc = parts_dev + k * kMaxGridCrc;
    w.dst = ss->ext.ptr + off;
    w.meta_host = meta_host_dev + off / kSliceBytes;
    hipEvent_t ev = nullptr;
    hipError_t e = launch_write_copy(w, dtables_, p.grid, l->stream);
    launches_++;
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(ev, l->stream);
    if (e != hipSuccess) {
      if (ev) (void)hipEventDestroy(ev);
      *err = std::string("sliced stage launch: ") + hipGetErrorString(e);
      (void)hipStreamSynchronize(l->stream);
      stage_slices_end(ss);
      return false;
    }
    ss->done.push_back(ev);
    ss->grids.push_back(p.grid);
  }
  sliced_stages_++;
  return true;
}

WriteResult ChunkStore::stage_slices_finish(const std::string& id, SliceStage* ss, uint32_t expected_crc, int pins) {
  TraceRange tr("dfs.store.stage_slices");
  WriteResult res;
  auto* l = static_cast<Lane*>(ss->lane);
  HIP_OK(hipSetDevice(cfg_.device));
  HIP_OK(hipStreamSynchronize(l->stream));
  const uint64_t n = ss->n, S = num_slices(n);
  const uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
  const auto* parts = reinterpret_cast<const uint32_t*>(l->hscratch + sliced_partials_off(S));
  uint32_t raw = 0;
  for (size_t k = 0; k < ss->grids.size(); ++k) {
    const uint64_t off = k * ss->slice, len = std::min(ss->slice, n - off);
    uint32_t r = 0;
    for (int g = 0; g < ss->grids[k]; ++g) r ^= parts[k * kMaxGridCrc + g];
    const uint64_t tail = len % kSliceBytes;
    if (tail) {  // only the last slice: its short tail slice, from the host .meta image
      const uint32_t tail_crc = __builtin_bswap32(reinterpret_cast<const uint32_t*>(hmeta)[(off + len) / kSliceBytes]);
      r = crc_shift(r, tail) ^ (tail_crc ^ crc_init_term(tail));
    }
    raw = crc_shift(raw, len) ^ r;
  }
  const uint32_t crc = raw ^ crc_init_term(n);
  res.actual_crc = crc;
  if (expected_crc != 0 && crc != expected_crc) {
    {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.crc_mismatches;
    }
    res.error = "Checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " + std::to_string(crc);
    return res;  // the extent stays reserved: end() once the sends drained
  }
  auto meta = std::make_shared<std::vector<uint8_t>>(hmeta, hmeta + S * 4);
  release_lane(l);
  ss->lane = nullptr;
  insert_resident(id, ss->ext, n, crc, false, meta, pins);
  ss->ext = DevExtent{};  // owned by the index now
  res.ok = true;
  return res;
}

void ChunkStore::stage_slices_end(SliceStage* ss) {
  if (ss->lane) {
    auto* l = static_cast<Lane*>(ss->lane);
    (void)hipStreamSynchronize(l->stream);
    release_lane(l);
    ss->lane = nullptr;
  }
  for (hipEvent_t e : ss->done) (void)hipEventDestroy(e);
  ss->done.clear();
  release(ss->ext);
  ss->ext = DevExtent{};
}

bool ChunkStore::register_host(const void* p, uint64_t n) {
  if (!gpu() || !p || !n) return false;
  HIP_OK(hipSetDevice(cfg_.device));
  if (hipHostRegister(const_cast<void*>(p), n, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, const_cast<void*>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    dp = nullptr;
  }
  std::lock_guard<std::mutex> g(reg_mu_);
  reg_.emplace_back(reinterpret_cast<uintptr_t>(p), n);
  reg_dev_.push_back(reinterpret_cast<uintptr_t>(dp));
  return true;
}

uint8_t* ChunkStore::device_view(const void* p, uint64_t n) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> g(reg_mu_);
  for (size_t k = 0; k < reg_.size(); ++k) {
    const auto& r = reg_[k];
    if (a >= r.first && n <= r.second && a - r.first <= r.second - n)
      return reg_dev_[k] ? reinterpret_cast<uint8_t*>(reg_dev_[k] + (a - r.first)) : nullptr;
  }
  return nullptr;
}

void ChunkStore::unregister_host(const void* p) {
  if (!gpu()) return;
  std::lock_guard<std::mutex> g(reg_mu_);
  for (auto it = reg_.begin(); it != reg_.end(); ++it)
    if (it->first == reinterpret_cast<uintptr_t>(p)) {
      (void)hipSetDevice(cfg_.device);
      (void)hipHostUnregister(const_cast<void*>(p));
      reg_dev_.erase(reg_dev_.begin() + (it - reg_.begin()));
      reg_.erase(it);
      return;
    }
}

bool ChunkStore::host_registered(const void* p, uint64_t n) {
  uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> g(reg_mu_);
  for (auto& r : reg_)
    if (a >= r.first && n <= r.second && a - r.first <= r.second - n) return true;
  return false;
}

bool ChunkStore::h2d_chunked(Lane* l, uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (host_registered(src, n)) {  // one DMA straight from the client's pinned slot
    HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, l->stream));
    direct_dma_++;
    return true;
  }
  staged_dma_++;
  int i = 0;
  for (uint64_t off = 0; off < n; off += kChunk, i ^= 1) {
    uint64_t len = std::min<uint64_t>(kChunk, n - off);
    HIP_OK(hipEventSynchronize(l->ev[i]));
    std::memcpy(l->pinned[i], src + off, len);
    HIP_OK(hipMemcpyAsync(dst + off, l->pinned[i], len, hipMemcpyHostToDevice, l->stream));
    HIP_OK(hipEventRecord(l->ev[i], l->stream));
  }
  return true;
}

bool ChunkStore::d2h_chunked(Lane* l, uint8_t* dst, const uint8_t* src, uint64_t n) {
  if (host_registered(dst, n)) {  // straight into the client's pinned slot; caller syncs
    HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, l->stream));
    direct_dma_++;
    return true;
  }
  staged_dma_++;
  uint64_t nch = (n + kChunk - 1) / kChunk;
  auto issue = [&](uint64_t c) {
    uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, n - off);
    HIP_OK(hipMemcpyAsync(l->pinned[c & 1], src + off, len, hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipEventRecord(l->ev[c & 1], l->stream));
  };
  if (nch) issue(0);
  for (uint64_t c = 0; c < nch; ++c) {
    if (c + 1 < nch) issue(c + 1);
    HIP_OK(hipEventSynchronize(l->ev[c & 1]));
    uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, n - off);
    std::memcpy(dst + off, l->pinned[c & 1], len);
  }
  return true;
}

bool ChunkStore::persist(const std::string& id, bool cold, const uint8_t* data, uint64_t n, const uint8_t* meta_be,
                         uint64_t nslices, std::string* err) {
  std::string dp = data_path(id, cold), mp = meta_path(id, cold);
  DiskGate::Slot slot = gate_ ? gate_->acquire() : DiskGate::Slot{};
  int fd = ::open(dp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) {
    *err = errno_str("open " + dp);
    return false;
  }
  bool ok = write_all(fd, data, n, 0);
  if (!ok) {
    *err = errno_str("write " + dp);
    ::close(fd);
    return false;
  }
  int mfd = ::open(mp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (mfd < 0) {
    *err = errno_str("open " + mp);
    ::close(fd);
    return false;
  }
  ok = write_all(mfd, meta_be, nslices * 4, 0);
  if (!ok) *err = errno_str("write " + mp);
  if (ok && !make_durable(fd, mfd, cold)) {
    ok = false;
    *err = errno_str("sync " + dp);
  }
  if (ok && cfg_.sync_writes && gpu()) drop_cached(fd);
  ::close(fd);
  ::close(mfd);
  return ok;
}

bool ChunkStore::make_durable(int data_fd, int meta_fd, bool cold) {
  if (!cfg_.sync_writes) return true;
  // Group commit: one syncfs() covers the data + .meta of every writer that finished
  // writing before it started (one device cache flush for a whole burst of blocks,
  // instead of two fdatasync flushes per block). Cold-tier files may live on another
  // filesystem: they take the per-file path.
  if (gsync_ && !cold) return gsync_->sync();
  // The two flushes are independent: issue them concurrently (NVMe queues them side by
  // side) instead of paying two device round trips back to back.
  auto meta = io_.submit([meta_fd] { return ::fdatasync(meta_fd) == 0; });
  bool ok = ::fdatasync(data_fd) == 0;
  return meta.get() && ok;
}

bool ChunkStore::sync_dir(bool cold) {
  GroupSync* g = cold ? dsync_cold_.get() : dsync_hot_.get();
  return g == nullptr || g->sync();
}

bool ChunkStore::write_fd_durable(int fd, const uint8_t* p, uint64_t n, const std::string& what, std::string* err) {
  if (!write_all(fd, p, n, 0)) {
    *err = errno_str(what);
    return false;
  }
  if (cfg_.sync_writes && ::fdatasync(fd) != 0) {
    *err = errno_str("sync: " + what);
    return false;
  }
  return true;
}

bool ChunkStore::claim_fresh(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  if (index_.count(id) || writing_.count(id)) return false;
  writing_.insert(id);
  return true;
}

void ChunkStore::unclaim_fresh(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  writing_.erase(id);
}

bool ChunkStore::write_file_durable(const std::string& path, const uint8_t* p, uint64_t n, std::string* err) {
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) {
    *err = errno_str("open " + path);
    return false;
  }
  bool ok = write_all(fd, p, n, 0);
  if (!ok) *err = errno_str("write " + path);
  if (ok && cfg_.sync_writes && ::fdatasync(fd) != 0) {
    ok = false;
    *err = errno_str("sync " + path);
  }
  if (ok && cfg_.sync_writes) drop_cached(fd);
  ::close(fd);
  return ok;
}

// ---------------------------------------------------------------- write
// Block ids become file names under the storage directories: accept only a plain name
// (letters, digits, '-', '_', '.', not starting with '.'), so no id reaches outside them.
bool valid_block_id(const std::string& id) {
  if (id.empty() || id.size() > 200 || id[0] == '.') return false;
  for (char c : id) {
    bool ok = (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
              c == '.';
    if (!ok) return false;
  }
  return !ends_with(id, ".meta") && !ends_with(id, ".tmp");
}

static WriteResult bad_id(const std::string& id) {
  WriteResult r;
  r.error = "invalid block id: " + id.substr(0, 64);
  return r;
}

WriteResult ChunkStore::write(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc) {
  if (!valid_block_id(id)) return bad_id(id);
  if (!gpu()) return write_host(id, data, n, expected_crc);
  return stage_impl(id, data, n, expected_crc, true);
}

WriteResult ChunkStore::stage(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc) {
  if (!valid_block_id(id)) return bad_id(id);
  if (!gpu()) return write_host(id, data, n, expected_crc);
  return stage_impl(id, data, n, expected_crc, false);
}

void ChunkStore::insert_resident(const std::string& id, const DevExtent& ext, uint64_t n, uint32_t crc, bool on_disk,
                                 std::shared_ptr<std::vector<uint8_t>> meta, int pins, const JournalRec* jr) {
  bool hbm_ack = cfg_.durability == Durability::HbmAck;
  JournalRec old;  // the replaced version's journal record, if any: no longer referenced
  {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = index_.find(id);
    if (it != index_.end()) {
      cv_.wait(lk, [&] { return it->second.pins == 0; });
      free_extent_locked(it->second);
      lru_remove_locked(it->second);
      drop_mirror_locked(it->second);
      old = it->second.jrec;
      if (it->second.cold) {  // the new version lives in the hot dir
        ::unlink(data_path(id, true).c_str());
        ::unlink(meta_path(id, true).c_str());
      }
    }
    Block& b = index_[id];
    b = Block{};
    b.size = n;
    b.crc = crc;
    b.crc_known = true;
    b.on_disk = on_disk;
    b.dirty = !on_disk;
    b.dev_off = ext.off;
    b.dev_bytes = ext.bytes;
    b.pins = pins;
    if (jr) {  // durable in the journal: clean, and queued for its own files
      b.dirty = false;
      b.jrec = *jr;
      b.jmeta = std::move(meta);
      enqueue_materialize_locked(id, b);
    } else if (!on_disk) {
      // nvme-sync: persist_staged's .meta image; hbm-ack: the spill's, which then needs no
      // device-to-host copy of it
      b.staged_meta = std::move(meta);
    }
    touch_locked(id, b);
    if (!on_disk && !jr && hbm_ack) spill_q_.push_back(id);
  }
  cv_.notify_all();
  if (old.seg) journal_->release(old);
}

// H2D + checksum of a host buffer into `ext` on one lane; the BE .meta image comes back in
// *meta_be and the whole-block CRC in co->block_crc.
bool ChunkStore::device_stage(const uint8_t* data, uint64_t n, const DevExtent& ext, std::vector<uint8_t>* meta_be,
                              CrcOut* co, std::string* err) {
  Lane* l = acquire_lane();
  uint64_t S = num_slices(n);
  auto* dmeta = reinterpret_cast<uint32_t*>(ext.ptr + align_up(std::max<uint64_t>(n, 1), 256));
  ensure_hscratch(l, S * 4 + 16);
  uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
  bool ok = true;
  static const bool fused_ok = [] {  // DFS_FUSED_WRITE=0: SDMA copy + checksum kernel (A/B)
    const char* e = std::getenv("DFS_FUSED_WRITE");
    return !(e && e[0] == '0');
  }();
  // The fused kernel loads the block over PCIe with the waves' own reads: lowest latency for
  // one write (1 MiB: 39 vs 57 us, profiles/archive/r3_fused_write), but GPU-initiated host reads top
  // out well below the copy engines once several writes overlap (10 x 1 MiB: 29 vs 46 GB/s,
  // profiles/r4_roofline). Past this many stagings in flight the SDMA engines take the copy.
  static const int fused_max = [] {
    const char* e = std::getenv("DFS_FUSED_WRITE_MAX_INFLIGHT");
    return e ? std::atoi(e) : 2;
  }();
  struct Inflight {
    std::atomic<int>& c;
    int v;
    explicit Inflight(std::atomic<int>& x) : c(x), v(x.fetch_add(1) + 1) {}
    ~Inflight() { c.fetch_sub(1); }
  } inflight(staging_);
  const bool fused_now = fused_ok && (fused_max <= 0 || inflight.v <= fused_max);
  const uint8_t* src_dev =
      fused_now && n > kMirrorMax && crc_mfma_enabled() && l->hscratch_dev ? device_view(data, n) : nullptr;
  if (src_dev && reinterpret_cast<uintptr_t>(src_dev) % 16 == 0) {
    ok = write_copy(l, src_dev, ext.ptr, n, dmeta, hmeta, co, err);
  } else if (h2d_chunked(l, ext.ptr, data, n) && n <= kMirrorMax) {
    // a few slices: PCLMUL on the host bytes beats a kernel launch plus the .meta readback;
    // the image goes up with the data in the same stream round trip
    std::vector<uint32_t> sums(S);
    crc32_slices(data, n, sums.data());
    for (uint64_t i = 0; i < S; ++i) reinterpret_cast<uint32_t*>(hmeta)[i] = __builtin_bswap32(sums[i]);
    co->block_crc = crc32_from_slices(sums.data(), n);
    if (S) HIP_OK(hipMemcpyAsync(dmeta, hmeta, S * 4, hipMemcpyHostToDevice, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
  } else {
    bool md = false;
    ok = run_crc(l, ext.ptr, n, dmeta, nullptr, true, 0, n, co, err, hmeta, &md);
    if (ok && S && !md) {
      HIP_OK(hipMemcpyAsync(hmeta, dmeta, S * 4, hipMemcpyDeviceToHost, l->stream));
      HIP_OK(hipStreamSynchronize(l->stream));
    }
  }
  if (ok) meta_be->assign(hmeta, hmeta + S * 4);
  release_lane(l);
  return ok;
}

// H2D (double-buffered pinned chunks) + fused K1/K2 kernel + D2H of the .meta image, then
// verification against the client's whole-block CRC. With durable_now the data and .meta
// are fdatasync'ed from the caller's host buffer before the block becomes visible.
WriteResult ChunkStore::stage_impl(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc,
                                   bool durable_now) {
  TraceRange tr(durable_now ? "dfs.store.write" : "dfs.store.stage");
  HIP_OK(hipSetDevice(cfg_.device));
  WriteResult res;
  DevExtent ext = reserve(n);
  if (ext.off < 0) {
    res.error = "HBM arena full";
    return res;
  }
  bool sync_now = durable_now && cfg_.durability == Durability::NvmeSync;
  if (sync_now && journal_takes(n, num_slices(n))) return stage_journal(id, data, n, expected_crc, ext);
  std::unique_ptr<FileClaim> claim;  // the exporter keeps off the id's files until indexed
  if (sync_now && journal_) claim = std::make_unique<FileClaim>(this, id);
  // nvme-sync: the data file (the slow part: page-cache write + device flush) is written
  // and fdatasync'ed on a helper thread WHILE the GPU stages and checksums the block; the
  // .meta (known only after the CRC kernel) follows. A checksum mismatch removes the file.
  std::future<bool> data_file, dir_file;
  std::string data_err;
  // A re-written id goes to private temporary names, renamed over the block only after the
  // checksum verified: a rejected or failed write never destroys an earlier durable copy
  // (e.g. a retry on gRPC after a fast-path punt). A fresh id — the common case, block ids
  // are unique per allocation — is written under its final names like the reference's
  // write-then-sync_all (chunkserver.rs:192-209): both names exist before any flush, so
  // the directory fsync that makes them durable runs BESIDE the data and .meta flushes
  // instead of after a rename (one device round trip on the ack path instead of two).
  static const bool final_names = [] {  // DFS_FINAL_NAMES=0: every write via tmp + rename (A/B)
    const char* e = std::getenv("DFS_FINAL_NAMES");
    return !(e && e[0] == '0');
  }();
  const bool fresh = final_names && sync_now && !gsync_ && claim_fresh(id);
  const std::string tmp_sfx = fresh ? "" : "." + std::to_string(tmp_seq_.fetch_add(1)) + ".tmp";
  const std::string dp_tmp = data_path(id, false) + tmp_sfx, mp_tmp = meta_path(id, false) + tmp_sfx;
  int dfd = -1, mfd = -1;
  bool direct = fresh && odirect_enabled() && cfg_.sync_writes && n >= 4096 &&
                reinterpret_cast<uintptr_t>(data) % 4096 == 0;
  if (fresh) {
    dfd = ::open(dp_tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC | (direct ? O_DIRECT : 0), 0644);
    if (dfd < 0 && direct) {  // the filesystem refuses O_DIRECT: buffered
      direct = false;
      dfd = ::open(dp_tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    }
    mfd = dfd < 0 ? -1 : ::open(mp_tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (mfd < 0) {
      res.error = errno_str("open " + (dfd < 0 ? dp_tmp : mp_tmp));
      if (dfd >= 0) ::close(dfd);
      ::unlink(dp_tmp.c_str());
      unclaim_fresh(id);
      release(ext);
      return res;
    }
    dir_file = io_.submit([this] { return sync_dir(false); });
    data_file = io_.submit([this, dfd, data, n, direct, &data_err] {
      DiskGate::Slot slot = gate_ ? gate_->acquire() : DiskGate::Slot{};
      if (!direct) return write_fd_durable(dfd, data, n, "write " + std::to_string(n) + " bytes", &data_err);
      if (!write_direct(dfd, data, n) || ::fdatasync(dfd) != 0) {
        data_err = errno_str("write (O_DIRECT) " + std::to_string(n) + " bytes");
        return false;
      }
      std::lock_guard<std::mutex> g(mu_);
      ++st_.direct_writes;
      return true;
    });
  } else if (sync_now && !gsync_) {
    data_file = io_.submit([this, dp_tmp, data, n, &data_err] {
      DiskGate::Slot slot = gate_ ? gate_->acquire() : DiskGate::Slot{};
      return write_file_durable(dp_tmp, data, n, &data_err);
    });
  }
  // the page-cache drop and the closes are off the ack path
  auto close_fresh = [&] {
    if (dfd < 0) return;
    const bool drop = cfg_.sync_writes && gpu();
    io_.submit([dfd, mfd, drop] {
      if (drop) drop_cached(dfd);
      ::close(dfd);
      ::close(mfd);
    });
    dfd = mfd = -1;
  };
  auto abandon_data_file = [&] {
    if (data_file.valid()) {
      data_file.get();
      ::unlink(dp_tmp.c_str());
    }
    if (dir_file.valid()) dir_file.get();
    if (fresh) {
      close_fresh();
      ::unlink(mp_tmp.c_str());
      unclaim_fresh(id);
    }
  };
  uint64_t S = num_slices(n);
  std::string err;
  CrcOut co;
  auto meta = std::make_shared<std::vector<uint8_t>>();
  bool ok = device_stage(data, n, ext, meta.get(), &co, &err);
  if (!ok) {
    release(ext);
    abandon_data_file();
    res.error = err;
    return res;
  }
  res.actual_crc = co.block_crc;
  if (expected_crc != 0 && co.block_crc != expected_crc) {
    release(ext);
    abandon_data_file();
    {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.crc_mismatches;
    }
    res.error = "Checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " +
                std::to_string(co.block_crc);
    return res;
  }
  if (fresh) {
    bool mok = write_fd_durable(mfd, meta->data(), S * 4, "write " + mp_tmp, &err);
    bool dok = data_file.get();
    bool sok = dir_file.get();
    if (!sok) err = errno_str("fsync " + cfg_.storage_dir);
    close_fresh();
    if (!mok || !dok || !sok) {
      ::unlink(dp_tmp.c_str());
      ::unlink(mp_tmp.c_str());
      unclaim_fresh(id);
      release(ext);
      res.error = dok ? err : data_err;
      return res;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.final_name_writes;
    }
  } else if (data_file.valid()) {
    bool mok = write_file_durable(mp_tmp, meta->data(), S * 4, &err);
    bool dok = data_file.get();
    if (mok && dok) {
      // data first: a crash between the renames leaves new data under the old .meta,
      // which verification reports as corrupt (recovered from a replica), never silently
      if (::rename(dp_tmp.c_str(), data_path(id, false).c_str()) != 0 ||
          ::rename(mp_tmp.c_str(), meta_path(id, false).c_str()) != 0) {
        mok = false;
        err = errno_str("rename " + dp_tmp);
      } else if (!sync_dir(false)) {  // the ack promises the names, not just the bytes
        mok = false;
        err = errno_str("fsync " + cfg_.storage_dir);
      }
    }
    if (!mok || !dok) {
      ::unlink(dp_tmp.c_str());
      ::unlink(mp_tmp.c_str());
      release(ext);
      res.error = dok ? err : data_err;
      return res;
    }
  } else if (sync_now && !persist(id, false, data, n, meta->data(), S, &err)) {
    release(ext);
    res.error = err;
    return res;
  }
  if (sync_now && !supersede_file(id, &err)) {
    if (fresh) unclaim_fresh(id);
    release(ext);
    res.error = err;
    return res;
  }
  insert_resident(id, ext, n, co.block_crc, sync_now, meta);
  if (fresh) unclaim_fresh(id);  // indexed now: a later write of the id takes the tmp path
  if (n <= kMirrorMax) set_mirror(id, data, n, *meta);
  res.ok = true;
  return res;
}

void ChunkStore::drop_mirror_locked(Block& b) {
  if (!b.mirror) return;
  mirror_bytes_ -= std::min<uint64_t>(mirror_bytes_, b.mirror->size());
  b.mirror.reset();
  b.mirror_meta.reset();
}

void ChunkStore::set_mirror(const std::string& id, const uint8_t* data, uint64_t n, const std::vector<uint8_t>& meta_be) {
  auto bytes = std::make_shared<std::vector<uint8_t>>(data, data + n);
  auto sums = std::make_shared<std::vector<uint32_t>>(meta_be.size() / 4);
  for (size_t i = 0; i < sums->size(); ++i) {
    uint32_t be;
    std::memcpy(&be, meta_be.data() + 4 * i, 4);
    (*sums)[i] = __builtin_bswap32(be);
  }
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(id);
  if (it == index_.end() || it->second.size != n) return;
  drop_mirror_locked(it->second);
  it->second.mirror = std::move(bytes);
  it->second.mirror_meta = std::move(sums);
  mirror_bytes_ += n;
  mirror_fifo_.push_back(id);
  while (mirror_bytes_ > mirror_budget_ && !mirror_fifo_.empty()) {
    auto v = index_.find(mirror_fifo_.front());
    mirror_fifo_.pop_front();
    if (v != index_.end()) drop_mirror_locked(v->second);
  }
}

// Served from the small-block mirror: every 512 B slice the range touches is re-checked
// against its CRC on the CPU (PCLMUL) before a byte is returned; a mismatch drops the mirror
// and the caller takes the device path (which verifies and reports corruption as usual).
bool ChunkStore::read_mirror(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out, ReadResult* r) {
  std::shared_ptr<std::vector<uint8_t>> m;
  std::shared_ptr<std::vector<uint32_t>> sums;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end() || !it->second.mirror) return false;
    m = it->second.mirror;
    sums = it->second.mirror_meta;
  }
  const uint64_t size = m->size();
  if (offset >= size || offset + bytes > size) return false;  // the device path reports it
  if (bytes) {
    for (uint64_t s = offset / kSliceBytes, last = (offset + bytes - 1) / kSliceBytes; s <= last; ++s) {
      uint64_t so = s * kSliceBytes, sl = std::min<uint64_t>(kSliceBytes, size - so);
      if (s >= sums->size() || crc32(m->data() + so, sl) != (*sums)[s]) {
        std::lock_guard<std::mutex> g(mu_);
        auto it = index_.find(id);
        if (it != index_.end() && it->second.mirror == m) drop_mirror_locked(it->second);
        return false;
      }
    }
    std::memcpy(out, m->data() + offset, bytes);
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    ++mirror_hits_;
  }
  r->status = ReadStatus::Ok;
  r->total_size = size;
  r->bytes = bytes;
  return true;
}

bool ChunkStore::persist(const std::string& id, const uint8_t* host_data, uint64_t n, std::string* err) {
  TraceRange tr("dfs.store.persist");
  if (!gpu() || cfg_.durability == Durability::HbmAck) return true;
  std::shared_ptr<std::vector<uint8_t>> meta;
  const uint8_t* d = nullptr;
  uint64_t size = 0;
  uint32_t crc = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) {
      *err = "Block not found";
      return false;
    }
    Block& b = it->second;
    if (!b.dirty) return true;
    if (b.dev_off < 0 || !b.staged_meta) {
      *err = "block not staged";
      return false;
    }
    meta = b.staged_meta;
    size = b.size;
    crc = b.crc;
    d = arena_ + b.dev_off;
    b.pins++;
  }
  bool ok, jok = false;
  JournalRec jr;
  const bool from_host = host_data && n == size;
  std::unique_ptr<FileClaim> claim;
  if (journal_takes(size, meta->size() / 4)) {
    ok = jok = journal_block(id, from_host ? host_data : nullptr, from_host ? nullptr : d, size, crc, *meta, &jr, err);
  } else {
    if (journal_) claim = std::make_unique<FileClaim>(this, id);
    ok = from_host ? persist(id, false, host_data, size, meta->data(), meta->size() / 4, err)
                   : persist_from_device(id, d, size, meta->data(), meta->size() / 4, err);
    ok = ok && supersede_file(id, err);
  }
  bool obsolete = jok;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end()) {
      it->second.pins--;
      if (ok && it->second.staged_meta == meta) {
        it->second.dirty = false;
        it->second.staged_meta.reset();
        if (jok) {
          it->second.jrec = jr;
          it->second.jmeta = meta;
          enqueue_materialize_locked(id, it->second);
          obsolete = false;
        } else {
          it->second.on_disk = true;
        }
      }
    }
  }
  if (obsolete) journal_->release(jr);  // the block changed meanwhile: record unused
  cv_.notify_all();
  return ok;
}

bool ChunkStore::persist_from_device(const std::string& id, const uint8_t* d, uint64_t n, const uint8_t* meta_be,
                                     uint64_t nslices, std::string* err) {
  HIP_OK(hipSetDevice(cfg_.device));
  DiskGate::Slot slot = gate_ ? gate_->acquire() : DiskGate::Slot{};
  Lane* l = acquire_lane();
  std::string dp = data_path(id, false);
  // replicas: the pinned bounce chunks are page aligned, so with DFS_ODIRECT=1 they go to the
  // device without a page-cache copy (see odirect_enabled)
  bool direct = odirect_enabled() && cfg_.sync_writes && n >= 4096;
  int fd = ::open(dp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC | (direct ? O_DIRECT : 0), 0644);
  if (fd < 0 && direct) {
    direct = false;
    fd = ::open(dp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  }
  bool ok = fd >= 0;
  uint64_t nch = (n + kChunk - 1) / kChunk;
  for (uint64_t c = 0; ok && c < nch; ++c) {
    uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, n - off);
    HIP_OK(hipMemcpyAsync(l->pinned[c & 1], d + off, len, hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
    ok = direct ? write_direct(fd, l->pinned[c & 1], len, off) : write_all(fd, l->pinned[c & 1], len, off);
  }
  if (ok && direct) {
    std::lock_guard<std::mutex> g(mu_);
    ++st_.direct_writes;
  }
  release_lane(l);
  int mfd = -1;
  if (ok) {
    std::string mp = meta_path(id, false);
    mfd = ::open(mp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    ok = mfd >= 0 && write_all(mfd, meta_be, nslices * 4, 0);
  }
  if (ok) ok = make_durable(fd, mfd, false);
  if (ok && cfg_.sync_writes) drop_cached(fd);
  if (fd >= 0) ::close(fd);
  if (mfd >= 0) ::close(mfd);
  if (!ok) *err = errno_str("persist " + id);
  return ok;
}

WriteResult ChunkStore::write_host(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc) {
  if (!valid_block_id(id)) return bad_id(id);
  WriteResult res;
  uint32_t actual = crc32(data, n);
  res.actual_crc = actual;
  if (expected_crc != 0 && actual != expected_crc) {
    std::lock_guard<std::mutex> g(mu_);
    ++st_.crc_mismatches;
    res.error = "Checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " + std::to_string(actual);
    return res;
  }
  uint64_t S = num_slices(n);
  std::vector<uint32_t> sl(S);
  crc32_slices(data, n, sl.data());
  for (auto& v : sl) v = __builtin_bswap32(v);
  std::string err;
  JournalRec jr, old;
  std::shared_ptr<std::vector<uint8_t>> jmeta;
  std::unique_ptr<FileClaim> claim;
  const bool jok = journal_takes(n, S);
  if (jok) {
    jmeta = std::make_shared<std::vector<uint8_t>>(reinterpret_cast<const uint8_t*>(sl.data()),
                                                   reinterpret_cast<const uint8_t*>(sl.data()) + S * 4);
    if (!journal_block(id, data, nullptr, n, actual, *jmeta, &jr, &err)) {
      res.error = err;
      return res;
    }
  } else {
    if (journal_) claim = std::make_unique<FileClaim>(this, id);
    if (!persist(id, false, data, n, reinterpret_cast<const uint8_t*>(sl.data()), S, &err) ||
        !supersede_file(id, &err)) {
      res.error = err;
      return res;
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = index_.find(id);
    if (it != index_.end()) cv_.wait(lk, [&] { return it->second.pins == 0; });  // exporter / readers
    if (it != index_.end()) old = it->second.jrec;
    if (it != index_.end() && it->second.cold) {
      ::unlink(data_path(id, true).c_str());
      ::unlink(meta_path(id, true).c_str());
    }
    Block& b = index_[id];
    lru_remove_locked(b);
    b = Block{};
    b.size = n;
    b.crc = actual;
    b.crc_known = true;
    b.on_disk = !jok;
    if (jok) {
      b.jrec = jr;
      b.jmeta = std::move(jmeta);
      enqueue_materialize_locked(id, b);
    }
  }
  cv_.notify_all();
  if (old.seg) journal_->release(old);
  res.ok = true;
  return res;
}

// ---------------------------------------------------------------- read
ReadResult ChunkStore::stat(const std::string& id, uint64_t offset, uint64_t length) {
  ReadResult r;
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(id);
  if (it == index_.end()) {
    r.status = ReadStatus::NotFound;
    r.error = "Block not found";
    return r;
  }
  r.total_size = it->second.size;
  uint64_t len = length == 0 ? (r.total_size > offset ? r.total_size - offset : 0) : length;
  if (offset >= r.total_size) {
    r.status = ReadStatus::OutOfRange;
    r.error = "Offset " + std::to_string(offset) + " exceeds block size " + std::to_string(r.total_size);
    return r;
  }
  r.bytes = std::min<uint64_t>(len, r.total_size - offset);
  return r;
}

ReadResult ChunkStore::read_into(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out) {
  TraceRange tr("dfs.store.read");
  if (!gpu()) return read_host(id, offset, bytes, out);
  ReadResult r;
  if (read_mirror(id, offset, bytes, out, &r)) return r;
  HIP_OK(hipSetDevice(cfg_.device));
  uint64_t size = 0;
  const uint8_t* d = pin_device(id, &size);
  if (!d) {
    r.status = ReadStatus::NotFound;
    r.error = "Block not found";
    return r;
  }
  r.total_size = size;
  if (offset >= size || offset + bytes > size) {
    unpin(id);
    r.status = ReadStatus::OutOfRange;
    r.error = "Offset " + std::to_string(offset) + " exceeds block size " + std::to_string(size);
    return r;
  }
  auto* dmeta = reinterpret_cast<const uint32_t*>(d + align_up(std::max<uint64_t>(size, 1), 256));
  Lane* l = acquire_lane();
  std::string err;
  CrcOut co;
  CrcPlan p = plan_crc(d, size, nullptr, dmeta, false, offset, offset + bytes);
  static const bool fused_ok = [] {
    const char* e = std::getenv("DFS_FUSED_READ");
    return !(e && e[0] == '0');
  }();
  uint8_t* dout = fused_ok && crc_mfma_enabled() ? device_view(out, bytes) : nullptr;
  void* dbad = l->hscratch_dev;
  if (dout && dbad && (reinterpret_cast<uintptr_t>(dout) - offset) % 16 == 0 && p.grid > 0 && p.grid <= kMaxGridCrc) {
    // K3 fused: one kernel verifies the touched slices and stores the range into the
    // reader's registered slot; its verdicts land in the lane's pinned scratch
    ReadCopyLaunch rc;
    rc.c = p.a;
    rc.out = dout;
    rc.off = offset;
    rc.len = bytes;
    rc.part_bad = static_cast<uint32_t*>(dbad);
    hipError_t e = launch_read_copy(rc, dtables_, p.grid, l->stream);
    launches_++;
    if (e != hipSuccess) err = hipGetErrorString(e);
    HIP_OK(hipStreamSynchronize(l->stream));
    fused_reads_++;
  } else {
    if (p.grid > 0) {
      p.a.part_bad = l->dscratch + kMaxGridCrc;
      hipError_t e = launch_crc(p.a, dtables_, p.grid, l->stream);
      launches_++;
      if (e != hipSuccess) err = hipGetErrorString(e);
      HIP_OK(hipMemcpyAsync(l->hscratch, l->dscratch + kMaxGridCrc, p.grid * 4, hipMemcpyDeviceToHost, l->stream));
    }
    d2h_chunked(l, out, d + offset, bytes);  // overlaps with verification on the same stream order
    HIP_OK(hipStreamSynchronize(l->stream));
  }
  uint32_t bad = 0xFFFFFFFFu;
  for (int g = 0; g < p.grid; ++g) bad = std::min(bad, reinterpret_cast<uint32_t*>(l->hscratch)[g]);
  release_lane(l);
  unpin(id);
  r.bytes = bytes;
  if (!err.empty()) {
    r.status = ReadStatus::IoError;
    r.error = err;
    return r;
  }
  if (bad != 0xFFFFFFFFu) {
    std::lock_guard<std::mutex> g(mu_);
    ++st_.crc_mismatches;
    r.bad_slice = bad;
    r.error = "Checksum mismatch at chunk " + std::to_string(bad);
    if (offset == 0 && bytes == size) r.status = ReadStatus::Corrupt;
    else r.partial_corrupt = true;
  }
  return r;
}

std::vector<uint32_t> ChunkStore::load_meta_file(const std::string& id, bool cold, bool* ok) {
  std::vector<uint32_t> m;
  *ok = false;
  std::string mp = meta_path(id, cold);
  int fd = ::open(mp.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return m;
  struct stat st;
  if (::fstat(fd, &st) == 0) {
    m.resize(static_cast<size_t>(st.st_size) / 4);
    if (read_all(fd, reinterpret_cast<uint8_t*>(m.data()), m.size() * 4, 0)) {
      for (auto& v : m) v = __builtin_bswap32(v);
      *ok = true;
    }
  }
  ::close(fd);
  return m;
}

ReadResult ChunkStore::read_host(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out) {
  ReadResult r;
  bool cold = false;
  uint64_t size = 0;
  bool full = false;
  JournalRec jrec;
  std::shared_ptr<std::vector<uint8_t>> jmeta;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) {
      r.status = ReadStatus::NotFound;
      r.error = "Block not found";
      return r;
    }
    Block& b = it->second;
    size = b.size;
    cold = b.cold;
    r.total_size = size;
    if (offset >= size || offset + bytes > size) {
      r.status = ReadStatus::OutOfRange;
      r.error = "Offset " + std::to_string(offset) + " exceeds block size " + std::to_string(size);
      return r;
    }
    full = offset == 0 && bytes == size;
    if (full && b.host) {  // LRU hit (reference: no re-verification on cache hit)
      std::memcpy(out, b.host->data(), bytes);
      touch_locked(id, b);
      r.bytes = bytes;
      return r;
    }
    jrec = b.jrec;
    jmeta = b.jmeta;
    if (jrec.seg) jrec.seg->readers++;  // released by DurableSrc
  }
  DurableSrc src;
  const bool opened = open_durable(id, cold, jrec, jmeta, &src);
  if (src.fd < 0) {
    r.status = errno == ENOENT ? ReadStatus::NotFound : ReadStatus::IoError;
    r.error = errno == ENOENT ? "Block not found" : errno_str("Failed to read block");
    return r;
  }
  const int fd = src.fd;
  const uint64_t base = src.base;
  bool ok = read_all(fd, out, bytes, base + offset);
  if (!ok) {
    r.status = ReadStatus::IoError;
    r.error = errno_str("Failed to read block");
    return r;
  }
  r.bytes = bytes;
  bool mok = opened && src.meta_ok;
  std::vector<uint32_t>& meta = src.meta;
  if (!mok) {
    r.error = "Checksum file missing";
    if (full) r.status = ReadStatus::Corrupt;
    else r.partial_corrupt = true;
    return r;
  }
  if (full) {
    std::vector<uint32_t> act(num_slices(size));
    crc32_slices(out, size, act.data());
    if (act.size() != meta.size()) {
      r.status = ReadStatus::Corrupt;
      r.error = "Checksum count mismatch";
    } else {
      for (size_t i = 0; i < act.size(); ++i)
        if (act[i] != meta[i]) {
          r.status = ReadStatus::Corrupt;
          r.bad_slice = static_cast<int64_t>(i);
          r.error = "Checksum mismatch at chunk " + std::to_string(i);
          break;
        }
    }
    if (r.status == ReadStatus::Ok) {
      std::lock_guard<std::mutex> g(mu_);
      auto it = index_.find(id);
      if (it != index_.end()) {
        it->second.host = std::make_shared<std::vector<uint8_t>>(out, out + bytes);
        touch_locked(id, it->second);
        while (static_cast<int>(lru_.size()) > std::max(0, cfg_.cache_blocks)) {
          auto& victim = index_[lru_.back()];
          victim.host.reset();
          victim.in_lru = false;
          lru_.pop_back();
        }
      }
    } else {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.crc_mismatches;
    }
  } else {
    uint64_t first = offset / kSliceBytes, last = (offset + bytes - 1) / kSliceBytes;
    std::vector<uint8_t> buf(kSliceBytes);
    for (uint64_t s = first; s <= last && s < meta.size(); ++s) {
      uint64_t so = s * kSliceBytes, sl = std::min<uint64_t>(kSliceBytes, size - so);
      if (!read_all(fd, buf.data(), sl, base + so)) break;
      if (crc32(buf.data(), sl) != meta[s]) {
        r.partial_corrupt = true;
        r.bad_slice = static_cast<int64_t>(s);
        r.error = "Checksum mismatch at chunk " + std::to_string(s);
        std::lock_guard<std::mutex> g(mu_);
        ++st_.crc_mismatches;
        break;
      }
    }
  }
  return r;
}

// ---------------------------------------------------------------- residency
DevExtent ChunkStore::reserve(uint64_t n) {
  DevExtent e;
  if (!gpu()) return e;
  uint64_t bytes = alloc_bytes(n);
  std::unique_lock<std::mutex> lk(mu_);
  e.off = alloc_locked(lk, bytes);
  if (e.off >= 0) {
    e.bytes = bytes;
    e.ptr = arena_ + e.off;
  }
  return e;
}

void ChunkStore::release(const DevExtent& e) {
  if (e.off < 0) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    alloc_.free(static_cast<uint64_t>(e.off), e.bytes);
  }
  cv_.notify_all();
}

bool ChunkStore::promote(const std::string& id, std::string* err) {
  uint64_t size = 0;
  bool cold = false;
  JournalRec jrec;
  std::shared_ptr<std::vector<uint8_t>> jmeta;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) {
      *err = "Block not found";
      return false;
    }
    if (it->second.dev_off >= 0) return true;
    if (!it->second.on_disk && !it->second.jrec.seg) {
      *err = "block neither resident nor on disk";
      return false;
    }
    size = it->second.size;
    cold = it->second.cold;
    jrec = it->second.jrec;
    jmeta = it->second.jmeta;
    if (jrec.seg) jrec.seg->readers++;  // released by DurableSrc
  }
  DurableSrc src;
  if (!open_durable(id, cold, jrec, jmeta, &src)) {
    *err = src.meta_ok ? "Block not found" : "Checksum file missing";
    return false;
  }
  std::vector<uint32_t>& meta = src.meta;
  uint64_t S = num_slices(size);
  if (meta.size() != S) {
    *err = "Checksum count mismatch";
    return false;
  }
  DevExtent ext = reserve(size);
  if (ext.off < 0) {
    *err = "HBM arena full";
    return false;
  }
  Lane* l = acquire_lane();
  bool ok = true;
  int i = 0;
  for (uint64_t off = 0; off < size; off += kChunk, i ^= 1) {
    uint64_t len = std::min<uint64_t>(kChunk, size - off);
    HIP_OK(hipEventSynchronize(l->ev[i]));
    if (!read_all(src.fd, l->pinned[i], len, src.base + off)) {
      ok = false;
      break;
    }
    HIP_OK(hipMemcpyAsync(ext.ptr + off, l->pinned[i], len, hipMemcpyHostToDevice, l->stream));
    HIP_OK(hipEventRecord(l->ev[i], l->stream));
  }
  ensure_hscratch(l, S * 4 + 16);
  uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
  for (uint64_t s = 0; s < S; ++s) reinterpret_cast<uint32_t*>(hmeta)[s] = __builtin_bswap32(meta[s]);
  if (S)
    HIP_OK(hipMemcpyAsync(ext.ptr + align_up(std::max<uint64_t>(size, 1), 256), hmeta, S * 4,
                          hipMemcpyHostToDevice, l->stream));
  HIP_OK(hipStreamSynchronize(l->stream));
  release_lane(l);
  if (!ok) {
    release(ext);
    *err = errno_str("Failed to read block");
    return false;
  }
  bool keep = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end() && it->second.dev_off < 0 && it->second.size == size) {
      Block& b = it->second;
      b.dev_off = ext.off;
      b.dev_bytes = ext.bytes;
      if (!b.crc_known) {
        b.crc = crc32_from_slices(meta.data(), size);
        b.crc_known = true;
      }
      touch_locked(id, b);
      ++st_.promotions;
      keep = true;
    }
  }
  if (!keep) release(ext);
  return true;
}

const uint8_t* ChunkStore::pin_device(const std::string& id, uint64_t* size) {
  if (!gpu()) return nullptr;
  for (int attempt = 0; attempt < 3; ++attempt) {
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = index_.find(id);
      if (it == index_.end()) return nullptr;
      Block& b = it->second;
      if (b.dev_off >= 0) {
        b.pins++;
        touch_locked(id, b);
        *size = b.size;
        return arena_ + b.dev_off;
      }
    }
    std::string err;
    if (!promote(id, &err)) return nullptr;
  }
  return nullptr;
}

void ChunkStore::unpin(const std::string& id) {
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end() && it->second.pins > 0) it->second.pins--;
  }
  cv_.notify_all();
}

WriteResult ChunkStore::commit_device(const std::string& id, const DevExtent& ext, uint64_t n, uint32_t expected_crc,
                                      hipStream_t s, bool persist_now) {
  WriteResult res;
  HIP_OK(hipSetDevice(cfg_.device));
  if (s) HIP_OK(hipStreamSynchronize(s));
  Lane* l = acquire_lane();
  uint64_t S = num_slices(n);
  auto* dmeta = reinterpret_cast<uint32_t*>(ext.ptr + align_up(std::max<uint64_t>(n, 1), 256));
  ensure_hscratch(l, S * 4 + 16);
  uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
  std::string err;
  CrcOut co;
  bool md = false;
  bool ok = run_crc(l, ext.ptr, n, dmeta, nullptr, true, 0, n, &co, &err, hmeta, &md);
  if (ok && S && !md) {
    HIP_OK(hipMemcpyAsync(hmeta, dmeta, S * 4, hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
  }
  auto meta = std::make_shared<std::vector<uint8_t>>(hmeta, hmeta + S * 4);
  release_lane(l);
  if (!ok) {
    release(ext);
    res.error = err;
    return res;
  }
  res.actual_crc = co.block_crc;
  if (expected_crc != 0 && co.block_crc != expected_crc) {
    release(ext);
    res.error = "Replication checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " +
                std::to_string(co.block_crc);
    return res;
  }
  bool sync_now = persist_now && cfg_.durability == Durability::NvmeSync;
  JournalRec jr;
  const bool jok = sync_now && journal_takes(n, S);
  std::unique_ptr<FileClaim> claim;
  if (sync_now && !jok && journal_) claim = std::make_unique<FileClaim>(this, id);
  if (jok ? !journal_block(id, nullptr, ext.ptr, n, co.block_crc, *meta, &jr, &err)
          : sync_now && (!persist_from_device(id, ext.ptr, n, meta->data(), S, &err) || !supersede_file(id, &err))) {
    release(ext);
    res.error = err;
    return res;
  }
  insert_resident(id, ext, n, co.block_crc, sync_now && !jok, meta, 0, jok ? &jr : nullptr);
  res.ok = true;
  return res;
}

// Receiver-pull scratch: pinned host buffers (hipHostMalloc is ~ms) reused across receives.
// Held through shared_ptr by every launch closure, so a buffer goes back to the pool only
// when no kernel of an abandoned receive can still write it.
struct ChunkStore::PinnedPool {
  std::mutex mu;
  std::vector<std::pair<uint8_t*, uint64_t>> free;
  ~PinnedPool() {
    for (auto& f : free) (void)hipHostFree(f.first);
  }
};
struct ChunkStore::PullScratch {
  std::shared_ptr<PinnedPool> pool;
  uint8_t* host = nullptr;  // [0, S*4): the .meta image; [data_off, data_off + n): the bytes
  uint8_t* dev = nullptr;
  uint64_t cap = 0;
  uint64_t data_off = 0;  // 0: no host copy of the bytes
  ~PullScratch() {
    if (!host) return;
    std::lock_guard<std::mutex> g(pool->mu);
    pool->free.emplace_back(host, cap);
  }
};

bool ChunkStore::can_pull() const { return gpu() && crc_mfma_enabled() && dtables_ && pull_parts_dev_; }

bool ChunkStore::recv_begin(RecvVerify* rv, const DevExtent& e, uint64_t n, bool pull, bool persist_now) {
  rv->ext = e;
  rv->n = n;
  rv->pull.reset();
  if (pull) {
    if (!can_pull()) return false;
    // DFS_PULL_HOST=1: the pull kernel also leaves an nvme-sync replica's bytes in pinned host
    // memory and the journal appends from there, instead of from HBM through a lane's pinned
    // chunks. Measured a wash at 2 ranks (landing +30 us, the append's copy -30 us, inside a
    // ~2 ms fdatasync round: profiles/r6/pull/n2_pullhost*.json vs n2_pulldev.json), so off.
    static const bool host_ok = env_int("DFS_PULL_HOST", 0) != 0;
    const bool host_copy = host_ok && persist_now && cfg_.durability == Durability::NvmeSync && journal_ &&
                           n <= (16ull << 20) && n > 0;
    const uint64_t meta_bytes = align_up(num_slices(n) * 4 + 16, 4096);
    const uint64_t want = meta_bytes + (host_copy ? align_up(n, 4096) : 0);
    auto sc = std::make_shared<PullScratch>();
    sc->pool = pull_pool_;
    {
      std::lock_guard<std::mutex> g(pull_pool_->mu);
      auto& fr = pull_pool_->free;
      size_t best = fr.size();
      for (size_t i = 0; i < fr.size(); ++i)  // best fit: meta-only and host-copy receives share the pool
        if (fr[i].second >= want && (best == fr.size() || fr[i].second < fr[best].second)) best = i;
      if (best < fr.size()) {
        sc->host = fr[best].first;
        sc->cap = fr[best].second;
        fr[best] = fr.back();
        fr.pop_back();
      }
    }
    if (host_copy) sc->data_off = meta_bytes;
    if (!sc->host) {
      (void)hipSetDevice(cfg_.device);
      if (hipHostMalloc(reinterpret_cast<void**>(&sc->host), want, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        sc->host = nullptr;
        return false;
      }
      sc->cap = want;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, sc->host, 0) != hipSuccess) {
      (void)hipGetLastError();
      return false;  // sc goes back to the pool
    }
    sc->dev = static_cast<uint8_t*>(d);
    rv->pull = std::move(sc);
    rv->lane = nullptr;
    return true;
  }
  // no lane yet: a receive waits for its bytes without holding one of the store's streams
  // (at 10 writers per rank the waiting receives held the lanes the heads' stagings needed);
  // DFS_RECV_LANE_EAGER=1 takes it here, as before (A/B)
  static const bool eager = [] {
    const char* e = std::getenv("DFS_RECV_LANE_EAGER");
    return e && e[0] == '1';
  }();
  rv->lane = nullptr;
  if (eager) recv_lane(rv);
  return true;
}

void* ChunkStore::recv_lane(RecvVerify* rv) {
  if (!rv->lane) {
    rv->lane = acquire_lane();
    ensure_hscratch(static_cast<Lane*>(rv->lane), num_slices(rv->n) * 4 + 16);
  }
  return rv->lane;
}

bool ChunkStore::recv_slice(RecvVerify* rv, uint64_t lo, uint64_t hi) {
  if (rv->failed || hi <= lo) return !rv->failed;
  Lane* l = static_cast<Lane*>(recv_lane(rv));
  (void)hipSetDevice(cfg_.device);
  auto* dmeta = reinterpret_cast<uint32_t*>(rv->ext.ptr + align_up(std::max<uint64_t>(rv->n, 1), 256));
  // range mode writing (not verifying) the slices of [lo, hi): full slices via the tile
  // loop, the short tail slice when the range reaches the end of the block
  CrcPlan p = plan_crc(rv->ext.ptr, rv->n, dmeta, nullptr, false, lo, hi);
  if (p.grid == 0) return true;
  // the slice's .meta words also go straight into the lane's pinned scratch (LDS kernel), so
  // recv_finish needs no readback copy
  if (rv->host_meta && l->hscratch_dev && crc_meta_host_ok(p.a.ntiles))
    p.a.meta_host = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(l->hscratch_dev) + 2 * kMaxGridCrc * sizeof(uint32_t) + 16);
  else
    rv->host_meta = false;
  hipError_t e = launch_crc(p.a, dtables_, p.grid, l->stream);
  launches_++;
  if (e != hipSuccess) {
    rv->failed = true;
    rv->error = std::string("crc kernel launch: ") + hipGetErrorString(e);
  }
  return !rv->failed;
}

std::function<int(const uint8_t*, void*)> ChunkStore::recv_pull(RecvVerify* rv, uint64_t lo, uint64_t hi) {
  const uint64_t len = hi > lo ? hi - lo : 0;
  uint8_t* dst = rv->ext.ptr + lo;
  uint32_t* dmeta = reinterpret_cast<uint32_t*>(rv->ext.ptr + align_up(std::max<uint64_t>(rv->n, 1), 256)) +
                    lo / kSliceBytes;
  std::shared_ptr<PullScratch> sc = rv->pull;
  uint32_t* mh = sc ? reinterpret_cast<uint32_t*>(sc->dev) + lo / kSliceBytes : nullptr;
  uint8_t* hdst = sc && sc->data_off ? sc->dev + sc->data_off + lo : nullptr;
  const DevCrcTables* tables = dtables_;
  uint32_t* parts = pull_parts_dev_;
  return [=](const uint8_t* src, void* stream) -> int {
    if (!sc || lo % kSliceBytes || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) % 16))
      return -1;  // the kernel moves 16-byte vectors from slice-aligned offsets
    if (len == 0) return 0;
    CrcPlan p = plan_crc(src, len, dmeta, nullptr, true, 0, len);
    WriteCopyLaunch w;
    w.c = p.a;
    w.c.part_crc = parts;  // partials of the slice: unread (recv_finish combines the .meta words)
    w.dst = dst;
    w.meta_host = mh;
    w.dst_host = hdst;
    return launch_write_copy(w, tables, p.grid, static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -1;
  };
}

WriteResult ChunkStore::recv_finish(RecvVerify* rv, const std::string& id, uint32_t expected_crc, bool persist_now) {
  TraceRange tr("dfs.store.recv_commit");
  WriteResult res;
  uint64_t n = rv->n, S = num_slices(n);
  std::shared_ptr<std::vector<uint8_t>> meta;
  std::shared_ptr<PullScratch> pulled;  // holds the host copy of the bytes until the append
  if (rv->pull) {
    // every slice's kernel finished before the transport completed the receive: the .meta
    // image (and, for an nvme-sync replica, the bytes) are already in the pinned scratch
    meta = std::make_shared<std::vector<uint8_t>>(rv->pull->host, rv->pull->host + S * 4);
    pulled = std::move(rv->pull);
    pulled_recvs_++;
  } else {
    Lane* l = static_cast<Lane*>(recv_lane(rv));
    (void)hipSetDevice(cfg_.device);
    auto* dmeta = reinterpret_cast<uint32_t*>(rv->ext.ptr + align_up(std::max<uint64_t>(n, 1), 256));
    ensure_hscratch(l, S * 4 + 16);
    uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
    if (!rv->failed && S && !rv->host_meta)
      HIP_OK(hipMemcpyAsync(hmeta, dmeta, S * 4, hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
    meta = std::make_shared<std::vector<uint8_t>>(hmeta, hmeta + S * 4);
    release_lane(l);
    rv->lane = nullptr;
  }
  if (rv->failed) {
    release(rv->ext);
    res.error = rv->error;
    return res;
  }
  std::vector<uint32_t> native(S);
  for (uint64_t i = 0; i < S; ++i) {
    uint32_t be;
    std::memcpy(&be, meta->data() + 4 * i, 4);
    native[i] = __builtin_bswap32(be);
  }
  uint32_t crc = crc32_from_slices(native.data(), n);
  res.actual_crc = crc;
  if (expected_crc != 0 && crc != expected_crc) {
    release(rv->ext);
    {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.crc_mismatches;
    }
    res.error = "Replication checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " +
                std::to_string(crc);
    return res;
  }
  std::string err;
  bool sync_now = persist_now && cfg_.durability == Durability::NvmeSync;
  JournalRec jr;
  const bool jok = sync_now && journal_takes(n, S);
  std::unique_ptr<FileClaim> claim;
  if (sync_now && !jok && journal_) claim = std::make_unique<FileClaim>(this, id);
  const uint8_t* host_bytes = pulled && pulled->data_off ? pulled->host + pulled->data_off : nullptr;
  if (host_bytes) pulled_host_appends_++;
  if (jok ? !journal_block(id, host_bytes, host_bytes ? nullptr : rv->ext.ptr, n, crc, *meta, &jr, &err)
          : sync_now && (!persist_from_device(id, rv->ext.ptr, n, meta->data(), S, &err) ||
                         !supersede_file(id, &err))) {
    release(rv->ext);
    res.error = err;
    return res;
  }
  insert_resident(id, rv->ext, n, crc, sync_now && !jok, meta, 0, jok ? &jr : nullptr);
  res.ok = true;
  return res;
}

void ChunkStore::recv_abandon(RecvVerify* rv) {
  rv->pull.reset();  // launches still queued keep the scratch until they are dropped
  if (!rv->lane) return;
  Lane* l = static_cast<Lane*>(rv->lane);
  // kernels already queued on the lane only read the extent: they finish on their own
  (void)hipSetDevice(cfg_.device);
  (void)hipStreamSynchronize(l->stream);
  release_lane(l);
  rv->lane = nullptr;
}

void ChunkStore::spill_worker() {
  (void)hipSetDevice(cfg_.device);
  for (;;) {
    std::string id;
    uint64_t size = 0;
    const uint8_t* d = nullptr;
    std::shared_ptr<std::vector<uint8_t>> smeta;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || (!spill_paused_ && !spill_q_.empty()); });
      if (stop_ && spill_q_.empty()) return;
      id = spill_q_.front();
      spill_q_.pop_front();
      auto it = index_.find(id);
      if (it == index_.end() || !it->second.dirty || it->second.dev_off < 0) continue;
      it->second.pins++;
      size = it->second.size;
      d = arena_ + it->second.dev_off;
      smeta = it->second.staged_meta;
    }
    DiskGate::Slot slot = gate_ ? gate_->acquire() : DiskGate::Slot{};
    Lane* l = acquire_lane();
    uint64_t S = num_slices(size);
    ensure_hscratch(l, S * 4 + 16);
    uint8_t* hmeta = l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16;
    bool ok = true;
    // private temporary names, renamed into place once both are durable: a crash mid-spill
    // leaves only .tmp files (removed by scan_dirs), never a torn block under its real name
    const std::string tmp_sfx = "." + std::to_string(tmp_seq_.fetch_add(1)) + ".tmp";
    const std::string dp_tmp = data_path(id, false) + tmp_sfx, mp_tmp = meta_path(id, false) + tmp_sfx;
    int fd = ::open(dp_tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    ok = fd >= 0;
    uint64_t nch = (size + kChunk - 1) / kChunk;
    for (uint64_t c = 0; ok && c < nch; ++c) {
      uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, size - off);
      if (hipMemcpyAsync(l->pinned[c & 1], d + off, len, hipMemcpyDeviceToHost, l->stream) != hipSuccess ||
          hipStreamSynchronize(l->stream) != hipSuccess) {
        ok = false;
        break;
      }
      ok = write_all(fd, l->pinned[c & 1], len, off);
    }
    if (ok && S && smeta && smeta->size() == S * 4) {
      std::memcpy(hmeta, smeta->data(), S * 4);  // kept from the write: no readback
    } else if (ok && S) {
      ok = hipMemcpyAsync(hmeta, d + align_up(std::max<uint64_t>(size, 1), 256), S * 4, hipMemcpyDeviceToHost,
                          l->stream) == hipSuccess &&
           hipStreamSynchronize(l->stream) == hipSuccess;
    }
    int mfd = -1;
    if (ok) {
      mfd = ::open(mp_tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
      ok = mfd >= 0 && write_all(mfd, hmeta, S * 4, 0);
    }
    if (ok) ok = make_durable(fd, mfd, false);
    if (ok && cfg_.sync_writes) drop_cached(fd);
    if (fd >= 0) ::close(fd);
    if (mfd >= 0) ::close(mfd);
    // .meta first: a crash between the renames leaves a .meta with no data file, which
    // scan_dirs ignores (the block reads as missing, never as torn data)
    if (ok && (::rename(mp_tmp.c_str(), meta_path(id, false).c_str()) != 0 ||
               ::rename(dp_tmp.c_str(), data_path(id, false).c_str()) != 0))
      ok = false;
    if (ok) ok = sync_dir(false);  // the block stays dirty (and retried) until its names are durable
    if (!ok) {
      ::unlink(dp_tmp.c_str());
      ::unlink(mp_tmp.c_str());
    }
    release_lane(l);
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = index_.find(id);
      if (it != index_.end()) {
        it->second.pins--;
        if (ok && it->second.size == size) {
          it->second.dirty = false;
          it->second.on_disk = true;
          it->second.staged_meta.reset();
        } else if (!ok) {
          spill_q_.push_back(id);  // retry later
        }
      }
    }
    cv_.notify_all();
  }
}

// ---------------------------------------------------------------- misc ops
void ChunkStore::debug_pause_spill(bool on) {
  {
    std::lock_guard<std::mutex> g(mu_);
    spill_paused_ = on;
  }
  cv_.notify_all();
}

bool ChunkStore::exists(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  return index_.count(id) > 0;
}

int64_t ChunkStore::block_size(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(id);
  return it == index_.end() ? -1 : static_cast<int64_t>(it->second.size);
}

uint32_t ChunkStore::block_crc(const std::string& id) {
  bool cold = false;
  uint64_t size = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) return 0;
    if (it->second.crc_known) return it->second.crc;
    cold = it->second.cold;
    size = it->second.size;
  }
  bool ok = false;
  auto m = load_meta_file(id, cold, &ok);
  if (!ok) return 0;
  uint32_t c = crc32_from_slices(m.data(), size);
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(id);
  if (it != index_.end()) {
    it->second.crc = c;
    it->second.crc_known = true;
  }
  return c;
}

bool ChunkStore::remove(const std::string& id) {
  bool cold = false, durable = true;
  JournalRec old;
  {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) return false;
    durable = it->second.on_disk || it->second.jrec.seg != nullptr;
    old = it->second.jrec;
  }
  // an unretired journal record of the block would bring it back on replay (a block that
  // never became durable, e.g. an EC gather copy, has none): the tombstone is committed
  // before the block leaves the index. If it cannot be (journal failed, or no room even in
  // the markers' reserve), the block stays and the delete fails, so the master retries it
  // instead of the block coming back at the next restart.
  if (journal_ && durable) {
    std::string err;
    if (!journal_->marker(kJrTomb, id, &err)) {
      std::fprintf(stderr, "[store] delete %s kept: tombstone not durable: %s\n", id.c_str(), err.c_str());
      std::lock_guard<std::mutex> g(mu_);
      ++tomb_failures_;
      return false;
    }
  }
  {
    std::unique_lock<std::mutex> lk(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) return true;  // a concurrent delete won
    cv_.wait(lk, [&] {
      it = index_.find(id);
      return it == index_.end() || it->second.pins == 0;
    });
    if (it == index_.end()) return true;
    // (a rewrite that landed while the tombstone committed took a smaller LSN only if it
    // finished first; either way the id is gone after replay, as it is here)
    cold = it->second.cold;
    old = it->second.jrec;
    free_extent_locked(it->second);
    lru_remove_locked(it->second);
    drop_mirror_locked(it->second);
    index_.erase(it);
  }
  cv_.notify_all();
  ::unlink(data_path(id, cold).c_str());
  ::unlink(meta_path(id, cold).c_str());
  if (old.seg) journal_->release(old);
  return true;
}

bool ChunkStore::move_to_cold(const std::string& id) {
  if (cfg_.cold_dir.empty()) return false;
  std::unique_lock<std::mutex> lk(mu_);
  auto it = index_.find(id);
  if (it == index_.end() || it->second.cold) return false;
  if (it->second.jrec.seg) {  // its own files first
    lk.unlock();
    materialize_all();
    lk.lock();
    it = index_.find(id);
    if (it == index_.end() || it->second.jrec.seg) return false;
  }
  if (it->second.dirty) {
    lk.unlock();
    flush();
    lk.lock();
    it = index_.find(id);
    if (it == index_.end()) return false;
  }
  if (::rename(data_path(id, false).c_str(), data_path(id, true).c_str()) != 0) return false;
  if (::rename(meta_path(id, false).c_str(), meta_path(id, true).c_str()) != 0) return false;
  // both directory entries changed: flush the new one before the old (a crash in between
  // leaves the block reachable under at least one tier)
  (void)sync_dir(true);
  (void)sync_dir(false);
  it->second.cold = true;
  // cold blocks leave the fast tier
  if (it->second.pins == 0) {
    free_extent_locked(it->second);
    lru_remove_locked(it->second);
    it->second.host.reset();
  }
  return true;
}

std::string ChunkStore::verify_on_disk(const std::string& id) {
  bool cold = false;
  JournalRec jrec;
  std::shared_ptr<std::vector<uint8_t>> jmeta;
  int64_t sz = -1;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end()) {
      cold = it->second.cold;
      jrec = it->second.jrec;
      jmeta = it->second.jmeta;
      if (jrec.seg) jrec.seg->readers++;  // released by DurableSrc
      if (jrec.seg) sz = static_cast<int64_t>(it->second.size);
    } else if (!cfg_.cold_dir.empty() && file_exists(data_path(id, true))) {
      cold = true;
    }
  }
  DurableSrc src;
  if (!open_durable(id, cold, jrec, jmeta, &src)) return src.fd < 0 ? "Block not found" : "Checksum file missing";
  auto& meta = src.meta;
  if (!jrec.seg) {
    struct stat stt;
    if (::fstat(src.fd, &stt) != 0) return "Block not found";
    sz = stt.st_size;
  }
  std::vector<uint8_t> data(static_cast<size_t>(sz));
  bool ok = read_all(src.fd, data.data(), data.size(), src.base);
  if (!ok && sz > 0) return "read failed";
  std::vector<uint32_t> act(num_slices(data.size()));
  crc32_slices(data.data(), data.size(), act.data());
  if (act.size() != meta.size()) return "Checksum count mismatch";
  for (size_t i = 0; i < act.size(); ++i)
    if (act[i] != meta[i]) return "Checksum mismatch at chunk " + std::to_string(i);
  return "";
}

std::vector<uint32_t> ChunkStore::meta(const std::string& id) {
  uint64_t size = 0;
  bool cold = false;
  int64_t off = -1;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end()) return {};
    size = it->second.size;
    cold = it->second.cold;
    off = it->second.dev_off;
    if (off >= 0) it->second.pins++;
  }
  if (off >= 0) {
    HIP_OK(hipSetDevice(cfg_.device));
    std::vector<uint32_t> m(num_slices(size));
    if (!m.empty())
      HIP_OK(hipMemcpy(m.data(), arena_ + off + align_up(std::max<uint64_t>(size, 1), 256), m.size() * 4,
                       hipMemcpyDeviceToHost));
    for (auto& v : m) v = __builtin_bswap32(v);
    unpin(id);
    return m;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end() && it->second.jmeta) {
      std::vector<uint32_t> m(it->second.jmeta->size() / 4);
      for (size_t i = 0; i < m.size(); ++i) {
        uint32_t be;
        std::memcpy(&be, it->second.jmeta->data() + 4 * i, 4);
        m[i] = __builtin_bswap32(be);
      }
      return m;
    }
  }
  bool ok = false;
  return load_meta_file(id, cold, &ok);
}

// K1b: every resident block (pinned by the caller) verified against its HBM .meta image in
// one kernel launch per 64K blocks, one sync, one small D2H of the per-block verdicts.
std::vector<std::string> ChunkStore::scrub_resident(const std::vector<std::string>& ids) {
  TraceRange tr("dfs.store.scrub");
  std::vector<std::string> bad;
  if (!gpu() || ids.empty()) return bad;
  HIP_OK(hipSetDevice(cfg_.device));
  constexpr size_t kBatch = 65536;
  const size_t cap = std::min(kBatch, ids.size());
  ScrubBlock* dblocks = nullptr;
  uint32_t* dbad = nullptr;
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&dblocks), cap * sizeof(ScrubBlock)));
  HIP_OK(hipMalloc(reinterpret_cast<void**>(&dbad), cap * sizeof(uint32_t)));
  std::vector<ScrubBlock> hb;
  std::vector<size_t> which;
  std::vector<uint32_t> hbad;
  Lane* l = acquire_lane();
  for (size_t base = 0; base < ids.size(); base += kBatch) {
    size_t cnt = std::min(kBatch, ids.size() - base);
    hb.clear();
    which.clear();
    uint64_t tiles = 0;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t j = 0; j < cnt; ++j) {
        auto it = index_.find(ids[base + j]);
        if (it == index_.end() || it->second.dev_off < 0 || it->second.size == 0) continue;
        uint64_t size = it->second.size;
        const uint8_t* d = arena_ + it->second.dev_off;
        ScrubBlock b{};
        b.data = d;
        b.meta = reinterpret_cast<const uint32_t*>(d + align_up(size, 256));
        b.s_full = size / kSliceBytes;
        b.tile_start = tiles;
        b.tail_len = static_cast<uint32_t>(size % kSliceBytes);
        b.tail_init = b.tail_len ? crc_init_term(b.tail_len) : 0;
        tiles += (b.s_full + kSlicesPerTile - 1) / kSlicesPerTile;
        hb.push_back(b);
        which.push_back(base + j);
      }
    }
    if (hb.empty()) continue;
    HIP_OK(hipMemcpyAsync(dblocks, hb.data(), hb.size() * sizeof(ScrubBlock), hipMemcpyHostToDevice, l->stream));
    HIP_OK(hipMemsetAsync(dbad, 0xFF, hb.size() * sizeof(uint32_t), l->stream));
    ScrubLaunch a{};
    a.blocks = dblocks;
    a.nblocks = static_cast<uint32_t>(hb.size());
    a.ntiles = tiles;
    a.full_init = crc_init_term(kSliceBytes);
    a.bad = dbad;
    HIP_OK(launch_scrub(a, dtables_, l->stream));
    launches_++;
    hbad.resize(hb.size());
    HIP_OK(hipMemcpyAsync(hbad.data(), dbad, hb.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
    for (size_t j = 0; j < hb.size(); ++j)
      if (hbad[j] != 0xFFFFFFFFu) bad.push_back(ids[which[j]]);
  }
  release_lane(l);
  (void)hipFree(dblocks);
  (void)hipFree(dbad);
  return bad;
}

std::vector<std::string> ChunkStore::scrub() {
  std::vector<std::string> bad;
  size_t hbm_bad = 0;  // bad[0, hbm_bad): HBM copies; the rest: durable copies
  std::vector<std::string> resident, disk;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : index_) {
      if (gpu() && kv.second.dev_off >= 0) {
        kv.second.pins++;
        resident.push_back(kv.first);
      } else if (kv.second.on_disk || kv.second.jrec.seg) {
        disk.push_back(kv.first);
      }
    }
  }
  if (!resident.empty()) {
    for (auto& id : scrub_resident(resident)) bad.push_back(id);
    hbm_bad = bad.size();
    for (auto& id : resident) unpin(id);
  }
  // durable copies (journal records, files): the non-resident blocks, and the resident
  // blocks' copies, verified by the same K1b kernel in staged batches (the CPU takes what
  // does not fit a batch)
  std::vector<std::string> cpu;
  if (gpu()) {
    std::vector<std::string> copies = disk;
    for (auto& id : resident) {
      std::lock_guard<std::mutex> g(mu_);
      auto it = index_.find(id);
      if (it != index_.end() && (it->second.on_disk || it->second.jrec.seg) && !it->second.dirty &&
          std::find(bad.begin(), bad.end(), id) == bad.end())
        copies.push_back(id);
    }
    for (auto& id : scrub_durable_gpu(copies, &cpu))
      if (std::find(bad.begin(), bad.end(), id) == bad.end()) bad.push_back(id);
  } else {
    cpu = disk;
  }
  for (auto& id : cpu)
    if (!verify_on_disk(id).empty() && std::find(bad.begin(), bad.end(), id) == bad.end()) bad.push_back(id);
  // a durable copy can change under the scan (exported to its files, relocated, rewritten by
  // a recovery): a durable-copy mismatch is reported only if the copy the index names now
  // fails again, so a scan racing those moves does not queue recoveries of healthy blocks
  std::vector<std::string> confirmed;
  uint64_t transient = 0;
  for (size_t i = 0; i < bad.size(); ++i) {
    if (i < hbm_bad || !verify_on_disk(bad[i]).empty()) confirmed.push_back(bad[i]);
    else ++transient;
  }
  std::lock_guard<std::mutex> g(mu_);
  st_.crc_mismatches += confirmed.size();
  st_.scrub_transient += transient;
  return confirmed;
}

std::vector<std::string> ChunkStore::list_blocks() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> v;
  v.reserve(index_.size());
  for (auto& kv : index_) v.push_back(kv.first);
  return v;
}

StoreStats ChunkStore::stats() {
  std::lock_guard<std::mutex> g(mu_);
  StoreStats s = st_;
  s.disk_gate_waits = gate_ ? gate_->waits() : 0;
  s.blocks = index_.size();
  s.bytes = 0;
  s.hbm_resident_blocks = 0;
  s.dirty_blocks = 0;
  for (auto& kv : index_) {
    s.bytes += kv.second.size;
    if (kv.second.dev_off >= 0) s.hbm_resident_blocks++;
    if (kv.second.dirty) s.dirty_blocks++;
  }
  s.hbm_used = alloc_.used();
  s.spill_queue = spill_q_.size();
  s.gpu_kernel_launches = launches_.load();
  s.direct_dma = direct_dma_.load();
  s.fused_reads = fused_reads_.load();
  s.fused_writes = fused_writes_.load();
  s.pulled_recvs = pulled_recvs_.load();
  s.pulled_host_appends = pulled_host_appends_.load();
  s.sliced_stages = sliced_stages_.load();
  s.staged_dma = staged_dma_.load();
  s.mirror_hits = mirror_hits_;
  s.mirror_bytes = mirror_bytes_;
  s.io_threads_spawned = io_.spawned();
  s.scrub_device_blocks = scrub_dev_blocks_.load();
  {
    std::lock_guard<std::mutex> lg(lane_mu_);
    s.lane_waits = lane_waits_;
    s.lane_wait_ns = lane_wait_ns_;
  }
  if (journal_) {
    JournalStats j = journal_->stats();
    s.journal = true;
    s.journal_records = j.records;
    s.journal_bytes = j.bytes;
    s.journal_commits = j.commits;
    s.journal_sync_rounds = j.sync_rounds;
    s.journal_mode = !store_mode_ ? "idle" : export_ ? "store" : "store-noexport";
    s.journal_tombstones = j.tombstones;
    s.journal_supersedes = j.supersedes;
    s.journal_full_waits = j.full_waits;
    s.journal_segs = j.segs_total;
    s.journal_segs_free = j.segs_free;
    s.journal_segs_in_use = j.segs_in_use;
    s.journal_segs_marked = j.segs_marked;
    s.journal_segs_retired = j.segs_retired;
    s.journal_replayed = j.replayed;
    s.journal_replay_skipped = j.replay_skipped;
    s.journal_replay_verified = j.replay_verified;
    s.journal_live_records = j.live_records;
    s.journal_live_bytes = j.live_bytes;
    s.journal_used_bytes = j.used_bytes;
    s.journal_failed = j.failed;
    s.journal_grow_blocked = j.grow_blocked;
    s.relocated_blocks = relocated_blocks_;
    s.relocated_bytes = relocated_bytes_;
    s.compactions = compactions_;
    s.export_deferred_headroom = export_deferred_;
    s.materialized_blocks = materialized_blocks_;
    s.materialized_bytes = materialized_bytes_;
    s.materialize_pending = mat_q_.size();
    s.materialize_batches = mat_batches_;
    s.materialize_errors = mat_errors_;
    s.materialize_last_error = mat_last_error_;
    s.journal_prepare_errors = j.prepare_errors;
    s.journal_segs_filled = j.filled;
    s.journal_fill_bytes = j.fill_bytes;
    s.journal_parts_unready = j.parts_unready;
    s.journal_spares_missing = j.spares_missing;
    s.journal_grow_deferred = j.grow_deferred;
    s.journal_mark_preflushes = j.mark_preflushes;
    s.journal_reserve_markers = j.reserve_markers;
    s.delete_tomb_failures = tomb_failures_;
    s.export_busy_polls = export_busy_polls_;
    s.journal_sync_ns = j.sync_ns;
    s.journal_bypassed = bypassed_.load();
    s.journal_commit_ns = j.commit_ns;
    s.journal_last_error = j.last_error;
  }
  {
    std::lock_guard<std::mutex> rg(reg_mu_);
    for (auto& r : reg_) s.host_registered_bytes += r.second;
  }
  return s;
}

void ChunkStore::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] {
    if (stop_) return true;
    for (auto& kv : index_)
      if (kv.second.dirty) return false;
    return true;
  });
}

void ChunkStore::drop_resident() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& kv : index_) {
    Block& b = kv.second;
    if (b.pins == 0 && !b.dirty && (b.on_disk || b.jrec.seg)) {
      free_extent_locked(b);
      lru_remove_locked(b);
      b.host.reset();
    }
  }
}

bool ChunkStore::debug_corrupt(const std::string& id, uint64_t offset) {
  bool cold = false;
  int64_t off = -1;
  uint64_t size = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end() || offset >= it->second.size) return false;
    cold = it->second.cold;
    off = it->second.dev_off;
    size = it->second.size;
    if (it->second.host) (*it->second.host)[offset] ^= 0xFF;
    if (it->second.mirror) (*it->second.mirror)[offset] ^= 0xFF;
    if (it->second.jrec.seg) {
      uint8_t c = 0;
      const int jfd = it->second.jrec.fd();
      const uint64_t at = it->second.jrec.data_off() + offset;
      if (read_all(jfd, &c, 1, at)) {
        c ^= 0xFF;
        write_all(jfd, &c, 1, at);
      }
    }
  }
  (void)size;
  std::string dp = data_path(id, cold);
  int fd = ::open(dp.c_str(), O_RDWR | O_CLOEXEC);
  if (fd >= 0) {
    uint8_t c = 0;
    if (read_all(fd, &c, 1, offset)) {
      c ^= 0xFF;
      write_all(fd, &c, 1, offset);
    }
    ::close(fd);
  }
  if (off >= 0) {
    HIP_OK(hipSetDevice(cfg_.device));
    uint8_t c = 0;
    HIP_OK(hipMemcpy(&c, arena_ + off + offset, 1, hipMemcpyDeviceToHost));
    c ^= 0xFF;
    HIP_OK(hipMemcpy(arena_ + off + offset, &c, 1, hipMemcpyHostToDevice));
  }
  return true;
}

bool ChunkStore::gf_matmul_gpu(const std::vector<std::vector<uint8_t>>& mat, const std::vector<const uint8_t*>& in,
                               const std::vector<uint8_t*>& out, uint64_t len) {
  TraceRange tr("dfs.store.rs_matmul");
  if (!gpu()) return false;
  int k = static_cast<int>(in.size()), rows = static_cast<int>(out.size());
  if (k > kMaxShards || rows > kMaxShards || static_cast<int>(mat.size()) != rows) return false;
  HIP_OK(hipSetDevice(cfg_.device));
  uint64_t stride = align_up(std::max<uint64_t>(len, 16), 256);
  const uint64_t tbytes = static_cast<uint64_t>(rows) * k * 32;
  DevExtent ext = reserve(stride * (k + rows) + align_up(tbytes, 256));
  if (ext.off < 0) return false;
  // split-nibble product tables of the matrix (32 B per coefficient), uploaded once
  std::vector<uint8_t> flat(static_cast<size_t>(rows) * k);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < k; ++c) flat[r * k + c] = mat[r][c];
  auto* dtab = reinterpret_cast<uint32_t*>(ext.ptr + stride * (k + rows));
  // Column-chunked pipeline over two lanes (streams): while chunk j computes and drains on
  // one lane, chunk j+1's inputs are already crossing PCIe on the other; with registered
  // (pinned) client buffers every copy is a single DMA in each direction, both directions busy.
  Lane* lanes[2];
  {
    // both lanes at once: two callers holding one lane each must not wait for each other
    std::unique_lock<std::mutex> lk(lane_mu_);
    lane_cv_.wait(lk, [&] { return free_lanes_.size() >= 2; });
    for (Lane*& l : lanes) {
      l = free_lanes_.back();
      free_lanes_.pop_back();
    }
  }
  ensure_hscratch(lanes[0], tbytes + 16);
  auto* htab = reinterpret_cast<uint32_t*>(lanes[0]->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16);
  gf_nibble_tables(flat.data(), rows, k, htab);
  HIP_OK(hipMemcpyAsync(dtab, htab, tbytes, hipMemcpyHostToDevice, lanes[0]->stream));
  HIP_OK(hipStreamSynchronize(lanes[0]->stream));
  // per shard per step: small enough that the pipeline's fill (first H2D) and drain (last
  // D2H) are short, large enough that each copy runs at full DMA rate (DFS_RS_CHUNK_KIB)
  static const uint64_t min_chunk = [] {
    const char* e = std::getenv("DFS_RS_CHUNK_KIB");
    long v = e ? std::atol(e) : 4096;
    return static_cast<uint64_t>(v > 64 ? v : 64) << 10;
  }();
  const uint64_t chunk = std::max<uint64_t>(min_chunk, align_up(len / 64, 4096));
  bool ok = true;
  for (uint64_t off = 0, j = 0; off < len && ok; off += chunk, ++j) {
    Lane* l = lanes[j & 1];
    const uint64_t n = std::min(chunk, len - off);
    GfLaunch a{};
    a.k = k;
    a.rows = rows;
    a.len = n;
    a.tables = dtab;
    for (int c = 0; c < k; ++c) {
      a.in[c] = ext.ptr + c * stride + off;
      h2d_chunked(l, ext.ptr + c * stride + off, in[c] + off, n);
    }
    for (int r = 0; r < rows; ++r) a.out[r] = ext.ptr + (k + r) * stride + off;
    ok = launch_gf_matmul(a, l->stream) == hipSuccess;
    launches_++;
    for (int r = 0; ok && r < rows; ++r) d2h_chunked(l, out[r] + off, a.out[r], n);
  }
  for (Lane* l : lanes) {
    HIP_OK(hipStreamSynchronize(l->stream));
    release_lane(l);
  }
  release(ext);
  return ok;
}

uint32_t ChunkStore::gpu_crc(const uint8_t* data, uint64_t n, std::vector<uint32_t>* slices) {
  if (!gpu()) throw std::runtime_error("gpu_crc: store has no GPU");
  HIP_OK(hipSetDevice(cfg_.device));
  DevExtent ext = reserve(n);
  if (ext.off < 0) throw std::runtime_error("HBM arena full");
  Lane* l = acquire_lane();
  uint64_t S = num_slices(n);
  auto* dmeta = reinterpret_cast<uint32_t*>(ext.ptr + align_up(std::max<uint64_t>(n, 1), 256));
  h2d_chunked(l, ext.ptr, data, n);
  CrcOut co;
  std::string err;
  bool ok = run_crc(l, ext.ptr, n, dmeta, nullptr, true, 0, n, &co, &err);
  if (ok && slices) {
    slices->resize(S);
    if (S) HIP_OK(hipMemcpy(slices->data(), dmeta, S * 4, hipMemcpyDeviceToHost));
    for (auto& v : *slices) v = __builtin_bswap32(v);
  }
  release_lane(l);
  release(ext);
  if (!ok) throw std::runtime_error(err);
  return co.block_crc;
}


// ---------------------------------------------------------------- block journal
ChunkStore::DurableSrc::~DurableSrc() {
  if (own_fd && fd >= 0) ::close(fd);
  if (seg) seg->readers--;
}

// `jrec.seg`, when set, was captured under mu_ with its reader count raised (the segment
// cannot retire until this DurableSrc lets go of it).
bool ChunkStore::open_durable(const std::string& id, bool cold, const JournalRec& jrec,
                              const std::shared_ptr<std::vector<uint8_t>>& jmeta, DurableSrc* s) {
  if (jrec.seg) {
    s->seg = jrec.seg;
    s->fd = jrec.fd();
    s->base = jrec.data_off();
    s->meta_ok = jmeta != nullptr;
    if (jmeta) {
      s->meta.resize(jmeta->size() / 4);
      for (size_t i = 0; i < s->meta.size(); ++i) {
        uint32_t be;
        std::memcpy(&be, jmeta->data() + 4 * i, 4);
        s->meta[i] = __builtin_bswap32(be);
      }
    }
    return s->meta_ok;
  }
  s->fd = ::open(data_path(id, cold).c_str(), O_RDONLY | O_CLOEXEC);
  if (s->fd < 0) return false;
  s->own_fd = true;
  s->meta = load_meta_file(id, cold, &s->meta_ok);
  return s->meta_ok;
}

ChunkStore::FileClaim::FileClaim(ChunkStore* st, const std::string& i) : s(st), id(i) {
  std::lock_guard<std::mutex> g(s->mu_);
  s->file_writers_[id]++;
}

ChunkStore::FileClaim::~FileClaim() {
  std::lock_guard<std::mutex> g(s->mu_);
  auto it = s->file_writers_.find(id);
  if (it != s->file_writers_.end() && --it->second <= 0) s->file_writers_.erase(it);
}

bool ChunkStore::supersede_file(const std::string& id, std::string* err) {
  if (!journal_) return true;
  return journal_->marker(kJrFile, id, err);
}

bool ChunkStore::journal_block(const std::string& id, const uint8_t* host, const uint8_t* dev, uint64_t n,
                               uint32_t crc, const std::vector<uint8_t>& meta_be, JournalRec* out, std::string* err) {
  TraceRange tr("dfs.store.journal");
  const uint64_t S = meta_be.size() / 4;
  JournalRec jr;
  bool ok = true;
  // DFS_JOURNAL_GATE=1: the append + commit holds a node-wide disk slot (taken before any
  // lane, so no slot holder ever waits for a lane holder that waits for a slot)
  DiskGate::Slot slot = journal_gate_ && gate_ ? gate_->acquire() : DiskGate::Slot{};
  if (dev) {
    // out of HBM through the lane's two pinned chunks: the D2H of chunk c+1 overlaps the
    // append of chunk c. The lane is taken before the record so a writer never holds a
    // reserved record while it waits for a lane (commit() waits on earlier records).
    HIP_OK(hipSetDevice(cfg_.device));
    Lane* l = acquire_lane();
    if (!journal_->reserve(n, S, &jr, err)) {
      release_lane(l);
      return false;
    }
    const uint64_t nch = (n + kChunk - 1) / kChunk;
    auto issue = [&](uint64_t c) {
      const uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, n - off);
      HIP_OK(hipMemcpyAsync(l->pinned[c & 1], dev + off, len, hipMemcpyDeviceToHost, l->stream));
      HIP_OK(hipEventRecord(l->ev[c & 1], l->stream));
    };
    if (nch) issue(0);
    for (uint64_t c = 0; c < nch; ++c) {
      if (c + 1 < nch) issue(c + 1);
      HIP_OK(hipEventSynchronize(l->ev[c & 1]));
      const uint64_t off = c * kChunk, len = std::min<uint64_t>(kChunk, n - off);
      if (ok) ok = journal_->write(jr, off, l->pinned[c & 1], len);
    }
    release_lane(l);
  } else {
    if (!journal_->reserve(n, S, &jr, err)) return false;
    ok = journal_->write(jr, 0, host, n);
  }
  if (!ok) {
    *err = errno_str("journal append");
    journal_->abandon(jr);
    return false;
  }
  if (!journal_->finish(&jr, id, n, crc, meta_be.data(), S) || !journal_->commit(jr)) {
    *err = "journal commit failed";
    journal_->release(jr);  // never indexed
    return false;
  }
  *out = jr;
  return true;
}

// The nvme-sync head write with the journal: the block bytes are appended to the reserved
// record (from the caller's buffer, on an I/O thread) while the GPU stages and checksums
// them; the header + .meta image follow once the kernel has produced them, and one group
// commit makes the record durable. The block is acked resident in HBM and durable in the
// journal, which stays its durable home until the exporter writes `<id>` + `<id>.meta`.
WriteResult ChunkStore::stage_journal(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc,
                                      const DevExtent& ext) {
  WriteResult res;
  const uint64_t S = num_slices(n);
  JournalRec jr;
  std::string err;
  DiskGate::Slot slot = journal_gate_ && gate_ ? gate_->acquire() : DiskGate::Slot{};  // see journal_block
  if (!journal_->reserve(n, S, &jr, &err)) {
    release(ext);
    res.error = err;
    return res;
  }
  std::future<bool> wf;
  bool wok = true;
  if (n <= kMirrorMax) wok = journal_->write(jr, 0, data, n);  // a thread hand-off costs more
  else wf = io_.submit([this, &jr, data, n] { return journal_->write(jr, 0, data, n); });
  CrcOut co;
  auto meta = std::make_shared<std::vector<uint8_t>>();
  bool ok = device_stage(data, n, ext, meta.get(), &co, &err);
  if (wf.valid()) wok = wf.get();
  res.actual_crc = co.block_crc;
  const bool mismatch = ok && expected_crc != 0 && co.block_crc != expected_crc;
  if (!ok || mismatch || !wok) {
    journal_->abandon(jr);
    release(ext);
    if (mismatch) {
      std::lock_guard<std::mutex> g(mu_);
      ++st_.crc_mismatches;
      res.error = "Checksum mismatch: expected " + std::to_string(expected_crc) + ", actual " +
                  std::to_string(co.block_crc);
    } else {
      res.error = ok ? errno_str("journal append") : err;
    }
    return res;
  }
  if (!journal_->finish(&jr, id, n, co.block_crc, meta->data(), S) || !journal_->commit(jr)) {
    journal_->release(jr);
    release(ext);
    res.error = "journal commit failed";
    return res;
  }
  insert_resident(id, ext, n, co.block_crc, false, meta, 0, &jr);
  if (n <= kMirrorMax) set_mirror(id, data, n, *meta);
  res.ok = true;
  return res;
}

// Store of record: every durable write that fits a segment part goes to the journal. Round-4
// mode: while the journal has room below the materializer's mark; past it the materializer
// is already writing every journaled block a second time, so a write through the journal
// would cost the volume twice; it takes the per-file path instead (written once).
bool ChunkStore::journal_takes(uint64_t n, uint64_t nslices) {
  if (!journal_ || !journal_->fits(n, nslices)) return false;
  last_durable_write_ns_.store(static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                         std::chrono::steady_clock::now().time_since_epoch())
                                                         .count()),
                               std::memory_order_relaxed);
  if (store_mode_ || !journal_bypass_ || journal_->pressure() < mat_pressure_) return true;
  bypassed_++;
  return false;
}

void ChunkStore::enqueue_materialize_locked(const std::string& id, const Block& b) {
  mat_q_.push_back(MatItem{id, b.jrec, b.size, b.jmeta});
  mat_cv_.notify_all();
}

// Round-4 mode: materialization competes with the acked writes for the volume, so it runs
// when the writers pause (idle: no durable write, journaled or not, for DFS_JOURNAL_IDLE_MS),
// not on every append. Without the bypass it also runs once the journal is at its mark (the
// writers would block on a full journal otherwise). With the bypass, writes past the mark
// already go to their own files, written once.
bool ChunkStore::materialize_due() {
  if (mat_idle_ns_ == 0) return true;
  const double p = journal_->pressure();
  if (p >= (journal_bypass_ ? 0.97 : mat_pressure_)) return true;
  const uint64_t now = static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                 std::chrono::steady_clock::now().time_since_epoch())
                                                 .count());
  const uint64_t last = std::max<uint64_t>(journal_->last_append_ns(), last_durable_write_ns_.load());
  return now - last >= mat_idle_ns_;
}

// Export doubles a block's footprint until its journal segment recycles; it runs only while
// the volume keeps export_headroom_ free besides the batch (a full node keeps its blocks in
// the journal, which holds them in about one copy's space).
bool ChunkStore::export_headroom(uint64_t bytes) {
  struct statvfs sv;
  if (::statvfs(cfg_.storage_dir.c_str(), &sv) != 0) return false;
  return static_cast<uint64_t>(sv.f_bavail) * sv.f_frsize >= export_headroom_ + bytes;
}

namespace {
// The record's bytes into a fresh file: copy_file_range keeps them in the kernel (page
// cache to page cache, or a reflink where the filesystem shares extents).
bool copy_range(int in_fd, uint64_t in_off, int out_fd, uint64_t n) {
  loff_t io = static_cast<loff_t>(in_off), oo = 0;
  uint64_t left = n;
  while (left) {
    ssize_t r = ::copy_file_range(in_fd, &io, out_fd, &oo, left, 0);
    if (r > 0) {
      left -= static_cast<uint64_t>(r);
      continue;
    }
    if (r < 0 && errno == EINTR) continue;
    break;  // unsupported here (EXDEV / ENOSYS / EINVAL): plain reads and writes
  }
  if (!left) return true;
  std::vector<uint8_t> buf(std::min<uint64_t>(left, 4ull << 20));
  while (left) {
    const uint64_t len = std::min<uint64_t>(left, buf.size());
    if (!read_all(in_fd, buf.data(), len, static_cast<uint64_t>(io)) ||
        !write_all(out_fd, buf.data(), len, static_cast<uint64_t>(oo)))
      return false;
    io += len;
    oo += len;
    left -= len;
  }
  return true;
}
}  // namespace

// Writes each pinned job as `<id>` + `<id>.meta` under private temporary names, starts the
// writeback of all of them at once (sync_file_range) and then flushes each file
// (fdatasync: per file, not the whole filesystem), renames each into place only while its
// record is still the block's current version and no per-file writer holds the id (checked
// and renamed under mu_, so an export never lands over a newer per-file version), and
// flushes the directory once. A block whose names are durable leaves the journal: its index
// entry points at the files and its record is released.
uint64_t ChunkStore::export_batch(std::vector<MatItem>& batch, bool retry) {
  TraceRange tr("dfs.store.export");
  struct Job {
    int fd = -1, mfd = -1;
    bool ok = false, renamed = false, claimed = false;
    std::string dtmp, mtmp, err;
  };
  std::vector<Job> jobs(batch.size());
  for (size_t i = 0; i < batch.size(); ++i) {
    Job& j = jobs[i];
    const MatItem& m = batch[i];
    const std::string sfx = ".x" + std::to_string(tmp_seq_.fetch_add(1)) + ".tmp";
    j.dtmp = data_path(m.id, false) + sfx;
    j.mtmp = meta_path(m.id, false) + sfx;
    j.fd = ::open(j.dtmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    j.mfd = j.fd < 0 ? -1 : ::open(j.mtmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    j.ok = j.mfd >= 0 && copy_range(m.rec.fd(), m.rec.data_off(), j.fd, m.n) &&
           write_all(j.mfd, m.meta->data(), m.meta->size(), 0);
    if (!j.ok) j.err = errno_str(j.dtmp.c_str());
  }
  if (cfg_.sync_writes) {
    for (auto& j : jobs)
      if (j.ok) {
        (void)::sync_file_range(j.fd, 0, 0, SYNC_FILE_RANGE_WRITE);
        (void)::sync_file_range(j.mfd, 0, 0, SYNC_FILE_RANGE_WRITE);
      }
    for (auto& j : jobs)
      if (j.ok && (::fdatasync(j.fd) != 0 || ::fdatasync(j.mfd) != 0)) {
        j.ok = false;
        j.err = errno_str("fdatasync " + j.dtmp);
      }
  }
  const bool drop = gpu();
  for (auto& j : jobs) {
    if (j.fd >= 0) {
      if (drop) drop_cached(j.fd);
      ::close(j.fd);
    }
    if (j.mfd >= 0) ::close(j.mfd);
  }
  bool any = false;
  for (size_t i = 0; i < batch.size(); ++i) {
    Job& j = jobs[i];
    if (j.ok) {
      std::lock_guard<std::mutex> g(mu_);
      auto it = index_.find(batch[i].id);
      const bool current = it != index_.end() && it->second.jrec.same(batch[i].rec);
      j.claimed = file_writers_.count(batch[i].id) > 0;
      if (current && !j.claimed) {
        // .meta first: a crash between the renames leaves a .meta with no data file (ignored)
        if (::rename(j.mtmp.c_str(), meta_path(batch[i].id, false).c_str()) == 0 &&
            ::rename(j.dtmp.c_str(), data_path(batch[i].id, false).c_str()) == 0) {
          j.renamed = any = true;
        } else {
          j.ok = false;
          j.err = errno_str("rename " + j.dtmp);
        }
      }
    }
    if (!j.renamed) {
      ::unlink(j.dtmp.c_str());
      ::unlink(j.mtmp.c_str());
    }
  }
  // the names are durable once the directory is: only then does the index leave the journal
  const bool dir_ok = !any || !cfg_.sync_writes || sync_dir(false);
  std::vector<JournalRec> released;
  uint64_t exported = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < batch.size(); ++i) {
      Job& j = jobs[i];
      MatItem& m = batch[i];
      auto it = index_.find(m.id);
      if (it == index_.end()) continue;
      it->second.pins--;
      if (!it->second.jrec.same(m.rec)) continue;  // rewritten meanwhile: that version counts
      if (j.renamed && dir_ok) {
        it->second.on_disk = true;
        it->second.jrec = JournalRec{};
        it->second.jmeta.reset();
        released.push_back(m.rec);
        ++materialized_blocks_;
        materialized_bytes_ += m.n;
        ++exported;
        continue;
      }
      if (!j.ok || !dir_ok) {
        ++mat_errors_;
        mat_last_error_ = j.ok ? errno_str("fsync " + cfg_.storage_dir) : j.err;
      }
      // still journal-resident: the record stays its durable copy; try again later (a
      // per-file writer that fails leaves the record current)
      if (retry) mat_q_.push_back(std::move(m));
    }
    ++mat_batches_;
  }
  cv_.notify_all();
  for (auto& r : released) journal_->release(r);
  return exported;
}

// Moves one journal-resident block's record to the head of the journal, keeping its LSN
// (a rewrite committed meanwhile has a larger one, so replay still prefers it). The block is
// pinned while it moves: writers of the id and remove() wait, so a tombstone is never
// appended before the copy it must cancel. A copy that lost the race with a rewrite is made
// durable padding before the old record is given up.
bool ChunkStore::relocate_one(const std::string& id, const JournalRec& old) {
  std::shared_ptr<std::vector<uint8_t>> meta;
  uint64_t n = 0;
  uint32_t crc = 0;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it == index_.end() || !it->second.jrec.same(old) || !it->second.jmeta) return false;
    it->second.pins++;
    meta = it->second.jmeta;
    n = it->second.size;
    crc = it->second.crc;
  }
  const uint64_t S = meta->size() / 4;
  std::vector<uint8_t> buf(n);
  bool ok = n == 0 || read_all(old.fd(), buf.data(), n, old.data_off());
  JournalRec nr;
  std::string err;
  bool appended = false;
  if (ok && journal_->reserve(n, S, &nr, &err)) {
    if (!journal_->write(nr, 0, buf.data(), n)) {
      journal_->abandon(nr);
    } else {
      appended = journal_->finish(&nr, id, n, crc, meta->data(), S, old.lsn) && journal_->commit(nr);
      if (!appended) journal_->release(nr);
    }
  }
  bool swapped = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    auto it = index_.find(id);
    if (it != index_.end()) {
      it->second.pins--;
      if (appended && it->second.jrec.same(old)) {
        it->second.jrec = nr;
        swapped = true;
        ++relocated_blocks_;
        relocated_bytes_ += n;
        enqueue_materialize_locked(id, it->second);  // the queued item names the old record
      }
    }
  }
  cv_.notify_all();
  if (swapped) {
    journal_->release(old);
  } else if (appended) {
    journal_->pad_durable(nr);
    journal_->release(nr);
  }
  return swapped;
}

uint64_t ChunkStore::relocate_segment(const SegRef& seg, uint64_t budget_bytes) {
  std::lock_guard<std::mutex> cg(compact_mu_);
  std::vector<std::pair<std::string, JournalRec>> todo;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& kv : index_)
      if (kv.second.jrec.seg == seg) todo.emplace_back(kv.first, kv.second.jrec);
  }
  // in record order: the copies land in the head in the order they were written
  std::sort(todo.begin(), todo.end(), [](const auto& a, const auto& b) {
    return a.second.part != b.second.part ? a.second.part < b.second.part : a.second.off < b.second.off;
  });
  uint64_t moved = 0, bytes = 0;
  for (auto& t : todo) {
    if (bytes >= budget_bytes) break;
    if (relocate_one(t.first, t.second)) {
      ++moved;
      bytes += t.second.bytes();
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (bytes < budget_bytes) ++compactions_;  // the segment is empty now (unless it raced)
  }
  journal_->retire_ready();
  return bytes;
}

uint64_t ChunkStore::compact(double max_live) {
  if (!journal_ || !store_mode_) return 0;
  uint64_t before;
  {
    std::lock_guard<std::mutex> g(mu_);
    before = relocated_blocks_;
  }
  for (;;) {
    SegRef seg = journal_->compaction_candidate(max_live);
    if (!seg) break;
    relocate_segment(seg, UINT64_MAX);
    if (journal_->compaction_candidate(max_live) == seg) break;  // pinned by readers / raced
  }
  std::lock_guard<std::mutex> g(mu_);
  return relocated_blocks_ - before;
}

// The exporter / compaction thread. Store mode: journal-resident blocks are exported as
// reference-format files through a token bucket (DFS_EXPORT_MBPS) at idle I/O priority,
// while the volume has headroom; without headroom (or with export off) the oldest segment is
// compacted once enough of the journal is dead. Round-4 mode: everything is materialized
// when the writers pause (materialize_due). Either way materialize_all() forces a full
// export, and a stop ends after at most one failed pass (what failed stays in the journal).
void ChunkStore::materializer_loop() {
  if (store_mode_) {
    // idle I/O class for this thread (honoured by the BFQ / CFQ schedulers; the token bucket
    // is what bounds it everywhere)
    constexpr long kWhoProcess = 1, kClassIdle = 3, kClassShift = 13;
    (void)::syscall(SYS_ioprio_set, kWhoProcess, 0L, kClassIdle << kClassShift);
  }
  const double burst = 64.0 * (1 << 20), kBusyBurst = 8.0 * (1 << 20);
  double tokens = burst;
  auto t_prev = std::chrono::steady_clock::now();
  bool headroom = false, stop_failed = false;
  bool want_compact = false, compact_urgent = false, reclaim = false;
  auto headroom_at = t_prev, compact_check_at = t_prev;
  std::vector<MatItem> batch;
  for (;;) {
    batch.clear();
    uint64_t bytes = 0;
    bool compact_now = false, forced = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      for (;;) {
        const auto t = std::chrono::steady_clock::now();
        const uint64_t last_append = store_mode_ ? journal_->last_append_ns() : 0;
        // Writers active: exports trickle (DFS_EXPORT_BUSY_MBPS, small bursts) so they stay out
        // of the acked writes' way. Not while segments wait for compaction: reclaim is what
        // keeps the writers from finding the journal full, and at the trickle rate it never
        // got the half burst it starts at (config 5's multipart phase: 6,371 writer waits,
        // uploads timing out at 120 s, profiles/r6/config5.json first run).
        const bool busy = last_append && mono_ns() - last_append < 50000000ull && !reclaim;
        const double cap = busy ? std::min(burst, kBusyBurst) : burst;
        tokens = std::min(cap, tokens + (busy ? export_busy_bps_ : export_bps_) *
                                            std::chrono::duration<double>(t - t_prev).count());
        if (busy) ++export_busy_polls_;
        t_prev = t;
        if (mat_q_.empty() && !mat_busy_) mat_cv_.notify_all();  // materialize_all() waiters
        if (mat_stop_ && (store_mode_ || mat_q_.empty() || stop_failed)) return;
        if (mat_paused_) {
          mat_cv_.wait_for(lk, std::chrono::milliseconds(50));
          continue;
        }
        forced = mat_force_ > 0 || mat_stop_;
        // Reclaim before export: while a quarter of the journal is dead and its oldest segment
        // can be compacted, the tokens go to relocation, not to exports. Segments are reused
        // oldest first, so one old segment holding a few live records keeps every dead one
        // behind it; with the exports spending every token as it arrived, compaction never
        // ran under sustained overwrites and the journal grew until the volume was full (config
        // 5's 10 s phases: 5,780 writer waits, multipart uploads timing out at 120 s, r5w). A
        // journal that can no longer grow compacts without waiting for tokens.
        if (store_mode_ && !forced && t >= compact_check_at) {
          compact_check_at = t + std::chrono::milliseconds(20);
          lk.unlock();
          const JournalStats j = journal_->stats();
          // dead space in the segments behind the active one (the active one's unwritten
          // tail is not dead): a quarter of them, and more than one segment's worth
          const uint64_t dead = j.sealed_used_bytes - std::min(j.sealed_used_bytes, j.sealed_live_bytes);
          reclaim = j.grow_blocked || (dead > j.sealed_used_bytes / 4 && dead > journal_->seg_bytes());
          // Segments retire oldest first, so an oldest segment that stays mostly live (blocks
          // nobody overwrites, exports behind) holds every dead segment behind it: under
          // reclaim it is relocated whatever its live share (config 5's multipart phase: 80 GB
          // of journal for 2.35 GB live, the volume full, writers waiting, r6c5).
          want_compact = reclaim && journal_->compaction_candidate(1.0) != nullptr;
          compact_urgent = j.grow_blocked;
          lk.lock();
        }
        if (want_compact && (tokens >= burst / 2 || compact_urgent) && !mat_paused_ && !mat_stop_) {
          compact_now = true;
          want_compact = false;  // re-evaluated after this pass
          compact_check_at = t;
          break;
        }
        if (!mat_q_.empty()) {
          if (forced) break;
          if (!store_mode_) {
            if (materialize_due()) break;
          } else if (export_ && !want_compact &&
                     tokens >= std::min<double>(burst, static_cast<double>(mat_q_.front().n))) {
            if (t >= headroom_at) {
              lk.unlock();
              headroom = export_headroom(64ull << 20);
              lk.lock();
              headroom_at = t + std::chrono::milliseconds(500);
              if (!headroom) ++export_deferred_;
            }
            if (headroom) break;
          }
        }
        if (!store_mode_ && mat_q_.empty()) {
          lk.unlock();
          journal_->retire_ready();  // segments whose readers have finished since
          lk.lock();
        }
        mat_cv_.wait_for(lk, std::chrono::milliseconds(store_mode_ ? 50 : mat_q_.empty() ? 200 : 5));
      }
      if (!compact_now) {
        // a drain in a pause goes in small batches and re-checks for writers between them;
        // under pressure, or when asked to drain, the batches are large; the store mode's
        // batches are what the token bucket allows
        const bool urgent = forced || (!store_mode_ && (mat_idle_ns_ == 0 ||
                                                         journal_->pressure() >= (journal_bypass_ ? 0.97 : mat_pressure_)));
        const uint64_t cap = urgent ? (256ull << 20) : store_mode_ ? static_cast<uint64_t>(std::max(tokens, 1.0))
                                                                   : (32ull << 20);
        while (!mat_q_.empty() && batch.size() < 1024 && (bytes < cap || batch.empty())) {
          MatItem m = std::move(mat_q_.front());
          mat_q_.pop_front();
          auto it = index_.find(m.id);
          if (it == index_.end() || !it->second.jrec.same(m.rec)) continue;  // superseded: nothing to do
          it->second.pins++;  // a rewrite or remove() of the id waits for the export
          bytes += m.n;
          batch.push_back(std::move(m));
        }
        mat_busy_ = !batch.empty();
      }
    }
    if (compact_now) {
      SegRef seg = journal_->compaction_candidate(1.0);
      // urgent (the journal cannot grow): one whole segment's live records whatever the tokens
      const double budget = compact_urgent ? static_cast<double>(journal_->seg_bytes()) : std::max(tokens, 1.0);
      if (seg) tokens -= static_cast<double>(relocate_segment(seg, static_cast<uint64_t>(budget)));
      tokens = std::max(tokens, -burst);  // an urgent pass's debt is bounded
      continue;
    }
    if (batch.empty()) continue;
    const size_t want = batch.size();
    const uint64_t done = export_batch(batch, !mat_stop_);
    tokens -= static_cast<double>(bytes);
    {
      std::lock_guard<std::mutex> g(mu_);
      mat_busy_ = false;
      if (done < want && mat_stop_) stop_failed = true;
    }
    mat_cv_.notify_all();
    if (done < want && !mat_stop_ && !forced) std::this_thread::sleep_for(std::chrono::milliseconds(100));
  }
}

void ChunkStore::materialize_all() {
  if (!journal_) return;
  std::unique_lock<std::mutex> lk(mu_);
  if (mat_paused_) return;
  ++mat_force_;
  mat_cv_.notify_all();
  // failures are requeued: give up once a pass made no progress for a while
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
  mat_cv_.wait_until(lk, deadline, [&] { return (mat_q_.empty() && !mat_busy_) || mat_paused_ || mat_stop_; });
  --mat_force_;
}

void ChunkStore::debug_pause_materializer(bool on) {
  {
    std::lock_guard<std::mutex> g(mu_);
    mat_paused_ = on;
  }
  mat_cv_.notify_all();
}

bool ChunkStore::journaled(const std::string& id) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = index_.find(id);
  return it != index_.end() && it->second.jrec.seg != nullptr;
}

void ChunkStore::replay_journal() {
  std::vector<ReplayRecord> recs = journal_->recover();
  // a replayed block record's data against its .meta image and whole-block CRC (K1/K2 on
  // the GPU for blocks past the host-mirror size)
  auto verify = [&](const ReplayRecord& r, std::vector<uint8_t>& buf) {
    buf.resize(r.n);
    if (r.n && !read_all(r.fd(), buf.data(), r.n, r.data_off())) return false;
    std::vector<uint32_t> sl;
    uint32_t whole;
    if (gpu() && r.n > kMirrorMax) {
      whole = gpu_crc(buf.data(), r.n, &sl);
    } else {
      sl.resize(num_slices(r.n));
      crc32_slices(buf.data(), r.n, sl.data());
      whole = crc32_from_slices(sl.data(), r.n);
    }
    bool good = whole == r.crc && sl.size() * 4 == r.meta_be.size();
    for (size_t i = 0; good && i < sl.size(); ++i) {
      uint32_t be;
      std::memcpy(&be, r.meta_be.data() + 4 * i, 4);
      good = __builtin_bswap32(be) == sl[i];
    }
    return good;
  };
  uint64_t replayed = 0, skipped = 0, verified = 0;
  bool cold_touched = false, hot_touched = false;
  std::vector<uint8_t> buf;
  auto drop_files = [&](const std::string& id) {
    if (!cfg_.cold_dir.empty() && file_exists(data_path(id, true))) {
      ::unlink(data_path(id, true).c_str());
      ::unlink(meta_path(id, true).c_str());
      cold_touched = true;
    }
    if (file_exists(data_path(id, false)) || file_exists(meta_path(id, false))) {
      ::unlink(data_path(id, false).c_str());
      ::unlink(meta_path(id, false).c_str());
      hot_touched = true;
    }
  };
  if (store_mode_) {
    // Store of record: per id, from its newest record back, the first tombstone, supersede
    // marker or intact block record decides. A block record is indexed where it lies (the
    // journal stays its home; the exporter may write its files later). Records of segments
    // sealed durable are trusted; the others' data is re-checked (a torn record was never
    // acknowledged: the id falls back to its previous version).
    std::unordered_map<std::string, std::vector<size_t>> by_id;
    for (size_t i = 0; i < recs.size(); ++i) by_id[recs[i].id].push_back(i);
    std::vector<char> keep(recs.size(), 0);
    std::vector<size_t> chosen_recs;  // indexed below, under the lock (verification takes it)
    for (auto& kv : by_id) {
      const std::string& id = kv.first;
      if (!valid_block_id(id)) {
        ++skipped;
        continue;
      }
      long chosen = -1;
      uint32_t decided = 0;
      for (auto it = kv.second.rbegin(); it != kv.second.rend(); ++it) {
        const ReplayRecord& r = recs[*it];
        if (r.type != kJrBlock) {
          decided = r.type;
          break;
        }
        if (!r.trusted) {
          ++verified;
          if (!verify(r, buf)) {
            ++skipped;
            continue;
          }
        }
        chosen = static_cast<long>(*it);
        decided = kJrBlock;
        break;
      }
      if (decided == kJrTomb) drop_files(id);
      if (decided != kJrBlock) continue;  // kJrFile: its files are the home (scan_dirs indexes them)
      const ReplayRecord& r = recs[static_cast<size_t>(chosen)];
      if (file_size(data_path(id, false)) == static_cast<int64_t>(r.n) &&
          file_size(meta_path(id, false)) == static_cast<int64_t>(r.meta_be.size())) {
        // an export of this very record that was durable before the crash (same size, same
        // .meta image): the files are the home, the record is released (scan_dirs indexes them)
        std::vector<uint8_t> m(r.meta_be.size());
        int fd = ::open(meta_path(id, false).c_str(), O_RDONLY | O_CLOEXEC);
        const bool same = fd >= 0 && (m.empty() || read_all(fd, m.data(), m.size(), 0)) && m == r.meta_be;
        if (fd >= 0) ::close(fd);
        if (same) continue;
      }
      keep[static_cast<size_t>(chosen)] = 1;
      drop_files(id);  // an older per-file version: the record is the latest, and the home
      chosen_recs.push_back(static_cast<size_t>(chosen));
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i : chosen_recs) {
        const ReplayRecord& r = recs[i];
        Block& b = index_[r.id];
        b = Block{};
        b.size = r.n;
        b.crc = r.crc;
        b.crc_known = true;
        b.jrec = r.rec;
        b.jmeta = std::make_shared<std::vector<uint8_t>>(r.meta_be);
        enqueue_materialize_locked(r.id, b);
        ++replayed;
      }
    }
    if ((hot_touched && !sync_dir(false)) || (cold_touched && !sync_dir(true)))
      throw std::runtime_error("journal replay: directory sync");
    std::vector<JournalRec> dead;
    for (size_t i = 0; i < recs.size(); ++i)
      if (recs[i].type == kJrBlock && !keep[i]) dead.push_back(recs[i].rec);
    recs.clear();
    journal_->note_replay(replayed, skipped, verified);
    // (release() takes only the journal's lock)
    for (auto& r : dead) journal_->release(r);
    return;
  }
  // Round-4 mode: the latest state per block id is verified and written out as `<id>` +
  // `<id>.meta`; tombstoned ids lose their files. Then every segment is retired and
  // scan_dirs() indexes the result.
  std::unordered_map<std::string, long> last;  // id -> index of its final record (-1: deleted, -2: own files)
  for (size_t i = 0; i < recs.size(); ++i)
    last[recs[i].id] = recs[i].type == kJrBlock ? static_cast<long>(i) : recs[i].type == kJrTomb ? -1 : -2;
  std::string err;
  for (auto& kv : last) {
    const std::string& id = kv.first;
    if (!valid_block_id(id)) {
      ++skipped;
      continue;
    }
    if (kv.second == -2) continue;
    if (kv.second < 0) {
      drop_files(id);
      continue;
    }
    const ReplayRecord& r = recs[static_cast<size_t>(kv.second)];
    ++verified;
    if (!verify(r, buf)) {  // torn: never acknowledged (prefix order), so dropping it loses nothing
      ++skipped;
      continue;
    }
    if (!cfg_.cold_dir.empty() && file_exists(data_path(id, true))) {
      // the journal holds the latest write of the id: it replaces a cold copy
      ::unlink(data_path(id, true).c_str());
      ::unlink(meta_path(id, true).c_str());
      cold_touched = true;
    }
    if (!write_file_durable(data_path(id, false), buf.data(), r.n, &err) ||
        !write_file_durable(meta_path(id, false), r.meta_be.data(), r.meta_be.size(), &err)) {
      throw std::runtime_error("journal replay: " + err);
    }
    ++replayed;
  }
  if (!sync_dir(false) || (cold_touched && !sync_dir(true))) throw std::runtime_error("journal replay: directory sync");
  journal_->note_replay(replayed, skipped, verified);
  recs.clear();
  journal_->retire_all();
}

// K1b over durable copies: blocks that are not resident (or resident blocks' journal / file
// copies) are read into a staging extent, batch by batch, laid out as in the arena (data,
// then the BE .meta image), and one launch of the scrub kernel verifies the batch. Blocks
// larger than a batch go to `rest` (CPU verify).
std::vector<std::string> ChunkStore::scrub_durable_gpu(const std::vector<std::string>& ids,
                                                       std::vector<std::string>* rest) {
  std::vector<std::string> bad;
  if (!gpu() || ids.empty()) {
    rest->insert(rest->end(), ids.begin(), ids.end());
    return bad;
  }
  HIP_OK(hipSetDevice(cfg_.device));
  // a batch is a staging extent of the arena (it may evict clean resident blocks): at most
  // an eighth of it, at most 64 MiB
  const uint64_t kBatchBytes = std::max<uint64_t>(1ull << 20, std::min<uint64_t>(64ull << 20, arena_bytes() / 8));
  size_t i = 0;
  std::vector<uint8_t> data;
  while (i < ids.size()) {
    struct Item {
      std::string id;
      uint64_t n = 0, off = 0;
      std::vector<uint8_t> bytes, meta_be;
    };
    std::vector<Item> items;
    uint64_t total = 0;
    for (; i < ids.size() && total < kBatchBytes; ++i) {
      const std::string& id = ids[i];
      bool cold = false;
      JournalRec jrec;
      std::shared_ptr<std::vector<uint8_t>> jmeta;
      uint64_t size = 0;
      {
        std::lock_guard<std::mutex> g(mu_);
        auto it = index_.find(id);
        if (it == index_.end()) continue;
        cold = it->second.cold;
        jrec = it->second.jrec;
        jmeta = it->second.jmeta;
        size = it->second.size;
        if (jrec.seg) jrec.seg->readers++;  // released by DurableSrc
      }
      const uint64_t need = align_up(std::max<uint64_t>(size, 1), 256) + align_up(num_slices(size) * 4 + 4, 256);
      if (size == 0 || need > kBatchBytes) {
        if (jrec.seg) jrec.seg->readers--;
        rest->push_back(id);
        continue;
      }
      if (!items.empty() && total + need > kBatchBytes) {  // the next batch takes it
        if (jrec.seg) jrec.seg->readers--;
        break;
      }
      DurableSrc src;
      if (!open_durable(id, cold, jrec, jmeta, &src) || src.meta.size() != num_slices(size)) {
        bad.push_back(id);  // missing, or its checksums are
        continue;
      }
      Item it;
      it.id = id;
      it.n = size;
      it.bytes.resize(size);
      if (!read_all(src.fd, it.bytes.data(), size, src.base)) {
        bad.push_back(id);
        continue;
      }
      it.meta_be.resize(src.meta.size() * 4);
      for (size_t s = 0; s < src.meta.size(); ++s) {
        const uint32_t be = __builtin_bswap32(src.meta[s]);
        std::memcpy(it.meta_be.data() + 4 * s, &be, 4);
      }
      it.off = total;
      total += need;
      items.push_back(std::move(it));
    }
    if (items.empty()) continue;
    DevExtent ext = reserve(total);
    if (ext.off < 0) {  // no room in the arena: CPU
      for (auto& it : items) rest->push_back(it.id);
      continue;
    }
    Lane* l = acquire_lane();
    std::vector<ScrubBlock> hb;
    uint64_t tiles = 0;
    for (auto& it : items) {
      uint8_t* d = ext.ptr + it.off;
      h2d_chunked(l, d, it.bytes.data(), it.n);
      uint8_t* dm = d + align_up(it.n, 256);
      HIP_OK(hipMemcpyAsync(dm, it.meta_be.data(), it.meta_be.size(), hipMemcpyHostToDevice, l->stream));
      HIP_OK(hipStreamSynchronize(l->stream));  // the pageable sources must outlive the copies
      ScrubBlock b{};
      b.data = d;
      b.meta = reinterpret_cast<const uint32_t*>(dm);
      b.s_full = it.n / kSliceBytes;
      b.tile_start = tiles;
      b.tail_len = static_cast<uint32_t>(it.n % kSliceBytes);
      b.tail_init = b.tail_len ? crc_init_term(b.tail_len) : 0;
      tiles += (b.s_full + kSlicesPerTile - 1) / kSlicesPerTile;
      hb.push_back(b);
    }
    ScrubBlock* dblocks = nullptr;
    uint32_t* dbad = nullptr;
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&dblocks), hb.size() * sizeof(ScrubBlock)));
    HIP_OK(hipMalloc(reinterpret_cast<void**>(&dbad), hb.size() * sizeof(uint32_t)));
    HIP_OK(hipMemcpyAsync(dblocks, hb.data(), hb.size() * sizeof(ScrubBlock), hipMemcpyHostToDevice, l->stream));
    HIP_OK(hipMemsetAsync(dbad, 0xFF, hb.size() * sizeof(uint32_t), l->stream));
    ScrubLaunch a{};
    a.blocks = dblocks;
    a.nblocks = static_cast<uint32_t>(hb.size());
    a.ntiles = tiles;
    a.full_init = crc_init_term(kSliceBytes);
    a.bad = dbad;
    HIP_OK(launch_scrub(a, dtables_, l->stream));
    launches_++;
    std::vector<uint32_t> hbad(hb.size());
    HIP_OK(hipMemcpyAsync(hbad.data(), dbad, hb.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
    release_lane(l);
    (void)hipFree(dblocks);
    (void)hipFree(dbad);
    release(ext);
    for (size_t j = 0; j < items.size(); ++j)
      if (hbad[j] != 0xFFFFFFFFu) bad.push_back(items[j].id);
    scrub_dev_blocks_ += items.size();
  }
  return bad;
}


// ---------------------------------------------------------------- device erasure coding
namespace {
uint64_t ec_meta_stride(uint64_t len) { return align_up(std::max<uint64_t>(num_slices(len) * 4, 4), 256); }
}  // namespace

bool ChunkStore::ec_encode(const uint8_t* host, uint64_t host_stride, uint64_t len, int k,
                           const std::vector<std::vector<uint8_t>>& parity, EcBuffers* out, std::string* err) {
  TraceRange tr("dfs.store.ec_encode");
  const int m = static_cast<int>(parity.size()), total = k + m;
  if (!gpu() || k <= 0 || m <= 0 || k > kMaxShards || m > kMaxShards || len == 0) {
    *err = "device EC needs a GPU store and 1..32 shards";
    return false;
  }
  HIP_OK(hipSetDevice(cfg_.device));
  const uint64_t stride = align_up(std::max<uint64_t>(len, 16), 256), ms = ec_meta_stride(len);
  const uint64_t tbytes = static_cast<uint64_t>(m) * k * 32;
  DevExtent ext = reserve(stride * total + ms * total + align_up(tbytes, 256));
  if (ext.off < 0) {
    *err = "HBM arena full";
    return false;
  }
  uint8_t* metas = ext.ptr + stride * total;
  auto* dtab = reinterpret_cast<uint32_t*>(metas + ms * total);
  Lane* l = acquire_lane();
  ensure_hscratch(l, tbytes + 16);
  std::vector<uint8_t> flat(static_cast<size_t>(m) * k);
  for (int r = 0; r < m; ++r)
    for (int c = 0; c < k; ++c) flat[r * k + c] = parity[r][c];
  auto* htab = reinterpret_cast<uint32_t*>(l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16);
  gf_nibble_tables(flat.data(), m, k, htab);
  HIP_OK(hipMemcpyAsync(dtab, htab, tbytes, hipMemcpyHostToDevice, l->stream));
  for (int c = 0; c < k; ++c) h2d_chunked(l, ext.ptr + c * stride, host + c * host_stride, len);
  GfLaunch a{};
  a.k = k;
  a.rows = m;
  a.len = len;
  a.tables = dtab;
  for (int c = 0; c < k; ++c) a.in[c] = ext.ptr + c * stride;
  for (int r = 0; r < m; ++r) a.out[r] = ext.ptr + (k + r) * stride;
  bool ok = launch_gf_matmul(a, l->stream) == hipSuccess;
  launches_++;
  out->crc.assign(total, 0);
  for (int i = 0; ok && i < total; ++i) {
    CrcOut co;
    ok = run_crc(l, ext.ptr + i * stride, len, reinterpret_cast<uint32_t*>(metas + i * ms), nullptr, true, 0, len,
                 &co, err);
    out->crc[i] = co.block_crc;
  }
  if (ok) {
    HIP_OK(hipEventCreateWithFlags(&out->done, hipEventDisableTiming));
    HIP_OK(hipEventRecord(out->done, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
  }
  release_lane(l);
  if (!ok) {
    release(ext);
    if (err->empty()) *err = "GPU erasure coding failed";
    return false;
  }
  out->ext = ext;
  out->len = len;
  out->stride = stride;
  out->count = total;
  return true;
}

bool ChunkStore::ec_decode(const std::vector<std::vector<uint8_t>>& rows, const std::vector<const uint8_t*>& in,
                           uint64_t len, EcBuffers* out, std::string* err) {
  TraceRange tr("dfs.store.ec_decode");
  const int k = static_cast<int>(in.size()), nr = static_cast<int>(rows.size());
  if (!gpu() || k <= 0 || nr <= 0 || k > kMaxShards || nr > kMaxShards || len == 0) {
    *err = "device EC needs a GPU store and 1..32 shards";
    return false;
  }
  HIP_OK(hipSetDevice(cfg_.device));
  const uint64_t stride = align_up(std::max<uint64_t>(len, 16), 256), ms = ec_meta_stride(len);
  const uint64_t tbytes = static_cast<uint64_t>(nr) * k * 32;
  DevExtent ext = reserve(stride * nr + ms * nr + align_up(tbytes, 256));
  if (ext.off < 0) {
    *err = "HBM arena full";
    return false;
  }
  uint8_t* metas = ext.ptr + stride * nr;
  auto* dtab = reinterpret_cast<uint32_t*>(metas + ms * nr);
  Lane* l = acquire_lane();
  ensure_hscratch(l, tbytes + 16);
  std::vector<uint8_t> flat(static_cast<size_t>(nr) * k);
  for (int r = 0; r < nr; ++r)
    for (int c = 0; c < k; ++c) flat[r * k + c] = rows[r][c];
  auto* htab = reinterpret_cast<uint32_t*>(l->hscratch + 2 * kMaxGridCrc * sizeof(uint32_t) + 16);
  gf_nibble_tables(flat.data(), nr, k, htab);
  HIP_OK(hipMemcpyAsync(dtab, htab, tbytes, hipMemcpyHostToDevice, l->stream));
  GfLaunch a{};
  a.k = k;
  a.rows = nr;
  a.len = len;
  a.tables = dtab;
  for (int c = 0; c < k; ++c) a.in[c] = in[c];
  for (int r = 0; r < nr; ++r) a.out[r] = ext.ptr + r * stride;
  bool ok = launch_gf_matmul(a, l->stream) == hipSuccess;
  launches_++;
  out->crc.assign(nr, 0);
  for (int i = 0; ok && i < nr; ++i) {
    CrcOut co;
    ok = run_crc(l, ext.ptr + i * stride, len, reinterpret_cast<uint32_t*>(metas + i * ms), nullptr, true, 0, len,
                 &co, err);
    out->crc[i] = co.block_crc;
  }
  if (ok) {
    HIP_OK(hipEventCreateWithFlags(&out->done, hipEventDisableTiming));
    HIP_OK(hipEventRecord(out->done, l->stream));
    HIP_OK(hipStreamSynchronize(l->stream));
  }
  release_lane(l);
  if (!ok) {
    release(ext);
    if (err->empty()) *err = "GPU erasure decoding failed";
    return false;
  }
  out->ext = ext;
  out->len = len;
  out->stride = stride;
  out->count = nr;
  return true;
}

void ChunkStore::ec_free(EcBuffers* b) {
  if (b->done) {
    (void)hipEventDestroy(b->done);
    b->done = nullptr;
  }
  if (b->ext.off >= 0) release(b->ext);
  b->ext = DevExtent{};
  b->count = 0;
}

bool ChunkStore::device_to_host(uint8_t* dst, const uint8_t* src_dev, uint64_t n) {
  if (!gpu()) return false;
  HIP_OK(hipSetDevice(cfg_.device));
  Lane* l = acquire_lane();
  d2h_chunked(l, dst, src_dev, n);
  HIP_OK(hipStreamSynchronize(l->stream));
  release_lane(l);
  return true;
}

WriteResult ChunkStore::commit_copy(const std::string& id, const uint8_t* src_dev, uint64_t n, uint32_t expected_crc,
                                    bool persist_now) {
  WriteResult res;
  if (!valid_block_id(id)) return bad_id(id);
  if (!gpu()) {
    res.error = "no GPU";
    return res;
  }
  HIP_OK(hipSetDevice(cfg_.device));
  DevExtent e = reserve(n);
  if (e.off < 0) {
    res.error = "HBM arena full";
    return res;
  }
  Lane* l = acquire_lane();
  if (n) HIP_OK(hipMemcpyAsync(e.ptr, src_dev, n, hipMemcpyDeviceToDevice, l->stream));
  HIP_OK(hipStreamSynchronize(l->stream));
  release_lane(l);
  return commit_device(id, e, n, expected_crc, nullptr, persist_now);
}

}  // namespace dfs
