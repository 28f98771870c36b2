// BlockJournal implementation. See journal.h for the format and the protocol.
#include "journal.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <chrono>
#include <cstring>

#include "crc32.h"

namespace dfs {

namespace {

constexpr uint32_t kSegMagic = 0x314a5344u;  // "DSJ1"
constexpr uint32_t kRecMagic = 0x524a5344u;  // "DSJR"
constexpr uint64_t kPage = 4096;
constexpr uint64_t kHdr = 512;

struct SegHdr {
  uint32_t magic;
  uint32_t version;
  uint64_t seq;
  uint64_t cap;
  uint32_t hdr_crc;
  uint32_t pad;
};

struct RecHdr {
  uint32_t magic;
  uint32_t type;
  uint64_t seq;
  uint64_t off;
  uint64_t rec_len;
  uint64_t hdr_bytes;
  uint64_t n;
  uint32_t crc;
  uint32_t nslices;
  uint32_t meta_crc;
  uint32_t id_len;
  char id[256];
  uint8_t pad[kHdr - 320 - 4];
  uint32_t hdr_crc;
};
static_assert(sizeof(RecHdr) == kHdr, "record header is 512 bytes");

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

uint64_t now_ns() {
  return static_cast<uint64_t>(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
          .count());
}

bool pwrite_all(int fd, const uint8_t* p, uint64_t n, uint64_t off) {
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

bool pread_all(int fd, uint8_t* p, uint64_t n, uint64_t off) {
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

void fsync_dir(const std::string& dir) {
  int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
  if (fd >= 0) {
    (void)::fsync(fd);
    ::close(fd);
  }
}

std::string parent_of(const std::string& p) {
  auto s = p.find_last_of('/');
  return s == std::string::npos || s == 0 ? std::string("/") : p.substr(0, s);
}

}  // namespace

JournalSeg::~JournalSeg() {
  if (fd >= 0) ::close(fd);
  if (dfd >= 0) ::close(dfd);
}

BlockJournal::BlockJournal(JournalConfig cfg) : cfg_(std::move(cfg)) {
  cfg_.seg_bytes = std::max<uint64_t>(align_up(cfg_.seg_bytes, kPage), 4 << 20);
  cfg_.max_segs = std::max(2, cfg_.max_segs);
  if (::mkdir(cfg_.dir.c_str(), 0755) == 0) fsync_dir(parent_of(cfg_.dir));
}

BlockJournal::~BlockJournal() {
  {
    std::lock_guard<std::mutex> g(mu_);
    prep_stop_ = true;
  }
  cv_.notify_all();
  if (preparer_.joinable()) preparer_.join();
}

// Creates every segment file up to the cap (fallocate: metadata only), then, with zero_fill,
// writes the free ones out while the writers are idle (8 MiB at a time, re-checking between
// chunks), so first-cycle appends are overwrites of written extents.
void BlockJournal::prepare_loop() {
  static const std::vector<uint8_t> zeros(8 << 20, 0);
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    if (prep_stop_) return;
    if (static_cast<int>(segs_.size()) + preparing_ < cfg_.max_segs) {
      ++preparing_;
      const std::string path = cfg_.dir + "/seg-" + std::to_string(next_file_++) + ".log";
      lk.unlock();
      errno = 0;
      SegRef s = open_seg(path, true);
      bool ok = s != nullptr;
      if (ok) {
        ok = !cfg_.sync || ::fdatasync(s->fd) == 0;
        fsync_dir(cfg_.dir);  // the name survives a crash before its first record is acked
      }
      const int e = errno;
      if (!ok) {
        s.reset();
        ::unlink(path.c_str());
      }
      lk.lock();
      --preparing_;
      if (ok) {
        segs_.push_back(s);
        free_.push_back(s);
        st_.prepared++;
      } else {
        st_.prepare_errors++;
        st_.last_error = "segment " + path + ": " + std::strerror(e ? e : EIO);
        std::fprintf(stderr, "[journal] preparing %s failed: %s (%s)\n", path.c_str(), std::strerror(e ? e : EIO),
                     describe_locked().c_str());
        if ((e == ENOSPC || e == EDQUOT) && !segs_.empty()) {
          // no room for another segment: run with the ones there are (a writer waits for the
          // materializer to recycle one instead of failing)
          cfg_.max_segs = std::max<int>(2, static_cast<int>(segs_.size()));
        } else {
          // transient (or nothing to fall back on): try again shortly
          cv_.wait_for(lk, std::chrono::milliseconds(500), [&] { return prep_stop_; });
        }
      }
      cv_.notify_all();
      continue;
    }
    SegRef t;
    if (cfg_.zero_fill)
      for (auto& f : free_)
        if (!f->filled) {
          t = f;
          break;
        }
    if (!t) {
      cv_.wait_for(lk, std::chrono::milliseconds(200));
      continue;
    }
    const uint64_t idle_ns = static_cast<uint64_t>(std::max(1, cfg_.idle_fill_ms)) * 1000000ull;
    const uint64_t since = now_ns() - last_append_ns_;
    if (last_append_ns_ && since < idle_ns) {  // writers active: wait until they pause
      cv_.wait_for(lk, std::chrono::nanoseconds(idle_ns - since + 1000000));
      continue;
    }
    t->filling = true;
    const uint64_t off = t->fill_off, len = std::min<uint64_t>(zeros.size(), t->cap - off);
    lk.unlock();
    bool ok = pwrite_all(t->fd, zeros.data(), len, off);
    const bool last = ok && off + len >= t->cap;
    if (last) {
      ok = !cfg_.sync || ::fdatasync(t->fd) == 0;
      (void)::posix_fadvise(t->fd, 0, 0, POSIX_FADV_DONTNEED);
    }
    lk.lock();
    t->filling = false;
    if (ok) {
      t->fill_off = off + len;
      st_.fill_bytes += len;
      if (last) {
        t->filled = true;
        st_.filled++;
      }
    } else {
      t->filled = true;  // give up on this one (appends still work on unwritten extents)
    }
    cv_.notify_all();
  }
}

std::string BlockJournal::describe_locked() const {
  char buf[512];
  int n = std::snprintf(buf, sizeof(buf), "segments %zu of max %d, in use %zu, free %zu, preparing %d",
                        segs_.size(), cfg_.max_segs, order_.size(), free_.size(), preparing_);
  if (!order_.empty() && n > 0 && n < static_cast<int>(sizeof(buf))) {
    const JournalSeg* f = order_.front().get();
    std::snprintf(buf + n, sizeof(buf) - n,
                  "; oldest seq %llu: live %llu, sealed %d, completed %llu of %llu, readers %d",
                  static_cast<unsigned long long>(f->seq), static_cast<unsigned long long>(f->live),
                  f->sealed ? 1 : 0, static_cast<unsigned long long>(f->done_upto),
                  static_cast<unsigned long long>(f->tail), f->readers.load());
  }
  return buf;
}

uint64_t BlockJournal::hdr_bytes_for(uint64_t nslices) { return align_up(kHdr + 4 * nslices, kPage); }

uint64_t BlockJournal::rec_bytes_for(uint64_t n, uint64_t nslices) {
  return hdr_bytes_for(nslices) + align_up(n, kPage);
}

bool BlockJournal::fits(uint64_t n, uint64_t nslices) const {
  return rec_bytes_for(n, nslices) + kPage <= cfg_.seg_bytes;
}

SegRef BlockJournal::open_seg(const std::string& path, bool create) {
  auto s = std::make_shared<JournalSeg>();
  s->path = path;
  s->fd = ::open(path.c_str(), O_RDWR | O_CLOEXEC | (create ? O_CREAT : 0), 0644);
  if (s->fd < 0) return nullptr;
  struct stat st;
  if (::fstat(s->fd, &st) != 0) return nullptr;
  if (create || static_cast<uint64_t>(st.st_size) < cfg_.seg_bytes) {
    // reserve the extent once; later appends are overwrites inside the file
    if (::fallocate(s->fd, 0, 0, static_cast<off_t>(cfg_.seg_bytes)) != 0 &&
        ::ftruncate(s->fd, static_cast<off_t>(cfg_.seg_bytes)) != 0)
      return nullptr;
    s->cap = cfg_.seg_bytes;
  } else {
    s->cap = static_cast<uint64_t>(st.st_size);
  }
  if (cfg_.direct) s->dfd = ::open(path.c_str(), O_RDWR | O_CLOEXEC | O_DIRECT);
  return s;
}

bool BlockJournal::write_seg_header(JournalSeg* s, uint64_t seq) {
  alignas(4096) static thread_local uint8_t page[kPage];
  std::memset(page, 0, kPage);
  if (seq) {
    SegHdr h{};
    h.magic = kSegMagic;
    h.version = 1;
    h.seq = seq;
    h.cap = s->cap;
    h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(SegHdr, hdr_crc));
    std::memcpy(page, &h, sizeof(h));
  }
  return pwrite_all(s->fd, page, kPage, 0);
}

std::vector<ReplayRecord> BlockJournal::recover() {
  std::vector<ReplayRecord> out;
  std::vector<std::pair<std::string, int>> files;
  if (DIR* d = ::opendir(cfg_.dir.c_str())) {
    while (dirent* e = ::readdir(d)) {
      int idx = -1;
      if (std::sscanf(e->d_name, "seg-%d.log", &idx) == 1 && idx >= 0) files.emplace_back(e->d_name, idx);
    }
    ::closedir(d);
  }
  std::vector<SegRef> live;
  for (auto& f : files) {
    SegRef s = open_seg(cfg_.dir + "/" + f.first, false);
    if (!s) continue;
    next_file_ = std::max(next_file_, f.second + 1);
    segs_.push_back(s);
    SegHdr h{};
    if (pread_all(s->fd, reinterpret_cast<uint8_t*>(&h), sizeof(h), 0) && h.magic == kSegMagic && h.seq > 0 &&
        h.hdr_crc == crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(SegHdr, hdr_crc))) {
      s->seq = h.seq;
      next_seq_ = std::max(next_seq_, h.seq + 1);
      live.push_back(s);
    } else {
      free_.push_back(s);
    }
  }
  std::sort(live.begin(), live.end(), [](const SegRef& a, const SegRef& b) { return a->seq < b->seq; });
  std::vector<uint8_t> hdr_area;
  for (auto& s : live) {
    uint64_t off = kPage;
    while (off + kPage <= s->cap) {
      RecHdr h;
      if (!pread_all(s->fd, reinterpret_cast<uint8_t*>(&h), kHdr, off)) break;
      if (h.magic != kRecMagic || h.hdr_crc != crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc)))
        break;
      if (h.seq != s->seq || h.off != off || h.rec_len < kPage || h.rec_len % kPage || off + h.rec_len > s->cap)
        break;
      if (h.type == kJrBlock || h.type == kJrTomb) {
        ReplayRecord r;
        r.type = h.type;
        r.id.assign(h.id, std::min<uint32_t>(h.id_len, sizeof(h.id)));
        r.seg = s;
        if (h.type == kJrBlock) {
          if (h.hdr_bytes != hdr_bytes_for(h.nslices) || h.nslices != num_slices(h.n) ||
              h.hdr_bytes + align_up(h.n, kPage) != h.rec_len)
            break;
          r.meta_be.resize(4 * h.nslices);
          if (h.nslices && !pread_all(s->fd, r.meta_be.data(), r.meta_be.size(), off + kHdr)) break;
          if (crc32(r.meta_be.data(), r.meta_be.size()) != h.meta_crc) break;
          r.n = h.n;
          r.crc = h.crc;
          r.data_off = off + h.hdr_bytes;
        }
        out.push_back(std::move(r));
      }
      off += h.rec_len;
    }
    s->tail = s->done_upto = s->durable_upto = off;
    s->sealed = true;
    order_.push_back(s);
  }
  st_.segs_total = segs_.size();
  preparer_ = std::thread([this] { prepare_loop(); });  // spares get ready while the caller replays
  return out;
}

void BlockJournal::note_replay(uint64_t replayed, uint64_t skipped) {
  std::lock_guard<std::mutex> g(mu_);
  st_.replayed += replayed;
  st_.replay_skipped += skipped;
}

void BlockJournal::retire_all() {
  std::vector<SegRef> segs;
  {
    std::lock_guard<std::mutex> g(mu_);
    segs.swap(order_);
  }
  for (auto& s : segs) {
    (void)write_seg_header(s.get(), 0);
    if (cfg_.sync) (void)::fdatasync(s->fd);
    (void)::posix_fadvise(s->fd, 0, 0, POSIX_FADV_DONTNEED);
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& s : segs) {
    s->seq = 0;
    s->tail = s->done_upto = s->durable_upto = s->syncing_upto = s->live = 0;
    s->done_out.clear();
    s->sealed = false;
    free_.push_back(s);
    ++st_.segs_retired;
  }
  cv_.notify_all();
}

// Caller holds the lock. Seals nothing; takes a free segment (or creates one while under
// the cap) and makes it the active one. Waits for the materializer when all are in use.
SegRef BlockJournal::activate_locked(std::unique_lock<std::mutex>& lk, std::string* err) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(cfg_.full_timeout_s);
  auto next_report = std::chrono::steady_clock::now() + std::chrono::seconds(5);
  for (;;) {
    if (failed_) {
      *err = "journal failed";
      return nullptr;
    }
    if (!preparer_.joinable()) preparer_ = std::thread([this] { prepare_loop(); });
    // another writer activated a segment while this one waited: append there instead (two
    // activations would leave the first one unsealed behind the second, and retirement,
    // which goes oldest first, would stop at it for good)
    if (!order_.empty() && !order_.back()->sealed) return order_.back();
    SegRef s;
    {
      // a written-out segment first; never one the preparer is writing zeros into right now
      int pick = -1;
      for (int i = static_cast<int>(free_.size()) - 1; i >= 0; --i) {
        if (free_[i]->filling) continue;
        if (pick < 0 || (free_[i]->filled && !free_[pick]->filled)) pick = i;
      }
      if (pick >= 0) {
        s = free_[pick];
        free_.erase(free_.begin() + pick);
        cv_.notify_all();  // the preparer may create / fill another
      }
    }
    if (s) {
      const uint64_t seq = next_seq_++;
      // no flush of its own: the first commit's fdatasync of this segment covers the header
      if (!write_seg_header(s.get(), seq)) {
        *err = std::string("journal header: ") + std::strerror(errno);
        free_.push_back(s);
        return nullptr;
      }
      s->seq = seq;
      s->tail = s->done_upto = s->durable_upto = s->syncing_upto = kPage;
      s->done_out.clear();
      s->live = 0;
      s->sealed = false;
      order_.push_back(s);
      return s;
    }
    const bool full = static_cast<int>(segs_.size()) + preparing_ >= cfg_.max_segs &&
                      std::none_of(free_.begin(), free_.end(), [](const SegRef& f) { return f->filling; });
    if (full) ++st_.full_waits;  // not just waiting for the preparer
    if (std::chrono::steady_clock::now() >= next_report) {
      std::fprintf(stderr, "[journal] writer waiting for a free segment (%s)\n", describe_locked().c_str());
      next_report += std::chrono::seconds(10);
    }
    if (cv_.wait_until(lk, std::min(deadline, next_report)) == std::cv_status::timeout &&
        std::chrono::steady_clock::now() >= deadline) {
      *err = std::string(full ? "journal full (materializer behind): " : "no journal segment ready: ") +
             describe_locked() + (st_.last_error.empty() ? "" : "; last error: " + st_.last_error);
      return nullptr;
    }
  }
}

bool BlockJournal::reserve(uint64_t n, uint64_t nslices, JournalRec* r, std::string* err) {
  const uint64_t len = rec_bytes_for(n, nslices);
  if (len + kPage > cfg_.seg_bytes) {
    *err = "block larger than a journal segment";
    return false;
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (failed_) {
    *err = "journal failed";
    return false;
  }
  SegRef s;
  for (;;) {
    s = order_.empty() || order_.back()->sealed ? nullptr : order_.back();
    if (s && s->tail + len <= s->cap) break;
    if (s) {
      s->sealed = true;
      cv_.notify_all();
    }
    // activate_locked may wait (and drop the lock): whatever it returns is checked again
    if (!activate_locked(lk, err)) return false;
  }
  r->seg = s;
  r->off = s->tail;
  r->hdr_bytes = hdr_bytes_for(nslices);
  r->end = s->tail + len;
  s->tail += len;
  s->live++;
  last_append_ns_ = now_ns();
  return true;
}

bool BlockJournal::write(const JournalRec& r, uint64_t at, const uint8_t* p, uint64_t len) {
  const uint64_t off = r.data_off() + at;
  const JournalSeg* s = r.seg.get();
  if (s->dfd >= 0 && off % kPage == 0 && reinterpret_cast<uintptr_t>(p) % kPage == 0) {
    const uint64_t full = len & ~(kPage - 1);
    if (full && !pwrite_all(s->dfd, p, full, off)) return false;
    return full == len || pwrite_all(s->fd, p + full, len - full, off + full);
  }
  return pwrite_all(s->fd, p, len, off);
}

bool BlockJournal::finish(const JournalRec& r, const std::string& id, uint64_t n, uint32_t crc,
                          const uint8_t* meta_be, uint64_t nslices) {
  std::vector<uint8_t> area(kHdr + 4 * nslices);
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = kJrBlock;
  h.seq = r.seg->seq;
  h.off = r.off;
  h.rec_len = r.end - r.off;
  h.hdr_bytes = r.hdr_bytes;
  h.n = n;
  h.crc = crc;
  h.nslices = static_cast<uint32_t>(nslices);
  h.meta_crc = crc32(meta_be, 4 * nslices);
  h.id_len = static_cast<uint32_t>(std::min<size_t>(id.size(), sizeof(h.id)));
  std::memcpy(h.id, id.data(), h.id_len);
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  std::memcpy(area.data(), &h, kHdr);
  if (nslices) std::memcpy(area.data() + kHdr, meta_be, 4 * nslices);
  bool ok = pwrite_all(r.seg->fd, area.data(), area.size(), r.off);
  std::lock_guard<std::mutex> g(mu_);
  if (!ok) failed_ = true;  // the prefix cannot advance past a record that is not on disk
  complete_locked(r.seg.get(), r.off, r.end);
  st_.records++;
  st_.bytes += n;
  cv_.notify_all();
  return ok;
}

void BlockJournal::abandon(const JournalRec& r) {
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = kJrPad;
  h.seq = r.seg->seq;
  h.off = r.off;
  h.rec_len = r.end - r.off;
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  bool ok = pwrite_all(r.seg->fd, reinterpret_cast<const uint8_t*>(&h), kHdr, r.off);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!ok) failed_ = true;
    complete_locked(r.seg.get(), r.off, r.end);
    st_.pads++;
  }
  materialized(r.seg, 1);
}

void BlockJournal::complete_locked(JournalSeg* s, uint64_t off, uint64_t end) {
  if (off != s->done_upto) {
    s->done_out[off] = end;
    return;
  }
  s->done_upto = end;
  for (auto it = s->done_out.begin(); it != s->done_out.end() && it->first == s->done_upto;) {
    s->done_upto = it->second;
    it = s->done_out.erase(it);
  }
}

bool BlockJournal::commit(const JournalRec& r) {
  const uint64_t t_in = now_ns();
  std::unique_lock<std::mutex> lk(mu_);
  st_.commits++;
  struct Acc {  // the caller's wait, whichever way it returns (lock held at every return)
    JournalStats& st;
    uint64_t t0;
    ~Acc() { st.commit_ns += now_ns() - t0; }
  } acc{st_, t_in};
  JournalSeg* seg = r.seg.get();
  const int max_syncers = std::max(1, cfg_.syncers);
  for (;;) {
    if (failed_) return false;
    if (seg->durable_upto >= r.end) return true;
    // wait while an earlier record of the segment is still being written, while a running
    // round already covers this record, or while every flush slot is busy
    if (seg->done_upto < r.end || seg->syncing_upto >= r.end || syncers_ >= max_syncers) {
      cv_.wait(lk);
      continue;
    }
    ++syncers_;
    std::vector<std::pair<SegRef, uint64_t>> targets;
    for (auto& s : order_)
      if (s->done_upto > std::max(s->durable_upto, s->syncing_upto)) {
        targets.emplace_back(s, s->done_upto);
        s->syncing_upto = s->done_upto;
      }
    lk.unlock();
    bool ok = true;
    if (cfg_.sync_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(cfg_.sync_delay_us));
    const uint64_t t_sync = now_ns();
    if (cfg_.sync)
      for (auto& t : targets) ok = ::fdatasync(t.first->fd) == 0 && ok;
    const uint64_t d_sync = now_ns() - t_sync;
    lk.lock();
    --syncers_;
    st_.sync_rounds++;
    st_.sync_ns += d_sync;
    // a round that finishes flushed everything dirty when it started, i.e. every record
    // completed before its snapshot, whatever rounds started earlier still run
    if (ok)
      for (auto& t : targets) t.first->durable_upto = std::max(t.first->durable_upto, t.second);
    else
      failed_ = true;  // after a failed flush the page state is unknown: refuse further acks
    cv_.notify_all();
  }
}

void BlockJournal::tombstone(const std::string& id) {
  JournalRec r;
  std::string err;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (failed_) return;
    SegRef s;
    for (;;) {
      s = order_.empty() || order_.back()->sealed ? nullptr : order_.back();
      if (s && s->tail + kPage <= s->cap) break;
      if (s) {
        s->sealed = true;
        cv_.notify_all();
      }
      if (!activate_locked(lk, &err)) return;
    }
    r.seg = s;
    r.off = s->tail;
    r.end = s->tail + kPage;
    s->tail += kPage;
  }
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = kJrTomb;
  h.seq = r.seg->seq;
  h.off = r.off;
  h.rec_len = kPage;
  h.id_len = static_cast<uint32_t>(std::min<size_t>(id.size(), sizeof(h.id)));
  std::memcpy(h.id, id.data(), h.id_len);
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  bool ok = pwrite_all(r.seg->fd, reinterpret_cast<const uint8_t*>(&h), kHdr, r.off);
  std::lock_guard<std::mutex> g(mu_);
  if (!ok) failed_ = true;
  complete_locked(r.seg.get(), r.off, r.end);
  st_.tombstones++;
  cv_.notify_all();
}

void BlockJournal::materialized(const SegRef& s, uint64_t count) {
  {
    std::lock_guard<std::mutex> g(mu_);
    s->live -= std::min(s->live, count);
  }
  retire_ready();
}

void BlockJournal::retire_ready() {
  std::vector<SegRef> retire;
  {
    std::lock_guard<std::mutex> g(mu_);
    // oldest first: a segment retires only after every older one did, so a tombstone is
    // never dropped while a record it cancels could still be replayed; a segment somebody
    // is still reading from waits for the next call
    while (!order_.empty()) {
      SegRef f = order_.front();
      if (!f->sealed && f != order_.back()) f->sealed = true;  // only the newest segment takes appends
      if (!f->sealed || f->live || f->done_upto < f->tail || f->readers.load() > 0) break;
      retire.push_back(f);
      order_.erase(order_.begin());
    }
  }
  if (retire.empty()) return;
  // the invalidated header must be durable before the segment is reused: otherwise a crash
  // could replay its old records over newer materialized versions
  for (auto& f : retire) {
    (void)write_seg_header(f.get(), 0);
    if (cfg_.sync) (void)::fdatasync(f->fd);
    (void)::posix_fadvise(f->fd, 0, 0, POSIX_FADV_DONTNEED);
  }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& f : retire) {
    if (f->tail + (8ull << 20) >= f->cap) f->filled = true;  // appends wrote (almost) all of it
    f->seq = 0;
    f->tail = f->done_upto = f->durable_upto = f->syncing_upto = 0;
    f->done_out.clear();
    f->sealed = false;
    free_.push_back(f);
    ++st_.segs_retired;
  }
  cv_.notify_all();
}

double BlockJournal::pressure() {
  std::lock_guard<std::mutex> g(mu_);
  const double cap = static_cast<double>(cfg_.max_segs);
  return std::min(1.0, static_cast<double>(order_.size()) / cap);
}

uint64_t BlockJournal::last_append_ns() {
  std::lock_guard<std::mutex> g(mu_);
  return last_append_ns_;
}

JournalStats BlockJournal::stats() {
  std::lock_guard<std::mutex> g(mu_);
  JournalStats s = st_;
  s.segs_total = segs_.size();
  s.segs_free = free_.size();
  s.failed = failed_;
  return s;
}

}  // namespace dfs
