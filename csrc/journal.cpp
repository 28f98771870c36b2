// BlockJournal implementation. See journal.h for the format and the protocol.
#include "journal.h"
#include "thread_name.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstddef>
#include <cstdio>
#include <cstring>

#include "crc32.h"

namespace dfs {

namespace {

constexpr uint32_t kSegMagic = 0x324a5344u;  // "DSJ2" (striped segments)
constexpr uint32_t kRecMagic = 0x524a5344u;  // "DSJR"
constexpr uint64_t kPage = 4096;
constexpr uint64_t kHdr = 512;
constexpr uint32_t kFlagSealed = 1, kFlagRetired = 2;
// the tail of every part that block records leave free: room for 16 tombstone / supersede
// markers per part when no free segment is left (a delete must not wait for journal space
// that only deletes can free)
constexpr uint64_t kMarkerReserve = 16 * kPage;

// version 3; version 2 (round 4: no flags, no LSN mark, retirement zeroed the page) still reads
struct PartHdr {
  uint32_t magic;
  uint32_t version;
  uint64_t seq;
  uint64_t cap;
  uint32_t part;
  uint32_t nparts;
  uint32_t flags;
  uint32_t pad0;
  uint64_t lsn_hw;  // every LSN in the journal is below this when the header is written
  uint32_t hdr_crc;
  uint32_t pad;
};
struct PartHdrV2 {
  uint32_t magic;
  uint32_t version;
  uint64_t seq;
  uint64_t cap;
  uint32_t part;
  uint32_t nparts;
  uint32_t hdr_crc;
  uint32_t pad;
};

struct RecHdr {
  uint32_t magic;
  uint32_t type;
  uint64_t seq;   // segment sequence number
  uint64_t off;   // record offset in its part
  uint64_t rec_len;
  uint64_t hdr_bytes;
  uint64_t n;
  uint32_t crc;
  uint32_t nslices;
  uint32_t meta_crc;
  uint32_t id_len;
  char id[256];
  uint64_t lsn;   // journal-wide order (replay order across parts)
  uint32_t part;
  uint32_t pad0;
  uint8_t pad[kHdr - 336 - 4];
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

// A part header as read back: valid, its segment sequence number, flags and LSN mark.
struct HdrView {
  bool ok = false;
  uint64_t seq = 0, lsn_hw = 0;
  uint32_t flags = 0;
};

HdrView read_part_header(int fd, size_t k, size_t nparts) {
  HdrView v;
  uint8_t raw[sizeof(PartHdr)];
  if (!pread_all(fd, raw, sizeof(raw), 0)) return v;
  uint32_t magic, version;
  std::memcpy(&magic, raw, 4);
  std::memcpy(&version, raw + 4, 4);
  if (magic != kSegMagic) return v;
  if (version == 3) {
    PartHdr h;
    std::memcpy(&h, raw, sizeof(h));
    if (h.hdr_crc != crc32(raw, offsetof(PartHdr, hdr_crc)) || h.part != k || h.nparts != nparts || h.seq == 0)
      return v;
    v.ok = true;
    v.seq = h.seq;
    v.flags = h.flags;
    v.lsn_hw = h.lsn_hw;
  } else if (version == 2) {
    PartHdrV2 h;
    std::memcpy(&h, raw, sizeof(h));
    if (h.hdr_crc != crc32(raw, offsetof(PartHdrV2, hdr_crc)) || h.part != k || h.nparts != nparts || h.seq == 0)
      return v;
    v.ok = true;
    v.seq = h.seq;
  }
  return v;
}

}  // namespace

JournalPart::~JournalPart() {
  if (fd >= 0) ::close(fd);
  if (dfd >= 0) ::close(dfd);
}

bool JournalSeg::complete() const {
  for (auto& p : parts)
    if (p->done_upto < p->tail) return false;
  return true;
}

bool JournalSeg::filled() const {
  for (auto& p : parts)
    if (!p->filled) return false;
  return true;
}

bool JournalSeg::filling() const {
  for (auto& p : parts)
    if (p->filling) return true;
  return false;
}

uint64_t JournalSeg::capacity() const {
  uint64_t c = 0;
  for (auto& p : parts) c += p->cap;
  return c;
}

BlockJournal::BlockJournal(JournalConfig cfg) : cfg_(std::move(cfg)) {
  cfg_.parts = std::max(1, std::min(cfg_.parts, 64));
  cfg_.seg_bytes = std::max<uint64_t>(align_up(cfg_.seg_bytes, kPage), 4 << 20);
  part_bytes_ = std::max<uint64_t>(cfg_.seg_bytes / cfg_.parts / kPage * kPage, 1 << 20);
  if (cfg_.grow) {
    if (cfg_.max_segs > 0) cfg_.max_segs = std::max(2, cfg_.max_segs);
    cfg_.spares = std::max(1, cfg_.spares);
  } else {
    cfg_.max_segs = std::max(2, cfg_.max_segs);
  }
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

bool BlockJournal::room_for_segment() {
  struct statvfs sv;
  if (::statvfs(cfg_.dir.c_str(), &sv) != 0) return true;  // unknown: let the create itself fail
  const uint64_t avail = static_cast<uint64_t>(sv.f_bavail) * sv.f_frsize;
  return avail >= capacity_bytes() + cfg_.reserve_bytes;
}

// Marks the oldest sealed, complete, unmarked segment: its part headers get the `sealed` flag
// and each part is flushed (which also flushes any record bytes a writer has not committed,
// e.g. padding). Called with the lock held; drops it around the I/O.
bool BlockJournal::mark_one(std::unique_lock<std::mutex>& lk) {
  SegRef s;
  for (auto& f : order_)
    if (f->sealed && !f->marked && !f->marking && f->complete()) {
      s = f;
      break;
    }
  if (!s) return false;
  s->marking = true;
  const uint64_t seq = s->seq, lsn = next_lsn_;
  // complete() only says every record's bytes were written, not that they were flushed: a
  // record whose commit is still running (or that nobody commits, e.g. padding) may sit in
  // the page cache, and writeback could persist the sealed header before it — replay would
  // then trust a torn record. So the parts not yet durable up to their tail are flushed
  // first, and only then is the sealed header written and flushed.
  std::vector<uint64_t> flush_to(s->parts.size(), 0);
  for (size_t k = 0; k < s->parts.size(); ++k) {
    const JournalPart* p = s->parts[k].get();
    if (p->durable_upto < p->tail || p->syncers > 0) flush_to[k] = p->tail;
  }
  lk.unlock();
  bool ok = true;
  for (size_t k = 0; k < s->parts.size(); ++k)
    if (flush_to[k] && cfg_.sync) ok = ok && ::fdatasync(s->parts[k]->fd) == 0;
  if (ok) {
    lk.lock();
    for (size_t k = 0; k < s->parts.size(); ++k)
      if (flush_to[k]) s->parts[k]->durable_upto = std::max(s->parts[k]->durable_upto, flush_to[k]);
    lk.unlock();
  }
  for (size_t k = 0; ok && k < s->parts.size(); ++k) {
    JournalPart* p = s->parts[k].get();
    ok = ok && write_part_header(p, seq, static_cast<int>(k), static_cast<int>(s->parts.size()), kFlagSealed, lsn);
    ok = ok && (!cfg_.sync || ::fdatasync(p->fd) == 0);
  }
  lk.lock();
  s->marking = false;
  st_.mark_preflushes += std::count_if(flush_to.begin(), flush_to.end(), [](uint64_t v) { return v != 0; });
  if (ok) {
    s->marked = true;
    st_.segs_marked++;
  }
  cv_.notify_all();
  return ok;
}

void BlockJournal::mark_sealed_now() {
  std::unique_lock<std::mutex> lk(mu_);
  if (!order_.empty() && !order_.back()->sealed && order_.back()->complete()) order_.back()->sealed = true;
  while (mark_one(lk)) {
  }
}

// Creates segments (fallocate: metadata only) — all up to max_segs, or in grow mode enough
// to keep `spares` free ones ready while the volume has room — and, in the writers' idle
// windows, flushes the `sealed` headers of finished segments and (zero_fill) writes the free
// parts out once (8 MiB at a time, re-checking between chunks), so first-cycle appends are
// overwrites of written extents.
void BlockJournal::prepare_loop() {
  name_thread("jr-prepare");
  static const std::vector<uint8_t> zeros(8 << 20, 0);
  std::unique_lock<std::mutex> lk(mu_);
  auto grow_check_ns = 0ull;
  bool deferring = false;
  const uint64_t idle_ns = static_cast<uint64_t>(std::max(1, cfg_.idle_fill_ms)) * 1000000ull;
  for (;;) {
    if (prep_stop_) return;
    const int have = static_cast<int>(segs_.size()) + preparing_;
    const int ready = static_cast<int>(free_.size()) + preparing_;
    bool want = cfg_.grow ? ready < cfg_.spares && (cfg_.max_segs <= 0 || have < cfg_.max_segs)
                          : have < cfg_.max_segs;
    if (want && cfg_.grow && ready >= cfg_.spares_low && last_append_ns_ && now_ns() - last_append_ns_ < idle_ns) {
      // enough spares for now and the writers are active: top up in their next idle window,
      // so no segment creation (and its flushes) shares the volume with acked writes
      if (!deferring) st_.grow_deferred++;
      deferring = true;
      want = false;
    } else if (want) {
      deferring = false;
    }
    if (want && cfg_.grow) {
      const uint64_t t = now_ns();
      if (grow_blocked_ && t < grow_check_ns) {
        want = false;
      } else {
        lk.unlock();
        const bool room = room_for_segment();
        lk.lock();
        grow_blocked_ = !room;
        grow_check_ns = t + 1000000000ull;
        want = room;
        if (!room) cv_.notify_all();  // writers waiting for a segment learn the journal is full
      }
    }
    if (want) {
      ++preparing_;
      const int index = next_file_++;
      lk.unlock();
      errno = 0;
      SegRef s = open_seg(index, true);
      bool ok = s != nullptr;
      if (ok) {
        for (auto& p : s->parts) ok = ok && (!cfg_.sync || ::fdatasync(p->fd) == 0);
        fsync_dir(cfg_.dir);  // the names survive a crash before the first record is acked
      }
      const int e = errno;
      if (!ok && s) {
        for (auto& p : s->parts) ::unlink(p->path.c_str());
        s.reset();
      }
      lk.lock();
      --preparing_;
      if (ok) {
        segs_.push_back(s);
        free_.push_back(s);
        st_.prepared++;
      } else {
        st_.prepare_errors++;
        st_.last_error = "segment " + std::to_string(index) + ": " + std::strerror(e ? e : EIO);
        std::fprintf(stderr, "[journal] preparing segment %d failed: %s (%s)\n", index, std::strerror(e ? e : EIO),
                     describe_locked().c_str());
        if ((e == ENOSPC || e == EDQUOT) && !segs_.empty()) {
          // no room for another segment: run with the ones there are (a writer waits for the
          // exporter / compaction to free one instead of failing)
          if (cfg_.grow) {
            grow_blocked_ = true;
            grow_check_ns = now_ns() + 1000000000ull;
          } else {
            cfg_.max_segs = std::max<int>(2, static_cast<int>(segs_.size()));
          }
        } else {
          // transient (or nothing to fall back on): try again shortly
          cv_.wait_for(lk, std::chrono::milliseconds(500), [&] { return prep_stop_; });
        }
      }
      cv_.notify_all();
      continue;
    }
    const uint64_t since = now_ns() - last_append_ns_;
    const bool idle = !last_append_ns_ || since >= idle_ns;
    if (idle && mark_one(lk)) continue;
    JournalPart* t = nullptr;
    if (cfg_.zero_fill)
      for (auto& f : free_) {
        for (auto& p : f->parts)
          if (!p->filled) {
            t = p.get();
            break;
          }
        if (t) break;
      }
    const bool sealed_pending = std::any_of(order_.begin(), order_.end(), [](const SegRef& f) {
      return f->sealed && !f->marked && !f->marking && f->complete();
    });
    if (!t && !sealed_pending) {
      // (a deferred top-up is re-checked once the writers have been idle for idle_ns)
      cv_.wait_for(lk, deferring ? std::chrono::nanoseconds(idle_ns + 1000000) : std::chrono::nanoseconds(200000000));
      continue;
    }
    if (!idle) {  // writers active: wait until they pause
      cv_.wait_for(lk, std::chrono::nanoseconds(idle_ns - since + 1000000));
      continue;
    }
    if (!t) {
      cv_.wait_for(lk, std::chrono::milliseconds(50));
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
  int n = std::snprintf(buf, sizeof(buf), "segments %zu of max %d%s (%d parts), in use %zu, free %zu, preparing %d",
                        segs_.size(), cfg_.max_segs, cfg_.grow ? (grow_blocked_ ? " grow, volume at reserve" : " grow")
                                                                : "",
                        cfg_.parts, order_.size(), free_.size(), preparing_);
  if (!order_.empty() && n > 0 && n < static_cast<int>(sizeof(buf))) {
    const JournalSeg* f = order_.front().get();
    std::snprintf(buf + n, sizeof(buf) - n, "; oldest seq %llu: live %llu, sealed %d, complete %d, readers %d",
                  static_cast<unsigned long long>(f->seq), static_cast<unsigned long long>(f->live),
                  f->sealed ? 1 : 0, f->complete() ? 1 : 0, f->readers.load());
  }
  return buf;
}

uint64_t BlockJournal::hdr_bytes_for(uint64_t nslices) { return align_up(kHdr + 4 * nslices, kPage); }

uint64_t BlockJournal::rec_bytes_for(uint64_t n, uint64_t nslices) {
  return hdr_bytes_for(nslices) + align_up(n, kPage);
}

bool BlockJournal::fits(uint64_t n, uint64_t nslices) const {
  return rec_bytes_for(n, nslices) + kPage + kMarkerReserve <= part_bytes_;
}

SegRef BlockJournal::open_seg(int index, bool create) {
  auto s = std::make_shared<JournalSeg>();
  s->index = index;
  for (int k = 0; k < cfg_.parts; ++k) {
    auto p = std::make_unique<JournalPart>();
    p->path = cfg_.dir + "/seg-" + std::to_string(index) + "." + std::to_string(k) + ".log";
    p->fd = ::open(p->path.c_str(), O_RDWR | O_CLOEXEC | (create ? O_CREAT : 0), 0644);
    if (p->fd < 0) return nullptr;
    struct stat st;
    if (::fstat(p->fd, &st) != 0) return nullptr;
    if (create || static_cast<uint64_t>(st.st_size) < part_bytes_) {
      // reserve the extent once; later appends are overwrites inside the file
      if (::fallocate(p->fd, 0, 0, static_cast<off_t>(part_bytes_)) != 0 &&
          ::ftruncate(p->fd, static_cast<off_t>(part_bytes_)) != 0)
        return nullptr;
    }
    p->cap = std::max<uint64_t>(part_bytes_, static_cast<uint64_t>(st.st_size));
    if (cfg_.direct) p->dfd = ::open(p->path.c_str(), O_RDWR | O_CLOEXEC | O_DIRECT);
    s->parts.push_back(std::move(p));
  }
  return s;
}

bool BlockJournal::write_part_header(JournalPart* p, uint64_t seq, int part, int nparts, uint32_t flags,
                                     uint64_t lsn_hw) {
  alignas(4096) static thread_local uint8_t page[kPage];
  std::memset(page, 0, kPage);
  PartHdr h{};
  h.magic = kSegMagic;
  h.version = 3;
  h.seq = seq;
  h.cap = p->cap;
  h.part = static_cast<uint32_t>(part);
  h.nparts = static_cast<uint32_t>(nparts);
  h.flags = flags;
  h.lsn_hw = lsn_hw;
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(PartHdr, hdr_crc));
  std::memcpy(page, &h, sizeof(h));
  return pwrite_all(p->fd, page, kPage, 0);
}

std::vector<ReplayRecord> BlockJournal::recover() {
  std::vector<ReplayRecord> out;
  std::map<int, int> indices;  // segment index -> part files seen
  if (DIR* d = ::opendir(cfg_.dir.c_str())) {
    while (dirent* e = ::readdir(d)) {
      int idx = -1, k = -1;
      if (std::sscanf(e->d_name, "seg-%d.%d.log", &idx, &k) == 2 && idx >= 0 && k >= 0) indices[idx]++;
    }
    ::closedir(d);
  }
  std::vector<SegRef> live;
  for (auto& kv : indices) {
    next_file_ = std::max(next_file_, kv.first + 1);
    SegRef s = open_seg(kv.first, false);  // (a segment short of parts gets them created)
    if (!s) continue;
    segs_.push_back(s);
    // the segment's sequence number is the largest valid header's; parts whose header does
    // not carry it (never flushed before a crash) hold no acknowledged record. Every header,
    // retired ones included, raises the sequence / LSN floors of this run.
    uint64_t seq = 0;
    bool retired = false, sealed = true, any_hdr = false;
    std::vector<bool> valid(s->parts.size(), false);
    std::vector<HdrView> hv(s->parts.size());
    for (size_t k = 0; k < s->parts.size(); ++k) {
      hv[k] = read_part_header(s->parts[k]->fd, k, s->parts.size());
      if (!hv[k].ok) continue;
      any_hdr = true;
      next_seq_ = std::max(next_seq_, hv[k].seq + 1);
      next_lsn_ = std::max(next_lsn_, hv[k].lsn_hw);
      seq = std::max(seq, hv[k].seq);
    }
    for (size_t k = 0; k < s->parts.size(); ++k) {
      if (hv[k].ok && hv[k].seq == seq) {
        valid[k] = true;
        retired = retired || (hv[k].flags & kFlagRetired);
        sealed = sealed && (hv[k].flags & kFlagSealed);
      } else {
        sealed = false;
      }
    }
    if (seq == 0 || retired) {
      // free (a retirement that reached any part decided that every record is dead)
      if (any_hdr)
        for (auto& p : s->parts) p->filled = true;  // used before: written extents
      free_.push_back(s);
      continue;
    }
    s->seq = seq;
    for (size_t k = 0; k < s->parts.size(); ++k) {
      JournalPart* p = s->parts[k].get();
      uint64_t off = kPage;
      while (valid[k] && off + kPage <= p->cap) {
        RecHdr h;
        if (!pread_all(p->fd, reinterpret_cast<uint8_t*>(&h), kHdr, off)) break;
        if (h.magic != kRecMagic || h.hdr_crc != crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc)))
          break;
        if (h.seq != seq || h.part != k || h.off != off || h.rec_len < kPage || h.rec_len % kPage ||
            off + h.rec_len > p->cap)
          break;
        if (h.type == kJrBlock || h.type == kJrTomb || h.type == kJrFile) {
          ReplayRecord r;
          r.type = h.type;
          r.id.assign(h.id, std::min<uint32_t>(h.id_len, sizeof(h.id)));
          r.lsn = h.lsn;
          r.trusted = sealed;
          r.rec.seg = s;
          r.rec.part = static_cast<int>(k);
          r.rec.off = off;
          r.rec.end = off + h.rec_len;
          r.rec.lsn = h.lsn;
          if (h.type == kJrBlock) {
            if (h.hdr_bytes != hdr_bytes_for(h.nslices) || h.nslices != num_slices(h.n) ||
                h.hdr_bytes + align_up(h.n, kPage) != h.rec_len)
              break;
            r.meta_be.resize(4 * h.nslices);
            if (h.nslices && !pread_all(p->fd, r.meta_be.data(), r.meta_be.size(), off + kHdr)) break;
            if (crc32(r.meta_be.data(), r.meta_be.size()) != h.meta_crc) break;
            r.n = h.n;
            r.crc = h.crc;
            r.rec.hdr_bytes = h.hdr_bytes;
            s->live++;
            s->live_bytes += h.rec_len;
          }
          next_lsn_ = std::max(next_lsn_, h.lsn + 1);
          out.push_back(std::move(r));
        }
        off += h.rec_len;
      }
      p->tail = p->done_upto = p->durable_upto = p->syncing_upto = off;
      p->filled = true;  // written once at least up to the tail; recycled later as written extents
    }
    s->sealed = true;
    s->marked = sealed;
    live.push_back(s);
  }
  std::sort(live.begin(), live.end(), [](const SegRef& a, const SegRef& b) { return a->seq < b->seq; });
  for (auto& s : live) order_.push_back(s);
  std::stable_sort(out.begin(), out.end(), [](const ReplayRecord& a, const ReplayRecord& b) { return a.lsn < b.lsn; });
  st_.segs_total = segs_.size();
  preparer_ = std::thread([this] { prepare_loop(); });  // spares get ready while the caller replays
  return out;
}

void BlockJournal::note_replay(uint64_t replayed, uint64_t skipped, uint64_t verified) {
  std::lock_guard<std::mutex> g(mu_);
  st_.replayed += replayed;
  st_.replay_skipped += skipped;
  st_.replay_verified += verified;
}

void BlockJournal::reset_seg_locked(JournalSeg* s) {
  s->seq = 0;
  s->live = 0;
  s->live_bytes = 0;
  s->sealed = false;
  s->marked = false;
  for (auto& p : s->parts) {
    p->tail = p->done_upto = p->durable_upto = p->syncing_upto = 0;
    p->done_out.clear();
  }
}

void BlockJournal::retire_all() {
  std::vector<SegRef> segs;
  uint64_t lsn;
  {
    std::lock_guard<std::mutex> g(mu_);
    segs.swap(order_);
    lsn = next_lsn_;
  }
  for (auto& s : segs)
    for (size_t k = 0; k < s->parts.size(); ++k) {
      JournalPart* p = s->parts[k].get();
      (void)write_part_header(p, s->seq, static_cast<int>(k), static_cast<int>(s->parts.size()), kFlagRetired, lsn);
      if (cfg_.sync) (void)::fdatasync(p->fd);
      (void)::posix_fadvise(p->fd, 0, 0, POSIX_FADV_DONTNEED);
    }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& s : segs) {
    reset_seg_locked(s.get());
    free_.push_back(s);
    ++st_.segs_retired;
  }
  cv_.notify_all();
}

// Caller holds the lock. Seals nothing; takes a free segment (or waits for the preparer /
// the exporter) and makes it the active one.
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
        if (free_[i]->filling()) continue;
        if (pick < 0 || (free_[i]->filled() && !free_[pick]->filled())) pick = i;
      }
      if (pick >= 0) {
        s = free_[pick];
        free_.erase(free_.begin() + pick);
        cv_.notify_all();  // the preparer may create / fill another
      }
    }
    if (s) {
      const uint64_t seq = next_seq_++;
      // no flush of their own: the first commit's fdatasync of each part covers its header
      for (size_t k = 0; k < s->parts.size(); ++k)
        if (!write_part_header(s->parts[k].get(), seq, static_cast<int>(k), static_cast<int>(s->parts.size()), 0,
                               next_lsn_)) {
          *err = std::string("journal header: ") + std::strerror(errno);
          free_.push_back(s);
          return nullptr;
        }
      s->seq = seq;
      for (auto& p : s->parts) {
        p->tail = p->done_upto = p->durable_upto = p->syncing_upto = kPage;
        p->done_out.clear();
      }
      s->live = 0;
      s->live_bytes = 0;
      s->sealed = false;
      s->marked = false;
      order_.push_back(s);
      return s;
    }
    const int have = static_cast<int>(segs_.size()) + preparing_;
    const bool capped = cfg_.grow ? grow_blocked_ || (cfg_.max_segs > 0 && have >= cfg_.max_segs)
                                  : have >= cfg_.max_segs;
    const bool full = capped && std::none_of(free_.begin(), free_.end(), [](const SegRef& f) { return f->filling(); });
    if (full) ++st_.full_waits;  // not just waiting for the preparer
    if (std::chrono::steady_clock::now() >= next_report) {
      std::fprintf(stderr, "[journal] writer waiting for a free segment (%s)\n", describe_locked().c_str());
      next_report += std::chrono::seconds(10);
    }
    if (cv_.wait_until(lk, std::min(deadline, next_report)) == std::cv_status::timeout &&
        std::chrono::steady_clock::now() >= deadline) {
      *err = std::string(full ? "journal full (no free segment and no room for another): "
                              : "no journal segment ready: ") +
             describe_locked() + (st_.last_error.empty() ? "" : "; last error: " + st_.last_error);
      return nullptr;
    }
  }
}

bool BlockJournal::place_locked(std::unique_lock<std::mutex>& lk, uint64_t len, JournalRec* r, std::string* err,
                                bool marker) {
  for (;;) {
    SegRef s = order_.empty() || order_.back()->sealed ? nullptr : order_.back();
    if (!s && marker && free_.empty() && !order_.empty() && order_.back()->marking) {
      cv_.wait(lk);  // its sealed header is being flushed: the reserve is usable right after
      continue;
    }
    if (!s && marker && free_.empty() && !order_.empty()) {
      // no active segment: a marker goes into the newest segment's reserve (it retires last,
      // so the marker still outlives every record it cancels); the segment is re-marked later
      SegRef b = order_.back();
      for (size_t k = 0; k < b->parts.size(); ++k) {
        JournalPart* p = b->parts[k].get();
        if (p->tail + len > p->cap) continue;
        r->seg = b;
        r->part = static_cast<int>(k);
        r->off = p->tail;
        r->end = p->tail + len;
        p->tail += len;
        b->marked = false;
        st_.reserve_markers++;
        return true;
      }
    }
    if (s) {
      // round robin over the parts, so concurrent appends land in different files; block
      // records leave each part's marker reserve free
      const uint64_t limit = marker ? 0 : kMarkerReserve;
      const size_t np = s->parts.size();
      for (size_t i = 0; i < np; ++i) {
        const size_t k = (rr_ + i) % np;
        JournalPart* p = s->parts[k].get();
        if (p->tail + len + limit > p->cap) continue;
        rr_ = k + 1;
        r->seg = s;
        r->part = static_cast<int>(k);
        r->off = p->tail;
        r->end = p->tail + len;
        p->tail += len;
        return true;
      }
      s->sealed = true;  // no part has room
      cv_.notify_all();
    }
    // activate_locked may wait (and drop the lock): whatever it returns is checked again
    if (!activate_locked(lk, err)) return false;
  }
}

bool BlockJournal::reserve(uint64_t n, uint64_t nslices, JournalRec* r, std::string* err) {
  const uint64_t len = rec_bytes_for(n, nslices);
  if (len + kPage + kMarkerReserve > part_bytes_) {
    *err = "block larger than a journal segment part";
    return false;
  }
  std::unique_lock<std::mutex> lk(mu_);
  if (failed_) {
    *err = "journal failed";
    return false;
  }
  if (!place_locked(lk, len, r, err)) return false;
  r->hdr_bytes = hdr_bytes_for(nslices);
  r->seg->live++;
  r->seg->live_bytes += len;
  last_append_ns_ = now_ns();
  return true;
}

bool BlockJournal::write(const JournalRec& r, uint64_t at, const uint8_t* p, uint64_t len) {
  const uint64_t off = r.data_off() + at;
  const JournalPart* part = r.seg->parts[r.part].get();
  if (part->dfd >= 0 && off % kPage == 0 && reinterpret_cast<uintptr_t>(p) % kPage == 0) {
    const uint64_t full = len & ~(kPage - 1);
    if (full && !pwrite_all(part->dfd, p, full, off)) return false;
    return full == len || pwrite_all(part->fd, p + full, len - full, off + full);
  }
  if (!cfg_.sync || cfg_.early_wb_bytes == 0 || len <= cfg_.early_wb_bytes)
    return pwrite_all(part->fd, p, len, off);
  // pieces end on multiples of early_wb_bytes (page-aligned), so a page handed to writeback is
  // never written again by the next piece
  const uint64_t piece = align_up(cfg_.early_wb_bytes, kPage);
  for (uint64_t o = off, e = off + len; o < e;) {
    const uint64_t next = std::min(e, (o / piece + 1) * piece);
    if (!pwrite_all(part->fd, p + (o - off), next - o, o)) return false;
    // only starts the write-out (no wait); the commit's fdatasync still makes it durable
    (void)::sync_file_range(part->fd, static_cast<off_t>(o), static_cast<off_t>(next - o), SYNC_FILE_RANGE_WRITE);
    o = next;
  }
  return true;
}

bool BlockJournal::finish(JournalRec* r, const std::string& id, uint64_t n, uint32_t crc, const uint8_t* meta_be,
                          uint64_t nslices, uint64_t keep_lsn) {
  std::vector<uint8_t> area(kHdr + 4 * nslices);
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = kJrBlock;
  h.seq = r->seg->seq;
  h.off = r->off;
  h.rec_len = r->end - r->off;
  h.hdr_bytes = r->hdr_bytes;
  h.n = n;
  h.crc = crc;
  h.nslices = static_cast<uint32_t>(nslices);
  h.meta_crc = crc32(meta_be, 4 * nslices);
  h.id_len = static_cast<uint32_t>(std::min<size_t>(id.size(), sizeof(h.id)));
  std::memcpy(h.id, id.data(), h.id_len);
  h.part = static_cast<uint32_t>(r->part);
  if (keep_lsn) {
    h.lsn = keep_lsn;
  } else {
    // the LSN is taken when the record is finished, after its bytes are written: a later
    // write of the same id (which can only start after this one returned) gets a larger one
    std::lock_guard<std::mutex> g(mu_);
    h.lsn = next_lsn_++;
  }
  r->lsn = h.lsn;
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  std::memcpy(area.data(), &h, kHdr);
  if (nslices) std::memcpy(area.data() + kHdr, meta_be, 4 * nslices);
  bool ok = pwrite_all(r->fd(), area.data(), area.size(), r->off);
  std::lock_guard<std::mutex> g(mu_);
  if (!ok) failed_ = true;  // the prefix cannot advance past a record that is not on disk
  complete_locked(r->seg->parts[r->part].get(), r->off, r->end);
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
  h.part = static_cast<uint32_t>(r.part);
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  bool ok = pwrite_all(r.fd(), reinterpret_cast<const uint8_t*>(&h), kHdr, r.off);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!ok) failed_ = true;
    complete_locked(r.seg->parts[r.part].get(), r.off, r.end);
    st_.pads++;
  }
  release(r);
}

void BlockJournal::pad_durable(const JournalRec& r) {
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = kJrPad;
  h.seq = r.seg->seq;
  h.off = r.off;
  h.rec_len = r.end - r.off;
  h.part = static_cast<uint32_t>(r.part);
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  bool ok = pwrite_all(r.fd(), reinterpret_cast<const uint8_t*>(&h), kHdr, r.off) &&
            (!cfg_.sync || ::fdatasync(r.fd()) == 0);
  std::lock_guard<std::mutex> g(mu_);
  if (!ok) failed_ = true;
  st_.pads++;
}

void BlockJournal::complete_locked(JournalPart* p, uint64_t off, uint64_t end) {
  if (off != p->done_upto) {
    p->done_out[off] = end;
    return;
  }
  p->done_upto = end;
  for (auto it = p->done_out.begin(); it != p->done_out.end() && it->first == p->done_upto;) {
    p->done_upto = it->second;
    it = p->done_out.erase(it);
  }
}

// Group commit per part: the first writer that finds its record complete but not durable
// (and no running round covering it) flushes the part for everyone whose record completed
// before; the others wait for that round. Parts commit independently, side by side.
bool BlockJournal::commit(const JournalRec& r) {
  const uint64_t t_in = now_ns();
  std::unique_lock<std::mutex> lk(mu_);
  st_.commits++;
  struct Acc {  // the caller's wait, whichever way it returns (lock held at every return)
    JournalStats& st;
    uint64_t t0;
    ~Acc() { st.commit_ns += now_ns() - t0; }
  } acc{st_, t_in};
  JournalPart* part = r.seg->parts[r.part].get();
  const int max_syncers = std::max(1, cfg_.syncers);
  for (;;) {
    if (failed_) return false;
    if (part->durable_upto >= r.end) return true;
    // wait while an earlier record of the part is still being written, while a running
    // round already covers this record, or while the part's flush slots are busy
    if (part->done_upto < r.end || part->syncing_upto >= r.end || part->syncers >= max_syncers) {
      cv_.wait(lk);
      continue;
    }
    ++part->syncers;
    const uint64_t snap = part->done_upto;
    part->syncing_upto = snap;
    lk.unlock();
    bool ok = true;
    if (cfg_.sync_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(cfg_.sync_delay_us));
    const uint64_t t_sync = now_ns();
    if (cfg_.sync) ok = ::fdatasync(part->fd) == 0;
    const uint64_t d_sync = now_ns() - t_sync;
    lk.lock();
    --part->syncers;
    st_.sync_rounds++;
    st_.sync_ns += d_sync;
    // a round that finishes flushed everything dirty when it started, i.e. every record
    // completed before its snapshot, whatever rounds started earlier still run
    if (ok) part->durable_upto = std::max(part->durable_upto, snap);
    else failed_ = true;  // after a failed flush the page state is unknown: refuse further acks
    cv_.notify_all();
  }
}

bool BlockJournal::marker(uint32_t type, const std::string& id, std::string* err) {
  JournalRec r;
  {
    std::unique_lock<std::mutex> lk(mu_);
    if (failed_) {
      *err = "journal failed";
      return false;
    }
    if (!place_locked(lk, kPage, &r, err, true)) return false;
    last_append_ns_ = now_ns();
  }
  RecHdr h{};
  h.magic = kRecMagic;
  h.type = type;
  h.seq = r.seg->seq;
  h.off = r.off;
  h.rec_len = kPage;
  h.id_len = static_cast<uint32_t>(std::min<size_t>(id.size(), sizeof(h.id)));
  std::memcpy(h.id, id.data(), h.id_len);
  h.part = static_cast<uint32_t>(r.part);
  {
    std::lock_guard<std::mutex> g(mu_);
    h.lsn = next_lsn_++;
  }
  h.hdr_crc = crc32(reinterpret_cast<const uint8_t*>(&h), offsetof(RecHdr, hdr_crc));
  bool ok = pwrite_all(r.fd(), reinterpret_cast<const uint8_t*>(&h), kHdr, r.off);
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!ok) failed_ = true;
    complete_locked(r.seg->parts[r.part].get(), r.off, r.end);
    if (type == kJrTomb) st_.tombstones++;
    else st_.supersedes++;
    cv_.notify_all();
  }
  if (!ok || !commit(r)) {
    *err = "journal marker append failed";
    return false;
  }
  return true;
}

void BlockJournal::release(const JournalRec& r) {
  if (!r.seg) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    r.seg->live -= std::min<uint64_t>(r.seg->live, 1);
    r.seg->live_bytes -= std::min(r.seg->live_bytes, r.bytes());
  }
  retire_ready();
}

void BlockJournal::retire_ready() {
  std::vector<SegRef> retire;
  uint64_t lsn;
  {
    std::lock_guard<std::mutex> g(mu_);
    // oldest first: a segment retires only after every older one did, so a tombstone or a
    // newer version is never dropped while a record it cancels could still be replayed; a
    // segment somebody is still reading from (or marking) waits for the next call
    while (!order_.empty()) {
      SegRef f = order_.front();
      if (!f->sealed && f != order_.back()) f->sealed = true;  // only the newest segment takes appends
      if (!f->sealed || f->live || !f->complete() || f->readers.load() > 0 || f->marking) break;
      retire.push_back(f);
      order_.erase(order_.begin());
    }
    lsn = next_lsn_;
  }
  if (retire.empty()) return;
  // the retired headers must be durable before the segment is reused: otherwise a crash
  // could replay its old records over newer versions
  for (auto& f : retire)
    for (size_t k = 0; k < f->parts.size(); ++k) {
      JournalPart* p = f->parts[k].get();
      (void)write_part_header(p, f->seq, static_cast<int>(k), static_cast<int>(f->parts.size()), kFlagRetired, lsn);
      if (cfg_.sync) (void)::fdatasync(p->fd);
      (void)::posix_fadvise(p->fd, 0, 0, POSIX_FADV_DONTNEED);
    }
  std::lock_guard<std::mutex> g(mu_);
  for (auto& f : retire) {
    for (auto& p : f->parts)
      if (p->tail + (8ull << 20) >= p->cap) p->filled = true;  // appends wrote (almost) all of it
    reset_seg_locked(f.get());
    free_.push_back(f);
    ++st_.segs_retired;
  }
  cv_.notify_all();
}

SegRef BlockJournal::compaction_candidate(double max_live) {
  std::lock_guard<std::mutex> g(mu_);
  if (order_.size() < 2) return nullptr;
  SegRef f = order_.front();
  if (!f->sealed || !f->complete() || f->live == 0) return nullptr;
  if (static_cast<double>(f->live_bytes) > max_live * static_cast<double>(f->capacity())) return nullptr;
  return f;
}

double BlockJournal::pressure() {
  std::lock_guard<std::mutex> g(mu_);
  const double cap = static_cast<double>(cfg_.max_segs > 0 ? cfg_.max_segs : std::max<size_t>(1, segs_.size()));
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
  s.segs_in_use = order_.size();
  s.failed = failed_;
  s.grow_blocked = grow_blocked_;
  for (auto& seg : order_) {
    s.live_records += seg->live;
    s.live_bytes += seg->live_bytes;
    s.used_bytes += seg->capacity();
    if (seg != order_.back()) {
      s.sealed_used_bytes += seg->capacity();
      s.sealed_live_bytes += seg->live_bytes;
    }
  }
  // parts_unready: what a writer activating a segment could be handed that is not ready (a
  // free segment not written out yet, or none at all below spares_low); spares_missing: the
  // grow-mode top-up still owed (done in idle windows)
  uint64_t missing = 0;
  if (cfg_.grow) {
    const bool can_grow = !grow_blocked_ && (cfg_.max_segs <= 0 || static_cast<int>(segs_.size()) < cfg_.max_segs);
    const int nfree = static_cast<int>(free_.size());
    if (can_grow && nfree < cfg_.spares) s.spares_missing = static_cast<uint64_t>(cfg_.spares - nfree);
    if (can_grow && nfree < cfg_.spares_low) missing = static_cast<uint64_t>(cfg_.spares_low - nfree);
  } else if (cfg_.max_segs > static_cast<int>(segs_.size())) {
    missing = cfg_.max_segs - segs_.size();
  }
  s.parts_unready = missing * static_cast<uint64_t>(cfg_.parts);
  if (cfg_.zero_fill)
    for (auto& seg : cfg_.grow ? free_ : segs_)
      for (auto& p : seg->parts) s.parts_unready += p->filled ? 0 : 1;
  return s;
}

}  // namespace dfs
