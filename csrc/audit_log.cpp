#include "audit_log.h"

#include <dirent.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "audit_json.h"

namespace dfs {

namespace {

using Clock = std::chrono::steady_clock;
constexpr int64_t kHourMs = 3'600'000;

int64_t wall_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

// audit.py::_idx_key: str(v or "") with tabs / newlines blanked (one token per index line)
std::string idx_key(const Json& v) {
  std::string s;
  if (v.is_string()) s = v.as_string();
  else if (v.is_number()) s = v.dump();
  else if (v.is_bool() && v.as_bool()) s = "True";
  for (char& c : s)
    if (c == '\t' || c == '\n') c = ' ';
  return s;
}

// audit.py::extract_bucket_name: the 6th ':' field of the ARN (or the whole string), up to '/'
std::string bucket_of(const std::string& resource) {
  std::string bid = resource;
  size_t pos = 0;
  int field = 0;
  for (size_t i = 0; i <= resource.size(); ++i) {
    if (i == resource.size() || resource[i] == ':') {
      if (field == 5) {
        bid = resource.substr(pos, i - pos);
        break;
      }
      ++field;
      pos = i + 1;
    }
  }
  size_t slash = bid.find('/');
  return slash == std::string::npos ? bid : bid.substr(0, slash);
}

std::vector<std::pair<int64_t, std::string>> list_segments(const std::string& dir) {
  std::vector<std::pair<int64_t, std::string>> out;
  DIR* d = ::opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    std::string n = e->d_name;
    if (n.size() <= 8 || n.compare(0, 4, "seg-") != 0 || n.compare(n.size() - 4, 4, ".log") != 0) continue;
    const std::string num = n.substr(4, n.size() - 8);
    char* end = nullptr;
    long long v = std::strtoll(num.c_str(), &end, 10);
    if (end && *end == '\0' && !num.empty()) out.emplace_back(v, dir + "/" + n);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

bool write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::write(fd, s.data() + off, s.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    off += static_cast<size_t>(n);
  }
  return true;
}

bool append_file(const std::string& path, const std::string& bytes, bool sync, off_t* base) {
  int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (fd < 0) return false;
  if (base) {
    struct stat st {};
    if (::fstat(fd, &st) != 0) {
      ::close(fd);
      return false;
    }
    *base = st.st_size;
  }
  bool ok = write_all(fd, bytes) && (!sync || ::fsync(fd) == 0);
  ::close(fd);
  return ok;
}

}  // namespace

AuditLog::AuditLog(std::string dir, int retention_days, int batch_size, std::string secret, size_t capacity,
                   int flush_interval_ms, bool sync)
    : dir_(std::move(dir)),
      retention_days_(retention_days),
      batch_size_(std::max(1, batch_size)),
      secret_(std::move(secret)),
      capacity_(std::max<size_t>(1, capacity)),
      flush_interval_ms_(std::max(10, flush_interval_ms)),
      sync_(sync) {
  ::mkdir(dir_.c_str(), 0755);
  recover();
  writer_ = std::thread([this] { run(); });
}

AuditLog::~AuditLog() { close(); }

void AuditLog::recover() {
  auto segs = list_segments(dir_);
  for (auto it = segs.rbegin(); it != segs.rend(); ++it) {
    FILE* f = std::fopen(it->second.c_str(), "rb");
    if (!f) continue;
    std::string data;
    char buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) data.append(buf, n);
    std::fclose(f);
    // the newest non-empty line (audit.py SegmentStore.last)
    size_t end = data.size();
    while (end > 0) {
      size_t start = data.rfind('\n', end - 1);
      start = start == std::string::npos ? 0 : start + 1;
      std::string line = data.substr(start, end - start);
      end = start == 0 ? 0 : start - 1;
      if (!line.empty() && line.back() == '\n') line.pop_back();
      bool blank = line.find_first_not_of(" \t\r") == std::string::npos;
      if (blank) continue;
      size_t tab = line.find('\t');
      if (tab == std::string::npos) break;
      try {
        Json rec = Json::parse(line.substr(tab + 1));
        last_ts_ = std::stoll(line.substr(0, tab));
        head_ = rec["record_hash"].str();
        return;
      } catch (...) {
        break;  // as last(): an unparsable newest line -> try the previous segment
      }
    }
  }
}

bool AuditLog::log(const std::string& json) {
  total_++;
  Json rec;
  try {
    rec = Json::parse(json);
  } catch (...) {
    dropped_++;
    return false;
  }
  if (!rec.is_object()) {
    dropped_++;
    return false;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_ || q_.size() >= capacity_) {
      dropped_++;
      return false;
    }
    q_.push_back(std::move(rec));
    pending_++;
    if (q_.size() < static_cast<size_t>(batch_size_)) return true;
  }
  cv_.notify_one();
  return true;
}

void AuditLog::start_ingest(int fd) {
  if (ingest_.joinable()) return;
  ingest_fd_ = ::fcntl(fd, F_DUPFD_CLOEXEC, 0);
  if (ingest_fd_ < 0) return;
  ingest_ = std::thread([this] { ingest_loop(ingest_fd_); });
}

void AuditLog::ingest_loop(int fd) {
  std::string buf(1 << 16, '\0');
  while (!ingest_stop_.load()) {
    pollfd p{fd, POLLIN, 0};
    int r = ::poll(&p, 1, 200);
    if (r <= 0) continue;
    ssize_t n = ::recv(fd, &buf[0], buf.size(), MSG_DONTWAIT);
    if (n <= 0) continue;
    ingested_++;
    log(std::string(buf.data(), static_cast<size_t>(n)));
  }
}

bool AuditLog::flush(int timeout_ms) {
  std::unique_lock<std::mutex> lk(mu_);
  flush_now_ = true;
  cv_.notify_one();
  return flushed_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return pending_ == 0; });
}

void AuditLog::close() {
  ingest_stop_ = true;
  if (ingest_.joinable()) ingest_.join();
  if (ingest_fd_ >= 0) {
    ::close(ingest_fd_);
    ingest_fd_ = -1;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_one();
  if (writer_.joinable()) writer_.join();
}

std::string AuditLog::head() const {
  std::lock_guard<std::mutex> g(mu_);
  return head_;
}

void AuditLog::run() {
  auto next_flush = Clock::now() + std::chrono::milliseconds(flush_interval_ms_);
  auto next_cleanup = Clock::now() + std::chrono::hours(1);
  for (;;) {
    std::deque<Json> batch;
    bool done = false;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait_until(lk, std::min(next_flush, next_cleanup), [&] {
        return stop_ || flush_now_ || q_.size() >= static_cast<size_t>(batch_size_);
      });
      const bool due = Clock::now() >= next_flush || flush_now_ || stop_;
      size_t take = q_.size() >= static_cast<size_t>(batch_size_) ? static_cast<size_t>(batch_size_)
                                                                   : (due ? q_.size() : 0);
      for (size_t i = 0; i < take; ++i) {
        batch.push_back(std::move(q_.front()));
        q_.pop_front();
      }
      if (q_.empty()) flush_now_ = false;
      done = stop_ && q_.empty();
    }
    auto now = Clock::now();
    if (now >= next_flush) next_flush = now + std::chrono::milliseconds(flush_interval_ms_);
    if (!batch.empty()) commit(batch);
    if (now >= next_cleanup) {
      next_cleanup = now + std::chrono::hours(1);
      cleanup(wall_ms());
    }
    if (done) break;
  }
}

void AuditLog::commit(std::deque<Json>& batch) {
  std::stable_sort(batch.begin(), batch.end(), [](const Json& a, const Json& b) {
    int64_t ta = a["timestamp_ms"].as_int(), tb = b["timestamp_ms"].as_int();
    if (ta != tb) return ta < tb;
    return a["request_id"].str() < b["request_id"].str();
  });
  std::string h;
  {
    std::lock_guard<std::mutex> g(mu_);
    h = head_;
  }
  int64_t last = last_ts_;
  std::vector<std::pair<int64_t, Json>> keyed;
  keyed.reserve(batch.size());
  for (auto& rec : batch) {
    int64_t key_ts = std::max(rec["timestamp_ms"].as_int(), last);
    last = key_ts;
    rec.set("previous_hash", h.empty() ? Json() : Json(h));
    rec.set("record_hash", Json());
    h = audit::hmac_hex(secret_, audit::canonical_json(rec, true));
    rec.set("record_hash", h);
    keyed.emplace_back(key_ts, std::move(rec));
  }
  bool ok = false;
  for (int attempt = 1; attempt <= 3 && !ok; ++attempt) {
    ok = append(keyed);
    if (!ok) {
      flush_errors_++;
      std::fprintf(stderr, "dfs audit: flush failed (attempt %d): %s\n", attempt, std::strerror(errno));
      if (attempt < 3) std::this_thread::sleep_for(std::chrono::milliseconds(500 * attempt));
    }
  }
  if (ok) {
    last_ts_ = last;
    committed_ += keyed.size();
  } else {
    std::fprintf(stderr, "dfs audit: flush failed after 3 attempts; %zu records lost\n", keyed.size());
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    if (ok) head_ = h;  // the chain head advances only after a successful write
    pending_ -= std::min<uint64_t>(pending_, batch.size());
  }
  flushed_cv_.notify_all();
}

bool AuditLog::append(const std::vector<std::pair<int64_t, Json>>& keyed) {
  std::map<int64_t, std::vector<std::pair<std::string, const Json*>>> by_seg;
  for (auto& kv : keyed) {
    std::string line = std::to_string(kv.first) + "\t" + audit::canonical_json(kv.second, false) + "\n";
    by_seg[kv.first / kHourMs * kHourMs].emplace_back(std::move(line), &kv.second);
  }
  // A failed attempt is rolled back before the caller retries: every file this batch touches
  // is cut back to its size before the attempt (or removed if the attempt created it), so a
  // retry never writes a record twice and a batch that fails for good leaves no trace of
  // records the chain head does not cover.
  std::vector<std::pair<std::string, off_t>> before;  // path, size (-1: did not exist)
  for (auto& sv : by_seg)
    for (const char* ext : {".log", ".uidx", ".ridx"}) {
      const std::string path = dir_ + "/seg-" + std::to_string(sv.first) + ext;
      struct stat st;
      before.emplace_back(path, ::stat(path.c_str(), &st) == 0 ? st.st_size : -1);
    }
  auto rollback = [&] {
    const int saved = errno;
    for (auto& b : before) {
      if (b.second < 0) ::unlink(b.first.c_str());
      else (void)::truncate(b.first.c_str(), b.second);
    }
    errno = saved;
    return false;
  };
  for (auto& sv : by_seg) {
    const std::string base_path = dir_ + "/seg-" + std::to_string(sv.first);
    std::string bytes;
    for (auto& it : sv.second) bytes += it.first;
    off_t base = 0;
    if (!append_file(base_path + ".log", bytes, sync_, &base)) return rollback();
    // index lines only after the records they point at are written
    std::string uidx, ridx;
    uint64_t off = static_cast<uint64_t>(base);
    for (auto& it : sv.second) {
      const std::string ref = "\t" + std::to_string(off) + "\t" + std::to_string(it.first.size()) + "\n";
      uidx += idx_key((*it.second)["user_id"]) + ref;
      ridx += idx_key(Json(bucket_of((*it.second)["resource"].str()))) + ref;
      off += it.first.size();
    }
    if (!append_file(base_path + ".uidx", uidx, sync_, nullptr) ||
        !append_file(base_path + ".ridx", ridx, sync_, nullptr))
      return rollback();
  }
  return true;
}

int AuditLog::cleanup(int64_t now_ms) {
  const int64_t cutoff = now_ms - static_cast<int64_t>(retention_days_) * 86'400'000;
  int n = 0;
  for (auto& s : list_segments(dir_)) {
    if (s.first + kHourMs > cutoff) continue;
    ::unlink(s.second.c_str());
    const std::string stem = dir_ + "/seg-" + std::to_string(s.first);
    ::unlink((stem + ".uidx").c_str());
    ::unlink((stem + ".ridx").c_str());
    ++n;
  }
  return n;
}

}  // namespace dfs
