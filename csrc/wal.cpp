#include "wal.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "crc32.h"

namespace dfs {

namespace {
std::string dirname_of(const std::string& p) {
  auto pos = p.find_last_of('/');
  return pos == std::string::npos ? "." : p.substr(0, pos);
}
void fsync_dir(const std::string& dir) {
  int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (fd >= 0) {
    ::fsync(fd);
    ::close(fd);
  }
}
void put32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }
std::string frame(const std::vector<std::string>& recs) {
  std::string out;
  size_t total = 0;
  for (auto& r : recs) total += r.size() + 8;
  out.reserve(total);
  for (auto& r : recs) {
    put32(out, static_cast<uint32_t>(r.size()));
    put32(out, crc32(reinterpret_cast<const uint8_t*>(r.data()), r.size()));
    out += r;
  }
  return out;
}
void write_fully(int fd, const std::string& buf, uint64_t off, const std::string& what) {
  size_t done = 0;
  while (done < buf.size()) {
    ssize_t w = ::pwrite(fd, buf.data() + done, buf.size() - done, static_cast<off_t>(off + done));
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(what + ": " + std::strerror(errno));
    }
    done += static_cast<size_t>(w);
  }
}
}  // namespace

Wal::Wal(std::string path, bool sync) : path_(std::move(path)), sync_(sync) {
  const char* e = std::getenv("DFS_WAL_PREFILL_MB");
  prefill_ = static_cast<uint64_t>(e && *e ? std::atoll(e) : 8) << 20;
}

Wal::~Wal() {
  if (fd_ >= 0) ::close(fd_);
}

// Opens the log, finds its valid end (the first torn / corrupt frame, or a zero length: the
// written-out zeros past the end), cuts everything after it and writes zeros ahead of it.
// Appends then overwrite written extents inside the file: their fdatasync flushes data only,
// with no size or extent change for the filesystem's journal to commit with it (the master's
// CompleteFile paid one such metadata commit per write).
void Wal::open_for_append(std::vector<std::string>* out) {
  if (fd_ >= 0) return;
  fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  if (fd_ < 0) throw std::runtime_error("wal open " + path_ + ": " + std::strerror(errno));
  struct stat st;
  ::fstat(fd_, &st);
  const uint64_t fsize = static_cast<uint64_t>(st.st_size);
  std::string buf(fsize, '\0');
  size_t got = 0;
  while (got < fsize) {
    ssize_t r = ::pread(fd_, &buf[got], fsize - got, static_cast<off_t>(got));
    if (r <= 0) break;
    got += static_cast<size_t>(r);
  }
  size_t pos = 0;
  while (pos + 8 <= got) {
    uint32_t len, crc;
    std::memcpy(&len, &buf[pos], 4);
    std::memcpy(&crc, &buf[pos + 4], 4);
    if (len == 0 || pos + 8 + len > got) break;
    if (crc32(reinterpret_cast<const uint8_t*>(&buf[pos + 8]), len) != crc) break;
    if (out) out->emplace_back(buf, pos + 8, len);
    pos += 8 + len;
  }
  size_ = pos;
  filled_ = pos;
  if (pos < got && std::all_of(buf.begin() + static_cast<std::ptrdiff_t>(pos), buf.begin() + static_cast<std::ptrdiff_t>(got),
                               [](char c) { return c == 0; })) {
    filled_ = got;  // a clean end: the zeros written ahead of it are still there
  } else if (pos != fsize && ::ftruncate(fd_, static_cast<off_t>(pos)) == 0 && sync_) {
    ::fdatasync(fd_);  // a torn tail goes, so no stale frame can ever follow new appends
  }
  extend_fill(pos);
}

void Wal::extend_fill(uint64_t need) {
  if (prefill_ == 0 || filled_ >= need + prefill_ / 2) return;
  const uint64_t to = need + prefill_;
  static const std::string zeros(1 << 20, '\0');
  for (uint64_t off = filled_; off < to; off += zeros.size()) {
    const uint64_t n = std::min<uint64_t>(zeros.size(), to - off);
    write_fully(fd_, n == zeros.size() ? zeros : zeros.substr(0, n), off, "wal prefill");
  }
  filled_ = to;
  if (sync_) ::fdatasync(fd_);  // the size and extents once, ahead of the appends
}

std::vector<std::string> Wal::replay() {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  if (fd_ >= 0) {  // already open: rescan from the start
    ::close(fd_);
    fd_ = -1;
  }
  open_for_append(&out);
  return out;
}

void Wal::append(const std::vector<std::string>& records) {
  if (records.empty()) return;
  for (auto& r : records)
    if (r.empty()) throw std::runtime_error("wal append: empty record");  // a zero length ends the log
  std::string buf = frame(records);
  std::lock_guard<std::mutex> g(mu_);
  open_for_append();
  extend_fill(size_ + buf.size());
  write_fully(fd_, buf, size_, "wal append");
  size_ += buf.size();
  if (sync_) {
    ::fdatasync(fd_);
    ++syncs_;
  }
}

void Wal::reset(const std::vector<std::string>& records) {
  std::string buf = frame(records);
  std::lock_guard<std::mutex> g(mu_);
  std::string tmp = path_ + ".compact";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("wal compact open: " + std::string(std::strerror(errno)));
  write_fully(fd, buf, 0, "wal compact");
  if (sync_) ::fdatasync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path_.c_str()) != 0)
    throw std::runtime_error("wal compact rename: " + std::string(std::strerror(errno)));
  if (sync_) fsync_dir(dirname_of(path_));
  if (fd_ >= 0) ::close(fd_);
  fd_ = -1;
  open_for_append();
}

void atomic_write_file(const std::string& path, const std::string& data, bool sync) {
  std::string tmp = path + ".tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw std::runtime_error("open " + tmp + ": " + std::strerror(errno));
  write_fully(fd, data, 0, "write " + tmp);
  if (sync) ::fdatasync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path.c_str()) != 0)
    throw std::runtime_error("rename " + tmp + ": " + std::strerror(errno));
  if (sync) fsync_dir(dirname_of(path));
}

}  // namespace dfs
