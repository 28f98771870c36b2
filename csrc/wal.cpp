#include "wal.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
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

Wal::Wal(std::string path, bool sync) : path_(std::move(path)), sync_(sync) {}

Wal::~Wal() {
  if (fd_ >= 0) ::close(fd_);
}

void Wal::open_for_append() {
  if (fd_ >= 0) return;
  fd_ = ::open(path_.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
  if (fd_ < 0) throw std::runtime_error("wal open " + path_ + ": " + std::strerror(errno));
  struct stat st;
  ::fstat(fd_, &st);
  size_ = static_cast<uint64_t>(st.st_size);
}

std::vector<std::string> Wal::replay() {
  std::lock_guard<std::mutex> g(mu_);
  open_for_append();
  std::vector<std::string> out;
  std::string buf(size_, '\0');
  size_t got = 0;
  while (got < size_) {
    ssize_t r = ::pread(fd_, &buf[got], size_ - got, static_cast<off_t>(got));
    if (r <= 0) break;
    got += static_cast<size_t>(r);
  }
  size_t pos = 0;
  while (pos + 8 <= got) {
    uint32_t len, crc;
    std::memcpy(&len, &buf[pos], 4);
    std::memcpy(&crc, &buf[pos + 4], 4);
    if (pos + 8 + len > got) break;
    if (crc32(reinterpret_cast<const uint8_t*>(&buf[pos + 8]), len) != crc) break;
    out.emplace_back(buf, pos + 8, len);
    pos += 8 + len;
  }
  if (pos != size_) {  // torn tail: cut it off so new appends follow valid records
    if (::ftruncate(fd_, static_cast<off_t>(pos)) == 0) {
      size_ = pos;
      if (sync_) ::fdatasync(fd_);
    }
  }
  return out;
}

void Wal::append(const std::vector<std::string>& records) {
  if (records.empty()) return;
  std::string buf = frame(records);
  std::lock_guard<std::mutex> g(mu_);
  open_for_append();
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
