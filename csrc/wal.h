// Append-only, CRC-framed write-ahead log for the Raft metadata plane. Replaces the
// reference's RocksDB column of `log:{i}` keys + term/vote keys
// (reference: dfs/metaserver/src/simple_raft.rs:809-991, 1033-1097).
//
// Frame: [u32 length LE][u32 crc32(payload) LE][payload]. A batch of records is written
// with one pwrite and made durable with ONE fdatasync (leader batching / group commit,
// simple_raft.rs:1689-1778). Replay stops at the first torn or corrupt frame (or a zero
// length) and truncates the tail, so a crash mid-append loses only the unacknowledged batch.
// The file is kept written out with zeros a few MiB past the last frame, so an append's
// fdatasync carries no file-size / extent metadata.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace dfs {

class Wal {
 public:
  Wal(std::string path, bool sync);
  ~Wal();
  std::vector<std::string> replay();
  void append(const std::vector<std::string>& records);
  // Replace the whole log (compaction after a snapshot): new file + fsync + rename.
  void reset(const std::vector<std::string>& records);
  uint64_t size_bytes() const { return size_; }
  uint64_t syncs() const { return syncs_; }

 private:
  void open_for_append(std::vector<std::string>* out = nullptr);
  void extend_fill(uint64_t need);  // zeros written (and flushed) at least prefill_/2 past `need`
  std::string path_;
  bool sync_;
  int fd_ = -1;
  uint64_t size_ = 0;    // end of the valid frames
  uint64_t filled_ = 0;  // the file's written bytes (frames, then zeros)
  uint64_t prefill_ = 8 << 20;  // DFS_WAL_PREFILL_MB (0: the file grows with every append)
  uint64_t syncs_ = 0;
  std::mutex mu_;
};

// temp file + fdatasync + rename + directory fsync.
void atomic_write_file(const std::string& path, const std::string& data, bool sync);

}  // namespace dfs
