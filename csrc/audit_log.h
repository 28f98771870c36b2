// Tamper-evident S3 audit log writer (C56) in C++: the gateway's record sink and the
// datagram ingest of every gateway worker and of the native S3 front (s3_front.cpp), so
// one process owns one hash chain without a Python thread on the record path.
//
// Reference: dfs/s3_server/src/audit.rs (bounded channel of 10 000 records, batches of
// `batch_size` or a 5 s flush, records sorted by (timestamp_ms, request_id), monotonic key
// timestamps, previous_hash -> record_hash = HMAC-SHA256(secret, JSON with record_hash =
// null), the chain head recovered from the newest stored record, 3 write attempts with
// 0.5 s * n backoff, hourly retention). The store is the segment directory of
// tests/models/s3_audit.py (seg-<hour_ms>.log lines "<key_ts>\t<canonical json>", plus .uidx / .ridx
// index lines "<key>\t<offset>\t<length>" appended after the bytes they point at), so the
// Python reader, the native audit_reader and this writer share it byte for byte.
//
// Threading: log() is non-blocking (a full queue counts a drop); one writer thread batches
// and appends; an optional ingest thread receives JSON datagrams on a UNIX socket.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>

#include "json.h"

namespace dfs {

class AuditLog {
 public:
  AuditLog(std::string dir, int retention_days, int batch_size, std::string secret, size_t capacity = 10000,
           int flush_interval_ms = 5000, bool sync = false);
  ~AuditLog();
  AuditLog(const AuditLog&) = delete;
  AuditLog& operator=(const AuditLog&) = delete;

  // One record as JSON text (an object with the audit.py::make_record fields). false = dropped
  // (queue full or not an object).
  bool log(const std::string& json);
  // Receive records as datagrams on `fd` (a bound SOCK_DGRAM socket; dup'ed, the caller keeps
  // its own) until close().
  void start_ingest(int fd);
  // Wait until every accepted record is committed (flushes immediately). false on timeout.
  bool flush(int timeout_ms);
  void close();  // drain the queue, stop the threads

  uint64_t total() const { return total_.load(); }
  uint64_t dropped() const { return dropped_.load(); }
  uint64_t flush_errors() const { return flush_errors_.load(); }
  uint64_t committed() const { return committed_.load(); }
  uint64_t ingested() const { return ingested_.load(); }
  std::string head() const;  // record_hash of the newest committed record ("" = none)

  // Segment retention (also run hourly by the writer): removes segments older than
  // retention_days relative to now_ms; returns how many.
  int cleanup(int64_t now_ms);

 private:
  void run();
  void ingest_loop(int fd);
  void commit(std::deque<Json>& batch);
  bool append(const std::vector<std::pair<int64_t, Json>>& keyed);
  void recover();

  const std::string dir_;
  const int retention_days_, batch_size_;
  const std::string secret_;
  const size_t capacity_;
  const int flush_interval_ms_;
  const bool sync_;

  mutable std::mutex mu_;
  std::condition_variable cv_, flushed_cv_;
  std::deque<Json> q_;
  uint64_t pending_ = 0;   // accepted, not yet committed (mu_)
  bool stop_ = false, flush_now_ = false;
  std::string head_;       // chain head (writer thread; read under mu_)
  int64_t last_ts_ = 0;    // newest key timestamp (writer thread)

  std::atomic<uint64_t> total_{0}, dropped_{0}, flush_errors_{0}, committed_{0}, ingested_{0};
  std::thread writer_;
  int ingest_fd_ = -1;
  std::atomic<bool> ingest_stop_{false};
  std::thread ingest_;
};

}  // namespace dfs
