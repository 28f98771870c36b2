// BlockJournal: the group-committed write-ahead journal of one ChunkServer's block store.
//
// Reference semantics kept: a replica is acknowledged only once its bytes and slice
// checksums are on stable storage (chunkserver.rs:192-209 writes `<id>` and `<id>.meta`
// and sync_all()s both before the WriteBlock/ReplicateBlock reply). The reference pays
// two file creations, two device flushes and (implicitly) a directory update per block;
// with many writers on one volume those flush storms are what bounds the node (VERDICT
// r3: N=7 on one volume reached 25 % of N=1). Here every durable write of the hot tier
// appends ONE record — header + big-endian .meta image + the block bytes — to a
// preallocated segment, and one fdatasync covers every record that completed before it
// started (group commit). A background materializer (chunk_store.cpp) later writes the
// reference's `<id>` + `<id>.meta` files from the record, makes them durable in batches and
// retires the segment; on restart, unretired segments are replayed (each record verified
// against its checksums before it is materialized).
//
// A segment is striped over `parts` files. Buffered writes to one file serialize on its
// inode lock, so concurrent 1 MiB appends to a single file queue behind each other
// (measured on the MI355X box's volume: 21 writers on one file p50 2.3 ms, the same load
// over 3 files p50 0.7 ms, profiles/r4_journal); records go to the parts round robin and
// each part has its own group commit, so the flushes of different parts run side by side.
//
// On-disk layout, `<storage_dir>/.journal/seg-<n>.<k>.log` (part k of segment n), each
// seg_bytes / parts long:
//   [part header, 4 KiB][record][record]...            records never span parts
//   record = [RecHdr 512 B][.meta image, S x u32 BE][pad to 4 KiB][data n B][pad to 4 KiB]
// Every record carries a journal-wide sequence number (LSN) that orders replay across parts.
// A record is valid when its header checksum, segment sequence number, part and offset match
// and (block records) the data's slice CRCs equal the .meta image. Acknowledgement is
// prefix-ordered per part: a record is acked only after every record before it in its part
// is complete and flushed, so replay may stop at the first invalid record of a part without
// losing anything that was acknowledged. Segments retire oldest first, whole.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

struct JournalConfig {
  std::string dir;                  // usually <storage_dir>/.journal
  uint64_t seg_bytes = 256ull << 20;
  int max_segs = 16;                // journal capacity = max_segs x seg_bytes
  int parts = 8;                    // files a segment is striped over
  bool direct = false;              // O_DIRECT appends (aligned sources only; else buffered)
  bool sync = true;                 // fdatasync on commit (false: tests / --no-fsync)
  // Segment files are created (fallocate) ahead of use by a background thread, all of them up
  // to max_segs. With zero_fill that thread also writes the free ones out once while the
  // writers are idle (no append for a few ms), so an append overwrites written extents and its
  // flush carries no unwritten-extent conversion (measured: 23 % at 10 writers, 2.6x at 70 on
  // the box's volume, profiles/r4_journal); a fill never competes with acked writes.
  // Recycled segments are written extents either way.
  int spares = 2;          // kept ready when segments must be created on demand
  bool zero_fill = true;
  int idle_fill_ms = 20;   // the writers count as idle after this long without an append
  // Flush rounds that may run at once per part. 1 = classic group commit (one leader, the
  // others wait for the next round); more = pipelined: a writer whose record came after a
  // running round's snapshot starts its own round instead of waiting for that one to finish.
  int syncers = 1;
  int sync_delay_us = 0;   // tests: the commit leader waits this long first (makes rounds shared)
  int full_timeout_s = 120;  // a writer waiting this long for a free segment fails
};

enum JournalRecType : uint32_t { kJrBlock = 1, kJrPad = 2, kJrTomb = 3 };

struct JournalPart {
  int fd = -1;
  int dfd = -1;  // O_DIRECT descriptor of the same file (-1: none)
  std::string path;
  uint64_t cap = 0;
  // append state (BlockJournal::mu_)
  uint64_t tail = 0;
  uint64_t done_upto = 0;                 // contiguous completed prefix
  std::map<uint64_t, uint64_t> done_out;  // completed [off, end) past the prefix
  uint64_t durable_upto = 0;
  uint64_t syncing_upto = 0;              // covered by a flush round in progress
  int syncers = 0;                        // flush rounds in progress on this part
  bool filled = false;   // every extent written once (zero fill done, or a full cycle of appends)
  bool filling = false;  // the preparer is writing zeros into it right now
  uint64_t fill_off = 0;
  ~JournalPart();
};

struct JournalSeg {
  uint64_t seq = 0;  // 0 = free (headers invalidated)
  int index = 0;     // n of seg-<n>.<k>.log
  std::vector<std::unique_ptr<JournalPart>> parts;
  uint64_t live = 0;                      // block records not yet materialized (or dropped)
  bool sealed = false;
  std::atomic<int> readers{0};            // reads in progress from this segment (defer retirement)
  bool complete() const;                  // every part's records are complete
  bool filled() const;
  bool filling() const;
};
using SegRef = std::shared_ptr<JournalSeg>;

struct JournalRec {
  SegRef seg;
  int part = 0;
  uint64_t off = 0;        // record start in the part
  uint64_t hdr_bytes = 0;  // header + .meta area (4 KiB multiple)
  uint64_t end = 0;
  uint64_t data_off() const { return off + hdr_bytes; }
  int fd() const { return seg->parts[part]->fd; }
};

struct ReplayRecord {
  uint32_t type = 0;
  std::string id;
  uint64_t n = 0;
  uint32_t crc = 0;
  uint64_t lsn = 0;
  SegRef seg;
  int part = 0;
  uint64_t data_off = 0;
  std::vector<uint8_t> meta_be;
  int fd() const { return seg->parts[part]->fd; }
};

struct JournalStats {
  uint64_t records = 0, bytes = 0, commits = 0, sync_rounds = 0, tombstones = 0, pads = 0;
  uint64_t segs_total = 0, segs_free = 0, segs_retired = 0, full_waits = 0;
  uint64_t replayed = 0, replay_skipped = 0, prepared = 0, prepare_errors = 0, filled = 0, fill_bytes = 0;
  uint64_t sync_ns = 0, commit_ns = 0;  // time in fdatasync rounds; time writers spent in commit()
  uint64_t parts_unready = 0;  // part files not yet created, or (zero_fill) not yet written out once
  bool failed = false;
  std::string last_error;  // the last segment preparation / header error, for /stats
};

class BlockJournal {
 public:
  explicit BlockJournal(JournalConfig cfg);
  ~BlockJournal();
  BlockJournal(const BlockJournal&) = delete;

  // Recovery: every record of the unretired segments in LSN order (each part up to its
  // first invalid record). Block records carry their segment and part so the caller can
  // read and verify the data. Call once, before any append; then retire_all() once the
  // caller has materialized what it needed.
  std::vector<ReplayRecord> recover();
  void retire_all();
  void note_replay(uint64_t replayed, uint64_t skipped);

  static uint64_t hdr_bytes_for(uint64_t nslices);
  static uint64_t rec_bytes_for(uint64_t n, uint64_t nslices);
  bool fits(uint64_t n, uint64_t nslices) const;

  // Append protocol: reserve -> write (any order, any thread) -> finish | abandon -> commit.
  // reserve() blocks while every segment is in use (the materializer frees them).
  bool reserve(uint64_t n, uint64_t nslices, JournalRec* r, std::string* err);
  bool write(const JournalRec& r, uint64_t at, const uint8_t* p, uint64_t len);
  bool finish(const JournalRec& r, const std::string& id, uint64_t n, uint32_t crc, const uint8_t* meta_be,
              uint64_t nslices);
  void abandon(const JournalRec& r);  // the record becomes padding (counts as materialized)
  bool commit(const JournalRec& r);   // returns once the record is on stable storage
  void tombstone(const std::string& id);

  // Materializer side: `count` block records of `s` are now durable in their own files
  // (or obsolete). Sealed segments whose records are all materialized are retired in
  // sequence order and become free for reuse.
  void materialized(const SegRef& s, uint64_t count);
  void retire_ready();  // retires what materialized() had to defer for readers
  // Used segments (holding live or unretired records) over the capacity, 0..1.
  double pressure();
  uint64_t last_append_ns();
  JournalStats stats();

 private:
  // reserves `len` bytes in a part of the active segment (activating one if needed); lock held
  bool place_locked(std::unique_lock<std::mutex>& lk, uint64_t len, JournalRec* r, std::string* err);
  SegRef activate_locked(std::unique_lock<std::mutex>& lk, std::string* err);
  std::string describe_locked() const;  // segment accounting, for errors and stall reports
  bool write_part_header(JournalPart* p, uint64_t seq, int part, int nparts);
  void complete_locked(JournalPart* p, uint64_t off, uint64_t end);
  SegRef open_seg(int index, bool create);
  void reset_seg_locked(JournalSeg* s);
  void prepare_loop();
  std::thread preparer_;
  bool prep_stop_ = false;
  int preparing_ = 0;  // segment files being created (mu_)

  JournalConfig cfg_;
  uint64_t part_bytes_ = 0;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<SegRef> segs_;   // every segment
  std::vector<SegRef> order_;  // in use, oldest first (the last one is active)
  std::vector<SegRef> free_;
  uint64_t next_seq_ = 1;
  uint64_t next_lsn_ = 1;
  uint64_t rr_ = 0;  // round robin over the active segment's parts
  int next_file_ = 0;
  bool failed_ = false;
  uint64_t last_append_ns_ = 0;
  JournalStats st_;
};

}  // namespace dfs
