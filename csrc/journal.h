// BlockJournal: the group-committed, log-structured block store of one ChunkServer.
//
// Reference semantics kept: a replica is acknowledged only once its bytes and slice
// checksums are on stable storage (chunkserver.rs:192-209 writes `<id>` and `<id>.meta`
// and sync_all()s both before the WriteBlock/ReplicateBlock reply). The reference pays
// two file creations, two device flushes and (implicitly) a directory update per block;
// with many writers on one volume those flush storms are what bounds the node (VERDICT
// r3: N=7 on one volume reached 25 % of N=1). Here every durable write of the hot tier
// appends ONE record — header + big-endian .meta image + the block bytes — to a
// preallocated segment, and one fdatasync covers every record that completed before it
// started (group commit).
//
// Since round 5 the journal is the block's home ("store of record", chunk_store.cpp):
// segments are created on demand while the volume keeps a reserve free, a record stays the
// durable copy until its block is deleted, rewritten, relocated by compaction or exported
// as the reference's `<id>` + `<id>.meta` files (by a rate-limited exporter, only while the
// volume has headroom, or on request). The round-4 mode (every record materialized once
// the writers pause, then the segment recycled) remains as `DFS_JOURNAL_EXPORT=idle`.
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
// The part header carries the segment's sequence number, an LSN high-water mark and flags:
//   live     records are appended / replayed;
//   sealed   every record of the segment was complete and flushed when this header was
//            written (replay trusts the record headers without re-reading the data);
//   retired  every record is dead; the sequence number is kept, so sequence numbers (and
//            LSNs) only grow across restarts and a reused segment's stale records can never
//            match its new sequence number.
// Every record carries a journal-wide sequence number (LSN) that orders replay across parts.
// A record is valid when its header checksum, segment sequence number, part and offset match
// and (block records in segments not sealed) the data's slice CRCs equal the .meta image.
// Acknowledgement is prefix-ordered per part: a record is acked only after every record
// before it in its part is complete and flushed, so replay may stop at the first invalid
// record of a part without losing anything that was acknowledged. Segments retire oldest
// first, whole: a tombstone or a newer version therefore outlives every older record it
// cancels.
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
  int max_segs = 16;                // cap on segment files (0: none; `grow` then stops at reserve_bytes)
  // grow: segments are created on demand, `spares` free ones kept ready, as long as the
  // volume keeps reserve_bytes free (the store of record). Otherwise every segment up to
  // max_segs is created up front (the round-4 ring).
  bool grow = false;
  uint64_t reserve_bytes = 2ull << 30;
  int parts = 8;                    // files a segment is striped over
  bool direct = false;              // O_DIRECT appends (aligned sources only; else buffered)
  bool sync = true;                 // fdatasync on commit (false: tests / --no-fsync)
  // Early writeback: a buffered append is written in pieces of this many bytes (page-aligned
  // file offsets), each handed to writeback at once (sync_file_range WRITE), so the device
  // is already writing the record's first pieces while the rest are copied and the header is
  // formed; the commit's fdatasync then waits for less. 0 = off (one pwrite, writeback
  // starts at the fdatasync).
  uint64_t early_wb_bytes = 0;
  // Segment files are created (fallocate) ahead of use by a background thread. With zero_fill
  // that thread also writes the free ones out once while the writers are idle (no append for
  // a few ms), so an append overwrites written extents and its flush carries no
  // unwritten-extent conversion (measured: 23 % at 10 writers, 2.6x at 70 on the box's
  // volume, profiles/r4_journal); a fill never competes with acked writes. The same idle
  // windows flush the `sealed` headers.
  int spares = 2;
  // grow: while the writers are active, a spare is created only when fewer than this many are
  // free (creating one is a fallocate + one flush per part + a directory flush on the volume
  // the acked writes use); the rest of the top-up waits for an idle window
  int spares_low = 2;
  bool zero_fill = true;
  int idle_fill_ms = 20;   // the writers count as idle after this long without an append
  // Flush rounds that may run at once per part. 1 = classic group commit (one leader, the
  // others wait for the next round); more = pipelined: a writer whose record came after a
  // running round's snapshot starts its own round instead of waiting for that one to finish.
  int syncers = 1;
  int sync_delay_us = 0;   // tests: the commit leader waits this long first (makes rounds shared)
  int full_timeout_s = 120;  // a writer waiting this long for a free segment fails
};

// kJrFile: "from this LSN on the id's current version lives in its own files" (written after
// a per-file durable write, so replay does not bring back an older journal version of it).
enum JournalRecType : uint32_t { kJrBlock = 1, kJrPad = 2, kJrTomb = 3, kJrFile = 4 };

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
  uint64_t seq = 0;  // 0 = free
  int index = 0;     // n of seg-<n>.<k>.log
  std::vector<std::unique_ptr<JournalPart>> parts;
  uint64_t live = 0;        // block records still referenced by the store
  uint64_t live_bytes = 0;  // their record bytes
  bool sealed = false;
  bool marked = false;      // the `sealed` headers are durable (replay trusts the records)
  bool marking = false;     // being marked right now (mu_)
  std::atomic<int> readers{0};  // reads in progress from this segment (defer retirement)
  bool complete() const;        // every part's records are complete
  bool filled() const;
  bool filling() const;
  uint64_t capacity() const;
};
using SegRef = std::shared_ptr<JournalSeg>;

struct JournalRec {
  SegRef seg;
  int part = 0;
  uint64_t off = 0;        // record start in the part
  uint64_t hdr_bytes = 0;  // header + .meta area (4 KiB multiple)
  uint64_t end = 0;
  uint64_t lsn = 0;        // set by finish() (or kept from the record it relocates)
  uint64_t data_off() const { return off + hdr_bytes; }
  uint64_t bytes() const { return end - off; }
  int fd() const { return seg->parts[part]->fd; }
  bool same(const JournalRec& o) const { return seg == o.seg && part == o.part && off == o.off; }
};

struct ReplayRecord {
  uint32_t type = 0;
  std::string id;
  uint64_t n = 0;
  uint32_t crc = 0;
  uint64_t lsn = 0;
  bool trusted = false;  // its segment was sealed durable: no need to re-read the data
  JournalRec rec;        // where it lives (block records)
  std::vector<uint8_t> meta_be;
  int fd() const { return rec.fd(); }
  uint64_t data_off() const { return rec.data_off(); }
};

struct JournalStats {
  uint64_t records = 0, bytes = 0, commits = 0, sync_rounds = 0, tombstones = 0, pads = 0, supersedes = 0;
  uint64_t segs_total = 0, segs_free = 0, segs_in_use = 0, segs_retired = 0, segs_marked = 0, full_waits = 0;
  uint64_t replayed = 0, replay_skipped = 0, replay_verified = 0, prepared = 0, prepare_errors = 0, filled = 0,
           fill_bytes = 0;
  uint64_t live_records = 0, live_bytes = 0, used_bytes = 0;  // used: in-use segments x capacity
  // the in-use segments behind the active one: what retiring or compacting them could free
  uint64_t sealed_used_bytes = 0, sealed_live_bytes = 0;
  uint64_t sync_ns = 0, commit_ns = 0;  // time in fdatasync rounds; time writers spent in commit()
  uint64_t parts_unready = 0;  // free segments' parts not yet written out once (zero_fill), or missing below spares_low
  uint64_t spares_missing = 0; // grow: segments short of `spares` (topped up in idle windows)
  uint64_t grow_deferred = 0;  // grow: spare creations put off while the writers were active
  uint64_t mark_preflushes = 0;  // parts flushed before a sealed header (records not yet durable)
  uint64_t reserve_markers = 0;  // markers placed in a sealed segment's reserve (no active segment)
  bool failed = false, grow_blocked = false;
  std::string last_error;  // the last segment preparation / header error, for /stats
};

class BlockJournal {
 public:
  explicit BlockJournal(JournalConfig cfg);
  ~BlockJournal();
  BlockJournal(const BlockJournal&) = delete;

  // Recovery: every record of the unretired segments in LSN order (each part up to its
  // first invalid record). Block records carry their location so the caller can read and
  // verify the data, or index it in place. Every block record starts out live: the caller
  // release()s the ones it does not keep. Call once, before any append.
  std::vector<ReplayRecord> recover();
  void retire_all();  // the round-4 mode: after replay materialized everything, and at a clean stop
  void note_replay(uint64_t replayed, uint64_t skipped, uint64_t verified);
  uint64_t capacity_bytes() const { return part_bytes_ * static_cast<uint64_t>(cfg_.parts); }

  static uint64_t hdr_bytes_for(uint64_t nslices);
  static uint64_t rec_bytes_for(uint64_t n, uint64_t nslices);
  bool fits(uint64_t n, uint64_t nslices) const;

  // Append protocol: reserve -> write (any order, any thread) -> finish | abandon -> commit.
  // reserve() blocks while no segment has room (the preparer / exporter / compaction frees one).
  bool reserve(uint64_t n, uint64_t nslices, JournalRec* r, std::string* err);
  bool write(const JournalRec& r, uint64_t at, const uint8_t* p, uint64_t len);
  // keep_lsn != 0: the record is a relocated copy and keeps the original's LSN
  bool finish(JournalRec* r, const std::string& id, uint64_t n, uint32_t crc, const uint8_t* meta_be,
              uint64_t nslices, uint64_t keep_lsn = 0);
  void abandon(const JournalRec& r);  // the record becomes padding (and is released)
  bool commit(const JournalRec& r);   // returns once the record is on stable storage
  // A durable tombstone (kJrTomb) or supersede marker (kJrFile) for `id`; returns after its
  // group commit. Markers may use the last kMarkerReserve bytes of every part, which block
  // records leave free, so a delete can still commit its tombstone when no segment is free.
  bool marker(uint32_t type, const std::string& id, std::string* err);
  // A committed record nobody references becomes durable padding (a relocated copy that lost
  // the race with a rewrite: replay must not see it).
  void pad_durable(const JournalRec& r);

  // The store no longer references the record (exported, rewritten, deleted, relocated):
  // sealed segments whose records are all released retire in sequence order.
  void release(const JournalRec& r);
  void retire_ready();  // retires what release() had to defer for readers
  // The oldest in-use segment, when it is sealed, complete and at most `max_live` of its
  // capacity is still live (compaction copies its live records forward); else nullptr.
  SegRef compaction_candidate(double max_live);
  uint64_t seg_bytes() const { return cfg_.seg_bytes; }
  // Used segments (holding live or unretired records) over the capacity, 0..1 (round-4 mode).
  double pressure();
  uint64_t last_append_ns();
  JournalStats stats();
  void mark_sealed_now();  // flush every sealed, complete segment's `sealed` headers (tests, stop)

 private:
  // reserves `len` bytes in a part of the active segment (activating one if needed); lock held
  bool place_locked(std::unique_lock<std::mutex>& lk, uint64_t len, JournalRec* r, std::string* err,
                    bool marker = false);
  SegRef activate_locked(std::unique_lock<std::mutex>& lk, std::string* err);
  std::string describe_locked() const;  // segment accounting, for errors and stall reports
  bool write_part_header(JournalPart* p, uint64_t seq, int part, int nparts, uint32_t flags, uint64_t lsn_hw);
  void complete_locked(JournalPart* p, uint64_t off, uint64_t end);
  SegRef open_seg(int index, bool create);
  void reset_seg_locked(JournalSeg* s);
  bool room_for_segment();  // grow: the volume keeps reserve_bytes after one more segment
  bool mark_one(std::unique_lock<std::mutex>& lk);  // marks one sealed segment; lock held on entry/exit
  void prepare_loop();
  std::thread preparer_;
  bool prep_stop_ = false;
  int preparing_ = 0;  // segment files being created (mu_)
  bool grow_blocked_ = false;  // grow: the last attempt found no room on the volume

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
