// ChunkStore: the ChunkServer's block store (reference: dfs/chunkserver/src/chunkserver.rs
// write_block_async/read_block_async/verify_block/verify_partial_read/move_block_to_cold,
// :110-143,192-351). On-disk format is identical to the reference:
//   <dir>/<block_id>        raw bytes
//   <dir>/<block_id>.meta   big-endian CRC-32/IEEE per 512 B slice
//
// Two backends behind one API:
//  * HBM mode (device >= 0): blocks live in a hipMalloc arena carved by an extent
//    allocator (host-side index + LRU). Checksums are computed/verified by the CDNA4
//    kernels in gpu_kernels.hip; persistence is either synchronous (nvme-sync: data and
//    .meta fdatasync'ed before ack, like the reference) or asynchronous spill threads
//    (hbm-ack: D2H into pinned buffers then pwrite/fdatasync). Non-dirty blocks are evicted
//    LRU when the arena is full and re-promoted from NVMe on the next read.
//  * Host mode (device < 0): reference semantics on the CPU (PCLMUL CRC, LRU of full
//    blocks, BLOCK_CACHE_SIZE).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "disk_gate.h"
#include "extent_alloc.h"
#include "gpu_kernels.h"
#include "io_pool.h"
#include "journal.h"

namespace dfs {

enum class Durability : int { NvmeSync = 0, HbmAck = 1 };

struct StoreConfig {
  std::string storage_dir = "/tmp/chunkserver_data";
  std::string cold_dir;          // empty = no cold tier
  int device = -1;               // < 0: host mode
  uint64_t hbm_capacity = 0;     // 0: auto (half of free HBM, capped at 64 GiB)
  Durability durability = Durability::NvmeSync;
  int cache_blocks = 100;        // host-mode LRU (BLOCK_CACHE_SIZE)
  int lanes = 8;                 // concurrent GPU stream contexts
  int spill_threads = 4;
  bool sync_writes = true;       // fdatasync data + .meta
  int journal = -1;              // group-committed block journal for nvme-sync writes (journal.h):
                                 // -1: DFS_JOURNAL (default on), 0: per-file fdatasync, 1: on
  int disk_inflight = -1;        // node-wide cap on durable writes per filesystem (disk_gate.h);
                                 // -1: DFS_DISK_INFLIGHT (default 12), 0: ungated
};

struct WriteResult {
  bool ok = false;
  uint32_t actual_crc = 0;
  std::string error;
};

enum class ReadStatus : int { Ok = 0, NotFound = 1, OutOfRange = 2, Corrupt = 3, IoError = 4 };

struct ReadResult {
  ReadStatus status = ReadStatus::Ok;
  uint64_t total_size = 0;
  uint64_t bytes = 0;
  bool partial_corrupt = false;  // partial read whose touched slices failed verification
  int64_t bad_slice = -1;
  std::string error;
};

struct StoreStats {
  uint64_t blocks = 0;
  uint64_t bytes = 0;
  uint64_t hbm_capacity = 0;
  uint64_t hbm_used = 0;
  uint64_t hbm_resident_blocks = 0;
  uint64_t dirty_blocks = 0;
  uint64_t spill_queue = 0;
  uint64_t evictions = 0;
  uint64_t promotions = 0;
  uint64_t crc_mismatches = 0;
  uint64_t scrub_transient = 0;  // durable-copy mismatches a re-check of the current copy did not confirm
  uint64_t gpu_kernel_launches = 0;
  uint64_t disk_gate_waits = 0;  // durable writes that queued for a node-wide disk slot
  uint64_t direct_dma = 0;       // host<->HBM copies done straight from registered memory
  uint64_t fused_reads = 0;      // reads delivered by the K3 verify+copy kernel (no SDMA copy)
  uint64_t fused_writes = 0;     // writes staged by the K1/K2 copy+checksum kernel (no SDMA copy)
  uint64_t pulled_recvs = 0;  // replica receives moved by the receiver's copy+checksum kernel
  uint64_t pulled_host_appends = 0;  // ... whose journal append read the kernel's host copy
  uint64_t sliced_stages = 0;    // pipelined head writes (per-slice fused kernels, sends overlap)
  uint64_t staged_dma = 0;       // copies bounced through pinned staging buffers
  uint64_t host_registered_bytes = 0;
  uint64_t mirror_hits = 0;      // small-block reads served from the verified host mirror
  uint64_t mirror_bytes = 0;
  uint64_t io_threads_spawned = 0;  // helper threads ever started (steady state: none per write)
  uint64_t final_name_writes = 0;   // durable writes of fresh ids straight to their final names
  uint64_t direct_writes = 0;       // of those, data files written with O_DIRECT (DFS_ODIRECT=1)
  // block journal (journal.h): group-committed durable writes; the store of record, with a
  // rate-limited exporter of reference-format files and compaction (or the round-4 mode)
  bool journal = false;
  std::string journal_mode = "none";  // "none" without fsync; "store" (export with headroom), "store-noexport", "idle" (round 4)
  uint64_t journal_records = 0, journal_bytes = 0, journal_commits = 0, journal_sync_rounds = 0;
  uint64_t journal_tombstones = 0, journal_supersedes = 0, journal_full_waits = 0, journal_segs = 0,
           journal_segs_free = 0, journal_segs_in_use = 0, journal_segs_marked = 0;
  uint64_t journal_segs_retired = 0, journal_replayed = 0, journal_replay_skipped = 0, journal_replay_verified = 0;
  uint64_t journal_live_records = 0, journal_live_bytes = 0, journal_used_bytes = 0;
  uint64_t materialized_blocks = 0, materialized_bytes = 0, materialize_pending = 0, materialize_batches = 0;
  uint64_t materialize_errors = 0, journal_prepare_errors = 0, journal_segs_filled = 0, journal_fill_bytes = 0,
           journal_parts_unready = 0, journal_spares_missing = 0, journal_grow_deferred = 0,
           journal_mark_preflushes = 0, journal_reserve_markers = 0;
  uint64_t delete_tomb_failures = 0;  // deletes refused: tombstone not durable (block kept)
  uint64_t export_busy_polls = 0;     // exporter wake-ups at the writers-active rate
  uint64_t journal_sync_ns = 0, journal_commit_ns = 0, journal_bypassed = 0;
  uint64_t relocated_blocks = 0, relocated_bytes = 0, compactions = 0, export_deferred_headroom = 0;
  uint64_t scrub_device_blocks = 0;  // durable (journal / file) copies verified by the K1b kernel
  uint64_t lane_waits = 0, lane_wait_ns = 0;  // callers that found every lane (stream context) busy
  bool journal_failed = false, journal_grow_blocked = false;
  std::string journal_last_error, materialize_last_error;
};

// Group commit: callers that finished writing share one flush round — syncfs() of the
// filesystem (data files, opt-in DFS_GROUP_SYNC) or fsync() of the directory itself (makes
// the renames of every block that finished before the round durable, one journal commit
// for a whole burst of writers instead of one per block).
class GroupSync {
 public:
  enum class Mode { FileSystem, Directory };
  explicit GroupSync(const std::string& dir, Mode mode = Mode::FileSystem);
  ~GroupSync();
  bool sync();  // returns once a flush that started after this call has completed
  uint64_t rounds() const { return rounds_; }

 private:
  int fd_ = -1;
  Mode mode_;
  std::mutex mu_;
  std::condition_variable cv_;
  uint64_t issued_ = 0, done_ = 0, rounds_ = 0;
  bool running_ = false;
  std::vector<std::pair<uint64_t, uint64_t>> failed_;  // ticket ranges of failed rounds
};

class ChunkStore;

// A region of the arena owned by an in-flight operation (RCCL receive target).
struct DevExtent {
  int64_t off = -1;
  uint64_t bytes = 0;
  uint8_t* ptr = nullptr;
};

class ChunkStore {
 public:
  explicit ChunkStore(StoreConfig cfg);
  ~ChunkStore();
  ChunkStore(const ChunkStore&) = delete;

  bool gpu() const { return cfg_.device >= 0; }
  const StoreConfig& config() const { return cfg_; }
  // The HBM arena (one hipMalloc): device transports export it to same-node peers, which
  // then DMA replica slices straight into the extents this store reserves.
  uint8_t* arena_base() const { return arena_; }
  uint64_t arena_bytes() const { return st_.hbm_capacity; }

  WriteResult write(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc);
  // Two-phase write used by pipelined chain replication: stage() lands the block in HBM
  // and verifies it (the block is then readable and can be forwarded over RCCL while
  // persist() makes it durable). persist() writes from `host_data` when given (no D2H),
  // otherwise streams the block out of HBM. In hbm-ack mode persist() returns at once and
  // the spill threads make the block durable.
  WriteResult stage(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc);
  bool persist(const std::string& id, const uint8_t* host_data, uint64_t n, std::string* err);
  // Resolves [offset, offset+length) against the block (length 0 = rest of block).
  ReadResult stat(const std::string& id, uint64_t offset, uint64_t length);
  ReadResult read_into(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out);
  bool exists(const std::string& id);
  int64_t block_size(const std::string& id);
  uint32_t block_crc(const std::string& id);
  bool remove(const std::string& id);
  bool move_to_cold(const std::string& id);
  // Reference verify_block against the on-disk .meta (CPU).
  std::string verify_on_disk(const std::string& id);
  std::vector<uint32_t> meta(const std::string& id);  // native-endian slice CRCs
  // Batched scrub (GPU verify of resident blocks + CPU verify of the rest).
  std::vector<std::string> scrub();
  // GPU part only: verify the given resident blocks (caller keeps them pinned), K1b.
  std::vector<std::string> scrub_resident(const std::vector<std::string>& ids);
  std::vector<std::string> list_blocks();
  StoreStats stats();
  void flush();          // wait until no dirty blocks remain
  void drop_resident();  // evict every clean resident block (tests / memory pressure)
  bool debug_corrupt(const std::string& id, uint64_t offset);  // flip a byte everywhere
  void debug_pause_spill(bool on);  // hbm-ack crash tests: hold dirty blocks in HBM only
  // Journal: export every journal-resident block as `<id>` + `<id>.meta` now and wait for it
  // (tests, tiering, `/export`); pause holds the exporter (crash tests).
  void materialize_all();
  void debug_pause_materializer(bool on);
  bool journaled(const std::string& id);  // durable in the journal, not in its own files
  // Relocates the live records of the oldest journal segment when at most `max_live` of it is
  // still live (or unconditionally with max_live >= 1); returns blocks moved (tests, /compact).
  uint64_t compact(double max_live);

  // ---- replication engine hooks (RCCL receive / send) ----
  DevExtent reserve(uint64_t n);
  void release(const DevExtent& e);
  WriteResult commit_device(const std::string& id, const DevExtent& e, uint64_t n, uint32_t expected_crc,
                            hipStream_t s, bool persist_now = true);
  // Zero-copy host<->HBM: host memory registered here (the clients' shared-memory arenas,
  // mapped by the fast path) is DMA'd directly by the copy engines; anything else bounces
  // through the lanes' pinned staging buffers.
  bool register_host(const void* p, uint64_t n);
  void unregister_host(const void* p);
  // Pipelined receive (replication.cpp): while slices of a block land in a reserved extent,
  // each landed byte range is checksummed on a store lane (K1 into the extent's .meta image)
  // so verification overlaps the transfer; finish() folds the slice CRCs into the block CRC,
  // compares, and commits (or releases the extent on mismatch).
  struct PullScratch;  // pinned host memory a pulled receive's kernels write its .meta image to
  struct RecvVerify {
    DevExtent ext;
    uint64_t n = 0;
    void* lane = nullptr;
    bool failed = false;
    bool host_meta = true;  // every slice kernel mirrored its .meta words into the lane's scratch
    std::string error;
    std::shared_ptr<PullScratch> pull;  // receiver pull (recv_begin(..., true))
  };
  // pull: the slices arrive through recv_pull's kernels (the transport launches them), not
  // recv_slice; returns false if the store cannot (no matrix-core CRC path, no pinned memory).
  // persist_now (pull only): an nvme-sync receive whose record the journal appends — the
  // kernels also leave the bytes in pinned host memory, so no device-to-host copy follows
  bool recv_begin(RecvVerify* rv, const DevExtent& e, uint64_t n, bool pull = false, bool persist_now = false);
  // Receiver pull: the launch of bytes [lo, hi) of the receive (lo a multiple of 512): one
  // crc_write_copy_kernel that reads the sender's bytes (a device pointer into its mapped
  // arena), stores them into the extent and writes the slices' .meta words to HBM and to the
  // receive's pinned scratch. The closure owns the scratch it writes to.
  std::function<int(const uint8_t*, void*)> recv_pull(RecvVerify* rv, uint64_t lo, uint64_t hi);
  bool can_pull() const;
  void* recv_lane(RecvVerify* rv);  // the receive's lane, taken at its first slice
  bool recv_slice(RecvVerify* rv, uint64_t lo, uint64_t hi);  // lo, hi: byte range, lo % 512 == 0
  WriteResult recv_finish(RecvVerify* rv, const std::string& id, uint32_t expected_crc, bool persist_now);
  // Gives the lane back without touching the extent (a late DMA may still land in it).
  void recv_abandon(RecvVerify* rv);
  // Pipelined head write (fast path, large replicated blocks): slice k of a block in
  // registered host memory is copied into HBM and checksummed by its own fused kernel
  // (crc_write_copy_kernel) and signals done[k], so the replica sends of slice k start while
  // slice k+1 is still crossing PCIe. finish() waits, folds the slice partials into the
  // block CRC, verifies, and indexes the block resident (not yet durable) holding `pins`
  // pins; on failure the extent stays reserved. end() — once no send can still wait on the
  // slice events or read the extent — frees the events and, after a failure, the extent.
  struct SliceStage {
    DevExtent ext;
    uint64_t n = 0, slice = 0;
    void* lane = nullptr;
    std::vector<hipEvent_t> done;
    std::vector<int> grids;
  };
  bool stage_slices_begin(const uint8_t* data, uint64_t n, uint64_t slice, SliceStage* ss, std::string* err);
  WriteResult stage_slices_finish(const std::string& id, SliceStage* ss, uint32_t expected_crc, int pins);
  void stage_slices_end(SliceStage* ss);
  // Pin a resident block (promoting it if needed) and return its device pointer.
  const uint8_t* pin_device(const std::string& id, uint64_t* size);
  void unpin(const std::string& id);

  // ---- device-resident erasure coding (EC writes, degraded reads, reconstruction): the
  // shards stay in HBM between the codec kernel (K4/K5), the per-shard checksum (K2) and the
  // replication engine that scatters / gathers them (reference client mod.rs:308-412,
  // 1110-1165; chunkserver.rs:503-640 move every shard through host memory).
  struct EcBuffers {
    DevExtent ext;
    uint64_t len = 0, stride = 0;
    int count = 0;
    std::vector<uint32_t> crc;   // whole-shard CRC-32 of each shard (K2)
    hipEvent_t done = nullptr;   // recorded after the kernels that produced the shards
    uint8_t* shard(int i) const { return ext.ptr + static_cast<uint64_t>(i) * stride; }
  };
  // k data stripes (host_stride apart in host memory; registered memory moves in one DMA
  // each) into HBM, the rows of `parity` x data computed next to them: out holds k + rows shards.
  bool ec_encode(const uint8_t* host, uint64_t host_stride, uint64_t len, int k,
                 const std::vector<std::vector<uint8_t>>& parity, EcBuffers* out, std::string* err);
  // `rows` x the k device inputs -> rows new shards in HBM.
  bool ec_decode(const std::vector<std::vector<uint8_t>>& rows, const std::vector<const uint8_t*>& in, uint64_t len,
                 EcBuffers* out, std::string* err);
  void ec_free(EcBuffers* b);
  // Device bytes into host memory (registered: one DMA) and synchronously complete.
  bool device_to_host(uint8_t* dst, const uint8_t* src_dev, uint64_t n);
  // A copy of device bytes committed as block `id` (checksummed, verified, made durable).
  WriteResult commit_copy(const std::string& id, const uint8_t* src_dev, uint64_t n, uint32_t expected_crc,
                          bool persist_now);

  // GPU-resident RS codec: shards are host buffers; returns false when no GPU.
  bool gf_matmul_gpu(const std::vector<std::vector<uint8_t>>& mat, const std::vector<const uint8_t*>& in,
                     const std::vector<uint8_t*>& out, uint64_t len);
  // Device checksum of a host buffer (K1+K2) for benchmarks / tests.
  uint32_t gpu_crc(const uint8_t* data, uint64_t n, std::vector<uint32_t>* slices);

 private:
  struct Block {
    uint64_t size = 0;
    uint32_t crc = 0;
    bool crc_known = false;
    bool cold = false;
    bool on_disk = false;
    bool dirty = false;
    int64_t dev_off = -1;
    uint64_t dev_bytes = 0;
    int pins = 0;
    bool doomed = false;  // removed while pinned: free on last unpin
    std::list<std::string>::iterator lru;
    bool in_lru = false;
    std::shared_ptr<std::vector<uint8_t>> host;  // host-mode cache
    std::shared_ptr<std::vector<uint8_t>> staged_meta;  // BE .meta image awaiting persist()
    // small blocks (<= kMirrorMax): host copy of the bytes + slice CRCs, so a 4 KiB read is a
    // verified memcpy instead of a GPU round trip (kernel launch + DMA + sync, ~30 us)
    std::shared_ptr<std::vector<uint8_t>> mirror;
    std::shared_ptr<std::vector<uint32_t>> mirror_meta;
    // durable in the block journal, not yet materialized into <id> + <id>.meta
    JournalRec jrec;
    std::shared_ptr<std::vector<uint8_t>> jmeta;  // BE .meta image of the journal record
  };
  struct Lane {
    hipStream_t stream = nullptr;
    uint8_t* pinned[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    uint32_t* dscratch = nullptr;  // device: part_crc[kMaxGridCrc], part_bad[kMaxGridCrc]
    uint8_t* hscratch = nullptr;   // pinned: meta image + partials
    uint64_t hscratch_cap = 0;
    void* hscratch_dev = nullptr;  // device-visible alias of hscratch (fused-read verdicts)
  };
  static constexpr uint64_t kChunk = 4ull << 20;

  std::string data_path(const std::string& id, bool cold) const;
  std::string meta_path(const std::string& id, bool cold) const;
  void scan_dirs();
  uint64_t alloc_bytes(uint64_t n) const;
  int64_t alloc_locked(std::unique_lock<std::mutex>& lk, uint64_t bytes);
  void free_extent_locked(Block& b);
  void touch_locked(const std::string& id, Block& b);
  void lru_remove_locked(Block& b);
  Lane* acquire_lane();
  uint64_t lane_waits_ = 0, lane_wait_ns_ = 0;  // under lane_mu_
  uint64_t tomb_failures_ = 0;  // deletes refused because their tombstone could not be committed (mu_)
  bool journal_gate_ = false;  // journal appends + commits take a DiskGate slot (DFS_JOURNAL_GATE)
  void release_lane(Lane* l);
  void ensure_hscratch(Lane* l, uint64_t bytes);
  // Device pass: CRC (and meta write or verify) over [slice range] of a resident block.
  struct CrcOut {
    uint32_t block_crc = 0;
    int64_t bad_slice = -1;
  };
  // hmeta (nullable, inside the lane's hscratch): where the caller wants the .meta image on
  // the host; *meta_done says whether the kernel wrote it there itself (no readback copy)
  bool run_crc(Lane* l, const uint8_t* dptr, uint64_t n, uint32_t* meta_out, const uint32_t* meta_expect,
               bool want_block, uint64_t byte_lo, uint64_t byte_hi, CrcOut* out, std::string* err,
               uint8_t* hmeta = nullptr, bool* meta_done = nullptr);
  bool h2d_chunked(Lane* l, uint8_t* dst, const uint8_t* src, uint64_t n);
  bool d2h_chunked(Lane* l, uint8_t* dst, const uint8_t* src, uint64_t n);
  bool promote(const std::string& id, std::string* err);  // load from NVMe into HBM
  WriteResult stage_impl(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc,
                         bool durable_now);
  void insert_resident(const std::string& id, const DevExtent& ext, uint64_t n, uint32_t crc, bool on_disk,
                       std::shared_ptr<std::vector<uint8_t>> meta, int pins = 0, const JournalRec* jr = nullptr);
  // GPU staging of a host buffer into `ext`: fused copy+checksum kernel (registered memory),
  // PCLMUL for small blocks, or SDMA copy + checksum kernel. Fills the BE .meta image.
  bool device_stage(const uint8_t* data, uint64_t n, const DevExtent& ext, std::vector<uint8_t>* meta_be,
                    CrcOut* co, std::string* err);
  WriteResult stage_journal(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc,
                            const DevExtent& ext);
  // Appends a verified block (from host memory, or streamed out of HBM when dev != nullptr)
  // to the journal and waits for its group commit.
  bool journal_block(const std::string& id, const uint8_t* host, const uint8_t* dev, uint64_t n, uint32_t crc,
                     const std::vector<uint8_t>& meta_be, JournalRec* out, std::string* err);
  void enqueue_materialize_locked(const std::string& id, const Block& b);
  bool journal_takes(uint64_t n, uint64_t nslices);
  std::atomic<uint64_t> bypassed_{0};  // durable writes sent past a journal at its materialize mark
  std::atomic<uint64_t> last_durable_write_ns_{0};  // any durable write, journaled or bypassed
  bool journal_bypass_ = true;
  // store of record (round 5): no bypass, no drain at stop, replay indexes records in place;
  // export_ = rate-limited export of reference-format files while the volume has headroom
  bool store_mode_ = false;
  bool export_ = true;
  double export_bps_ = 256e6;        // exporter token bucket (bytes / s)
  double export_busy_bps_ = 64e6;    // ... while writers are active (DFS_EXPORT_BUSY_MBPS)
  uint64_t export_busy_polls_ = 0;   // exporter wake-ups that found the writers active (mu_)
  uint64_t export_headroom_ = 0;     // export only while the volume keeps this much free
  void materializer_loop();
  bool materialize_due();
  bool export_headroom(uint64_t bytes);
  struct MatItem;
  // Exports the jobs (pins held) as `<id>` + `<id>.meta`: tmp names, per-file flush, rename
  // only while the record is still current and no per-file writer owns the id, one
  // directory flush. Returns the number exported; failures are requeued (retry = true).
  uint64_t export_batch(std::vector<MatItem>& batch, bool retry);
  uint64_t relocate_segment(const SegRef& seg, uint64_t budget_bytes);
  bool relocate_one(const std::string& id, const JournalRec& old);
  void replay_journal();
  void replay_store(std::vector<ReplayRecord>& recs);
  // After a durable per-file write of `id`: a supersede marker, so replay keeps the file
  // instead of an older journal version (no-op without a journal).
  bool supersede_file(const std::string& id, std::string* err);
  // Per-file writers of an id hold a claim while they write and index; the exporter never
  // renames over a claimed id (mu_).
  std::unordered_map<std::string, int> file_writers_;
  struct FileClaim {
    ChunkStore* s = nullptr;
    std::string id;
    FileClaim(ChunkStore* st, const std::string& i);
    ~FileClaim();
  };
  std::vector<std::string> scrub_durable_gpu(const std::vector<std::string>& ids, std::vector<std::string>* rest);
  // Where a block's durable bytes are read from: its own file or its journal record.
  struct DurableSrc {
    int fd = -1;
    bool own_fd = false;
    uint64_t base = 0;
    SegRef seg;  // keeps a journal segment open while it is read
    std::vector<uint32_t> meta;
    bool meta_ok = false;
    ~DurableSrc();
  };
  bool open_durable(const std::string& id, bool cold, const JournalRec& jrec,
                    const std::shared_ptr<std::vector<uint8_t>>& jmeta, DurableSrc* s);
  bool persist_from_device(const std::string& id, const uint8_t* d, uint64_t n, const uint8_t* meta_be,
                           uint64_t nslices, std::string* err);
  bool persist(const std::string& id, bool cold, const uint8_t* data, uint64_t n, const uint8_t* meta_be,
               uint64_t nslices, std::string* err);
  void spill_worker();
  bool make_durable(int data_fd, int meta_fd, bool cold);
  bool write_file_durable(const std::string& path, const uint8_t* p, uint64_t n, std::string* err);
  bool write_fd_durable(int fd, const uint8_t* p, uint64_t n, const std::string& what, std::string* err);
  WriteResult write_host(const std::string& id, const uint8_t* data, uint64_t n, uint32_t expected_crc);
  ReadResult read_host(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out);
  std::vector<uint32_t> load_meta_file(const std::string& id, bool cold, bool* ok);

  StoreConfig cfg_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::unordered_map<std::string, Block> index_;
  std::list<std::string> lru_;  // front = most recent
  ExtentAllocator alloc_;
  uint8_t* arena_ = nullptr;
  DevCrcTables* dtables_ = nullptr;
  std::vector<std::unique_ptr<Lane>> lanes_;
  std::vector<Lane*> free_lanes_;
  std::mutex lane_mu_;
  std::condition_variable lane_cv_;
  std::deque<std::string> spill_q_;
  static constexpr uint64_t kMirrorMax = 64ull << 10;
  uint64_t mirror_budget_ = 256ull << 20, mirror_bytes_ = 0;  // mu_
  std::deque<std::string> mirror_fifo_;                       // mu_: eviction order
  uint64_t mirror_hits_ = 0;                                  // mu_
  void set_mirror(const std::string& id, const uint8_t* data, uint64_t n, const std::vector<uint8_t>& meta_be);
  void drop_mirror_locked(Block& b);
  bool read_mirror(const std::string& id, uint64_t offset, uint64_t bytes, uint8_t* out, ReadResult* r);
  bool spill_paused_ = false;  // mu_
  std::vector<std::thread> spillers_;
  bool stop_ = false;
  StoreStats st_;
  std::atomic<uint64_t> launches_{0};
  std::atomic<uint64_t> tmp_seq_{0};  // unique temporary file names for in-flight writes
  std::unordered_set<std::string> writing_;  // mu_: fresh ids being written under their final names
  bool claim_fresh(const std::string& id);
  void unclaim_fresh(const std::string& id);
  bool host_registered(const void* p, uint64_t n);
  std::mutex reg_mu_;
  std::vector<std::pair<uintptr_t, uint64_t>> reg_;  // registered host ranges
  std::vector<uintptr_t> reg_dev_;  // device-visible address of each reg_ range (0 = none)
  // device-visible alias of registered host memory [p, p + n), nullptr if not registered
  uint8_t* device_view(const void* p, uint64_t n);
  std::atomic<uint64_t> fused_reads_{0};  // K3 fused verify+copy reads
  std::atomic<uint64_t> fused_writes_{0};  // K1/K2 fused copy+checksum writes
  struct PinnedPool;
  std::shared_ptr<PinnedPool> pull_pool_;  // receiver-pull .meta scratch (outlives closures)
  uint32_t* pull_parts_dev_ = nullptr;    // the pull kernels' whole-block partials (unread)
  std::atomic<uint64_t> pulled_recvs_{0};
  std::atomic<uint64_t> pulled_host_appends_{0};  // pulled replicas appended from their host copy
  std::atomic<int> staging_{0};            // device stagings in flight (fused vs SDMA choice)
  std::atomic<uint64_t> sliced_stages_{0};
  bool write_copy(Lane* l, const uint8_t* src_dev, uint8_t* dst, uint64_t n, uint32_t* dmeta, uint8_t* hmeta,
                  CrcOut* out, std::string* err);
  std::atomic<uint64_t> direct_dma_{0}, staged_dma_{0};
  std::unique_ptr<GroupSync> gsync_;
  IoPool io_{8, 30000, "store-io"};  // data-file writes and .meta flushes beside the GPU staging (no per-write threads)
  std::unique_ptr<GroupSync> dsync_hot_, dsync_cold_;  // directory fsync after renames
  bool sync_dir(bool cold);
  std::unique_ptr<DiskGate> gate_;
  // ---- block journal
  struct MatItem {
    std::string id;
    JournalRec rec;
    uint64_t n = 0;
    std::shared_ptr<std::vector<uint8_t>> meta;
  };
  std::unique_ptr<BlockJournal> journal_;
  std::deque<MatItem> mat_q_;         // mu_, append order
  std::condition_variable mat_cv_;    // materializer wake-up / completion
  int mat_force_ = 0;                 // mu_: materialize_all() callers waiting
  bool mat_busy_ = false;             // mu_: a batch is being written
  bool mat_paused_ = false;           // mu_
  bool mat_stop_ = false;             // mu_
  double mat_pressure_ = 0.5;         // materialize when this share of the journal is in use
  uint64_t mat_idle_ns_ = 100000000;  // ... or after this long without an append
  std::thread materializer_;
  uint64_t materialized_blocks_ = 0, materialized_bytes_ = 0, mat_batches_ = 0, mat_errors_ = 0;  // mu_
  uint64_t relocated_blocks_ = 0, relocated_bytes_ = 0, compactions_ = 0, export_deferred_ = 0;   // mu_
  std::atomic<uint64_t> scrub_dev_blocks_{0};
  std::mutex compact_mu_;       // one compaction at a time (exporter thread, compact())
  std::string mat_last_error_;  // mu_
};

}  // namespace dfs
