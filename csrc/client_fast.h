// Native client data path for co-located writers/readers (C46-C48 hot path): the whole
// `create_file_from_buffer` / `get_file_content` sequence of the reference client
// (dfs/client/src/mod.rs:225-494, 856-917) runs in C++ without the GIL:
//
//   write: CRC-32 (PCLMUL) + MD5 on a worker thread, overlapped with
//          CreateFile{allocate, deferred} -> shared-memory slot -> ChunkServer fast path
//          (the server chains the replicas over RCCL/xGMI) -> CompleteFile{create}
//   read:  GetFileInfo -> ChunkServer fast path DMAs the block from HBM into our slot
//
// Metadata RPCs go to the shard's master over its same-host socket (localrpc.h) with the
// generated proto3 codec; the payload travels through a /dev/shm arena that the
// chunkserver maps (utils/shm.py protocol). Anything this path does not own — a remote or
// non-leader master, a redirect, EC files, multi-block files, a remote chain head —
// returns NotHandled and the Python client takes over, so semantics never change.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <future>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "dfs_pb.h"
#include "grpc_client.h"
#include "io_pool.h"
#include "md5_mb.h"
#include "shard_map.h"

namespace dfs {

// A WriteBlockRequest with `data` (field 2) appended straight from the caller's buffer: one
// copy of the payload into the wire message instead of two (field order is free in proto3,
// and the server decodes field 2 as a view — cs_grpc.cpp decode_viewing). An
// `alignment_pad` (field 110) in front makes the payload start at a multiple of 16 bytes of
// the message, which the chunkserver receives into a page-aligned registered buffer: the
// fused write kernel then loads the block straight from where the socket put it.
inline std::string encode_with_payload(const pb::WriteBlockRequest& w, const uint8_t* data, size_t n) {
  std::string wire;
  wire.reserve(n + 256 + w.block_id.size());
  w.encode(wire);
  size_t vl = 1;
  for (uint64_t v = n; v >= 0x80; v >>= 7) ++vl;
  // pad field: tag (2 bytes for field 110) + length (1 byte) + L bytes, then tag 2 + varint(n)
  const size_t before = wire.size() + 3 + 1 + vl;
  const size_t pad = (16 - before % 16) % 16;
  pb::wire::tag(wire, 110, 2);
  pb::wire::varint(wire, pad);
  wire.append(pad, '\0');
  pb::wire::tag(wire, 2, 2);
  pb::wire::varint(wire, n);
  wire.append(reinterpret_cast<const char*>(data), n);
  return wire;
}

class FastClient {
 public:
  // Host aliases for the gRPC hops to other hosts (EC shards): see GrpcChannelPool.
  void set_host_aliases(std::vector<std::pair<std::string, std::string>> a) { grpc_.set_host_aliases(std::move(a)); }
  enum Status { Ok = 0, NotHandled = 1, Failed = 2 };
  struct Times {  // seconds, per phase (benchmark breakdown)
    double crc = 0, create = 0, write = 0, md5_wait = 0, complete = 0, getinfo = 0, read = 0;
    double copy = 0;  // write(): slot acquire + copy of the caller's buffer into it
    double acquire = 0;  // ... of which waiting for a free slot
  };

  FastClient(std::string fastpath_socket, std::string local_chunkserver, size_t arena_bytes, size_t slot_bytes,
             int hash_threads);
  ~FastClient();
  bool ok() const { return base_ != nullptr; }
  const std::string& arena_path() const { return arena_path_; }

  // Routing: shard map (serde JSON, "" = none) and the fallback master list.
  void set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters);

  // `rid`: the request id carried on every hop (minted here when empty).
  // `attrs`: FileMetadata.attributes set by the same CompleteFile (nullptr = none).
  Status write(const std::string& path, const uint8_t* data, size_t n, int* replicas, std::string* msg, Times* t,
               const std::string& rid = "", const std::map<std::string, std::string>* attrs = nullptr);
  // On Ok the block sits in slot `*slot` (`*n` bytes); the caller copies it out and calls
  // release(*slot).
  // `length` > 0: only [offset, offset + length) (clipped to the file), the K3 range read.
  Status read(const std::string& path, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
              const std::string& rid = "", uint64_t offset = 0, uint64_t length = 0);
  const uint8_t* slot_ptr(int64_t slot) const { return base_ + slot; }
  uint8_t* slot_mut(int64_t slot) { return base_ + slot; }
  size_t slot_bytes() const { return slot_bytes_; }
  void release(int64_t slot);

  // ---- gateway entry points (csrc/s3_front.cpp): the payload is produced / consumed in
  // place in a slot, so an HTTP body moves socket -> slot -> HBM with no staging copy.
  int64_t acquire_slot(size_t n);  // -1: none free within 5 s, or n > slot_bytes()
  // write() of bytes already in `slot`. When `etag_attr` is set, attrs[etag_attr] is
  // replaced by the quoted MD5 before CompleteFile (the S3 ETag). *md5_out = the MD5.
  // The caller keeps (and releases) the slot.
  Status write_slot(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg, Times* t,
                    const std::string& rid, const std::map<std::string, std::string>* attrs, const char* etag_attr,
                    std::string* md5_out);
  // The distinct next path components below `prefix` on every shard (ListFiles with the
  // delimiter extension: one entry per component from each master, not every path).
  Status list_components(const std::string& prefix, std::set<std::string>* out, const std::string& rid);
  // GetFileInfo on the path's shard: Ok with *found, or NotHandled (remote/non-leader master).
  Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg, const std::string& rid);
  // read() of a file whose metadata (serialized FileMetadata) the caller already holds.
  Status read_known(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, Times* t,
                    const std::string& rid, uint64_t offset, uint64_t length);
  Status remove(const std::string& path, std::string* msg, const std::string& rid);
  // Rename on the source's shard (a cross-shard destination runs the master's 2PC).
  Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid);
  // ListFiles{with_metadata} under `prefix` on every shard (one call per shard, its master's
  // same-host socket), merged: (path, serialized FileMetadata). NotHandled if a shard's master
  // is not local or does not return metadata.
  Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
              const std::string& rid);

  // Erasure-coded file (reference mod.rs:308-412): the data is striped into k shards in a
  // slot, the m parity shards are computed by the co-located chunkserver's GPU (fast-path op
  // 6, the CPU codec when it has none), and the k + m shards go to their servers in parallel
  // — same-host servers read them straight from our slot through their own fast path, others
  // get a gRPC WriteBlock. Degraded reads (mod.rs:1110-1165) gather the survivors into a slot
  // and decode the missing data shards on the GPU from the layout as fetched.
  Status write_ec(const std::string& path, const uint8_t* data, size_t n, int k, int m, std::string* msg,
                  const std::string& rid);
  uint64_t ec_gpu_ops() const { return ec_gpu_.load(); }
  uint64_t ec_cpu_ops() const { return ec_cpu_.load(); }
  uint64_t ec_degraded_reads() const { return ec_degraded_.load(); }
  // device-resident EC (fast-path ops 7/8): writes encoded + scattered HBM -> HBM by the
  // co-located chunkserver, degraded reads decoded in its HBM; and those that fell back
  uint64_t ec_device_writes() const { return ec_dev_writes_.load(); }
  uint64_t ec_device_reads() const { return ec_dev_reads_.load(); }
  uint64_t ec_host_fallbacks() const { return ec_host_.load(); }

  uint64_t writes() const { return writes_.load(); }
  uint64_t reads() const { return reads_.load(); }

 private:
  int64_t acquire(size_t n);
  std::string master_socket(const std::string& path);
  // one request/response on a pooled connection; false on a transport error
  bool call(const std::string& sock, const std::string& method_path, const std::string& rid, const std::string& req,
            int* code,
            std::string* resp);
  bool fp_call(uint8_t op, const std::string& body, uint8_t* status, uint64_t* total, uint64_t* nbytes,
               std::string* msg);
  bool fp_call_to(const std::string& sock, uint8_t op, const std::string& body, uint8_t* status, uint64_t* total,
                  uint64_t* nbytes, std::string* msg);
  std::string peer_fastpath(const std::string& addr) const;  // "" unless `addr` is on this host
  bool ec_matmul(const std::vector<std::vector<uint8_t>>& mat, int k, uint64_t len, uint64_t in_off, uint64_t out_off,
                 const std::vector<uint16_t>* idx, const std::string& rid);
  Status read_ec(const std::string& meta_pb, int64_t* slot, uint64_t* n, std::string* msg, const std::string& rid,
                 uint64_t offset, uint64_t length);
  int take_conn(const std::string& name);
  void give_conn(const std::string& name, int fd);
  void hash_loop();

  std::string fp_socket_, local_cs_, arena_path_;
  uint8_t* base_ = nullptr;
  size_t arena_bytes_ = 0, slot_bytes_ = 0;

  std::mutex slot_mu_;
  std::condition_variable slot_cv_;
  std::vector<int64_t> free_slots_;

  std::mutex route_mu_;
  ShardMap map_;
  bool have_map_ = false;
  std::vector<std::string> masters_;

  std::mutex conn_mu_;
  std::map<std::string, std::vector<int>> idle_;

  // Hashes of a write's payload, started on the hash workers: the MD5 (the etag, a strictly
  // sequential chain) and optionally the whole-buffer CRC (jumps the queue: it gates the
  // block transfer). write() starts both on the caller's buffer before copying it into the slot.
  struct Hashes {
    std::future<std::string> md5;
    std::future<uint32_t> crc;
    void wait() {  // never return while a worker still reads the buffer
      if (md5.valid()) md5.wait();
      if (crc.valid()) crc.wait();
    }
  };
  void start_hashes(const uint8_t* p, size_t n, bool with_crc, Hashes* h);
  Status write_slot_impl(const std::string& path, int64_t slot, size_t n, int* replicas, std::string* msg, Times* t,
                         const std::string& rid, const std::map<std::string, std::string>* attrs,
                         const char* etag_attr, std::string* md5_out, Hashes* pre);
  // MD5 workers (the etag is a strictly sequential hash: overlap it with the RPCs)
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<std::function<void()>> queue_;
  std::vector<std::thread> hashers_;
  bool stop_ = false;
  // the ETag MD5s on AVX-512 lanes, up to 16 messages per engine thread (md5_mb.h); null:
  // no AVX-512F (or DFS_MD5_MB=0): the hash workers run OpenSSL, one message each
  std::unique_ptr<Md5MultiBuffer> md5mb_;

 public:
  const char* md5_mode() const {
    return !md5mb_ ? "openssl" : md5mb_->kind() == Md5MultiBuffer::Kind::Avx512 ? "avx512-x16" : md5mb_->lanes() == 3 ? "scalar-x3" : md5mb_->lanes() == 2 ? "scalar-x2" : "scalar-x1";
  }

  std::atomic<uint64_t> writes_{0}, reads_{0}, ec_gpu_{0}, ec_cpu_{0}, ec_degraded_{0};
  std::atomic<uint64_t> ec_dev_writes_{0}, ec_dev_reads_{0}, ec_host_{0};
  GrpcChannelPool grpc_{120000};  // shard I/O with servers on other hosts
  IoPool shard_pool_{8};         // last: destroyed first, after in-flight shard I/O
};

}  // namespace dfs
