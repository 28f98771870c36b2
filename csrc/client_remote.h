// Native remote client: the reference client's write / read of a single-block file
// (dfs/client/src/mod.rs:225-494 write, 856-944 read) for a client on ANOTHER host — every
// RPC over gRPC/TCP (grpc_client.h), nothing through shared memory or local sockets:
//
//   write: CRC-32 (PCLMUL) + MD5 on a worker, overlapped with CreateFile{allocate, deferred}
//          -> WriteBlock(data, next_servers) to the chain head -> CompleteFile{create}
//   read:  GetFileInfo -> ReadBlock from the first location that answers
//
// Leader changes are followed (Not Leader hints, then the shard's other peers), and so are
// REDIRECT:<owner> answers to a stale shard map. Anything else it does not own (multi-block
// files) returns NotHandled and the Python client takes over, so semantics never change. It is what makes the
// "remote client" numbers of bench.py a native client against native servers, like the
// reference's Rust dfs_cli against its Rust servers.
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "client_fast.h"
#include "dfs_pb.h"
#include "grpc_client.h"
#include "md5_mb.h"
#include "io_pool.h"
#include "tls.h"
#include "shard_map.h"

namespace dfs {

class RemoteClient {
 public:
  using Status = FastClient::Status;
  using Times = FastClient::Times;

  // `tls`: TLS client context for https endpoints (nullptr = h2c).
  explicit RemoteClient(int hash_threads = 4, int timeout_ms = 120000, std::shared_ptr<TlsContext> tls = nullptr);
  ~RemoteClient();
  RemoteClient(const RemoteClient&) = delete;

  // Routing: shard map (serde JSON, "" = none) and the fallback master list (gRPC URLs).
  void set_routing(const std::string& shard_map_json, const std::vector<std::string>& masters);

  Status write(const std::string& path, const uint8_t* data, size_t n, int* replicas, std::string* msg, Times* t,
               const std::string& rid = "", const std::map<std::string, std::string>* attrs = nullptr);
  Status read(const std::string& path, std::string* out, std::string* msg, Times* t, const std::string& rid = "",
              uint64_t offset = 0, uint64_t length = 0);

  uint64_t writes() const { return writes_.load(); }
  uint64_t reads() const { return reads_.load(); }
  uint64_t connects() const { return pool_.connects(); }
  // Erasure-coded file from a client on another host (reference mod.rs:308-412): RS encode on
  // this host's CPU (gf256.cpp, bit-compatible with galois_8), k + m WriteBlock calls in
  // parallel; EC reads (mod.rs:1110-1165) gather the shards in parallel and decode when a
  // data shard is missing.
  Status write_ec(const std::string& path, const uint8_t* data, size_t n, int k, int m, std::string* msg,
                  const std::string& rid);
  uint64_t ec_degraded_reads() const { return ec_degraded_.load(); }
  // Hedged reads (Client::with_hedge_delay): 0 = off.
  void set_hedge_delay(int ms) { hedge_ms_.store(ms); }
  void set_host_aliases(std::vector<std::pair<std::string, std::string>> a) { pool_.set_host_aliases(std::move(a)); }
  uint64_t hedged() const { return hedged_.load(); }

  // ---- the S3 front's entry points for a gateway on another host (front_store.h), the
  // remote twins of FastClient's: same statuses, same NotHandled cases (the gateway's Python
  // path follows redirects and reports range errors).
  // write() that also sets attrs[etag_attr] to the quoted MD5 (the S3 ETag); *md5_out = the MD5.
  Status write_etag(const std::string& path, const uint8_t* data, size_t n, int* replicas, std::string* msg, Times* t,
                    const std::string& rid, const std::map<std::string, std::string>* attrs, const char* etag_attr,
                    std::string* md5_out);
  Status stat(const std::string& path, bool* found, std::string* meta_pb, std::string* msg, const std::string& rid);
  // read() of a file whose metadata the caller already holds
  Status read_meta(const pb::FileMetadata& m, std::string* out, std::string* msg, Times* t, const std::string& rid,
                   uint64_t offset, uint64_t length);
  Status remove(const std::string& path, std::string* msg, const std::string& rid);
  Status rename(const std::string& src, const std::string& dst, std::string* msg, const std::string& rid);
  // ListFiles{with_metadata} under `prefix` on every shard (one call per shard), merged by path
  Status list(const std::string& prefix, std::vector<std::pair<std::string, pb::FileMetadata>>* out,
              const std::string& rid);

 private:
  // A MasterService call on the path's shard, following Not Leader hints; `*code` = -1 on
  // transport failure everywhere.
  bool master_call(const std::string& path, const std::string& method, const std::string& req,
                   const std::string& rid, int* code, std::string* resp);
  // the same over an explicit candidate list (the shard's peers, its last known leader first)
  bool call_candidates(std::vector<std::string> cands, const std::string& shard, const std::string& method,
                       const std::string& req, const std::string& rid, int* code, std::string* resp);
  std::vector<std::string> masters_for(const std::string& path, std::string* shard);
  void hash_loop();

  GrpcChannelPool pool_;
  std::mutex route_mu_;
  ShardMap map_;
  bool have_map_ = false;
  std::vector<std::string> masters_;
  std::map<std::string, std::string> leader_;  // shard ("" = no map) -> last known leader

  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<std::function<void()>> queue_;
  std::vector<std::thread> hashers_;
  std::unique_ptr<Md5MultiBuffer> md5mb_;  // the ETag MD5s on AVX-512 lanes (null: OpenSSL workers)
  bool stop_ = false;

  Status read_ec(const pb::FileMetadata& m, std::string* out, std::string* msg, const std::string& rid, uint64_t offset,
                 uint64_t length);
  std::atomic<uint64_t> writes_{0}, reads_{0}, hedged_{0}, ec_degraded_{0};
  std::atomic<int> hedge_ms_{0};
  IoPool hedge_pool_{2};  // last: destroyed first, after its in-flight reads finished
};

}  // namespace dfs
