#include "cs_grpc.h"

#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <future>
#include <mutex>
#include <vector>

#include "cs_agent.h"
#include "dfs_pb.h"
#include "grpc_client.h"
#include "replication.h"
#include "trace.h"

namespace dfs {

namespace {
constexpr int kFailedPrecondition = 9, kNotFound = 5, kOutOfRange = 11, kInternal = 13;

void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(static_cast<char>((v & 0x7F) | 0x80));
    v >>= 7;
  }
  o.push_back(static_cast<char>(v));
}

size_t put_varint(uint8_t* o, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    o[n++] = static_cast<uint8_t>((v & 0x7F) | 0x80);
    v >>= 7;
  }
  o[n++] = static_cast<uint8_t>(v);
  return n;
}

// Decodes `s` into `m` except for the bytes field `field`, which comes back as a view into
// `s` (last occurrence wins, as protobuf merges). The payload of a WriteBlock /
// ReplicateBlock — up to a whole block — is then never copied between the HTTP/2 DATA
// frames and the store. The generated decoders only assign what they meet, so the
// segments around the field decode one after another into the same message.
template <class M>
bool decode_viewing(M& m, const uint8_t* p, size_t size, uint32_t field, const uint8_t** q, size_t* l) {
  const uint8_t* e = p + size;
  pb::wire::Reader r{p, e};
  const uint8_t* seg = p;
  *q = reinterpret_cast<const uint8_t*>("");
  *l = 0;
  while (r.more()) {
    const uint8_t* at = r.p;
    const uint64_t t = r.varint();
    if (!r.ok) return false;
    if ((t >> 3) == field && (t & 7) == 2) {
      if (!r.len(q, l)) return false;
      if (at > seg && !m.decode(seg, static_cast<size_t>(at - seg))) return false;
      seg = r.p;
    } else {
      r.skip(static_cast<uint32_t>(t & 7));
    }
  }
  if (!r.ok) return false;
  return seg == e || m.decode(seg, static_cast<size_t>(e - seg));
}
}  // namespace

// Registered reply buffers for ReadBlock. A read that lands in memory the store has pinned
// is one fused verify+copy kernel straight into the reply (K3, crc_read_copy_kernel) —
// instead of a zero-filled std::string plus the staged bounce copy an unregistered
// destination needs. Buffers are made on demand (at most kMax, one per in-flight read),
// registered once, recycled when nghttp2 has sent the last byte, and live as long as the
// process (the chunkserver's store outlives every reply).
class ReplyPool : public std::enable_shared_from_this<ReplyPool> {
 public:
  static constexpr size_t kBytes = (4u << 20) + 4096;  // reads up to 4 MiB
  static constexpr size_t kMax = 64;
  static constexpr size_t kHead = 64;  // data starts at kHead + offset % 16 (fused-read alignment)
  explicit ReplyPool(ChunkStore* s) : store_(s) {}

  // Registers `n` buffers up front. Registering pinned memory costs about a millisecond
  // per buffer; paid lazily it landed on the first reads of every new concurrency level and
  // made dfs.grpc.read_block's p99 ~50x its p50.
  void prewarm(size_t n) {
    for (size_t i = 0; i < n; ++i) {
      void* p = nullptr;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (made_ >= kMax) return;
        ++made_;
      }
      if (::posix_memalign(&p, 4096, kBytes) != 0) {
        std::lock_guard<std::mutex> g(mu_);
        --made_;
        return;
      }
      (void)store_->register_host(p, kBytes);
      std::lock_guard<std::mutex> g(mu_);
      free_.push_back(static_cast<uint8_t*>(p));
    }
  }

  std::shared_ptr<uint8_t> take() {
    uint8_t* b = nullptr;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        b = free_.back();
        free_.pop_back();
      } else if (made_ < kMax) {
        ++made_;
      } else {
        return nullptr;
      }
    }
    if (!b) {
      void* p = nullptr;
      if (::posix_memalign(&p, 4096, kBytes) != 0) {
        std::lock_guard<std::mutex> g(mu_);
        --made_;
        return nullptr;
      }
      b = static_cast<uint8_t*>(p);
      (void)store_->register_host(b, kBytes);  // CPU store: plain memory, still no zero fill
    }
    // the deleter keeps the pool alive until the last reply using it is sent
    return std::shared_ptr<uint8_t>(b, [self = shared_from_this()](uint8_t* x) {
      std::lock_guard<std::mutex> g(self->mu_);
      self->free_.push_back(x);
    });
  }

 private:
  ChunkStore* store_;
  std::mutex mu_;
  std::vector<uint8_t*> free_;
  size_t made_ = 0;
};

NativeChunkService::NativeChunkService(ChunkStore* store, FastPathServer* fp, Fallback fallback)
    : store_(store),
      fp_(fp),
      fallback_(std::move(fallback)),
      replies_(std::make_shared<ReplyPool>(store)),
      requests_(std::make_shared<ReplyPool>(store)) {
  const char* e = std::getenv("DFS_GRPC_REPLY_PREWARM");
  if (store_->gpu()) {
    replies_->prewarm(e ? static_cast<size_t>(std::atoi(e)) : 16);
    requests_->prewarm(e ? static_cast<size_t>(std::atoi(e)) : 16);
  }
}

// Registered buffers for large requests (WriteBlock payloads): the HTTP/2 DATA frames land
// in memory the store can DMA from (or the fused write kernel can load over PCIe), and the
// client's alignment_pad makes the payload 16-byte aligned in it. nullptr: the server keeps
// its std::string body (CPU store, request larger than a pool buffer, pool exhausted).
std::shared_ptr<uint8_t> NativeChunkService::request_buffer(size_t n) {
  if (!store_->gpu() || n + 16 > ReplyPool::kBytes) return nullptr;
  return requests_->take();
}

CsGrpcStats NativeChunkService::stats() const {
  CsGrpcStats t;
  t.native_writes = writes_.load();
  t.native_reads = reads_.load();
  t.native_replicates = replicates_.load();
  t.fallbacks = fallbacks_.load();
  t.grpc_forwards = grpc_forwards_.load();
  t.grpc_forward_failures = grpc_forward_failures_.load();
  t.recoveries = recoveries_.load();
  t.shm_writes = shm_writes_.load();
  t.shm_reads = shm_reads_.load();
  return t;
}

void NativeChunkService::set_native(CsAgent* agent, std::shared_ptr<GrpcChannelPool> peers) {
  agent_ = agent;
  peers_ = std::move(peers);
  native_ = true;
}

bool NativeChunkService::fence(uint64_t term, std::string* msg) {
  uint64_t known = 0;
  if (fp_->fence(term, &known)) return true;
  *msg = "Stale master term: request has " + std::to_string(term) + " but known term is " + std::to_string(known);
  return false;
}

GrpcReply NativeChunkService::handle(const GrpcCall& call) {
  RequestScope rs(call.request_id);
  fp_->note_rid(call.request_id);
  bool handled = false;
  GrpcReply r;
  if (call.path == "/dfs.ChunkServerService/WriteBlock") r = write_block(call, &handled);
  else if (call.path == "/dfs.ChunkServerService/ReadBlock") r = read_block(call, &handled);
  else if (call.path == "/dfs.ChunkServerService/ReplicateBlock") r = replicate_block(call, &handled);
  if (handled) return r;
  fallbacks_++;
  if (!fallback_) return {12, "method not implemented natively: " + call.path};
  return fallback_(call);  // the fallback reads call.data() / call.size()
}

// The reference's chain hop (chunkserver.rs:777-829): the block goes to next[0] with the
// rest of the chain, on a pooled connection (the reference dials a new channel per hop).
// A same-node hop at the end of the chain takes the replication engine when its pair is up.
int NativeChunkService::forward(const std::string& id, const uint8_t* data, uint64_t n,
                                const std::vector<std::string>& next, uint32_t crc, uint64_t term, bool heal,
                                const std::string& rid) {
  if (next.empty()) return 0;
  RequestScope rs(rid);
  TraceRange tr("dfs.grpc.forward");
  const std::string& nxt = next[0];
  const std::vector<std::string> rest(next.begin() + 1, next.end());
  if (rest.empty() && fp_->p2p_ready({nxt})) {
    const int r = fp_->replicate_to(nxt, id, crc, term, store_->gpu() ? nullptr : data, n, heal);
    if (r > 0) return r;
  }
  if (!peers_) return 0;
  pb::ReplicateBlockRequest req;
  req.block_id = id;
  if (data) {
    req.data.assign(reinterpret_cast<const char*>(data), n);
  } else {  // received over the engine: the bytes are read back (verified) from the store
    ReadResult st = store_->stat(id, 0, 0);
    if (st.status != ReadStatus::Ok) return 0;
    req.data.resize(st.bytes);
    ReadResult rr = store_->read_into(id, 0, st.bytes, reinterpret_cast<uint8_t*>(&req.data[0]));
    if (rr.status != ReadStatus::Ok || rr.partial_corrupt) return 0;
  }
  req.next_servers = rest;
  req.expected_checksum_crc32c = crc;
  req.master_term = term;
  req.heal = heal;
  GrpcResult r = peers_->call(nxt, "/dfs.ChunkServerService/ReplicateBlock", req.str(), rid);
  if (!r.transport_ok || r.status != 0) {
    grpc_forward_failures_++;
    std::fprintf(stderr, "[cs] failed to replicate %s to %s: %s\n", id.c_str(), nxt.c_str(),
                 r.transport_ok ? r.message.c_str() : "transport error");
    return 0;
  }
  pb::ReplicateBlockResponse resp;
  if (!resp.decode(r.message)) return 0;
  grpc_forwards_++;
  if (!resp.success) {
    std::fprintf(stderr, "[cs] downstream replication failed at %s: %s\n", nxt.c_str(), resp.error_message.c_str());
    return 0;
  }
  return resp.replicas_written;
}

// Local durability and the downstream hop run side by side; the ack waits for both (the
// reference writes, fsyncs, then forwards: chunkserver.rs:777-819).
GrpcReply NativeChunkService::store_and_forward(const std::string& id, const uint8_t* data, uint64_t n,
                                                const std::vector<std::string>& next, uint32_t crc, uint64_t term,
                                                bool heal, const std::string& rid, int* replicas, std::string* err,
                                                bool staged) {
  auto down = std::async(std::launch::async, [&] { return forward(id, data, n, next, crc, term, heal, rid); });
  const bool pok = !staged || store_->persist(id, data, data ? n : 0, err);
  const int d = down.get();
  *replicas = pok ? 1 + d : 0;
  return {};
}

GrpcReply NativeChunkService::write_block(const GrpcCall& call, bool* handled) {
  pb::WriteBlockRequest req;
  const uint8_t* data;
  size_t n;
  if (!decode_viewing(req, call.data(), call.size(), 2, &data, &n)) {
    *handled = true;
    return {kInternal, "malformed WriteBlockRequest"};
  }
  const bool p2p = req.next_servers.empty() || fp_->p2p_ready(req.next_servers);
  // shm-in-gRPC writes and chains that leave the host (or lack a P2P pair) go to the Python
  // service inside its shell; the native chunkserver serves them here
  if (!native_ && (!req.shm_path.empty() || !p2p)) return {};
  *handled = true;
  TraceRange tr("dfs.grpc.write_block");
  std::string msg;
  if (!fence(req.master_term, &msg)) return {kFailedPrecondition, msg};
  if (!req.shm_path.empty()) {
    std::string e;
    uint8_t* base = fp_->map_client_shm(req.shm_path, req.shm_offset, req.shm_length, &e);
    if (!base) return {kFailedPrecondition, "short-circuit unavailable: " + e};
    data = base + req.shm_offset;
    n = req.shm_length;
    shm_writes_++;
  }
  pb::WriteBlockResponse resp;
  if (req.next_servers.empty()) {
    WriteResult w = store_->write(req.block_id, data, n, req.expected_checksum_crc32c);
    resp.success = w.ok;
    resp.error_message = w.error;
    resp.replicas_written = w.ok ? 1 : 0;
  } else {
    WriteResult w = store_->stage(req.block_id, data, n, req.expected_checksum_crc32c);
    if (!w.ok) {
      resp.error_message = w.error;
    } else if (p2p) {
      int down = 0;
      std::string perr;
      bool pok = fp_->persist_and_replicate(req.block_id, data, n, req.expected_checksum_crc32c, req.master_term,
                                            req.next_servers, &down, &perr);
      resp.success = pok;
      resp.error_message = pok ? "" : perr;
      resp.replicas_written = pok ? 1 + down : 0;
    } else {
      int replicas = 0;
      std::string perr;
      store_and_forward(req.block_id, data, n, req.next_servers, req.expected_checksum_crc32c, req.master_term, false,
                        call.request_id, &replicas, &perr, store_->gpu());
      resp.success = replicas > 0;
      resp.error_message = replicas > 0 ? "" : perr;
      resp.replicas_written = replicas;
    }
  }
  if (resp.success && !req.shm_path.empty()) resp.fastpath_socket = fp_->name();
  if (resp.success) writes_++;
  return {0, resp.str()};
}

// A full read that failed verification: recover the block from another replica (checked
// against our .meta) and read again, or DATA_LOSS (reference chunkserver.rs:913-949).
static GrpcReply read_failure(const ReadResult& rr) {
  if (rr.status == ReadStatus::NotFound) return {kNotFound, "Block not found"};
  if (rr.status == ReadStatus::OutOfRange) return {kOutOfRange, rr.error};
  return {kInternal, "Failed to read block: " + rr.error};
}

GrpcReply NativeChunkService::read_block(const GrpcCall& call, bool* handled) {
  pb::ReadBlockRequest req;
  if (!req.decode(call.data(), call.size())) {
    *handled = true;
    return {kInternal, "malformed ReadBlockRequest"};
  }
  if (!req.shm_path.empty() && !native_) return {};
  TraceRange tr("dfs.grpc.read_block");
  ReadResult st = store_->stat(req.block_id, req.offset, req.length);
  if (st.status == ReadStatus::NotFound) {
    *handled = true;
    return {kNotFound, "Block not found"};
  }
  if (st.status == ReadStatus::OutOfRange) {
    *handled = true;
    return {kOutOfRange, st.error};
  }
  if (st.status != ReadStatus::Ok && !native_) return {};
  *handled = native_;
  // the read itself, once more after a recovery when the block was corrupt
  auto read_to = [&](uint8_t* dst, ReadResult* out) -> GrpcReply {
    for (int attempt = 0;; ++attempt) {
      *out = store_->read_into(req.block_id, req.offset, st.bytes, dst);
      if (out->status == ReadStatus::Ok) return {};
      if (!native_) return {-1, ""};
      if (out->status != ReadStatus::Corrupt) return read_failure(*out);
      if (attempt > 0) return {15, "Recovered block is still corrupted: " + out->error};
      std::fprintf(stderr, "[cs] CRITICAL: data corruption detected for block %s: %s\n", req.block_id.c_str(),
                   out->error.c_str());
      recoveries_++;
      const std::string rerr = agent_ ? agent_->recover(req.block_id) : std::string("no recovery agent");
      if (!rerr.empty()) return {15, "Data corruption detected: " + out->error + ". Recovery failed: " + rerr};
    }
  };
  if (!req.shm_path.empty()) {
    std::string e;
    uint8_t* base = fp_->map_client_shm(req.shm_path, req.shm_offset, req.shm_capacity, &e);
    if (!base) return {kFailedPrecondition, "short-circuit unavailable: " + e};
    if (st.bytes > req.shm_capacity) return {kOutOfRange, "read larger than the shared-memory slot"};
    ReadResult rr;
    GrpcReply bad = read_to(base + req.shm_offset, &rr);
    if (bad.status) return bad;
    if (rr.partial_corrupt) fp_->add_suspect(req.block_id);
    pb::ReadBlockResponse resp;
    resp.bytes_read = rr.bytes;
    resp.total_size = rr.total_size;
    resp.shm_filled = true;
    resp.fastpath_socket = fp_->name();
    reads_++;
    shm_reads_++;
    return {0, resp.str()};
  }
  // ReadBlockResponse encoded by hand so the verified range lands in the reply buffer
  // directly: field 1 (data) header, the bytes, then bytes_read and total_size
  static const bool pool_on = [] {
    const char* e = std::getenv("DFS_GRPC_REPLY_POOL");
    return !(e && e[0] == '0');
  }();
  std::shared_ptr<uint8_t> buf =
      pool_on && st.bytes + ReplyPool::kHead + 16 + 32 <= ReplyPool::kBytes ? replies_->take() : nullptr;
  if (buf) {
    uint8_t hdr[16];
    size_t hl = 0;
    hdr[hl++] = 0x0A;
    hl += put_varint(hdr + hl, st.bytes);
    uint8_t* data = buf.get() + ReplyPool::kHead + req.offset % 16;
    std::memcpy(data - hl, hdr, hl);
    ReadResult rr;
    GrpcReply bad = read_to(data, &rr);
    if (bad.status > 0) return bad;
    if (bad.status < 0) return {};  // corrupt / vanished: the Python service recovers
    if (rr.partial_corrupt) fp_->add_suspect(req.block_id);
    *handled = true;
    uint8_t* end = data + st.bytes;
    if (rr.bytes) {
      *end++ = 0x10;
      end += put_varint(end, rr.bytes);
    }
    if (rr.total_size) {
      *end++ = 0x18;
      end += put_varint(end, rr.total_size);
    }
    reads_++;
    GrpcReply r;
    r.ext = data - hl;
    r.ext_len = static_cast<size_t>(end - (data - hl));
    r.keep = std::move(buf);
    return r;
  }
  std::string out;
  out.reserve(st.bytes + 32);
  out.push_back(0x0A);
  put_varint(out, st.bytes);
  const size_t at = out.size();
  out.resize(at + st.bytes);
  ReadResult rr;
  GrpcReply bad = read_to(reinterpret_cast<uint8_t*>(&out[at]), &rr);
  if (bad.status > 0) return bad;
  if (bad.status < 0) return {};  // corrupt / vanished: the Python service recovers
  if (rr.partial_corrupt) fp_->add_suspect(req.block_id);  // data served, block repaired in the background
  *handled = true;
  if (rr.bytes) {
    out.push_back(0x10);
    put_varint(out, rr.bytes);
  }
  if (rr.total_size) {
    out.push_back(0x18);
    put_varint(out, rr.total_size);
  }
  reads_++;
  return {0, std::move(out)};
}

GrpcReply NativeChunkService::replicate_block(const GrpcCall& call, bool* handled) {
  pb::ReplicateBlockRequest req;
  const uint8_t* data;
  size_t n;
  if (!decode_viewing(req, call.data(), call.size(), 2, &data, &n)) {
    *handled = true;
    return {kInternal, "malformed ReplicateBlockRequest"};
  }
  if (!native_ && (req.rccl || req.heal || !req.next_servers.empty())) return {};
  *handled = true;
  TraceRange tr("dfs.grpc.replicate_block");
  std::string msg;
  if (!fence(req.master_term, &msg)) return {kFailedPrecondition, msg};
  pb::ReplicateBlockResponse resp;
  WriteResult w;
  int replicas = 0;
  std::string perr;
  if (req.rccl) {
    // the payload is on the replication engine; this call carries its descriptor
    ReplicationEngine* e = fp_->replication();
    if (!e) {
      resp.error_message = "RCCL transport not enabled";
      return {0, resp.str()};
    }
    w = e->recv(req.rccl_src_rank, req.rccl_gen, req.rccl_channel, req.rccl_seq, req.block_id, req.rccl_size,
                req.rccl_slice, req.expected_checksum_crc32c, req.next_servers.empty());
    if (w.ok && req.next_servers.empty()) replicas = 1;
    else if (w.ok)
      store_and_forward(req.block_id, nullptr, req.rccl_size, req.next_servers, req.expected_checksum_crc32c,
                        req.master_term, req.heal, call.request_id, &replicas, &perr, true);
  } else if (req.next_servers.empty()) {
    w = store_->write(req.block_id, data, n, req.expected_checksum_crc32c);
    replicas = w.ok ? 1 : 0;
  } else {
    w = store_->stage(req.block_id, data, n, req.expected_checksum_crc32c);
    if (w.ok)
      store_and_forward(req.block_id, data, n, req.next_servers, req.expected_checksum_crc32c, req.master_term,
                        req.heal, call.request_id, &replicas, &perr, store_->gpu());
  }
  resp.success = w.ok && replicas > 0;
  resp.replicas_written = resp.success ? replicas : 0;
  if (!w.ok) resp.error_message = w.error.rfind("Checksum mismatch", 0) == 0 ? "Replication c" + w.error.substr(1) : w.error;
  else if (!resp.success) resp.error_message = perr;
  if (resp.success) {
    replicates_++;
    if (req.heal && agent_) agent_->report_new_block(req.block_id);  // a new location for the masters
  }
  return {0, resp.str()};
}

}  // namespace dfs
