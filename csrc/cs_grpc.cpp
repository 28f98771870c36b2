#include "cs_grpc.h"

#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "dfs_pb.h"
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
  return {writes_.load(), reads_.load(), replicates_.load(), fallbacks_.load()};
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

GrpcReply NativeChunkService::write_block(const GrpcCall& call, bool* handled) {
  pb::WriteBlockRequest req;
  const uint8_t* data;
  size_t n;
  if (!decode_viewing(req, call.data(), call.size(), 2, &data, &n)) {
    *handled = true;
    return {kInternal, "malformed WriteBlockRequest"};
  }
  // shm-in-gRPC writes and chains that leave the host (or lack a P2P pair) stay in Python
  if (!req.shm_path.empty() || !(req.next_servers.empty() || fp_->p2p_ready(req.next_servers))) return {};
  *handled = true;
  TraceRange tr("dfs.grpc.write_block");
  std::string msg;
  if (!fence(req.master_term, &msg)) return {kFailedPrecondition, msg};
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
    } else {
      int down = 0;
      std::string perr;
      bool pok = fp_->persist_and_replicate(req.block_id, data, n, req.expected_checksum_crc32c, req.master_term,
                                            req.next_servers, &down, &perr);
      resp.success = pok;
      resp.error_message = pok ? "" : perr;
      resp.replicas_written = pok ? 1 + down : 0;
    }
  }
  if (resp.success) writes_++;
  return {0, resp.str()};
}

GrpcReply NativeChunkService::read_block(const GrpcCall& call, bool* handled) {
  pb::ReadBlockRequest req;
  if (!req.decode(call.data(), call.size())) {
    *handled = true;
    return {kInternal, "malformed ReadBlockRequest"};
  }
  if (!req.shm_path.empty()) return {};
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
  if (st.status != ReadStatus::Ok) return {};
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
    ReadResult rr = store_->read_into(req.block_id, req.offset, st.bytes, data);
    if (rr.status != ReadStatus::Ok) return {};  // corrupt / vanished: the Python service recovers
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
  ReadResult rr = store_->read_into(req.block_id, req.offset, st.bytes, reinterpret_cast<uint8_t*>(&out[at]));
  if (rr.status != ReadStatus::Ok) return {};  // corrupt / vanished: the Python service recovers
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
  if (req.rccl || req.heal || !req.next_servers.empty()) return {};
  *handled = true;
  TraceRange tr("dfs.grpc.replicate_block");
  std::string msg;
  if (!fence(req.master_term, &msg)) return {kFailedPrecondition, msg};
  WriteResult w = store_->write(req.block_id, data, n, req.expected_checksum_crc32c);
  pb::ReplicateBlockResponse resp;
  resp.success = w.ok;
  resp.replicas_written = w.ok ? 1 : 0;
  if (!w.ok) resp.error_message = w.error.rfind("Checksum mismatch", 0) == 0 ? "Replication c" + w.error.substr(1) : w.error;
  if (w.ok) replicates_++;
  return {0, resp.str()};
}

}  // namespace dfs
