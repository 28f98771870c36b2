#include "cs_grpc.h"

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
}  // namespace

NativeChunkService::NativeChunkService(ChunkStore* store, FastPathServer* fp, Fallback fallback)
    : store_(store), fp_(fp), fallback_(std::move(fallback)) {}

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
  return fallback_(call);
}

GrpcReply NativeChunkService::write_block(const GrpcCall& call, bool* handled) {
  pb::WriteBlockRequest req;
  if (!req.decode(call.message)) {
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
  const auto* data = reinterpret_cast<const uint8_t*>(req.data.data());
  const uint64_t n = req.data.size();
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
  if (!req.decode(call.message)) {
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
  if (!req.decode(call.message)) {
    *handled = true;
    return {kInternal, "malformed ReplicateBlockRequest"};
  }
  if (req.rccl || req.heal || !req.next_servers.empty()) return {};
  *handled = true;
  TraceRange tr("dfs.grpc.replicate_block");
  std::string msg;
  if (!fence(req.master_term, &msg)) return {kFailedPrecondition, msg};
  WriteResult w = store_->write(req.block_id, reinterpret_cast<const uint8_t*>(req.data.data()), req.data.size(),
                                req.expected_checksum_crc32c);
  pb::ReplicateBlockResponse resp;
  resp.success = w.ok;
  resp.replicas_written = w.ok ? 1 : 0;
  if (!w.ok) resp.error_message = w.error.rfind("Checksum mismatch", 0) == 0 ? "Replication c" + w.error.substr(1) : w.error;
  if (w.ok) replicates_++;
  return {0, resp.str()};
}

}  // namespace dfs
