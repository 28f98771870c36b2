// aws-chunked body decoding (the SigV4 streaming upload framing, reference
// dfs/common/src/auth/chunked.rs:5-57 and handlers.rs:291-320,931-935): a sequence of
//   <hex size>[;chunk-signature=<sig>]\r\n<size bytes>\r\n
// ending with a zero-size chunk, then optional trailers. With a chain (a signed stream,
// x-amz-content-sha256 = STREAMING-AWS4-HMAC-SHA256-PAYLOAD) every chunk's signature must
// extend the seed signature's chain, and the stream must end with its signed empty chunk.
//
// The source is anything with
//   int line(std::string* out, size_t max);   // one CRLF-terminated line (max 0: must be empty)
//   int read(uint8_t* dst, uint64_t n);       // exactly n bytes
//   int drain();                              // whatever follows (trailers, closing CRLF)
// each returning 1 ok, 0 connection error, -1 malformed / ended early. The S3 front decodes
// straight from the socket into a transfer slot; the unit tests decode from memory.
#pragma once
#include <cstdint>
#include <string>

#include "sigv4.h"

namespace dfs {

struct AwsChunkedResult {
  int rc = 0;          // 1 ok, 0 connection error, -1 bad framing / signature
  uint64_t bytes = 0;  // decoded payload bytes
  uint64_t sigs = 0;   // chunk signatures verified
};

namespace aws_chunked_detail {
inline std::string trim(const std::string& s) {
  size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t\r");
  return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}
}  // namespace aws_chunked_detail

template <class Src>
AwsChunkedResult decode_aws_chunked(Src& in, sigv4::ChunkChain* chain, uint8_t* dst, uint64_t cap) {
  using aws_chunked_detail::trim;
  AwsChunkedResult res;
  uint64_t n = 0;
  bool final_chunk = false;
  for (;;) {
    std::string h;
    int rc = in.line(&h, 4096);
    if (rc == -1 && !chain && n > 0) break;  // the body ended without its empty chunk
    if (rc != 1) {
      res.rc = rc;
      return res;
    }
    const size_t semi = h.find(';');
    const std::string hex = trim(h.substr(0, semi));
    if (hex.size() > 15 || hex.find_first_not_of("0123456789abcdefABCDEF") != std::string::npos) {
      res.rc = -1;
      return res;
    }
    const uint64_t size = hex.empty() ? 0 : std::stoull(hex, nullptr, 16);
    if (size > cap || n > cap - size) {
      res.rc = -1;
      return res;
    }
    if ((rc = in.read(dst + n, size)) != 1) {
      res.rc = rc;
      return res;
    }
    if (chain) {
      std::string sig;
      if (semi != std::string::npos) {
        size_t k = h.find("chunk-signature=", semi);
        if (k != std::string::npos) sig = trim(h.substr(k + 16));
      }
      if (!chain->verify(dst + n, size, sig)) {
        res.rc = -1;
        return res;
      }
      ++res.sigs;
    }
    if (size == 0) {
      final_chunk = true;
      break;
    }
    n += size;
    std::string crlf;
    if ((rc = in.line(&crlf, 0)) != 1) {
      res.rc = rc;
      return res;
    }
    if (!crlf.empty()) {
      res.rc = -1;
      return res;
    }
  }
  if (chain && !final_chunk) {  // a signed stream ends with its signed empty chunk
    res.rc = -1;
    return res;
  }
  res.rc = in.drain();  // trailers (x-amz-checksum-*) and the closing CRLF
  res.bytes = n;
  return res;
}

}  // namespace dfs
