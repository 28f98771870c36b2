// Native S3 front end; design notes in s3_front.h.
#include "s3_front.h"
#include "audit_json.h"
#include "aws_chunked.h"
#include <unordered_set>
#include <unordered_map>
#include <set>
#include "crypto.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstring>
#include <ctime>
#include <future>
#include <random>

#include "dfs_pb.h"
#include "json.h"
#include "sigv4.h"
#include "trace.h"

namespace dfs {

namespace {

constexpr size_t kMaxHead = 64 << 10;
constexpr size_t kRelayChunk = 256 << 10;
const char* kEmptyEtag = "\"d41d8cd98f00b204e9800998ecf8427e\"";
const char* kUnsigned = "UNSIGNED-PAYLOAD";
const char* kHidden[] = {".s3keep", ".s3_mpu_completed", ".meta", ".s3_bucket_policy"};

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

std::string lower(std::string s) {
  for (auto& ch : s) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
  return s;
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace(static_cast<unsigned char>(s[a]))) ++a;
  while (b > a && std::isspace(static_cast<unsigned char>(s[b - 1]))) --b;
  return s.substr(a, b - a);
}

// " ".join(v.split()): the SigV4 canonical header value
std::string collapse_ws(const std::string& v) {
  std::string o;
  bool sp = false;
  for (char ch : v) {
    if (std::isspace(static_cast<unsigned char>(ch))) {
      sp = !o.empty();
    } else {
      if (sp) o.push_back(' ');
      sp = false;
      o.push_back(ch);
    }
  }
  return o;
}

bool ends_with(const std::string& s, const char* suf) {
  size_t n = std::strlen(suf);
  return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

bool reserved_key(const std::string& key) {
  for (const char* h : kHidden)
    if (ends_with(key, h)) return true;
  return false;
}

bool send_all(int fd, const void* p, size_t n) {
  const auto* b = static_cast<const uint8_t*>(p);
  while (n) {
    ssize_t w = ::send(fd, b, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    b += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

bool send_head_body(int fd, const std::string& head, const uint8_t* body, size_t n) {
  if (n == 0 || n + head.size() <= (16 << 10)) {
    if (n == 0) return send_all(fd, head.data(), head.size());
    std::string all = head;
    all.append(reinterpret_cast<const char*>(body), n);
    return send_all(fd, all.data(), all.size());
  }
  iovec iv[2] = {{const_cast<char*>(head.data()), head.size()}, {const_cast<uint8_t*>(body), n}};
  msghdr mh{};
  mh.msg_iov = iv;
  mh.msg_iovlen = 2;
  ssize_t w;
  do {
    w = ::sendmsg(fd, &mh, MSG_NOSIGNAL);
  } while (w < 0 && errno == EINTR);
  if (w < 0) return false;
  size_t done = static_cast<size_t>(w);
  if (done < head.size()) {
    if (!send_all(fd, head.data() + done, head.size() - done)) return false;
    done = head.size();
  }
  size_t bo = done - head.size();
  return send_all(fd, body + bo, n - bo);
}

// One end of a relay or response: a plain socket, or a TLS session on it (the front's
// client connections when the gateway terminates TLS; the backend socket is always plain).
struct Io {
  int fd = -1;
  TlsConn* tls = nullptr;
};

long io_recv(Io io, void* p, size_t n) {
  if (io.tls) return io.tls->read(p, n);  // blocking socket: >0 bytes, -1 closed / error
  for (;;) {
    ssize_t k = ::recv(io.fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    return k;
  }
}

bool send_all(Io io, const void* p, size_t n) {
  if (!io.tls) return send_all(io.fd, p, n);
  return io.tls->write_all(p, n, std::chrono::steady_clock::now() + std::chrono::seconds(300));
}

bool send_head_body(Io io, const std::string& head, const uint8_t* body, size_t n) {
  if (!io.tls) return send_head_body(io.fd, head, body, n);
  if (n + head.size() <= (16 << 10)) {  // one TLS record for a small response
    std::string all = head;
    if (n) all.append(reinterpret_cast<const char*>(body), n);
    return send_all(io, all.data(), all.size());
  }
  return send_all(io, head.data(), head.size()) && send_all(io, body, n);
}

std::string http_date(uint64_t ms) {
  if (ms == 0) return "Wed, 01 Jan 2025 00:00:00 GMT";
  time_t t = static_cast<time_t>(ms / 1000);
  tm g{};
  gmtime_r(&t, &g);
  char b[64];
  std::strftime(b, sizeof b, "%a, %d %b %Y %H:%M:%S GMT", &g);
  return b;
}

std::string iso_now(double t, int64_t* ms_out) {
  time_t s = static_cast<time_t>(t);
  long us = static_cast<long>((t - static_cast<double>(s)) * 1e6);
  tm g{};
  gmtime_r(&s, &g);
  char b[64];
  std::strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%S", &g);
  std::string o = b;
  if (us) {
    char u[16];
    std::snprintf(u, sizeof u, ".%06ld", us);
    o += u;
  }
  *ms_out = static_cast<int64_t>(t * 1000);
  return o + "+00:00";
}

std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (unsigned char ch : s) {
    switch (ch) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (ch < 0x20) {
          char u[8];
          std::snprintf(u, sizeof u, "\\u%04x", ch);
          o += u;
        } else {
          o.push_back(static_cast<char>(ch));
        }
    }
  }
  return o + "\"";
}

std::string uuid4() {
  static thread_local std::mt19937_64 rng{std::random_device{}()};
  uint64_t a = rng(), b = rng();
  a = (a & 0xffffffffffff0fffull) | 0x4000ull;
  b = (b & 0x3fffffffffffffffull) | 0x8000000000000000ull;
  char s[40];
  std::snprintf(s, sizeof s, "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
                static_cast<unsigned>((a >> 16) & 0xffff), static_cast<unsigned>(a & 0xffff),
                static_cast<unsigned>(b >> 48), static_cast<unsigned long long>(b & 0xffffffffffffull));
  return s;
}

bool all_digits(const std::string& s) {
  if (s.empty() || s.size() > 18) return false;
  for (char ch : s)
    if (ch < '0' || ch > '9') return false;
  return true;
}

// parse_range of tests/models/s3_gateway.py: 0 = no (or ignored) range, 1 = [*s, *e], 2 = unsatisfiable,
// 3 = a form this path does not decide (handed to Python)
int parse_range(const std::string* v, uint64_t size, uint64_t* s, uint64_t* e) {
  if (!v || v->compare(0, 6, "bytes=") != 0) return 0;
  std::string spec = trim(v->substr(6));
  if (spec.find(',') != std::string::npos || spec.find('-') == std::string::npos) return 0;
  std::string a = spec.substr(0, spec.find('-')), b = spec.substr(spec.find('-') + 1);
  if (a.empty()) {
    if (!all_digits(b)) return 3;
    uint64_t n = std::stoull(b);
    if (n == 0 || size == 0) return 2;
    *s = size > n ? size - n : 0;
    *e = size - 1;
    return 1;
  }
  if (!all_digits(a) || (!b.empty() && !all_digits(b))) return 3;
  uint64_t start = std::stoull(a);
  uint64_t end = b.empty() ? (size ? size - 1 : 0) : std::stoull(b);
  if (start >= size) return 2;
  end = std::min(end, size - 1);
  if (end < start) return 0;
  *s = start;
  *e = end;
  return 1;
}

// parse_qsl(keep_blank_values=True) for the keys this path looks at (no '%' or '+' handled:
// such queries go to Python)
bool simple_query(const std::string& q, std::map<std::string, std::string>* out) {
  size_t i = 0;
  while (i <= q.size() && !q.empty()) {
    size_t amp = q.find('&', i);
    std::string kv = q.substr(i, amp == std::string::npos ? std::string::npos : amp - i);
    if (kv.find('%') != std::string::npos || kv.find('+') != std::string::npos) return false;
    if (!kv.empty()) {
      size_t eq = kv.find('=');
      (*out)[kv.substr(0, eq)] = eq == std::string::npos ? "" : kv.substr(eq + 1);
    }
    if (amp == std::string::npos) break;
    i = amp + 1;
  }
  return true;
}

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

// parse_qsl(raw, keep_blank_values=True) of the Python gateway: '+' is a space, %XX a byte,
// a malformed escape stays as written. False on bytes that are not UTF-8 (Python would
// substitute U+FFFD; the request goes there).
// The request path percent-decoded as the gateway routes it ('+' stays itself in a path);
// false for a bad escape, a NUL or invalid UTF-8.
bool decode_path(const std::string& raw, std::string* o) {
  o->clear();
  for (size_t i = 0; i < raw.size(); ++i) {
    if (raw[i] != '%') {
      o->push_back(raw[i]);
      continue;
    }
    if (i + 2 >= raw.size() || hexval(raw[i + 1]) < 0 || hexval(raw[i + 2]) < 0) return false;
    o->push_back(static_cast<char>(hexval(raw[i + 1]) * 16 + hexval(raw[i + 2])));
    i += 2;
  }
  for (size_t i = 0; i < o->size();) {
    unsigned char c0 = static_cast<unsigned char>((*o)[i]);
    int n = c0 < 0x80 ? 1 : (c0 >> 5) == 6 ? 2 : (c0 >> 4) == 14 ? 3 : (c0 >> 3) == 30 ? 4 : 0;
    if (!n || c0 == 0 || i + n > o->size()) return false;
    for (int k = 1; k < n; ++k)
      if ((static_cast<unsigned char>((*o)[i + k]) >> 6) != 2) return false;
    i += static_cast<size_t>(n);
  }
  return true;
}

bool decode_query(const std::string& q, std::map<std::string, std::string>* out) {
  auto dec = [](const std::string& v, std::string* o) {
    o->clear();
    for (size_t i = 0; i < v.size(); ++i) {
      if (v[i] == '+') {
        o->push_back(' ');
      } else if (v[i] == '%' && i + 2 < v.size() && hexval(v[i + 1]) >= 0 && hexval(v[i + 2]) >= 0) {
        o->push_back(static_cast<char>(hexval(v[i + 1]) * 16 + hexval(v[i + 2])));
        i += 2;
      } else {
        o->push_back(v[i]);
      }
    }
    // strict UTF-8
    for (size_t i = 0; i < o->size();) {
      unsigned char c0 = static_cast<unsigned char>((*o)[i]);
      int n = c0 < 0x80 ? 1 : (c0 >> 5) == 6 ? 2 : (c0 >> 4) == 14 ? 3 : (c0 >> 3) == 30 ? 4 : 0;
      if (!n || i + n > o->size()) return false;
      for (int k = 1; k < n; ++k)
        if ((static_cast<unsigned char>((*o)[i + k]) >> 6) != 2) return false;
      i += static_cast<size_t>(n);
    }
    return true;
  };
  size_t i = 0;
  while (!q.empty() && i <= q.size()) {
    size_t amp = q.find('&', i);
    std::string kv = q.substr(i, amp == std::string::npos ? std::string::npos : amp - i);
    if (!kv.empty()) {
      size_t eq = kv.find('=');
      std::string k, v;
      if (!dec(kv.substr(0, eq), &k) || !dec(eq == std::string::npos ? "" : kv.substr(eq + 1), &v)) return false;
      (*out)[k] = v;
    }
    if (amp == std::string::npos) break;
    i = amp + 1;
  }
  return true;
}

// xml.sax.saxutils.escape
std::string xml_escape(const std::string& v) {
  std::string o;
  o.reserve(v.size());
  for (char ch : v) {
    if (ch == '&') o += "&amp;";
    else if (ch == '<') o += "&lt;";
    else if (ch == '>') o += "&gt;";
    else o.push_back(ch);
  }
  return o;
}

std::string xel(const char* tag, const std::string& v) {
  return std::string("<") + tag + ">" + xml_escape(v) + "</" + tag + ">";
}

// _iso_ms: seconds precision, ".000Z"
std::string iso_ms(uint64_t ms) {
  if (!ms) return "2025-01-01T00:00:00.000Z";
  time_t t = static_cast<time_t>(ms / 1000);
  tm g{};
  gmtime_r(&t, &g);
  char b[40];
  std::strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%S.000Z", &g);
  return b;
}

}  // namespace

struct S3Front::Conn {
  int fd = -1;
  std::string ip;
  std::string buf;
  size_t pos = 0;
  std::unique_ptr<TlsConn> tls;  // TLS terminated here (cfg_.tls_cert)
  Io io() const { return Io{fd, tls.get()}; }
};

struct S3Front::Req {
  std::string method, target, raw_path, raw_query, version;
  std::string path;  // raw_path percent-decoded (the signature covers raw_path)
  std::vector<std::pair<std::string, std::string>> headers;  // (lower-case name, value)
  std::vector<std::string> names;                            // names as sent
  bool keep_alive = true, chunked = false, expect_continue = false;
  bool secure = false;  // arrived over the front's own TLS
  int64_t content_length = 0;
  double started = 0;
  std::string rid;
  std::string action;  // s3:<Action> once resolved for authorization (audit records)
  int status = 0;
  std::map<std::string, std::string> presign;  // X-Amz-* query authentication (presigned URL)
  // why authentication failed, as the gateway reports it (auth/errors.py kind, the audit
  // record's error code when it differs, the access key / role that were presented)
  std::string auth_kind, auth_audit, auth_user = "anonymous", auth_role;
  sigv4::ChunkChain chain;                      // set by a verified signature: aws-chunked bodies
  bool chain_set = false;
  const std::string* get(const char* lname) const {
    for (auto& h : headers)
      if (h.first == lname) return &h.second;
    return nullptr;
  }
};

namespace {

// an aws-chunked body (x-amz-content-sha256: STREAMING-..., or Content-Encoding: aws-chunked)
bool aws_chunked(const S3Front::Req& r) {
  const std::string* sha = r.get("x-amz-content-sha256");
  const std::string* enc = r.get("content-encoding");
  return (sha && sha->compare(0, 10, "STREAMING-") == 0) || (enc && enc->find("aws-chunked") != std::string::npos);
}

// repr() of a Python str, for the messages the gateway formats with {key!r}
std::string py_repr(const std::string& v) {
  const char q = v.find('\'') != std::string::npos && v.find('"') == std::string::npos ? '"' : '\'';
  std::string o(1, q);
  for (unsigned char ch : v) {
    if (ch == '\\') o += "\\\\";
    else if (ch == static_cast<unsigned char>(q)) o += std::string("\\") + q;
    else if (ch == '\n') o += "\\n";
    else if (ch == '\r') o += "\\r";
    else if (ch == '\t') o += "\\t";
    else if (ch < 0x20 || ch == 0x7f) {
      char u[8];
      std::snprintf(u, sizeof u, "\\x%02x", ch);
      o += u;
    } else {
      o.push_back(static_cast<char>(ch));
    }
  }
  return o + q;
}

// urllib.parse.unquote for the copy source: %XX decoded, '+' kept; false when the result is
// not UTF-8 (Python would substitute U+FFFD: the request goes there)
bool unquote(const std::string& v, std::string* o) {
  std::map<std::string, std::string> m;
  std::string enc;
  for (char ch : v) enc += ch == '+' ? std::string("%2B") : ch == '&' ? std::string("%26") : ch == '=' ? std::string("%3D") : std::string(1, ch);
  if (!decode_query("k=" + enc, &m)) return false;
  *o = m["k"];
  return true;
}

// "n:size,..." of a completion marker (x-dfs-mpu-layout)
bool parse_layout(const std::string& lay, std::vector<std::pair<uint64_t, uint64_t>>* parts) {
  parts->clear();
  for (size_t a = 0; a < lay.size();) {
    size_t b = lay.find(',', a);
    std::string kv = lay.substr(a, b == std::string::npos ? std::string::npos : b - a);
    size_t colon = kv.find(':');
    if (colon == std::string::npos || !all_digits(kv.substr(0, colon)) || !all_digits(kv.substr(colon + 1)))
      return false;
    parts->emplace_back(std::stoull(kv.substr(0, colon)), std::stoull(kv.substr(colon + 1)));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  return true;
}

// A small XML reader for request bodies (DeleteObjects): elements by local name (namespace
// prefix dropped, as tests/models/s3_xml.py's _local does), each with ElementTree's .text (character data
// before the first child). False for anything outside this subset — comments, CDATA, DTDs,
// unknown entities, mismatched tags: Python's ElementTree decides those.
struct XNode {
  std::string qname, name, text;
  std::vector<XNode> kids;
  const XNode* child(const char* n) const {
    for (auto& k : kids)
      if (k.name == n) return &k;
    return nullptr;
  }
};

bool xml_unescape(const std::string& raw, std::string* o) {
  o->clear();
  for (size_t k = 0; k < raw.size(); ++k) {
    char ch = raw[k];
    if (ch == '\r') {  // XML end-of-line handling: \r\n and lone \r become \n
      if (k + 1 < raw.size() && raw[k + 1] == '\n') ++k;
      o->push_back('\n');
      continue;
    }
    if (ch != '&') {
      o->push_back(ch);
      continue;
    }
    size_t e = raw.find(';', k);
    if (e == std::string::npos || e - k > 12) return false;
    const std::string ent = raw.substr(k + 1, e - k - 1);
    k = e;
    if (ent == "amp") o->push_back('&');
    else if (ent == "lt") o->push_back('<');
    else if (ent == "gt") o->push_back('>');
    else if (ent == "quot") o->push_back('"');
    else if (ent == "apos") o->push_back('\'');
    else if (ent.size() > 1 && ent[0] == '#') {
      const bool hx = ent[1] == 'x';
      const std::string num = ent.substr(hx ? 2 : 1);
      if (num.empty() || num.find_first_not_of(hx ? "0123456789abcdefABCDEF" : "0123456789") != std::string::npos)
        return false;
      unsigned long cp = std::stoul(num, nullptr, hx ? 16 : 10);
      if (cp == 0 || cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
      if (cp < 0x80) {
        o->push_back(static_cast<char>(cp));
      } else if (cp < 0x800) {
        o->push_back(static_cast<char>(0xC0 | (cp >> 6)));
        o->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
      } else if (cp < 0x10000) {
        o->push_back(static_cast<char>(0xE0 | (cp >> 12)));
        o->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
        o->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
      } else {
        o->push_back(static_cast<char>(0xF0 | (cp >> 18)));
        o->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
        o->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
        o->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
      }
    } else {
      return false;
    }
  }
  return true;
}

bool parse_xml(const std::string& b, XNode* root) {
  std::vector<XNode*> stack;
  bool have_root = false, closed = false;
  std::string text;
  auto flush = [&]() {
    if (stack.empty() || !stack.back()->kids.empty()) {  // outside the root, or a tail
      bool ws = text.find_first_not_of(" \t\r\n") == std::string::npos;
      text.clear();
      return ws || !stack.empty();
    }
    std::string v;
    if (!xml_unescape(text, &v)) return false;
    stack.back()->text += v;
    text.clear();
    return true;
  };
  size_t i = 0;
  while (i < b.size()) {
    if (b[i] != '<') {
      text.push_back(b[i++]);
      continue;
    }
    if (!flush()) return false;
    size_t j = i + 1;
    char quote = 0;
    for (; j < b.size(); ++j) {
      if (quote) {
        if (b[j] == quote) quote = 0;
      } else if (b[j] == '"' || b[j] == '\'') {
        quote = b[j];
      } else if (b[j] == '>') {
        break;
      }
    }
    if (j >= b.size()) return false;
    std::string tag = b.substr(i + 1, j - i - 1);
    i = j + 1;
    if (tag.empty() || tag[0] == '!') return false;
    if (tag[0] == '?') {
      if (have_root) return false;
      continue;
    }
    const bool closing = tag[0] == '/', empty_el = !closing && tag.back() == '/';
    std::string qn = closing ? tag.substr(1) : empty_el ? tag.substr(0, tag.size() - 1) : tag;
    qn = qn.substr(0, qn.find_first_of(" \t\r\n"));
    if (qn.empty()) return false;
    if (closing) {
      if (stack.empty() || stack.back()->qname != qn) return false;
      stack.pop_back();
      if (stack.empty()) closed = true;
      continue;
    }
    if (closed || (stack.empty() && have_root)) return false;
    XNode* node;
    if (stack.empty()) {
      *root = XNode{};
      node = root;
      have_root = true;
    } else {
      stack.back()->kids.emplace_back();
      node = &stack.back()->kids.back();
    }
    node->qname = qn;
    size_t colon = qn.find(':');
    node->name = colon == std::string::npos ? qn : qn.substr(colon + 1);
    if (!empty_el) stack.push_back(node);
    else if (stack.empty()) closed = true;
  }
  if (!text.empty() && text.find_first_not_of(" \t\r\n") != std::string::npos) return false;
  return have_root && closed && stack.empty();
}

// Runs fn(i) for i in [0, n) on up to `width` pool threads (the pool grows per task, so a
// bulk request must not submit one task per item).
template <class F>
void parallel_for(IoPool& pool, size_t n, size_t width, F fn) {
  if (n <= 1) {
    if (n) fn(0);
    return;
  }
  std::atomic<size_t> next{0};
  std::vector<std::future<void>> fs;
  for (size_t w = 0; w < std::min(n, width); ++w)
    fs.push_back(pool.submit([&] {
      for (size_t i; (i = next.fetch_add(1)) < n;) fn(i);
    }));
  for (auto& f : fs) f.get();
}

}  // namespace

S3Front::S3Front(S3FrontConfig cfg, FastClient* fc)
    : cfg_(std::move(cfg)), own_store_(std::make_unique<FastFrontStore>(fc)), fc_(own_store_.get()) {}

S3Front::S3Front(S3FrontConfig cfg, FrontStore* store) : cfg_(std::move(cfg)), fc_(store) {}

S3Front::~S3Front() {
  stop();
  if (epoch_map_) ::munmap(epoch_map_, 4096);
}

bool S3Front::start(std::string* err) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  int one = 1;
  ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (cfg_.reuse_port) ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(cfg_.port));
  if (cfg_.host.empty() || cfg_.host == "0.0.0.0") a.sin_addr.s_addr = INADDR_ANY;
  else if (::inet_pton(AF_INET, cfg_.host == "localhost" ? "127.0.0.1" : cfg_.host.c_str(), &a.sin_addr) != 1) {
    *err = "bad bind address " + cfg_.host;
    return false;
  }
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || ::listen(lfd_, 1024) != 0) {
    *err = std::string("bind/listen: ") + std::strerror(errno);
    ::close(lfd_);
    lfd_ = -1;
    return false;
  }
  socklen_t al = sizeof a;
  ::getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &al);
  cfg_.port = ntohs(a.sin_port);
  for (auto& kv : cfg_.sts_keys) {
    std::string k = kv.second;
    k.resize(32, '\0');  // _key32: zero-padded / truncated to 32 bytes
    sts_keys_[kv.first] = k;
  }
  if (!cfg_.iam_config.empty()) {
    try {
      iam_ = std::make_unique<s3policy::IamPolicy>(s3policy::IamPolicy::parse(cfg_.iam_config));
    } catch (const std::exception& e) {
      *err = std::string("IAM config: ") + e.what();
      ::close(lfd_);
      lfd_ = -1;
      return false;
    }
  }
  if (!cfg_.oidc_issuer.empty() && !cfg_.oidc_client_id.empty())
    oidc_ = std::make_unique<sts::OidcValidator>(cfg_.oidc_issuer, cfg_.oidc_client_id, cfg_.oidc_allow_hs256,
                                                 cfg_.oidc_ca);
  if (!cfg_.tls_cert.empty()) {
    tls_ = TlsContext::server_http1(cfg_.tls_cert, cfg_.tls_key, err);
    if (!tls_) {
      ::close(lfd_);
      lfd_ = -1;
      return false;
    }
  }
  if (!cfg_.audit_socket.empty()) audit_fd_ = ::socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
  if (!cfg_.policy_epoch_path.empty()) {
    int efd = ::open(cfg_.policy_epoch_path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
    if (efd >= 0) {
      struct stat sb {};
      if (::fstat(efd, &sb) == 0 && sb.st_size < 4096 && ::ftruncate(efd, 4096) != 0) {
        ::close(efd);
        efd = -1;
      }
    }
    void* m = efd < 0 ? MAP_FAILED : ::mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, efd, 0);
    if (efd >= 0) ::close(efd);
    if (m == MAP_FAILED) {
      *err = "policy epoch " + cfg_.policy_epoch_path + ": " + std::strerror(errno);
      ::close(lfd_);
      lfd_ = -1;
      return false;
    }
    epoch_map_ = static_cast<uint64_t*>(m);
    cache_epoch_ = policy_epoch();
  }
  epfd_ = ::epoll_create1(EPOLL_CLOEXEC);
  evfd_ = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.u64 = 0;  // the listener
  ::epoll_ctl(epfd_, EPOLL_CTL_ADD, lfd_, &ev);
  ev.data.u64 = 1;  // stop
  ::epoll_ctl(epfd_, EPOLL_CTL_ADD, evfd_, &ev);
  for (int i = 0; i < std::max(1, cfg_.workers); ++i) workers_.emplace_back([this] { worker_loop(); });
  epoller_ = std::thread([this] { epoll_loop(); });
  return true;
}

void S3Front::stop() {
  if (stop_.exchange(true)) return;
  if (evfd_ >= 0) {
    uint64_t one = 1;
    (void)!::write(evfd_, &one, sizeof one);
  }
  if (epoller_.joinable()) epoller_.join();
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (auto& kv : conns_) ::shutdown(kv.first, SHUT_RDWR);
  }
  q_cv_.notify_all();
  for (auto& t : workers_)
    if (t.joinable()) t.join();
  workers_.clear();
  {
    std::lock_guard<std::mutex> g(conns_mu_);
    for (auto& kv : conns_) {
      ::close(kv.first);
      delete kv.second;
    }
    conns_.clear();
  }
  ready_.clear();  // the connections themselves were owned (and freed) through conns_
  {
    std::lock_guard<std::mutex> g(be_mu_);
    for (int fd : be_idle_) ::close(fd);
    be_idle_.clear();
  }
  for (int* fd : {&lfd_, &epfd_, &evfd_, &audit_fd_})
    if (*fd >= 0) {
      ::close(*fd);
      *fd = -1;
    }
}

S3FrontStats S3Front::stats() {
  std::lock_guard<std::mutex> g(st_mu_);
  return st_;
}

void S3Front::epoll_loop() {
  epoll_event evs[64];
  while (!stop_.load()) {
    int n = ::epoll_wait(epfd_, evs, 64, 500);
    for (int i = 0; i < n; ++i) {
      if (evs[i].data.u64 == 1) return;
      if (evs[i].data.u64 == 0) {
        for (;;) {
          sockaddr_in pa{};
          socklen_t pl = sizeof pa;
          int fd = ::accept4(lfd_, reinterpret_cast<sockaddr*>(&pa), &pl, SOCK_CLOEXEC);
          if (fd < 0) break;
          int one = 1;
          ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
          timeval tv{300, 0};
          ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
          ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
          auto* c = new Conn();
          c->fd = fd;
          char ip[INET_ADDRSTRLEN] = "unknown";
          ::inet_ntop(AF_INET, &pa.sin_addr, ip, sizeof ip);
          c->ip = ip;
          {
            std::lock_guard<std::mutex> g(conns_mu_);
            conns_[fd] = c;
          }
          {
            std::lock_guard<std::mutex> g(st_mu_);
            st_.connections++;
          }
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP | EPOLLONESHOT;
          ev.data.ptr = c;
          ::epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev);
        }
        continue;
      }
      {
        std::lock_guard<std::mutex> g(q_mu_);
        ready_.push_back(static_cast<Conn*>(evs[i].data.ptr));
      }
      q_cv_.notify_one();
    }
  }
}

void S3Front::worker_loop() {
  for (;;) {
    Conn* c;
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      q_cv_.wait(lk, [this] { return stop_.load() || !ready_.empty(); });
      if (stop_.load()) return;
      c = ready_.front();
      ready_.pop_front();
    }
    serve(c);
  }
}

// ---------------------------------------------------------------- request loop
void S3Front::serve(Conn* c) {
  auto close_conn = [&] {
    ::epoll_ctl(epfd_, EPOLL_CTL_DEL, c->fd, nullptr);
    std::lock_guard<std::mutex> g(conns_mu_);
    conns_.erase(c->fd);
    ::close(c->fd);
    delete c;
  };
  char tmp[64 << 10];
  if (tls_ && !c->tls) {  // first time this connection is served: the TLS handshake
    c->tls = std::make_unique<TlsConn>(tls_, c->fd);
    std::string err;
    if (!c->tls->handshake("", std::chrono::steady_clock::now() + std::chrono::seconds(10), &err)) {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.tls_failures++;
      return close_conn();
    }
    std::lock_guard<std::mutex> g(st_mu_);
    st_.tls_handshakes++;
  }
  for (;;) {
    if (c->pos == c->buf.size()) {
      c->buf.clear();
      c->pos = 0;
      ssize_t n;
      if (c->tls) {
        // decrypted bytes may already sit in the session; otherwise poll the socket once
        pollfd pf{c->fd, POLLIN, 0};
        if (!c->tls->pending() && ::poll(&pf, 1, 0) <= 0) {
          n = -1;
          errno = EAGAIN;
        } else {
          n = c->tls->read(tmp, sizeof tmp);
          if (n < 0) n = 0;  // closed
        }
      } else {
        n = ::recv(c->fd, tmp, sizeof tmp, MSG_DONTWAIT);
      }
      if (n == 0 || (n < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) return close_conn();
      if (n < 0) {  // idle: back to the epoll thread
        epoll_event ev{};
        ev.events = EPOLLIN | EPOLLRDHUP | EPOLLONESHOT;
        ev.data.ptr = c;
        if (stop_.load() || ::epoll_ctl(epfd_, EPOLL_CTL_MOD, c->fd, &ev) != 0) return close_conn();
        return;
      }
      c->buf.append(tmp, static_cast<size_t>(n));
    }
    size_t end;
    while ((end = c->buf.find("\r\n\r\n", c->pos)) == std::string::npos) {
      if (c->buf.size() - c->pos > kMaxHead) return close_conn();
      long n = io_recv(c->io(), tmp, sizeof tmp);
      if (n <= 0) return close_conn();
      c->buf.append(tmp, static_cast<size_t>(n));
    }
    Req r;
    r.started = now_s();
    r.secure = c->tls != nullptr;
    const std::string head = c->buf.substr(c->pos, end - c->pos);
    c->pos = end + 4;
    size_t le = head.find("\r\n");
    std::string line = head.substr(0, le);
    size_t s1 = line.find(' '), s2 = line.rfind(' ');
    if (s1 == std::string::npos || s2 == s1) return close_conn();
    r.method = line.substr(0, s1);
    r.target = line.substr(s1 + 1, s2 - s1 - 1);
    r.version = line.substr(s2 + 1);
    size_t q = r.target.find('?');
    r.raw_path = r.target.substr(0, q);
    r.raw_query = q == std::string::npos ? "" : r.target.substr(q + 1);
    size_t p = le == std::string::npos ? head.size() : le + 2;
    while (p < head.size()) {
      size_t e = head.find("\r\n", p);
      if (e == std::string::npos) e = head.size();
      std::string h = head.substr(p, e - p);
      size_t colon = h.find(':');
      if (colon != std::string::npos) {
        r.names.push_back(h.substr(0, colon));
        r.headers.emplace_back(lower(h.substr(0, colon)), trim(h.substr(colon + 1)));
      }
      p = e + 2;
    }
    const std::string* conn = r.get("connection");
    std::string cl = conn ? lower(*conn) : "";
    r.keep_alive = r.version == "HTTP/1.1" ? cl.find("close") == std::string::npos
                                             : cl.find("keep-alive") != std::string::npos;
    if (const std::string* te = r.get("transfer-encoding")) r.chunked = lower(*te).find("chunked") != std::string::npos;
    if (const std::string* len = r.get("content-length")) {
      if (!all_digits(*len)) return close_conn();
      r.content_length = static_cast<int64_t>(std::stoull(*len));
    }
    if (const std::string* ex = r.get("expect")) r.expect_continue = lower(*ex) == "100-continue";
    const std::string* rid = r.get("x-request-id");
    r.rid = rid ? *rid : std::string();
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.requests++;
    }
    if (!handle(c, r) || !r.keep_alive) return close_conn();
  }
}

// Reads the request body (content_length bytes) into dst: buffered bytes first, then the
// socket straight into the destination (a FastClient slot for PUTs).
static bool read_body(S3Front::Conn* c, uint8_t* dst, uint64_t n);

bool S3Front::handle(Conn* c, Req& r) {
  // keys are routed by their decoded path (as the reference's axum path extractor decodes
  // them); the signature is checked over the path as sent
  if (!decode_path(r.raw_path, &r.path)) return proxy(c, r, nullptr, 0, "uri");
  const bool plain_path = r.path.size() > 1 && r.path[0] == '/';
  std::map<std::string, std::string> q;
  if (r.raw_path == "/metrics" || r.raw_path == "/health") return proxy(c, r, nullptr, 0, "metrics");
  if (r.raw_path == "/" && cfg_.backend.empty()) {  // STS at the root (tests/models/s3_gateway.py dispatch)
    std::map<std::string, std::string> sq;
    const std::string* ct = r.get("content-type");
    const bool form = r.method == "POST" && ct && lower(*ct).compare(0, 33, "application/x-www-form-urlencoded") == 0;
    if (decode_query(r.raw_query, &sq) && (sq["Action"] == "AssumeRoleWithWebIdentity" || form))
      return native_sts(c, r, sq);
  }
  if (fc_ && r.raw_path == "/" && r.method == "GET" && r.content_length <= 0 && !r.chunked)
    return native_list_buckets(c, r);  // ListBuckets takes no query parameters of its own (as the gateway)
  if (!fc_ || !plain_path || !decode_query(r.raw_query, &q)) return proxy(c, r, nullptr, 0, "route");
  // a presigned URL's authentication parameters are not part of the operation
  for (auto it = q.begin(); it != q.end();) {
    if (it->first.compare(0, 6, "X-Amz-") == 0) {
      r.presign.insert(*it);
      it = q.erase(it);
    } else {
      ++it;
    }
  }
  std::string p = r.path.substr(1);
  size_t slash = p.find('/');
  if (slash != 0 && (slash == std::string::npos || slash + 1 == p.size())) {
    const std::string bucket = p.substr(0, slash);
    if (bucket.empty()) return proxy(c, r, nullptr, 0, "route");
    const bool small_body = !r.chunked && r.content_length <= (1 << 20) && !aws_chunked(r);
    const bool policy = q.size() == 1 && q.count("policy");
    if (r.method == "GET" && q.size() == 1 && q.count("location") && small_body) return native_bucket(c, r, bucket, q);
    if (policy && small_body && (r.method == "GET" || r.method == "PUT" || r.method == "DELETE"))
      return native_bucket(c, r, bucket, q);
    if (r.method == "GET") {
      // ListObjects (v1, or v2 with list-type=2) unless it is a sub-resource
      if (q.count("location") || q.count("policy") || r.content_length > 0 || r.chunked)
        return proxy(c, r, nullptr, 0, "route");
      return native_list(c, r, bucket, q);
    }
    if (r.method == "POST" && q.size() == 1 && q.count("delete")) return native_delete_objects(c, r, bucket, q);
    if ((r.method == "PUT" || r.method == "HEAD" || r.method == "DELETE") && q.empty() && small_body &&
        r.content_length <= (64 << 10))
      return native_bucket(c, r, bucket, q);
    return proxy(c, r, nullptr, 0, "route");
  }
  if (slash == std::string::npos || slash == 0 || slash + 1 >= p.size()) return proxy(c, r, nullptr, 0, "route");
  const std::string bucket = p.substr(0, slash), key = p.substr(slash + 1);
  if (reserved_key(key)) return proxy(c, r, nullptr, 0, "route");
  q.erase("x-id");  // SDK operation tag, no meaning to S3 itself
  if (r.method == "POST" && q.size() == 1 && q.count("uploadId") && !r.chunked && r.content_length <= (1 << 20) &&
      !aws_chunked(r))
    return native_complete(c, r, bucket, key, q);
  if (r.method == "POST" && q.size() == 1 && q.count("uploads") && q["uploads"].empty() && !r.chunked &&
      r.content_length <= 0)
    return native_initiate(c, r, bucket, key, q);
  if (r.method == "POST" && q.size() == 1 && q.count("delete")) return native_delete_objects(c, r, bucket, q);
  const bool part = q.size() == 2 && q.count("partNumber") && q.count("uploadId");
  const bool is_put = r.method == "PUT", is_get = r.method == "GET", is_head = r.method == "HEAD",
             is_delete = r.method == "DELETE";
  const bool abort = is_delete && q.size() == 1 && q.count("uploadId");
  if (!q.empty() && !part && !abort) return proxy(c, r, nullptr, 0, "query");
  if (!(is_put || is_delete || ((is_get || is_head) && !part))) return proxy(c, r, nullptr, 0, "method");
  // SSE-S3: whole objects are encrypted / decrypted here (AES-256-GCM, the gateway's DEK
  // envelope). Multipart parts are stored as sent, as the reference's UploadPart does
  // (handlers.rs encrypts in PutObject and CopyObject only), so they stay native too.
  if (cfg_.sse_enabled && cfg_.sse_kek.size() != 32) return proxy(c, r, nullptr, 0, "sse");
  const std::string* copy_src = is_put ? r.get("x-amz-copy-source") : nullptr;
  if (is_put) {
    const bool aws = aws_chunked(r);
    const std::string* dl = aws ? r.get("x-amz-decoded-content-length") : nullptr;
    const bool sized = dl && all_digits(*dl);
    // Transfer-Encoding: chunked is served for aws-chunked bodies of a stated size (the SDKs'
    // streaming uploads); a plain chunked body of unknown size goes to Python
    if ((r.chunked && !(aws && sized)) || (copy_src && (part || r.content_length > 0 || r.chunked)))
      return proxy(c, r, nullptr, 0, "put-form");
    uint64_t body = static_cast<uint64_t>(r.content_length);
    if (sized) body = r.chunked ? std::stoull(*dl) : std::min<uint64_t>(body, std::stoull(*dl));
    if (body + (cfg_.sse_enabled ? 28 : 0) > fc_->slot_bytes()) return proxy(c, r, nullptr, 0, "large");
  } else if (r.content_length > 0 || r.chunked) {
    return proxy(c, r, nullptr, 0, "body");
  }
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return proxy(c, r, nullptr, 0, why);
  std::string path = "/" + bucket + "/" + key;
  bool ok;
  if (is_put && part) {
    const std::string& uid = q["uploadId"];
    const std::string& pn = q["partNumber"];
    if (uid.empty() || uid.find('/') != std::string::npos || uid == "." || uid == ".." || !all_digits(pn) ||
        std::stoull(pn) < 1 || std::stoull(pn) > 10000)
      return proxy(c, r, nullptr, 0, "part-args");
    path = "/.s3_mpu/" + uid + "/" + std::to_string(std::stoull(pn));
    ok = native_put(c, r, path, true);
  } else if (copy_src) {
    ok = native_copy(c, r, path);
  } else if (is_put) {
    ok = native_put(c, r, path, false);
  } else if (abort) {
    const std::string& uid = q["uploadId"];
    if (uid.empty() || uid.find('/') != std::string::npos || uid == "." || uid == "..")
      return proxy(c, r, nullptr, 0, "part-args");
    ok = native_abort(c, r, uid);
  } else if (is_delete) {
    ok = native_delete(c, r, path);
  } else {
    ok = native_get(c, r, path, is_head);
  }
  if (r.status > 0 && cfg_.auth_enabled) audit(c, r, user, r.status, sess.role_arn);
  return ok;
}

// Signature, session role policy and bucket policy of an authenticated gateway; false with
// the hand-over reason when Python must answer (a denial, or anything not verified here).
bool S3Front::authorize(Req& r, const std::string& bucket, const std::map<std::string, std::string>& q,
                        std::string* user, Session* sess_out, std::string* why) {
  Session& sess = *sess_out;
  if (cfg_.auth_enabled) {
    if (cfg_.require_tls && !r.secure) {
      r.auth_kind = "insecure_transport";
      return (*why = "insecure", false);
    }
    if (!verify_auth(r, user, &sess)) return (*why = "auth", false);
    std::vector<std::string> keys;
    for (auto& kv : q) keys.push_back(kv.first);
    auto ar = s3policy::resolve_action_and_resource(r.method, r.path, keys);
    r.action = ar.first;
    // an STS session's role policy (reference auth_middleware.rs: IAM evaluation for
    // sessions only); a denial goes to the gateway, which answers 403 + audit
    if (!sess.role_arn.empty() && iam_) {
      bool allowed = iam_->evaluate(ar.first, ar.second, sess.role_arn, sess.ctx);
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.policy_results[(allowed ? "allow|" : "deny|") + ar.first]++;
        if (allowed) st_.iam_native++;
      }
      if (!allowed) {
        r.auth_kind = "missing_auth";
        r.auth_audit = "AccessDenied";
        return (*why = "iam-deny", false);
      }
    }
    // bucket policy (reference auth_middleware.rs + bucket_policy.rs): a static-key caller has
    // no role ARN, so only a Principal "*" Deny can apply to it; a session is matched by its role
    // the gateway evaluates no bucket policy for the policy sub-resource itself (so a Deny
    // cannot lock its owner out) and none at the root
    if (q.count("policy") || bucket.empty()) return true;
    bool known = false;
    auto pol = bucket_policy(bucket, &known);
    if (!known) return (*why = "bucket-policy", false);
    if (pol) {
      if (pol->evaluate(sess.role_arn.empty() ? nullptr : &sess.role_arn, ar.first, ar.second) ==
          s3policy::PolicyResult::ExplicitDeny) {
        {
          std::lock_guard<std::mutex> g(st_mu_);
          st_.policy_results["deny|" + ar.first]++;
        }
        r.auth_kind = "missing_auth";
        r.auth_audit = "AccessDenied";
        return (*why = "bucket-policy-deny", false);
      }
      std::lock_guard<std::mutex> g(st_mu_);
      st_.policy_native++;
    }
  }
  return true;
}

// ListObjects / ListObjectsV2 (reference handlers.rs:1536-1697, tests/models/s3_gateway.py list_objects):
// one ListFiles{with_metadata} per shard over the masters' local sockets, the keys sorted
// and paged (prefix, delimiter, marker / continuation-token / start-after, max-keys) and
// the reference XML written here. Buckets that are missing or empty, and objects whose
// headers live in a sidecar file, are Python's.
bool S3Front::native_list(Conn* c, Req& r, const std::string& bucket, std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.list");
  const bool v2 = q.count("list-type") && q["list-type"] == "2";
  const std::string prefix = q.count("prefix") ? q["prefix"] : "";
  const std::string delim = q.count("delimiter") ? q["delimiter"] : "";
  int64_t max_keys = 1000;
  if (q.count("max-keys")) {
    const std::string& mk = q["max-keys"];
    if (mk.empty() || mk.size() > 9 || !all_digits(mk)) return proxy(c, r, nullptr, 0, "list-args");
    max_keys = std::min<int64_t>(std::stoll(mk), 1000);
  }
  auto opt = [&](const char* k) { return q.count(k) ? q[k] : std::string(); };
  const std::string marker = v2 ? (!opt("continuation-token").empty() ? opt("continuation-token") : opt("start-after"))
                                : opt("marker");
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return proxy(c, r, nullptr, 0, why);
  const std::string bp = "/" + bucket + "/";
  std::vector<std::pair<std::string, pb::FileMetadata>> files;
  if (fc_->list(bp, &files, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "list");
  if (files.empty()) return proxy(c, r, nullptr, 0, "list-empty");  // NoSuchBucket, or none at all
  static const char* kHiddenSfx[] = {".s3keep", ".s3_mpu_completed", ".meta", ".s3_bucket_policy"};
  auto hidden = [](const std::string& f) {
    for (const char* h : kHiddenSfx)
      if (ends_with(f, h)) return true;
    return false;
  };
  std::unordered_set<std::string> fileset;
  std::unordered_map<std::string, const pb::FileMetadata*> by_path;
  std::set<std::string> mpu_dirs;
  for (auto& f : files) {
    fileset.insert(f.first);
    by_path[f.first] = &f.second;
    if (ends_with(f.first, "/.s3_mpu_completed")) mpu_dirs.insert(f.first.substr(0, f.first.size() - 18));
  }
  std::map<std::string, const pb::FileMetadata*> entries;  // key -> metadata (nullptr: MPU object)
  for (auto& f : files) {
    if (f.first.compare(0, bp.size(), bp) != 0 || hidden(f.first)) continue;
    if (mpu_dirs.count(f.first.substr(0, f.first.rfind('/')))) continue;
    entries[f.first.substr(bp.size())] = &f.second;
  }
  for (auto& d : mpu_dirs)
    if (d.compare(0, bp.size(), bp) == 0) entries[d.substr(bp.size())] = nullptr;
  std::vector<std::string> objects, cps;
  std::set<std::string> seen;
  bool truncated = false;
  std::string next_marker;
  int64_t nkeys = 0;
  for (auto it = entries.upper_bound(marker); it != entries.end(); ++it) {
    const std::string& k = it->first;
    if (k.compare(0, prefix.size(), prefix) != 0) continue;
    if (!delim.empty()) {
      size_t i = k.find(delim, prefix.size());
      if (i != std::string::npos) {
        std::string cp = k.substr(0, i + delim.size());
        if (seen.count(cp)) continue;
        if (nkeys >= max_keys) {
          truncated = true;
          break;
        }
        seen.insert(cp);
        cps.push_back(cp);
        ++nkeys;
        next_marker = cp;
        continue;
      }
    }
    if (nkeys >= max_keys) {
      truncated = true;
      break;
    }
    objects.push_back(k);
    ++nkeys;
    next_marker = k;
  }
  std::string contents;
  for (auto& k : objects) {
    const pb::FileMetadata* info = entries[k];
    std::string etag = "\"d41d8cd98f00b204e9800998ecf8427e\"", lm = "2025-01-01T00:00:00.000Z";
    uint64_t size = 0;
    if (info == nullptr) {  // a completed multipart object: its marker's recorded headers
      auto mk = by_path.find(bp + k + "/.s3_mpu_completed");
      if (mk == by_path.end()) return proxy(c, r, nullptr, 0, "list-mpu");
      std::map<std::string, std::string> side;
      if (mk->second->attributes.empty() && !read_sidecar(bp + k, r.rid, &side)) return proxy(c, r, nullptr, 0, "list-sidecar");
      const auto& at = mk->second->attributes.empty() ? side : mk->second->attributes;
      auto e = at.find("ETag");
      etag = e != at.end() ? e->second : "\"000-MPU\"";
      auto sz = at.find("x-dfs-mpu-size");
      if (sz != at.end() && !sz->second.empty() && all_digits(sz->second)) {
        size = std::stoull(sz->second);
      } else {  // (a reference-completed object: the sum of its parts)
        const std::string pre = bp + k + "/";
        for (int part = 1; part <= 10000; ++part) {  // parts are numbered from 1 (S3)
          auto it = by_path.find(pre + std::to_string(part));
          if (it == by_path.end()) break;
          size += it->second->size;
        }
      }
    } else {
      size = info->size;
      if (!info->etag_md5.empty()) etag = "\"" + info->etag_md5 + "\"";
      lm = iso_ms(info->created_at_ms);
      if (!info->attributes.empty()) {
        auto e = info->attributes.find("ETag");
        if (e != info->attributes.end()) etag = e->second;
      } else if (fileset.count(bp + k + ".meta")) {
        std::map<std::string, std::string> side;
        if (!read_sidecar(bp + k, r.rid, &side)) return proxy(c, r, nullptr, 0, "list-sidecar");
        auto e = side.find("ETag");
        if (e != side.end()) etag = e->second;
      }
    }
    contents += "<Contents>" + xel("Key", k) + xel("LastModified", lm) + xel("ETag", etag) +
                xel("Size", std::to_string(size)) + xel("StorageClass", "STANDARD") +
                "<Owner><ID>dfs</ID><DisplayName>dfs</DisplayName></Owner></Contents>";
  }
  std::string prefixes;
  for (auto& cp : cps) prefixes += "<CommonPrefixes>" + xel("Prefix", cp) + "</CommonPrefixes>";
  const std::string trunc = truncated ? "true" : "false";
  std::string x = "<ListBucketResult>" + xel("Name", bucket) + xel("Prefix", prefix);
  if (v2) {
    x += xel("MaxKeys", std::to_string(max_keys)) + xel("IsTruncated", trunc) + contents + prefixes +
         xel("KeyCount", std::to_string(nkeys));
    if (q.count("continuation-token")) x += xel("ContinuationToken", q["continuation-token"]);
    if (truncated) x += xel("NextContinuationToken", next_marker);
    if (q.count("start-after")) x += xel("StartAfter", q["start-after"]);
  } else {
    x += xel("Marker", opt("marker"));
    if (truncated && !delim.empty()) x += xel("NextMarker", next_marker);
    x += xel("MaxKeys", std::to_string(max_keys)) + xel("IsTruncated", trunc) + contents + prefixes;
  }
  x += "</ListBucketResult>";
  std::string h = "HTTP/1.1 200 OK\r\nContent-Type: application/xml\r\nContent-Length: " + std::to_string(x.size()) +
                  "\r\n" + (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
  r.status = 200;
  count(r, 200);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.lists++;
  }
  const bool ok = send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(x.data()), x.size());
  if (cfg_.auth_enabled) audit(c, r, user, 200, sess.role_arn);
  return ok;
}

// ---------------------------------------------------------------- auth (static SigV4)
// An STS session token (StsTokenManager, reference auth/sts.rs:60-98):
// base64([kid u32 BE][nonce 12][AES-256-GCM(JSON StsSessionData)]). False when it does not
// open, has expired or is malformed: the request goes to Python for the exact error.
int S3Front::open_session(const std::string& token, Session* out) {
  std::string raw;
  if (!crypto::base64_decode(token, &raw) || raw.size() < 32) return 0;
  const uint32_t kid = (uint32_t(uint8_t(raw[0])) << 24) | (uint32_t(uint8_t(raw[1])) << 16) |
                       (uint32_t(uint8_t(raw[2])) << 8) | uint32_t(uint8_t(raw[3]));
  auto k = sts_keys_.find(kid);
  if (k == sts_keys_.end()) return 0;
  try {
    Json j = Json::parse(crypto::aes256gcm_decrypt(k->second, raw.substr(4, 12), raw.substr(16), ""));
    out->role_arn = j["role_arn"].str();
    out->secret = j["temp_secret_key"].str();
    if (out->role_arn.empty() || out->secret.empty()) return 0;
    if (j["expiration"].as_int() < static_cast<int64_t>(now_s())) return -1;
    const Json& cl = j["claims"];  // Claims.to_policy_context()
    out->ctx.principal_id = cl["sub"].str();
    out->ctx.groups.clear();
    if (cl["groups"].is_array())
      for (auto& g : cl["groups"].items()) out->ctx.groups.push_back(g.str());
    out->ctx.claims = {{"sub", cl["sub"].str()}, {"iss", cl["iss"].str()}};
    return 1;
  } catch (const std::exception&) {
    return 0;
  }
}

// SigV4 of the Authorization header, or of a presigned URL's query (reference
// auth_middleware.rs:19-365, presign.rs; tests/models/s3_gateway.py authenticate): the same canonical
// request either way — the query without X-Amz-Signature, the signed headers, the payload
// hash header or UNSIGNED-PAYLOAD. A presigned URL is bounded by X-Amz-Expires (at most 7
// days) instead of the 15-minute skew. Anything that does not verify is handed over, so
// Python answers with the exact error and audit record.
int S3Front::verify_auth(Req& r, std::string* user, Session* sess) {
  auto fail = [&r](const char* kind, const char* audit_code = "") {
    r.auth_kind = kind;
    r.auth_audit = audit_code;
    return 0;
  };
  const std::string* auth = r.get("authorization");
  auto qp = [&r](const char* k) -> const std::string* {
    auto it = r.presign.find(k);
    return it == r.presign.end() ? nullptr : &it->second;
  };
  const bool presigned = !auth && qp("X-Amz-Algorithm") && qp("X-Amz-Expires");
  std::string cred, sh, sig;
  const std::string* ts = nullptr;
  if (auth) {
    if (auth->compare(0, 16, "AWS4-HMAC-SHA256") != 0) return fail("missing_auth");
    std::vector<std::string> parts;
    size_t i = 0;
    while (i <= auth->size()) {
      size_t cm = auth->find(',', i);
      parts.push_back(trim(auth->substr(i, cm == std::string::npos ? std::string::npos : cm - i)));
      if (cm == std::string::npos) break;
      i = cm + 1;
    }
    if (parts.size() < 3) return fail("missing_auth");
    size_t k = parts[0].find("Credential=");
    if (k == std::string::npos) return fail("missing_auth");
    cred = parts[0].substr(k + 11);
    size_t sp = cred.find_first_of(" \t");
    if (sp != std::string::npos) cred = cred.substr(0, sp);
    auto after_eq = [](const std::string& v) {
      size_t e = v.find('=');
      return e == std::string::npos ? std::string() : trim(v.substr(e + 1));
    };
    sh = after_eq(parts[1]);
    sig = after_eq(parts[2]);
    ts = r.get("x-amz-date");
    if (!ts) ts = r.get("date");
  } else if (presigned) {
    if (*qp("X-Amz-Algorithm") != "AWS4-HMAC-SHA256" || !qp("X-Amz-Credential") || !qp("X-Amz-SignedHeaders") ||
        !qp("X-Amz-Signature") || !qp("X-Amz-Date"))
      return fail("missing_auth");
    cred = *qp("X-Amz-Credential");
    sh = *qp("X-Amz-SignedHeaders");
    sig = *qp("X-Amz-Signature");
    ts = qp("X-Amz-Date");
  } else {
    return fail("missing_auth");
  }
  std::vector<std::string> cp;
  for (size_t a = 0;;) {
    size_t b = cred.find('/', a);
    cp.push_back(cred.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    a = b + 1;
  }
  if (cp.size() < 5 || cp[4] != "aws4_request") return fail("missing_auth");
  r.auth_user = cp[0];
  if (!ts || sh.empty() || sig.empty()) return fail("missing_auth");
  tm t{};
  const bool ts_ok = ts->size() == 16 && strptime(ts->c_str(), "%Y%m%dT%H%M%SZ", &t);
  const double age = ts_ok ? now_s() - static_cast<double>(timegm(&t)) : 0;
  if (presigned) {
    // 0 < X-Amz-Expires <= 604800 and not yet expired
    if (!ts_ok) return fail("missing_auth", "InvalidArgument");
    const std::string& ex = *qp("X-Amz-Expires");
    if (!all_digits(ex) || ex.size() > 9 || std::stoull(ex) == 0) return fail("missing_auth", "InvalidArgument");
    const double expires = static_cast<double>(std::stoull(ex));
    if (expires > 604800) return fail("missing_auth", "AuthorizationQueryParametersError");
    if (age > expires) return fail("expired_token");
    // signed for the future (beyond the clock-skew window): not yet valid, and otherwise a way
    // to mint URLs that outlive the 7-day cap
    if (-age / 60.0 > 15.0) return fail("clock_skew");
  } else if (ts_ok && std::abs(age) / 60.0 > 15.0) {  // %Y%m%dT%H%M%SZ within 15 minutes of now
    return fail("clock_skew");
  }
  const std::string &ak = cp[0], &date = cp[1], &region = cp[2], &service = cp[3];
  if (region != cfg_.region || service != "s3") return fail("invalid_scope");
  const std::string* token = r.get("x-amz-security-token");
  if (!token) token = qp("X-Amz-Security-Token");
  std::string skey;
  if (token) {
    if (sts_keys_.empty()) return fail("internal");  // "STS is not enabled"
    const int os = open_session(*token, sess);
    if (os == 0) return fail("invalid_token");
    if (os < 0) {
      r.auth_role = sess->role_arn;
      return fail("expired_token");
    }
    r.auth_role = sess->role_arn;
    // a session's own secret: its signing key is never shared with the static key's slot
    skey = sigv4::signing_key(sess->secret, date, region, service);
  } else {
    if (cfg_.access_key.empty() || ak != cfg_.access_key) return fail("invalid_access_key");
    {
      std::lock_guard<std::mutex> g(key_mu_);
      auto it = key_cache_.find(date);
      if (it != key_cache_.end()) skey = it->second;
    }
    if (skey.empty()) {
      skey = sigv4::signing_key(cfg_.secret_key, date, region, service);
      std::lock_guard<std::mutex> g(key_mu_);
      if (key_cache_.size() > 8) key_cache_.clear();
      key_cache_[date] = skey;
    }
  }
  sigv4::Request sr;
  sr.method = r.method;
  sr.path = r.raw_path;
  sr.query = sigv4::normalize_query(r.raw_query);
  std::vector<std::string> names;
  for (size_t a = 0;;) {
    size_t b = sh.find(';', a);
    std::string n = lower(trim(sh.substr(a, b == std::string::npos ? std::string::npos : b - a)));
    if (!n.empty()) names.push_back(n);
    if (b == std::string::npos) break;
    a = b + 1;
  }
  std::sort(names.begin(), names.end());
  names.erase(std::unique(names.begin(), names.end()), names.end());
  std::string joined;
  for (auto& n : names) {
    std::string v;
    bool first = true;
    for (auto& h : r.headers)
      if (h.first == n) {
        if (!first) v += ",";
        v += collapse_ws(h.second);
        first = false;
      }
    sr.headers.emplace_back(n, v);
    joined += (joined.empty() ? "" : ";") + n;
  }
  sr.signed_headers = joined;
  const std::string* ph = r.get("x-amz-content-sha256");
  sr.payload_hash = ph && !ph->empty() ? *ph : kUnsigned;
  if (sr.payload_hash == kUnsigned && !cfg_.allow_unsigned_payload && !presigned) return fail("missing_auth");
  const std::string scope = date + "/" + region + "/" + service + "/aws4_request";
  std::string creq;
  if (!ts || !sigv4::verify(sr, *ts, scope, skey, sig, &creq)) return fail("signature_mismatch");
  *user = ak;
  if (cfg_.backend.empty()) {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.auth_results["success|none"]++;
  }
  // an aws-chunked body continues this signature's chain (seed = the request signature)
  r.chain = sigv4::ChunkChain{skey, *ts, scope, sig};
  r.chain_set = true;
  std::lock_guard<std::mutex> g(st_mu_);
  st_.auth_native++;
  if (presigned) st_.presigned++;
  return 1;
}

void S3Front::drop_policies() {
  std::lock_guard<std::mutex> g(pol_mu_);
  policy_cache_.clear();
  ++cache_epoch_;  // an answer fetched before this call is not cached
}

// PolicyEpoch.bump of tests/models/s3_gateway.py: strictly increasing across the gateway's processes (the
// system-wide monotonic clock, at least +1).
void S3Front::policy_changed() {
  if (epoch_map_) {
    timespec ts{};
    ::clock_gettime(CLOCK_MONOTONIC, &ts);
    const uint64_t mono = static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
    uint64_t cur = __atomic_load_n(epoch_map_, __ATOMIC_ACQUIRE);
    while (!__atomic_compare_exchange_n(epoch_map_, &cur, std::max(cur + 1, mono), false, __ATOMIC_ACQ_REL,
                                        __ATOMIC_ACQUIRE)) {
    }
  }
  drop_policies();
}

std::shared_ptr<const s3policy::BucketPolicy> S3Front::bucket_policy(const std::string& bucket, bool* known) {
  const double now = now_s();
  // the epoch is read BEFORE the policy file: a policy written before the bump is seen by
  // every fetch that starts after it, and an answer fetched under an older epoch is dropped
  const uint64_t ep = policy_epoch();
  uint64_t tag;
  {
    std::lock_guard<std::mutex> g(pol_mu_);
    if (epoch_map_ && ep != cache_epoch_) {
      policy_cache_.clear();
      cache_epoch_ = ep;
    }
    tag = cache_epoch_;
    auto it = policy_cache_.find(bucket);
    if (it != policy_cache_.end() && it->second.first > now) {
      *known = true;
      return it->second.second;
    }
  }
  *known = false;
  const std::string path = "/" + bucket + "/.s3_bucket_policy";
  bool found = false;
  std::string meta, msg;
  if (fc_->stat(path, &found, &meta, &msg, "") != FastClient::Ok) return nullptr;
  std::shared_ptr<const s3policy::BucketPolicy> pol;
  if (found) {
    int64_t slot = -1;
    uint64_t n = 0;
    FastClient::Times t;
    if (fc_->read_known(meta, &slot, &n, &msg, &t, "", 0, 0) != FastClient::Ok) return nullptr;
    std::string doc(reinterpret_cast<const char*>(fc_->slot_ptr(slot)), n);
    fc_->release(slot);
    try {
      pol = std::make_shared<const s3policy::BucketPolicy>(s3policy::BucketPolicy::parse(doc));
    } catch (const std::exception&) {
      pol = nullptr;  // the gateway ignores an unparsable policy as well
    }
  }
  *known = true;
  std::lock_guard<std::mutex> g(pol_mu_);
  if (tag == cache_epoch_ && (!epoch_map_ || policy_epoch() == ep)) {
    if (policy_cache_.size() >= kPolicyCacheMax) policy_cache_.clear();
    policy_cache_[bucket] = {now + 1.0, pol};  // the gateway's 1 s policy cache
  }
  return pol;
}

void S3Front::audit(const Conn* c, const Req& r, const std::string& user, int status, const std::string& role_arn,
                    const std::string& error_code, const std::string& action_in, const std::string& resource_in) {
  if (audit_fd_ < 0) return;
  std::string path = r.path.empty() ? r.raw_path : r.path;
  std::vector<std::string> segs;
  for (size_t a = 0; a < path.size();) {
    size_t b = path.find('/', a);
    std::string s = path.substr(a, b == std::string::npos ? std::string::npos : b - a);
    if (!s.empty()) segs.push_back(s);
    if (b == std::string::npos) break;
    a = b + 1;
  }
  std::string resource = "arn:dfs:s3:::";
  for (size_t i = 0; i < segs.size(); ++i) resource += (i ? "/" : "") + segs[i];
  if (!resource_in.empty()) resource = resource_in;
  std::string action = !action_in.empty() ? action_in : !r.action.empty() ? r.action
                       : r.method == "GET" ? "s3:GetObject" : r.method == "HEAD" ? "s3:HeadObject" : "s3:PutObject";
  const double t = now_s();
  int64_t ms;
  std::string ts = iso_now(t, &ms);
  const std::string* ua = r.get("user-agent");
  std::string rec = "{\"timestamp\":" + json_str(ts) + ",\"timestamp_ms\":" + std::to_string(ms) +
                    ",\"request_id\":" + json_str(r.rid.empty() ? uuid4() : r.rid) +
                    ",\"remote_ip\":" + json_str(c->ip) + ",\"user_id\":" + json_str(user) +
                    ",\"role_arn\":" + (role_arn.empty() ? std::string("null") : json_str(role_arn)) +
                    ",\"action\":" + json_str(action) + ",\"resource\":" + json_str(resource) +
                    ",\"status_code\":" + std::to_string(status) + ",\"error_code\":" +
                    (error_code.empty() ? std::string("null") : json_str(error_code)) + ",\"user_agent\":" +
                    (ua ? json_str(*ua) : std::string("null")) +
                    ",\"duration_ms\":" + std::to_string(static_cast<int64_t>((t - r.started) * 1000)) +
                    ",\"previous_hash\":null,\"record_hash\":null}";
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  std::snprintf(sa.sun_path, sizeof sa.sun_path, "%s", cfg_.audit_socket.c_str());
  bool ok = ::sendto(audit_fd_, rec.data(), rec.size(), 0, reinterpret_cast<sockaddr*>(&sa), sizeof sa) ==
            static_cast<ssize_t>(rec.size());
  std::lock_guard<std::mutex> g(st_mu_);
  (ok ? st_.audit_sent : st_.audit_dropped)++;
}

void S3Front::count(const Req& r, int status) {
  std::lock_guard<std::mutex> g(st_mu_);
  st_.native++;
  st_.by_status[r.method + " " + std::to_string(status)]++;
}

void S3Front::note_proxy(const std::string& why) {
  std::lock_guard<std::mutex> g(st_mu_);
  st_.proxied++;
  st_.proxy_reasons[why]++;
}

// ---------------------------------------------------------------- native object ops
static bool read_body(S3Front::Conn* c, uint8_t* dst, uint64_t n) {
  uint64_t have = std::min<uint64_t>(n, c->buf.size() - c->pos);
  if (have) std::memcpy(dst, c->buf.data() + c->pos, have);
  c->pos += have;
  uint64_t got = have;
  while (got < n) {
    long k = io_recv(c->io(), dst + got, n - got);
    if (k <= 0) return false;
    got += static_cast<uint64_t>(k);
  }
  return true;
}

bool S3Front::native_put(Conn* c, Req& r, const std::string& path, bool part) {
  TraceRange tr(part ? "dfs.s3.upload_part" : "dfs.s3.put");
  if (part) {  // the upload must exist before its body is accepted (NoSuchUpload from Python)
    const std::string marker = path.substr(0, path.rfind('/')) + "/.s3keep";
    bool found = false;
    std::string meta, msg;
    if (fc_->stat(marker, &found, &meta, &msg, r.rid) != FastClient::Ok || !found)
      return proxy(c, r, nullptr, 0, "no-upload");
  }
  uint64_t n = static_cast<uint64_t>(std::max<int64_t>(r.content_length, 0));
  const bool aws = aws_chunked(r);
  if (aws) {  // decoded into the slot below; its size bounded by what the client announced
    const std::string* dl = r.get("x-amz-decoded-content-length");
    if (dl && all_digits(*dl)) n = r.chunked ? std::stoull(*dl) : std::min<uint64_t>(n, std::stoull(*dl));
  }
  const bool sse = cfg_.sse_enabled && !part;  // handle() sent SSE parts to Python
  int64_t slot = fc_->acquire_slot(std::max<uint64_t>(sse ? n + 28 : n, 1));  // [nonce 12][ciphertext n][tag 16]
  if (slot < 0) return proxy(c, r, nullptr, 0, "no-slot");
  struct Release {
    FrontStore* fc;
    int64_t s;
    ~Release() { fc->release(s); }
  } rel{fc_, slot};
  if (r.expect_continue && !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
  uint8_t* dst = fc_->slot_mut(slot);
  if (aws) {
    const int rc = read_aws_chunked(c, r, sse ? dst + 12 : dst, n, &n);
    if (rc == 0) return false;
    if (rc < 0) {  // tests/models/s3_gateway.py route(): the body does not decode or its chain is broken
      r.keep_alive = false;
      s3_error(c, r, 403, "SignatureDoesNotMatch", "aws-chunked signature chain is invalid");
      return false;
    }
  } else if (!read_body(c, sse ? dst + 12 : dst, n)) {
    return false;
  }
  const uint64_t stored = sse ? n + 28 : n;
  std::map<std::string, std::string> attrs;
  std::string plain_md5, dk;
  if (sse) {
    // SseManager.encrypt_object (reference auth/sse.rs:10-62): a fresh DEK encrypts the
    // object in place, the KEK wraps the DEK; the ETag stays the plaintext's MD5
    plain_md5 = crypto::md5_hex(dst + 12, n);
    dk = crypto::random_bytes(32);
    const std::string n1 = crypto::random_bytes(12), n2 = crypto::random_bytes(12);
    std::memcpy(dst, n1.data(), 12);
    crypto::aes256gcm_encrypt_inplace(reinterpret_cast<const uint8_t*>(dk.data()), dst, dst + 12, n, dst + 12 + n);
    const std::string wrapped = n2 + crypto::aes256gcm_encrypt(cfg_.sse_kek, n2, dk, "");
    attrs["x-amz-sse-encrypted-dek"] = crypto::base64_encode(wrapped);
  }
  if (!part) {
    // put_object: ETag, x-amz-meta-* (lower-cased) and Content-Type become the attributes
    for (auto& h : r.headers)
      if (h.first.compare(0, 11, "x-amz-meta-") == 0) attrs[h.first] = h.second;
    if (const std::string* ct = r.get("content-type")) attrs["Content-Type"] = *ct;
    attrs["ETag"] = sse ? "\"" + plain_md5 + "\"" : "";
  }
  FastClient::Times t;
  std::string msg, md5;
  int reps = 0;
  // without SSE the ETag attribute is the MD5 the write computes of the stored bytes
  const char* etag_attr = part || sse ? nullptr : "ETag";
  auto st = fc_->write_slot(path, slot, stored, &reps, &msg, &t, r.rid, part ? nullptr : &attrs, etag_attr, &md5);
  if (st == FastClient::Failed && msg.find("already exists") != std::string::npos) {
    // _put_replace: an existing key is replaced (delete, then create again)
    std::string dmsg;
    if (fc_->remove(path, &dmsg, r.rid) != FastClient::NotHandled)
      st = fc_->write_slot(path, slot, stored, &reps, &msg, &t, r.rid, part ? nullptr : &attrs, etag_attr, &md5);
  }
  if (st != FastClient::Ok) {
    // a decoded aws-chunked body cannot be handed over under its signed STREAMING headers
    if (aws) {
      r.keep_alive = false;
      s3_error(c, r, 500, "InternalError", msg.empty() ? "write failed" : msg, path);
      return false;
    }
    if (!sse) return proxy(c, r, dst, n, "put-fallback");
    // the slot holds ciphertext: decrypt it back so Python gets the body it would have read
    if (!crypto::aes256gcm_decrypt_inplace(reinterpret_cast<const uint8_t*>(dk.data()), dst, dst + 12, n,
                                           dst + 12 + n))
      return false;
    return proxy(c, r, dst + 12, n, "put-fallback");
  }
  if (sse) {
    md5 = plain_md5;
    std::lock_guard<std::mutex> g(st_mu_);
    st_.sse_puts++;
  }
  if (!part && cfg_.metadata_sidecar) {
    attrs["ETag"] = "\"" + md5 + "\"";
    (void)write_sidecar(path, attrs, r.rid);
  }
  std::string head = "HTTP/1.1 200 OK\r\nETag: \"" + md5 + "\"\r\n" +
                     (sse ? "x-amz-server-side-encryption: AES256\r\n" : "") + "Content-Length: 0\r\n";
  head += r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
  r.status = 200;
  count(r, 200);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    (part ? st_.parts : st_.puts)++;
    st_.bytes_in += n;
    if (aws) st_.chunked_puts++;
  }
  return send_all(c->io(), head.data(), head.size());
}

namespace {

// _object_headers of tests/models/s3_gateway.py; false: a case Python owns (SSE, sidecar metadata)
bool object_headers(const pb::FileMetadata* m, const std::map<std::string, std::string>& attrs, std::string* out,
                    std::string* dek = nullptr) {
  std::string etag = m && !m->etag_md5.empty() ? "\"" + m->etag_md5 + "\"" : kEmptyEtag;
  std::string h = "Last-Modified: " + http_date(m ? m->created_at_ms : 0) + "\r\nAccept-Ranges: bytes\r\n";
  bool ctype = false;
  for (auto& kv : attrs) {
    if (kv.first == "ETag") {
      etag = kv.second;
    } else if (kv.first == "x-amz-sse-encrypted-dek") {
      if (!dek) return false;  // a caller that cannot decrypt
      *dek = kv.second;
      h += "x-amz-server-side-encryption: AES256\r\n";
    } else if (kv.first.compare(0, 11, "x-amz-meta-") == 0 || kv.first == "Content-Type") {
      if (kv.second.find_first_of("\r\n") != std::string::npos) return false;
      h += kv.first + ": " + kv.second + "\r\n";
      ctype |= kv.first == "Content-Type";
    }
  }
  h += "ETag: " + etag + "\r\n";
  if (!ctype) h += "Content-Type: application/octet-stream\r\n";
  *out = h;
  return true;
}

}  // namespace

// The reference gateway keeps an object's headers in a sidecar DFS file `<path>.meta` holding
// {"headers": {...}} (handlers.rs:984-1006 writes it, :1058-1079 reads it). Objects written
// here carry them as file attributes; a file without attributes (written by the reference's
// layout) is described by its sidecar. false: the store could not be asked.
bool S3Front::read_sidecar(const std::string& path, const std::string& rid, std::map<std::string, std::string>* out) {
  out->clear();
  bool found = false;
  std::string meta, msg;
  if (fc_->stat(path + ".meta", &found, &meta, &msg, rid) != FastClient::Ok) return false;
  if (!found) return true;
  pb::FileMetadata m;
  if (!m.decode(meta)) return true;
  std::string doc;
  if (m.size > 0) {
    int64_t slot = -1;
    uint64_t n = 0;
    FastClient::Times t;
    if (fc_->read_known(meta, &slot, &n, &msg, &t, rid, 0, 0) != FastClient::Ok) return false;
    doc.assign(reinterpret_cast<const char*>(fc_->slot_ptr(slot)), n);
    fc_->release(slot);
  }
  try {
    const Json j = Json::parse(doc);
    const Json& h = j["headers"];
    if (h.is_object())
      for (auto& kv : h.fields())
        if (kv.second.is_string()) (*out)[kv.first] = kv.second.str();
  } catch (const std::exception&) {
    out->clear();  // (an unreadable sidecar describes nothing, as in tests/models/s3_gateway.py _read_meta)
  }
  std::lock_guard<std::mutex> g(st_mu_);
  st_.sidecar_reads++;
  return true;
}

// S3_METADATA_SIDECAR=true: the object's headers are also written as the reference's sidecar,
// so a bucket the reference gateway must read back carries them where it looks. The JSON is
// the Python gateway's (json.dumps, compact, ASCII-escaped; ETag first, then x-amz-meta-*,
// Content-Type and the wrapped DEK); the old sidecar is deleted first, as both gateways do.
bool S3Front::write_sidecar(const std::string& path, const std::map<std::string, std::string>& attrs,
                            const std::string& rid) {
  if (!cfg_.metadata_sidecar) return true;
  std::string doc = "{\"headers\":{";
  bool first = true;
  auto add = [&](const std::string& k, const std::string& v) {
    if (!first) doc += ",";
    first = false;
    audit::put_string(doc, k, true);
    doc += ":";
    audit::put_string(doc, v, true);
  };
  auto et = attrs.find("ETag");
  if (et != attrs.end()) add(et->first, et->second);
  for (auto& kv : attrs)
    if (kv.first.compare(0, 11, "x-amz-meta-") == 0) add(kv.first, kv.second);
  for (const char* k : {"Content-Type", "x-amz-sse-encrypted-dek", "x-dfs-mpu-size", "x-dfs-mpu-layout"}) {
    auto it = attrs.find(k);
    if (it != attrs.end()) add(it->first, it->second);
  }
  doc += "}}";
  std::string msg;
  (void)fc_->remove(path + ".meta", &msg, rid);
  int64_t slot = fc_->acquire_slot(std::max<size_t>(doc.size(), 1));
  if (slot < 0) return false;
  std::memcpy(fc_->slot_mut(slot), doc.data(), doc.size());
  FastClient::Times t;
  std::string md5;
  int reps = 0;
  auto st = fc_->write_slot(path + ".meta", slot, doc.size(), &reps, &msg, &t, rid, nullptr, nullptr, &md5);
  fc_->release(slot);
  std::lock_guard<std::mutex> g(st_mu_);
  st_.sidecar_writes++;
  return st == FastClient::Ok;
}

bool S3Front::native_get(Conn* c, Req& r, const std::string& path, bool head) {
  TraceRange tr(head ? "dfs.s3.head" : "dfs.s3.get");
  bool found = false;
  std::string meta, msg;
  using SC = std::chrono::steady_clock;
  const auto t0 = SC::now();
  if (fc_->stat(path, &found, &meta, &msg, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "stat");
  const auto t1 = SC::now();
  if (!found) {
    // a completed multipart object, a "directory" probe, or NoSuchKey (tests/models/s3_gateway.py
    // get_object / head_object)
    std::string mm;
    if (fc_->stat(path + "/.s3_mpu_completed", &found, &mm, &msg, r.rid) != FastClient::Ok)
      return proxy(c, r, nullptr, 0, "stat");
    if (found && !head) return native_mpu_get(c, r, path, mm);
    if (found) {
      pb::FileMetadata mk;
      std::string hdrs;
      std::map<std::string, std::string> side;
      if (!mk.decode(mm)) return proxy(c, r, nullptr, 0, "attrs");
      if (mk.attributes.empty() && !read_sidecar(path, r.rid, &side)) return proxy(c, r, nullptr, 0, "sidecar");
      if (!object_headers(nullptr, mk.attributes.empty() ? side : mk.attributes, &hdrs))
        return proxy(c, r, nullptr, 0, "attrs");
      const size_t lm = hdrs.find("Last-Modified: ");
      hdrs.replace(lm, hdrs.find("\r\n", lm) - lm,
                   "Last-Modified: " + http_date(static_cast<uint64_t>(now_s() * 1000)));  // formatdate(): now
      auto sz = mk.attributes.find("x-dfs-mpu-size");
      const std::string size = sz != mk.attributes.end() && all_digits(sz->second) ? sz->second : "0";
      std::string h = "HTTP/1.1 200 OK\r\n" + hdrs + "Content-Length: " + size + "\r\n" +
                      (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
      r.status = 200;
      count(r, 200);
      {
        std::lock_guard<std::mutex> g(st_mu_);
        st_.heads++;
      }
      return send_all(c->io(), h.data(), h.size());
    }
    if (!head) return s3_error(c, r, 404, "NoSuchKey", "The specified key does not exist.", path);
    if (path.back() == '/') {  // a "directory" marker probe: 200 when anything lives under it
      std::vector<std::pair<std::string, pb::FileMetadata>> under;
      if (fc_->list(path, &under, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "list");
      if (!under.empty()) return respond(c, r, 200, "", "Content-Length: 0\r\n");
    }
    return respond(c, r, 404, "", "Content-Length: 0\r\n");
  }
  pb::FileMetadata m;
  if (!m.decode(meta)) return proxy(c, r, nullptr, 0, "decode");
  std::string hdrs, dek;
  std::map<std::string, std::string> side;
  if (m.attributes.empty() && !read_sidecar(path, r.rid, &side)) return proxy(c, r, nullptr, 0, "sidecar");
  if (!object_headers(&m, m.attributes.empty() ? side : m.attributes, &hdrs, &dek)) return proxy(c, r, nullptr, 0, "attrs");
  if (!dek.empty() && cfg_.sse_kek.size() != 32) return proxy(c, r, nullptr, 0, "sse");
  const std::string ka = r.keep_alive ? "Connection: keep-alive\r\n" : "Connection: close\r\n";
  if (!dek.empty() && !head) return sse_get(c, r, meta, m.size, hdrs, dek);
  if (head) {
    std::string h = "HTTP/1.1 200 OK\r\n" + hdrs + "Content-Length: " + std::to_string(m.size) + "\r\n" + ka + "\r\n";
    r.status = 200;
    count(r, 200);
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.heads++;
    }
    return send_all(c->io(), h.data(), h.size());
  }
  uint64_t s = 0, e = 0;
  int rng = parse_range(r.get("range"), m.size, &s, &e);
  if (rng == 2)  // _range_response: 416 with the size
    return respond(c, r, 416,
                   "<Error>" + xel("Code", "InvalidRange") + xel("Message", "The requested range is not satisfiable") +
                       "<Resource></Resource><RequestId></RequestId></Error>",
                   "Content-Range: bytes */" + std::to_string(m.size) + "\r\n");
  if (rng >= 2) return proxy(c, r, nullptr, 0, "range");
  int64_t slot = -1;
  uint64_t got = 0;
  FastClient::Times t;
  if (m.size > 0) {
    auto st = fc_->read_known(meta, &slot, &got, &msg, &t, r.rid, rng == 1 ? s : 0, rng == 1 ? e - s + 1 : 0);
    if (st != FastClient::Ok) return proxy(c, r, nullptr, 0, "read");
  }
  struct Release {
    FrontStore* fc;
    int64_t s;
    ~Release() {
      if (s >= 0) fc->release(s);
    }
  } rel{fc_, slot};
  const uint64_t want = rng == 1 ? e - s + 1 : m.size;
  if (got != want) return proxy(c, r, nullptr, 0, "short-read");
  const auto t2 = SC::now();
  std::string h;
  if (rng == 1) {
    h = "HTTP/1.1 206 Partial Content\r\n" + hdrs + "Content-Range: bytes " + std::to_string(s) + "-" +
        std::to_string(e) + "/" + std::to_string(m.size) + "\r\n";
    r.status = 206;
  } else {
    h = "HTTP/1.1 200 OK\r\n" + hdrs;
    r.status = 200;
  }
  h += "Content-Length: " + std::to_string(got) + "\r\n" + ka + "\r\n";
  count(r, r.status);
  const bool ok = send_head_body(c->io(), h, got ? fc_->slot_ptr(slot) : nullptr, got);
  const auto t3 = SC::now();
  auto us = [](SC::duration d) { return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::microseconds>(d).count()); };
  {
    std::lock_guard<std::mutex> g(st_mu_);
    (rng == 1 ? st_.range_gets : st_.gets)++;
    st_.bytes_out += got;
    st_.get_stat_us += us(t1 - t0);
    st_.get_read_us += us(t2 - t1);
    st_.get_send_us += us(t3 - t2);
    st_.get_timed++;
  }
  return ok;
}

namespace {

// ET.fromstring + _children/_text of tests/models/s3_xml.py for a CompleteMultipartUpload body, namespace
// agnostic: the (PartNumber, ETag) of every <Part> child of the root. False for anything
// this small scanner does not model (DTDs, CDATA, malformed XML): Python parses those.
bool parse_complete_body(const std::string& b, std::vector<std::pair<int64_t, std::string>>* parts) {
  parts->clear();
  size_t i = 0;
  auto local = [](const std::string& t) {
    size_t c = t.find(':');
    return c == std::string::npos ? t : t.substr(c + 1);
  };
  auto unescape = [](const std::string& v, std::string* o) {
    o->clear();
    for (size_t k = 0; k < v.size(); ++k) {
      if (v[k] != '&') {
        o->push_back(v[k]);
        continue;
      }
      size_t e = v.find(';', k);
      if (e == std::string::npos) return false;
      const std::string ent = v.substr(k + 1, e - k - 1);
      if (ent == "quot") o->push_back('"');
      else if (ent == "amp") o->push_back('&');
      else if (ent == "lt") o->push_back('<');
      else if (ent == "gt") o->push_back('>');
      else if (ent == "apos") o->push_back('\'');
      else return false;
      k = e;
    }
    return true;
  };
  std::vector<std::string> stack;
  std::string text, pn, et;
  bool have_pn = false, have_et = false, in_part = false, root_done = false;
  while (i < b.size()) {
    if (b[i] != '<') {
      text.push_back(b[i++]);
      continue;
    }
    size_t e = b.find('>', i);
    if (e == std::string::npos) return false;
    std::string tag = b.substr(i + 1, e - i - 1);
    i = e + 1;
    if (tag.empty() || tag[0] == '!') return false;     // comments, CDATA, DTD
    if (tag[0] == '?') {
      if (!stack.empty()) return false;
      continue;
    }
    const bool closing = tag[0] == '/';
    const bool empty_el = !closing && tag.back() == '/';
    std::string name = closing ? tag.substr(1) : (empty_el ? tag.substr(0, tag.size() - 1) : tag);
    name = name.substr(0, name.find_first_of(" \t\r\n"));
    if (name.empty()) return false;
    if (closing) {
      if (stack.empty() || stack.back() != name) return false;
      const std::string ln = local(name);
      if (stack.size() == 3 && in_part) {
        std::string v;
        if (!unescape(text, &v)) return false;
        if (ln == "PartNumber" && !have_pn) pn = v, have_pn = true;
        if (ln == "ETag" && !have_et) et = v, have_et = true;
      }
      if (stack.size() == 2 && in_part) {
        // int(_text(p, "PartNumber", "0")), _text(p, "ETag", "").strip()
        std::string num = have_pn ? pn : "0";
        auto trimws = [](std::string v) {
          size_t a = v.find_first_not_of(" \t\r\n"), z = v.find_last_not_of(" \t\r\n");
          return a == std::string::npos ? std::string() : v.substr(a, z - a + 1);
        };
        num = trimws(num);
        size_t d = num.size() && (num[0] == '+' || num[0] == '-') ? 1 : 0;
        if (num.size() == d || num.size() > 12 || num.find_first_not_of("0123456789", d) != std::string::npos)
          return false;
        parts->emplace_back(std::stoll(num), trimws(have_et ? et : ""));
        in_part = false;
      }
      stack.pop_back();
      if (stack.empty()) root_done = true;
      text.clear();
      continue;
    }
    if (root_done) return false;  // a second root element
    stack.push_back(name);
    text.clear();
    if (stack.size() == 2 && local(name) == "Part") {
      in_part = true;
      have_pn = have_et = false;
    }
    if (empty_el) {
      if (stack.size() == 3 && in_part) {
        const std::string ln = local(name);
        if (ln == "PartNumber" && !have_pn) pn.clear(), have_pn = true;
        if (ln == "ETag" && !have_et) et.clear(), have_et = true;
      }
      if (stack.size() == 2 && in_part) {
        parts->emplace_back(0, "");  // <Part/>: PartNumber "0" -> rejected below as invalid part
        in_part = false;
      }
      stack.pop_back();
      if (stack.empty()) root_done = true;
    }
  }
  return stack.empty() && root_done;
}

}  // namespace

// CompleteMultipartUpload (reference handlers.rs:322-432, tests/models/s3_gateway.py complete_mpu): the
// parts listed with their metadata in one ListFiles, validated against the request, the
// object's ETag md5(concat(md5s))-N, the completion marker written with the layout, and the
// parts renamed under the object in parallel (each rename one Raft entry, or the master's
// 2PC when the object's shard differs). Errors before anything changed are Python's.
// InitiateMultipartUpload (reference handlers.rs:234-262): a fresh upload id and its marker
// file /.s3_mpu/<id>/.s3keep (the Python gateway's initiate_mpu, same layout).
bool S3Front::native_initiate(Conn* c, Req& r, const std::string& bucket, const std::string& key,
                              std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.mpu_initiate");
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return proxy(c, r, nullptr, 0, why);
  const std::string uid = uuid4();
  {
    int64_t slot = fc_->acquire_slot(1);
    if (slot < 0) return proxy(c, r, nullptr, 0, "mpu-init");
    FastClient::Times t;
    std::string md5, msg;
    int reps = 0;
    auto st = fc_->write_slot("/.s3_mpu/" + uid + "/.s3keep", slot, 0, &reps, &msg, &t, r.rid, nullptr, nullptr, &md5);
    fc_->release(slot);
    if (st != FastClient::Ok) return proxy(c, r, nullptr, 0, "mpu-init");
  }
  const std::string x = "<InitiateMultipartUploadResult>" + xel("Bucket", bucket) + xel("Key", key) +
                        xel("UploadId", uid) + "</InitiateMultipartUploadResult>";
  std::string h = "HTTP/1.1 200 OK\r\nContent-Type: application/xml\r\nContent-Length: " + std::to_string(x.size()) +
                  "\r\n" + (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
  r.status = 200;
  count(r, 200);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.mpu_initiates++;
  }
  const bool ok = send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(x.data()), x.size());
  if (cfg_.auth_enabled) audit(c, r, user, 200, sess.role_arn);
  return ok;
}

bool S3Front::native_complete(Conn* c, Req& r, const std::string& bucket, const std::string& key,
                              std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.mpu_complete");
  const std::string upload_id = q["uploadId"];
  std::string body(static_cast<size_t>(r.content_length), '\0');
  if (r.expect_continue && !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
  if (!read_body(c, reinterpret_cast<uint8_t*>(&body[0]), body.size())) return false;
  r.expect_continue = false;  // the body is read: a hand-over sends it along
  auto hand_over = [&](const std::string& why) {
    return proxy(c, r, reinterpret_cast<const uint8_t*>(body.data()), body.size(), why);
  };
  if (upload_id.empty() || upload_id.find('/') != std::string::npos || upload_id == "." || upload_id == "..")
    return hand_over("mpu-args");
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return hand_over(why);
  std::vector<std::pair<int64_t, std::string>> requested;
  bool blank = body.find_first_not_of(" \t\r\n") == std::string::npos;
  if (!blank && !parse_complete_body(body, &requested)) return hand_over("mpu-xml");
  const std::string mpu_dir = "/.s3_mpu/" + upload_id, dest = "/" + bucket + "/" + key;
  std::vector<std::pair<std::string, pb::FileMetadata>> files;
  if (fc_->list(mpu_dir + "/", &files, r.rid) != FastClient::Ok) return hand_over("mpu-list");
  bool has_marker = false;
  std::map<int64_t, std::pair<std::string, uint64_t>> have;  // part -> (etag hex, size)
  for (auto& f : files) {
    if (f.first == mpu_dir + "/.s3keep") has_marker = true;
    const std::string tail = f.first.substr(std::min(f.first.size(), mpu_dir.size() + 1));
    if (f.first.compare(0, mpu_dir.size() + 1, mpu_dir + "/") == 0 && !tail.empty() && tail.size() <= 9 &&
        all_digits(tail))
      have[std::stoll(tail)] = {f.second.etag_md5, f.second.size};
  }
  if (!has_marker) return hand_over("mpu-missing");  // NoSuchUpload
  std::vector<int64_t> nums;
  if (!requested.empty()) {
    auto unq = [](std::string v) {
      while (!v.empty() && v.front() == '"') v.erase(v.begin());
      while (!v.empty() && v.back() == '"') v.pop_back();
      return v;
    };
    for (auto& rq : requested) {
      auto h = have.find(rq.first);
      if (h == have.end() || (!rq.second.empty() && unq(rq.second) != h->second.first)) return hand_over("mpu-part");
      nums.push_back(rq.first);
    }
    for (size_t i = 1; i < nums.size(); ++i)
      if (nums[i] <= nums[i - 1]) return hand_over("mpu-order");
  } else {
    for (auto& h : have) nums.push_back(h.first);
  }
  std::string md5s;
  uint64_t total = 0;
  std::string layout;
  for (int64_t n : nums) {
    const std::string& hx = have[n].first;
    if (hx.size() != 32) return hand_over("mpu-etag");
    for (size_t k = 0; k < 32; k += 2) md5s.push_back(static_cast<char>(hexval(hx[k]) * 16 + hexval(hx[k + 1])));
    total += have[n].second;
    layout += (layout.empty() ? "" : ",") + std::to_string(n) + ":" + std::to_string(have[n].second);
  }
  const std::string final_etag = "\"" + crypto::md5_hex(reinterpret_cast<const uint8_t*>(md5s.data()), md5s.size()) +
                                 "-" + std::to_string(nums.size()) + "\"";
  // from here on the namespace changes; a failure is answered 500 like the gateway's DfsError
  auto internal = [&](const std::string& msg) {
    const std::string x = "<Error>" + xel("Code", "InternalError") + xel("Message", msg) + xel("Resource", dest) +
                          "<RequestId></RequestId></Error>";
    std::string h = "HTTP/1.1 500 Internal Server Error\r\nContent-Type: application/xml\r\nContent-Length: " +
                    std::to_string(x.size()) + "\r\nConnection: close\r\n\r\n";
    r.status = 500;
    r.keep_alive = false;
    count(r, 500);
    if (cfg_.auth_enabled) audit(c, r, user, 500, sess.role_arn);
    send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(x.data()), x.size());
    return false;
  };
  std::string msg;
  // replace whatever object was at the destination (plain file or an older multipart one)
  (void)fc_->remove(dest, &msg, r.rid);
  std::vector<std::pair<std::string, pb::FileMetadata>> old;
  if (fc_->list(dest + "/", &old, r.rid) != FastClient::Ok) return internal("listing the destination failed");
  for (auto& f : old) (void)fc_->remove(f.first, &msg, r.rid);
  {
    std::map<std::string, std::string> attrs{{"ETag", final_etag}, {"x-dfs-mpu-size", std::to_string(total)},
                                             {"x-dfs-mpu-layout", layout}};
    int64_t slot = fc_->acquire_slot(1);
    if (slot < 0) return internal("no buffer");
    FastClient::Times t;
    std::string md5;
    int reps = 0;
    auto st = fc_->write_slot(dest + "/.s3_mpu_completed", slot, 0, &reps, &msg, &t, r.rid, &attrs, nullptr, &md5);
    fc_->release(slot);
    if (st != FastClient::Ok) return internal("Failed to create completion marker: " + msg);
    (void)write_sidecar(dest, attrs, r.rid);
  }
  // the parts move under the object concurrently (independent files, independent Raft entries)
  std::vector<std::future<std::string>> futs;
  for (int64_t n : nums)
    futs.push_back(pool_.submit([this, n, &mpu_dir, &dest, &r] {
      std::string m;
      const std::string num = std::to_string(n);
      auto st = fc_->rename(mpu_dir + "/" + num, dest + "/" + num, &m, r.rid);
      return st == FastClient::Ok ? std::string() : (m.empty() ? "rename of part " + num + " failed" : m);
    }));
  std::string first_err;
  for (auto& f : futs) {
    std::string e = f.get();
    if (!e.empty() && first_err.empty()) first_err = e;
  }
  if (!first_err.empty()) return internal(first_err);
  std::set<int64_t> used(nums.begin(), nums.end());
  for (auto& f : files) {
    const std::string tail = f.first.substr(std::min(f.first.size(), mpu_dir.size() + 1));
    const bool part = !tail.empty() && tail.size() <= 9 && all_digits(tail);
    if (ends_with(f.first, ".etag") || f.first == mpu_dir + "/.s3keep" || (part && !used.count(std::stoll(tail))))
      (void)fc_->remove(f.first, &msg, r.rid);
  }
  const std::string x = "<CompleteMultipartUploadResult>" +
                        xel("Location", "http://localhost:" + std::to_string(cfg_.port) + "/" + bucket + "/" + key) +
                        xel("Bucket", bucket) + xel("Key", key) + xel("ETag", final_etag) +
                        "</CompleteMultipartUploadResult>";
  std::string h = "HTTP/1.1 200 OK\r\nContent-Type: application/xml\r\nContent-Length: " + std::to_string(x.size()) +
                  "\r\n" + (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
  r.status = 200;
  count(r, 200);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.mpu_completes++;
  }
  const bool ok = send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(x.data()), x.size());
  if (cfg_.auth_enabled) audit(c, r, user, 200, sess.role_arn);
  return ok;
}

// GET of an SSE object (SseManager.decrypt_object, reference auth/sse.rs:64-110): the whole
// ciphertext is read into a slot, the DEK unwrapped with the KEK, the object decrypted in
// place (the GCM tag authenticates it) and the (range of the) plaintext sent from there.
bool S3Front::sse_get(Conn* c, Req& r, const std::string& meta, uint64_t size, const std::string& hdrs,
                      const std::string& dek_b64) {
  TraceRange tr("dfs.s3.get_sse");
  std::string wrapped, dk;
  if (size < 28 || size > fc_->slot_bytes() || !crypto::base64_decode(dek_b64, &wrapped) || wrapped.size() < 60)
    return proxy(c, r, nullptr, 0, "sse");
  try {
    dk = crypto::aes256gcm_decrypt(cfg_.sse_kek, wrapped.substr(0, 12), wrapped.substr(12), "");
  } catch (const std::exception&) {
    return proxy(c, r, nullptr, 0, "sse");  // Python answers 500 InternalError
  }
  if (dk.size() != 32) return proxy(c, r, nullptr, 0, "sse");
  int64_t slot = -1;
  uint64_t got = 0;
  std::string msg;
  FastClient::Times t;
  if (fc_->read_known(meta, &slot, &got, &msg, &t, r.rid, 0, 0) != FastClient::Ok) return proxy(c, r, nullptr, 0, "read");
  struct Release {
    FrontStore* fc;
    int64_t s;
    ~Release() {
      if (s >= 0) fc->release(s);
    }
  } rel{fc_, slot};
  if (got != size) return proxy(c, r, nullptr, 0, "short-read");
  uint8_t* b = fc_->slot_mut(slot);
  const uint64_t plen = size - 28;
  if (!crypto::aes256gcm_decrypt_inplace(reinterpret_cast<const uint8_t*>(dk.data()), b, b + 12, plen, b + 12 + plen))
    return proxy(c, r, nullptr, 0, "sse");
  uint64_t s = 0, e = 0;
  int rng = parse_range(r.get("range"), plen, &s, &e);
  if (rng >= 2) return proxy(c, r, nullptr, 0, "range");
  const uint64_t from = rng == 1 ? s : 0, want = rng == 1 ? e - s + 1 : plen;
  const std::string ka = r.keep_alive ? "Connection: keep-alive\r\n" : "Connection: close\r\n";
  std::string h;
  if (rng == 1) {
    h = "HTTP/1.1 206 Partial Content\r\n" + hdrs + "Content-Range: bytes " + std::to_string(s) + "-" +
        std::to_string(e) + "/" + std::to_string(plen) + "\r\n";
    r.status = 206;
  } else {
    h = "HTTP/1.1 200 OK\r\n" + hdrs;
    r.status = 200;
  }
  h += "Content-Length: " + std::to_string(want) + "\r\n" + ka + "\r\n";
  count(r, r.status);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    (rng == 1 ? st_.range_gets : st_.gets)++;
    st_.sse_gets++;
    st_.bytes_out += want;
  }
  return send_head_body(c->io(), h, b + 12 + from, want);
}

// GET of a completed multipart object: the parts' sizes come from the layout the completion
// recorded (x-dfs-mpu-layout), every part overlapping the range is checked first (so a
// missing part still turns into Python's answer), then the parts stream out in order while
// the next one is already being read.
bool S3Front::native_mpu_get(Conn* c, Req& r, const std::string& path, const std::string& marker_meta) {
  TraceRange tr("dfs.s3.mpu_get");
  pb::FileMetadata mk;
  if (!mk.decode(marker_meta)) return proxy(c, r, nullptr, 0, "decode");
  std::vector<std::pair<uint64_t, uint64_t>> parts;  // (number, size)
  auto lay = mk.attributes.find("x-dfs-mpu-layout");
  if (lay != mk.attributes.end()) {
    if (!parse_layout(lay->second, &parts)) return proxy(c, r, nullptr, 0, "mpu-layout");
  } else {
    // completed by the reference's gateway (no recorded layout): the parts are the numbered
    // files under the object, in number order (handlers.rs:1088-1176)
    std::vector<std::pair<std::string, pb::FileMetadata>> files;
    if (fc_->list(path + "/", &files, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "mpu-layout");
    for (auto& f : files) {
      const std::string tail = f.first.substr(path.size() + 1);
      if (!tail.empty() && tail.size() <= 9 && all_digits(tail)) parts.emplace_back(std::stoull(tail), f.second.size);
    }
    std::sort(parts.begin(), parts.end());
  }
  std::map<std::string, std::string> side;
  if (mk.attributes.empty() && !read_sidecar(path, r.rid, &side)) return proxy(c, r, nullptr, 0, "sidecar");
  std::string hdrs;
  if (!object_headers(nullptr, mk.attributes.empty() ? side : mk.attributes, &hdrs)) return proxy(c, r, nullptr, 0, "attrs");
  uint64_t total = 0;
  for (auto& p : parts) total += p.second;
  uint64_t s = 0, e = total ? total - 1 : 0;
  int rng = parse_range(r.get("range"), total, &s, &e);
  if (rng >= 2 || total == 0) return proxy(c, r, nullptr, 0, "mpu-range");
  if (rng == 0) {
    s = 0;
    e = total - 1;
  }
  struct Piece {
    std::string meta;
    uint64_t off, len;
    bool whole;
  };
  std::vector<Piece> pieces;
  uint64_t pos = 0;
  for (auto& p : parts) {
    uint64_t lo = std::max(s, pos), hi = std::min(e + 1, pos + p.second);
    if (lo < hi) {
      bool found = false;
      std::string pm, msg;
      if (fc_->stat(path + "/" + std::to_string(p.first), &found, &pm, &msg, r.rid) != FastClient::Ok || !found)
        return proxy(c, r, nullptr, 0, "mpu-part");
      pb::FileMetadata m;
      if (!m.decode(pm) || m.size != p.second) return proxy(c, r, nullptr, 0, "mpu-part");
      pieces.push_back({pm, lo - pos, hi - lo, lo == pos && hi == pos + p.second});
    }
    pos += p.second;
  }
  const std::string ka = r.keep_alive ? "Connection: keep-alive\r\n" : "Connection: close\r\n";
  std::string h;
  const uint64_t len = e - s + 1;
  if (rng == 1) {
    h = "HTTP/1.1 206 Partial Content\r\n" + hdrs + "Content-Range: bytes " + std::to_string(s) + "-" +
        std::to_string(e) + "/" + std::to_string(total) + "\r\n";
    r.status = 206;
  } else {
    h = "HTTP/1.1 200 OK\r\n" + hdrs;
    r.status = 200;
  }
  h += "Content-Length: " + std::to_string(len) + "\r\n" + ka + "\r\n";
  struct Got {
    int64_t slot = -1;
    uint64_t n = 0;
    bool ok = false;
  };
  auto fetch = [this, &r](const Piece& pc) {
    Got g;
    std::string msg;
    FastClient::Times t;
    g.ok = fc_->read_known(pc.meta, &g.slot, &g.n, &msg, &t, r.rid, pc.whole ? 0 : pc.off, pc.whole ? 0 : pc.len) ==
               FastClient::Ok &&
           g.n == pc.len;
    return g;
  };
  // the first part is read before the head goes out, so an unreadable object is still
  // answered by Python; later failures can only cut the connection
  std::deque<std::future<Got>> inflight;
  size_t next = 0;
  const size_t window = 3;
  while (next < pieces.size() && inflight.size() < window) {
    const Piece* pc = &pieces[next++];
    inflight.push_back(pool_.submit([fetch, pc] { return fetch(*pc); }));
  }
  bool sent_head = false, ok = true;
  while (!inflight.empty()) {
    Got g = inflight.front().get();
    inflight.pop_front();
    if (ok && next < pieces.size()) {
      const Piece* pc = &pieces[next++];
      inflight.push_back(pool_.submit([fetch, pc] { return fetch(*pc); }));
    }
    if (!g.ok || !ok) {
      if (g.slot >= 0) fc_->release(g.slot);
      if (!sent_head && ok) {
        ok = false;
        for (auto& f : inflight) {  // drain before handing the request over
          Got x = f.get();
          if (x.slot >= 0) fc_->release(x.slot);
        }
        inflight.clear();
        return proxy(c, r, nullptr, 0, "mpu-read");
      }
      ok = false;
      continue;
    }
    bool w = sent_head ? send_all(c->io(), fc_->slot_ptr(g.slot), g.n)
                       : send_head_body(c->io(), h, fc_->slot_ptr(g.slot), g.n);
    sent_head = true;
    fc_->release(g.slot);
    if (!w) ok = false;
  }
  if (!ok) return false;
  count(r, r.status);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.mpu_gets++;
    st_.bytes_out += len;
  }
  return true;
}

// ---------------------------------------------------------------- delete, copy, aws-chunked
bool S3Front::respond(Conn* c, Req& r, int status, const std::string& xml, const std::string& extra) {
  const char* reason = status == 200 ? "OK" : status == 204 ? "No Content" : status == 400 ? "Bad Request"
                       : status == 403 ? "Forbidden" : status == 404 ? "Not Found" : status == 409 ? "Conflict"
                       : status == 416 ? "Range Not Satisfiable" : status == 405 ? "Method Not Allowed"
                       : status == 501 ? "Not Implemented" : "Internal Server Error";
  std::string h = "HTTP/1.1 " + std::to_string(status) + " " + reason + "\r\n" + extra;
  if (!xml.empty()) h += "Content-Type: application/xml\r\n";
  if (status != 204 && extra.find("Content-Length:") == std::string::npos)
    h += "Content-Length: " + std::to_string(xml.size()) + "\r\n";
  h += r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
  r.status = status;
  count(r, status);
  return send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(xml.data()), xml.size());
}

// X.error of tests/models/s3_xml.py
bool S3Front::s3_error(Conn* c, Req& r, int status, const std::string& code, const std::string& msg,
                       const std::string& resource) {
  return respond(c, r, status,
                 "<Error>" + xel("Code", code) + xel("Message", msg) + xel("Resource", resource) +
                     "<RequestId></RequestId></Error>");
}

namespace {

// The request body as a byte stream: Content-Length framed, or in the HTTP/1.1 chunked transfer
// coding — what the AWS SDKs send for streaming uploads (Transfer-Encoding: chunked around an
// aws-chunked payload, x-amz-decoded-content-length giving the object size). Reads go through
// the connection buffer, then straight from the socket into the destination.
class BodyIn {
 public:
  BodyIn(S3Front::Conn* c, bool chunked, uint64_t content_length, Io io)
      : c_(c), io_(io), chunked_(chunked), left_(chunked ? 0 : content_length) {}
  // Exactly n bytes of the body into dst: 1 ok, 0 connection error, -1 the body ends first.
  int read(uint8_t* dst, uint64_t n) {
    while (n) {
      uint64_t a;
      int rc = avail(&a);
      if (rc != 1) return rc == 2 ? -1 : rc;
      uint64_t k = std::min(a, n), have = std::min<uint64_t>(k, buf_left());
      if (have) {
        std::memcpy(dst, c_->buf.data() + c_->pos, have);
        c_->pos += have;
      } else {
        long g = io_recv(io_, dst, k);
        if (g <= 0) return 0;
        have = static_cast<uint64_t>(g);
      }
      dst += have;
      n -= have;
      left_ -= have;
    }
    return 1;
  }
  // One CRLF-terminated line of the body (at most `max` bytes), without the CRLF.
  int line(std::string* out, size_t max) {
    out->clear();
    for (;;) {
      uint64_t a;
      int rc = avail(&a);
      if (rc != 1) return rc == 2 ? -1 : rc;
      if (!buf_left() && !fill()) return 0;
      const size_t lim = static_cast<size_t>(std::min<uint64_t>(a, buf_left()));
      const char* p = c_->buf.data() + c_->pos;
      const char* nl = static_cast<const char*>(std::memchr(p, '\n', lim));
      const size_t take = nl ? static_cast<size_t>(nl - p) + 1 : lim;
      out->append(p, take);
      c_->pos += take;
      left_ -= take;
      if (out->size() > max + 2) return -1;
      if (nl) {
        if (out->size() < 2 || (*out)[out->size() - 2] != '\r') return -1;
        out->resize(out->size() - 2);
        return 1;
      }
    }
  }
  // The rest of the body, discarded: 1 at its end, 0 connection error, -1 bad framing.
  int drain() {
    for (;;) {
      uint64_t a;
      int rc = avail(&a);
      if (rc == 2) return 1;
      if (rc != 1) return rc;
      if (!buf_left() && !fill()) return 0;
      const uint64_t k = std::min<uint64_t>(a, buf_left());
      c_->pos += k;
      left_ -= k;
    }
  }

 private:
  uint64_t buf_left() const { return c_->buf.size() - c_->pos; }
  bool fill() {
    char tmp[16 << 10];
    c_->buf.erase(0, c_->pos);
    c_->pos = 0;
    long k = io_recv(io_, tmp, sizeof tmp);
    if (k <= 0) return false;
    c_->buf.append(tmp, static_cast<size_t>(k));
    return true;
  }
  // A CRLF line of the HTTP framing itself (chunk sizes, trailers).
  int raw_line(std::string* out, size_t max) {
    for (;;) {
      size_t e = c_->buf.find("\r\n", c_->pos);
      if (e != std::string::npos) {
        if (e - c_->pos > max) return -1;
        out->assign(c_->buf, c_->pos, e - c_->pos);
        c_->pos = e + 2;
        return 1;
      }
      if (buf_left() > max + 1) return -1;
      char tmp[4096];
      long k = io_recv(io_, tmp, sizeof tmp);
      if (k <= 0) return 0;
      c_->buf.append(tmp, static_cast<size_t>(k));
    }
  }
  // 1: *n > 0 body bytes are next; 2: the body has ended; 0 connection error; -1 bad framing.
  int avail(uint64_t* n) {
    if (!chunked_) {
      if (!left_) return 2;
      *n = left_;
      return 1;
    }
    while (!left_) {
      if (eof_) return 2;
      std::string h;
      int rc;
      if (need_crlf_) {  // the CRLF after the previous chunk's data
        if ((rc = raw_line(&h, 0)) != 1) return rc;
        need_crlf_ = false;
      }
      if ((rc = raw_line(&h, 1024)) != 1) return rc;
      const std::string hex = trim(h.substr(0, h.find(';')));
      if (hex.empty() || hex.size() > 15 || hex.find_first_not_of("0123456789abcdefABCDEF") != std::string::npos)
        return -1;
      left_ = std::stoull(hex, nullptr, 16);
      if (!left_) {  // the last chunk: trailers up to the empty line
        for (;;) {
          if ((rc = raw_line(&h, 8192)) != 1) return rc;
          if (h.empty()) break;
        }
        eof_ = true;
        return 2;
      }
      need_crlf_ = true;
    }
    *n = left_;
    return 1;
  }

  S3Front::Conn* c_;
  Io io_;
  bool chunked_, eof_ = false, need_crlf_ = false;
  uint64_t left_;
};

}  // namespace

// aws-chunked framing, `<hex>[;chunk-signature=<sig>]\r\n<data>\r\n ... 0[;...]\r\n[trailers]`
// (s3/auth/sigv4.py decode_chunked, reference auth_middleware.rs streaming payloads), read
// straight from the connection — Content-Length framed, or inside HTTP chunked transfer
// coding as the SDKs send it: chunk headers through the connection buffer, chunk data into
// the slot. With STREAMING-AWS4-HMAC-SHA256-PAYLOAD on an authenticated gateway every chunk,
// the final empty one included, must continue the request signature's chain.
int S3Front::read_aws_chunked(Conn* c, Req& r, uint8_t* dst, uint64_t cap, uint64_t* n_out) {
  const std::string* sha = r.get("x-amz-content-sha256");
  sigv4::ChunkChain* chain =
      cfg_.auth_enabled && r.chain_set && sha && *sha == "STREAMING-AWS4-HMAC-SHA256-PAYLOAD" ? &r.chain : nullptr;
  BodyIn in(c, r.chunked, static_cast<uint64_t>(std::max<int64_t>(r.content_length, 0)), c->io());
  const AwsChunkedResult res = decode_aws_chunked(in, chain, dst, cap);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.chunk_sigs += res.sigs;
    if (res.rc < 0 && chain) st_.chunk_sig_failures++;
  }
  if (res.rc == 1) *n_out = res.bytes;
  return res.rc;
}

// CreateBucket / HeadBucket (reference handlers.rs:667-722; tests/models/s3_gateway.py create_bucket,
// head_bucket): the bucket is its marker file /<bucket>/.s3keep. A CreateBucketConfiguration
// body is read and ignored, as the gateway does.
bool S3Front::native_bucket(Conn* c, Req& r, const std::string& bucket, std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.bucket");
  std::string body;
  if (r.content_length > 0) {
    if (r.expect_continue && !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
    body.resize(static_cast<size_t>(r.content_length));
    if (!read_body(c, reinterpret_cast<uint8_t*>(&body[0]), body.size())) return false;
    r.expect_continue = false;
  }
  auto hand_over = [&](const std::string& why) {
    return proxy(c, r, body.empty() ? nullptr : reinterpret_cast<const uint8_t*>(body.data()), body.size(), why);
  };
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return hand_over(why);
  const std::string marker = "/" + bucket + "/.s3keep", polpath = "/" + bucket + "/.s3_bucket_policy";
  std::string msg;
  bool ok;
  auto write_small = [&](const std::string& path, const std::string& data, std::string* m) {
    int64_t slot = fc_->acquire_slot(std::max<size_t>(data.size(), 1));
    if (slot < 0) return FastClient::NotHandled;
    if (!data.empty()) std::memcpy(fc_->slot_mut(slot), data.data(), data.size());
    FastClient::Times t;
    std::string md5;
    int reps = 0;
    auto st = fc_->write_slot(path, slot, data.size(), &reps, m, &t, r.rid, nullptr, nullptr, &md5);
    fc_->release(slot);
    return st;
  };
  if (q.count("policy")) {
    // Get/Put/DeleteBucketPolicy (reference handlers.rs bucket policy; tests/models/s3_gateway.py)
    if (r.method == "GET") {
      bool found = false;
      std::string meta, doc;
      if (fc_->stat(polpath, &found, &meta, &msg, r.rid) != FastClient::Ok) return hand_over("policy");
      bool valid = false;
      if (found) {
        int64_t slot = -1;
        uint64_t n = 0;
        FastClient::Times t;
        if (fc_->read_known(meta, &slot, &n, &msg, &t, r.rid, 0, 0) != FastClient::Ok) return hand_over("policy");
        doc.assign(reinterpret_cast<const char*>(fc_->slot_ptr(slot)), n);
        fc_->release(slot);
        try {
          (void)Json::parse(doc);
          valid = true;
        } catch (const std::exception&) {
        }
      }
      if (!valid) {
        ok = respond(c, r, 404,
                     "<Error>" + xel("Code", "NoSuchBucketPolicy") + xel("Message", "The bucket policy does not exist") +
                         "<Resource></Resource><RequestId></RequestId>" + xel("BucketName", bucket) + "</Error>");
      } else {
        std::string h = "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: " +
                        std::to_string(doc.size()) + "\r\n" +
                        (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
        r.status = 200;
        count(r, 200);
        ok = send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(doc.data()), doc.size());
      }
    } else if (r.method == "PUT") {
      try {
        (void)s3policy::BucketPolicy::parse(body);
      } catch (const std::exception&) {
        ok = respond(c, r, 400, "<Error><Code>MalformedPolicy</Code><Message>Bucket policy must be valid JSON"
                                "</Message></Error>");
        goto done;
      }
      auto st = write_small(polpath, body, &msg);
      if (st == FastClient::Failed && msg.find("already exists") != std::string::npos) {
        std::string dm;
        if (fc_->remove(polpath, &dm, r.rid) == FastClient::NotHandled) return hand_over("policy");
        st = write_small(polpath, body, &msg);
      }
      if (st == FastClient::NotHandled) return hand_over("policy");
      if (st != FastClient::Ok) {
        ok = respond(c, r, 500, "<Error><Code>InternalError</Code><Message>Failed to store bucket policy"
                                "</Message></Error>");
        goto done;
      }
      policy_changed();
      ok = respond(c, r, 204, "");
    } else if (r.method == "DELETE") {
      if (fc_->remove(polpath, &msg, r.rid) == FastClient::NotHandled) return hand_over("policy");
      policy_changed();
      ok = respond(c, r, 204, "");
    } else {
      return hand_over("method");
    }
  } else if (q.count("location")) {
    ok = respond(c, r, 200, "<LocationConstraint>" + xml_escape(cfg_.region) + "</LocationConstraint>");
  } else if (r.method == "PUT") {
    auto st = write_small(marker, std::string(), &msg);
    if (st == FastClient::Failed && msg.find("already exists") != std::string::npos) ok = respond(c, r, 409, "");
    else if (st != FastClient::Ok) return hand_over("bucket");
    else ok = respond(c, r, 200, "", "Location: /" + bucket + "\r\n");
  } else if (r.method == "DELETE") {
    // DeleteBucket: empty (only the marker and policy) -> both removed; objects -> 409
    std::vector<std::pair<std::string, pb::FileMetadata>> files;
    if (fc_->list("/" + bucket + "/", &files, r.rid) != FastClient::Ok) return hand_over("bucket");
    bool objects = false;
    for (auto& f : files)
      if (!ends_with(f.first, ".s3keep") && !ends_with(f.first, ".s3_bucket_policy")) objects = true;
    if (objects) {
      ok = s3_error(c, r, 409, "BucketNotEmpty", "The bucket you tried to delete is not empty", bucket);
    } else if (files.empty()) {
      ok = s3_error(c, r, 404, "NoSuchBucket", "The specified bucket does not exist", bucket);
    } else {
      for (auto& f : files) {
        std::string dm;
        (void)fc_->remove(f.first, &dm, r.rid);
      }
      policy_changed();
      ok = respond(c, r, 204, "");
    }
  } else {  // HEAD
    bool found = false;
    std::string meta;
    if (fc_->stat(marker, &found, &meta, &msg, r.rid) != FastClient::Ok) return hand_over("bucket");
    if (!found) {  // a bucket of objects written without the marker still exists
      std::vector<std::pair<std::string, pb::FileMetadata>> files;
      if (fc_->list("/" + bucket + "/", &files, r.rid) != FastClient::Ok) return hand_over("bucket");
      found = !files.empty();
    }
    ok = respond(c, r, found ? 200 : 404, "", "Content-Length: 0\r\n");
  }
done:
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.bucket_ops++;
  }
  if (cfg_.auth_enabled) audit(c, r, user, r.status, sess.role_arn);
  return ok;
}

// ListBuckets (reference handlers.rs list_buckets; tests/models/s3_gateway.py list_buckets): the first path
// component of every file in the namespace, the multipart staging root left out.
bool S3Front::native_list_buckets(Conn* c, Req& r) {
  TraceRange tr("dfs.s3.list_buckets");
  std::map<std::string, std::string> q;
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, "", q, &user, &sess, &why)) return proxy(c, r, nullptr, 0, why);
  // one entry per bucket from each master (ListFiles with the "/" delimiter walks the ordered
  // path index bucket to bucket), not every file of the namespace
  std::set<std::string> names;
  if (fc_->list_components("/", &names, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "list");
  names.erase(".s3_mpu");
  std::string inner;
  for (auto& n : names) inner += "<Bucket>" + xel("Name", n) + xel("CreationDate", "2025-01-01T00:00:00.000Z") + "</Bucket>";
  const bool ok = respond(c, r, 200, "<ListAllMyBucketsResult><Owner><ID>dfs</ID><DisplayName>dfs</DisplayName></Owner>"
                                     "<Buckets>" + inner + "</Buckets></ListAllMyBucketsResult>");
  if (cfg_.auth_enabled) audit(c, r, user, 200, sess.role_arn);
  return ok;
}

// DeleteObject (reference handlers.rs delete_object; tests/models/s3_gateway.py delete_object): the object
// file, every file of a multipart object under "<key>/", and the sidecar "<key>.meta"; 204
// whether or not anything existed. The three lookups go out together; a master that cannot
// be reached here hands the (idempotent) request to Python.
bool S3Front::native_delete(Conn* c, Req& r, const std::string& path) {
  TraceRange tr("dfs.s3.delete");
  auto kids_f = pool_.submit([this, &path, &r] {
    std::vector<std::pair<std::string, pb::FileMetadata>> kids;
    const bool ok = fc_->list(path + "/", &kids, r.rid) == FastClient::Ok;
    return std::make_pair(ok, std::move(kids));
  });
  auto meta_f = pool_.submit([this, &path, &r] {
    std::string m;
    return fc_->remove(path + ".meta", &m, r.rid);
  });
  std::string msg;
  const bool main_ok = fc_->remove(path, &msg, r.rid) != FastClient::NotHandled;
  auto kids = kids_f.get();
  const bool meta_ok = meta_f.get() != FastClient::NotHandled;
  if (!main_ok || !meta_ok || !kids.first) return proxy(c, r, nullptr, 0, "delete");
  std::atomic<bool> handled{true};
  parallel_for(pool_, kids.second.size(), 16, [&](size_t i) {
    std::string m;
    if (fc_->remove(kids.second[i].first, &m, r.rid) == FastClient::NotHandled) handled = false;
  });
  if (!handled) return proxy(c, r, nullptr, 0, "delete");
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.deletes++;
  }
  return respond(c, r, 204, "");
}

// AbortMultipartUpload (reference handlers.rs:450-470; tests/models/s3_gateway.py abort_mpu): the upload's
// directory /.s3_mpu/<id>/ emptied; 204 whether or not it existed.
bool S3Front::native_abort(Conn* c, Req& r, const std::string& upload_id) {
  TraceRange tr("dfs.s3.mpu_abort");
  std::vector<std::pair<std::string, pb::FileMetadata>> files;
  if (fc_->list("/.s3_mpu/" + upload_id + "/", &files, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "abort");
  std::atomic<bool> handled{true};
  parallel_for(pool_, files.size(), 16, [&](size_t i) {
    std::string m;
    if (fc_->remove(files[i].first, &m, r.rid) == FastClient::NotHandled) handled = false;
  });
  if (!handled) return proxy(c, r, nullptr, 0, "abort");
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.mpu_aborts++;
  }
  return respond(c, r, 204, "");
}

// DeleteObjects (reference handlers.rs:1102-1180; tests/models/s3_gateway.py delete_objects): the
// <Delete><Object><Key>..</Key></Object>..<Quiet/></Delete> body parsed here, the keys removed
// 16 at a time, a missing key reported as deleted, the DeleteResult written here.
bool S3Front::native_delete_objects(Conn* c, Req& r, const std::string& bucket,
                                    std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.delete_objects");
  if (r.chunked || r.content_length <= 0 || r.content_length > (4 << 20) || aws_chunked(r))
    return proxy(c, r, nullptr, 0, "delete-body");
  std::string body(static_cast<size_t>(r.content_length), '\0');
  if (r.expect_continue && !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
  if (!read_body(c, reinterpret_cast<uint8_t*>(&body[0]), body.size())) return false;
  r.expect_continue = false;  // the body is read: a hand-over sends it along
  auto hand_over = [&](const std::string& why) {
    return proxy(c, r, reinterpret_cast<const uint8_t*>(body.data()), body.size(), why);
  };
  std::string user = "anonymous", why;
  Session sess;
  if (!authorize(r, bucket, q, &user, &sess, &why)) return hand_over(why);
  XNode root;
  if (!parse_xml(body, &root) || root.name != "Delete") return hand_over("delete-xml");  // MalformedXML there
  std::vector<std::string> keys;
  for (auto& o : root.kids)
    if (o.name == "Object") {
      const XNode* k = o.child("Key");
      keys.push_back(k ? k->text : std::string());
    }
  bool quiet = false;
  if (const XNode* qn = root.child("Quiet")) quiet = lower(trim(qn->text)) == "true";
  struct Res {
    int kind = 0;  // 0 deleted, 1 error, 2 not handled here
    std::string code, msg;
  };
  std::vector<Res> res(keys.size());
  parallel_for(pool_, keys.size(), 16, [&](size_t i) {
    const std::string& k = keys[i];
    Res& o = res[i];
    if (reserved_key(k)) {
      o = {1, "InvalidArgument", "object key " + py_repr(k) + " is reserved"};
      return;
    }
    const std::string path = "/" + bucket + "/" + k;
    std::string m;
    auto st = fc_->remove(path, &m, r.rid);
    if (st == FastClient::NotHandled) {
      o.kind = 2;
      return;
    }
    if (st == FastClient::Failed && lower(m).find("not found") == std::string::npos) {
      o = {1, "InternalError", m};
      return;
    }
    (void)fc_->remove(path + ".meta", &m, r.rid);
  });
  std::string deleted, errors;
  uint64_t nd = 0;
  for (size_t i = 0; i < keys.size(); ++i) {
    if (res[i].kind == 2) return hand_over("delete");  // every key again, in Python
    if (res[i].kind == 0) {
      ++nd;
      if (!quiet) deleted += "<Deleted>" + xel("Key", keys[i]) + "</Deleted>";
    } else {
      errors += "<Error>" + xel("Key", keys[i]) + xel("Code", res[i].code) + xel("Message", res[i].msg) + "</Error>";
    }
  }
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.multi_deletes++;
    st_.deleted_keys += nd;
  }
  const bool ok = respond(c, r, 200, "<DeleteResult>" + deleted + errors + "</DeleteResult>");
  if (cfg_.auth_enabled) audit(c, r, user, 200, sess.role_arn);
  return ok;
}

// CopyObject (reference handlers.rs:1182-1290; tests/models/s3_gateway.py copy_object): the source — a plain
// object, or a completed multipart one whose parts are read into one slot in parallel — is
// decrypted in place when SSE wrapped it, re-encrypted under a fresh DEK when the gateway is
// SSE, and written to the destination from the same slot with the source's (COPY) or the
// request's (REPLACE) x-amz-meta-* headers. A missing or sidecar-described source, and any
// error this path does not model, is Python's.
bool S3Front::native_copy(Conn* c, Req& r, const std::string& dest) {
  TraceRange tr("dfs.s3.copy");
  std::string src;
  {
    std::string raw = *r.get("x-amz-copy-source");
    raw = raw.substr(0, raw.find('?'));
    if (!unquote(raw, &src)) return proxy(c, r, nullptr, 0, "copy-args");
    if (src.empty() || src[0] != '/') src = "/" + src;
    if (reserved_key(src)) return proxy(c, r, nullptr, 0, "copy-args");
  }
  const bool sse = cfg_.sse_enabled;
  const uint64_t room = sse ? 28 : 0;
  bool found = false;
  std::string meta, msg;
  if (fc_->stat(src, &found, &meta, &msg, r.rid) != FastClient::Ok) return proxy(c, r, nullptr, 0, "copy-stat");
  int64_t slot = -1;
  struct Release {
    FrontStore* fc;
    int64_t* s;
    ~Release() {
      if (*s >= 0) fc->release(*s);
    }
  } rel{fc_, &slot};
  std::map<std::string, std::string> src_attrs;
  uint64_t n = 0;
  bool at12 = false;  // the plaintext sits after a 12-byte nonce (a decrypted SSE source)
  if (found) {
    pb::FileMetadata m;
    if (!m.decode(meta)) return proxy(c, r, nullptr, 0, "copy-attrs");
    if (m.attributes.empty() && !read_sidecar(src, r.rid, &src_attrs)) return proxy(c, r, nullptr, 0, "copy-attrs");
    if (!m.attributes.empty()) src_attrs = m.attributes;
    auto dk = src_attrs.find("x-amz-sse-encrypted-dek");
    const bool enc = dk != src_attrs.end();
    if (enc && !sse) return proxy(c, r, nullptr, 0, "sse");
    if (m.size + (enc ? 0 : room) > fc_->slot_bytes()) return proxy(c, r, nullptr, 0, "large");
    if (m.size > 0) {
      uint64_t got = 0;
      FastClient::Times t;
      if (fc_->read_known(meta, &slot, &got, &msg, &t, r.rid, 0, 0) != FastClient::Ok)
        return proxy(c, r, nullptr, 0, "copy-read");
      if (got != m.size) return proxy(c, r, nullptr, 0, "short-read");
    } else if ((slot = fc_->acquire_slot(std::max<uint64_t>(room, 1))) < 0) {
      return proxy(c, r, nullptr, 0, "no-slot");
    }
    n = m.size;
    if (enc) {
      std::string wrapped, key;
      if (m.size < 28 || !crypto::base64_decode(dk->second, &wrapped) || wrapped.size() < 60)
        return proxy(c, r, nullptr, 0, "sse");
      try {
        key = crypto::aes256gcm_decrypt(cfg_.sse_kek, wrapped.substr(0, 12), wrapped.substr(12), "");
      } catch (const std::exception&) {
        return proxy(c, r, nullptr, 0, "sse");
      }
      uint8_t* b = fc_->slot_mut(slot);
      n = m.size - 28;
      if (key.size() != 32 ||
          !crypto::aes256gcm_decrypt_inplace(reinterpret_cast<const uint8_t*>(key.data()), b, b + 12, n, b + 12 + n))
        return proxy(c, r, nullptr, 0, "sse");
      at12 = true;
    }
  } else {
    std::string mm;
    if (fc_->stat(src + "/.s3_mpu_completed", &found, &mm, &msg, r.rid) != FastClient::Ok || !found)
      return proxy(c, r, nullptr, 0, "copy-missing");  // NoSuchKey
    pb::FileMetadata mk;
    if (!mk.decode(mm)) return proxy(c, r, nullptr, 0, "copy-attrs");
    if (mk.attributes.empty() && !read_sidecar(src, r.rid, &src_attrs)) return proxy(c, r, nullptr, 0, "copy-attrs");
    if (!mk.attributes.empty()) src_attrs = mk.attributes;
    auto lay = src_attrs.find("x-dfs-mpu-layout");
    std::vector<std::pair<uint64_t, uint64_t>> parts;
    if (src_attrs.count("x-amz-sse-encrypted-dek") || lay == src_attrs.end() || !parse_layout(lay->second, &parts))
      return proxy(c, r, nullptr, 0, "copy-mpu");
    std::vector<uint64_t> offs;
    for (auto& p : parts) {
      offs.push_back(n);
      n += p.second;
    }
    if (n + room > fc_->slot_bytes()) return proxy(c, r, nullptr, 0, "large");
    if ((slot = fc_->acquire_slot(std::max<uint64_t>(n + room, 1))) < 0) return proxy(c, r, nullptr, 0, "no-slot");
    uint8_t* d = fc_->slot_mut(slot) + (sse ? 12 : 0);
    at12 = sse;
    std::atomic<bool> ok{true};
    parallel_for(pool_, parts.size(), 4, [&](size_t i) {
      if (!ok) return;
      bool f = false;
      std::string pm, e;
      pb::FileMetadata m;
      if (fc_->stat(src + "/" + std::to_string(parts[i].first), &f, &pm, &e, r.rid) != FastClient::Ok || !f ||
          !m.decode(pm) || m.size != parts[i].second) {
        ok = false;
        return;
      }
      if (m.size == 0) return;
      int64_t ps = -1;
      uint64_t got = 0;
      FastClient::Times t;
      if (fc_->read_known(pm, &ps, &got, &e, &t, r.rid, 0, 0) != FastClient::Ok || got != m.size) ok = false;
      else std::memcpy(d + offs[i], fc_->slot_ptr(ps), got);
      if (ps >= 0) fc_->release(ps);
    });
    if (!ok) return proxy(c, r, nullptr, 0, "copy-read");
  }
  uint8_t* b = fc_->slot_mut(slot);
  const std::string md5 = crypto::md5_hex(at12 ? b + 12 : b, n);
  const std::string etag = "\"" + md5 + "\"";
  std::map<std::string, std::string> attrs{{"ETag", etag}};
  const std::string* dir = r.get("x-amz-metadata-directive");
  std::string directive = dir ? *dir : "COPY";
  for (auto& ch : directive) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
  if (directive == "REPLACE") {
    for (auto& h : r.headers)
      if (h.first.compare(0, 11, "x-amz-meta-") == 0) attrs[h.first] = h.second;
  } else {
    for (auto& kv : src_attrs)
      if (kv.first.compare(0, 11, "x-amz-meta-") == 0 || kv.first == "Content-Type") attrs[kv.first] = kv.second;
  }
  uint64_t stored = n;
  if (sse) {  // SseManager.encrypt_object: a fresh DEK, wrapped by the KEK
    if (!at12) std::memmove(b + 12, b, n);
    const std::string dk = crypto::random_bytes(32), n1 = crypto::random_bytes(12), n2 = crypto::random_bytes(12);
    std::memcpy(b, n1.data(), 12);
    crypto::aes256gcm_encrypt_inplace(reinterpret_cast<const uint8_t*>(dk.data()), b, b + 12, n, b + 12 + n);
    attrs["x-amz-sse-encrypted-dek"] = crypto::base64_encode(n2 + crypto::aes256gcm_encrypt(cfg_.sse_kek, n2, dk, ""));
    stored = n + 28;
  }
  FastClient::Times t;
  std::string md5w;
  int reps = 0;
  auto st = fc_->write_slot(dest, slot, stored, &reps, &msg, &t, r.rid, &attrs, nullptr, &md5w);
  if (st == FastClient::Failed && msg.find("already exists") != std::string::npos) {
    std::string dmsg;
    if (fc_->remove(dest, &dmsg, r.rid) != FastClient::NotHandled)
      st = fc_->write_slot(dest, slot, stored, &reps, &msg, &t, r.rid, &attrs, nullptr, &md5w);
  }
  if (st != FastClient::Ok) return proxy(c, r, nullptr, 0, "copy-fallback");  // the copy again, in Python
  (void)write_sidecar(dest, attrs, r.rid);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.copies++;
    st_.copy_bytes += n;
  }
  int64_t ms;
  return respond(c, r, 200,
                 "<CopyObjectResult>" + xel("LastModified", iso_now(now_s(), &ms)) + xel("ETag", etag) +
                     "</CopyObjectResult>");
}

// ---------------------------------------------------------------- a front without Python
namespace {

struct AuthKind {
  const char *code, *message;
  int status;
  const char* error_type;
};

// auth/errors.py (reference common/src/auth/mod.rs:39-108)
const std::map<std::string, AuthKind>& auth_kinds() {
  static const std::map<std::string, AuthKind> k = {
      {"missing_auth", {"AccessDenied", "Access Denied", 403, "missing_auth"}},
      {"invalid_access_key",
       {"InvalidAccessKeyId", "The AWS Access Key Id you provided does not exist in our records.", 403,
        "invalid_access_key"}},
      {"signature_mismatch",
       {"SignatureDoesNotMatch", "The request signature we calculated does not match the signature you provided.",
        403, "signature_mismatch"}},
      {"clock_skew",
       {"RequestTimeTooSkewed", "The difference between the request time and the current time is too large.", 403,
        "clock_skew"}},
      {"invalid_scope",
       {"AuthorizationHeaderMalformed", "The authorization header is malformed; the region or service is wrong.", 400,
        "invalid_credential_scope"}},
      {"insecure_transport", {"AccessDenied", "Access Denied (Insecure Transport)", 403, "insecure_transport"}},
      {"invalid_token", {"InvalidTokenId", "The security token included in the request is invalid.", 403, "invalid_token"}},
      {"expired_token", {"ExpiredToken", "The provided token has expired.", 403, "expired_token"}},
      {"internal", {"InternalError", "An internal error occurred during authentication.", 500, "internal_error"}},
  };
  return k;
}

}  // namespace

bool S3Front::auth_error(Conn* c, Req& r) {
  auto it = auth_kinds().find(r.auth_kind);
  const AuthKind& k = it != auth_kinds().end() ? it->second : auth_kinds().at("missing_auth");
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.auth_results[std::string("failure|") + k.error_type]++;
  }
  const std::string x = std::string("<?xml version=\"1.0\" encoding=\"UTF-8\"?>\n<Error>\n  <Code>") + k.code +
                        "</Code>\n  <Message>" + xml_escape(k.message) + "</Message>\n  <Resource>/</Resource>\n</Error>";
  const bool ok = respond(c, r, k.status, x);
  if (cfg_.auth_enabled) {
    if (r.action.empty()) {
      std::map<std::string, std::string> q;
      std::vector<std::string> keys;
      if (decode_query(r.raw_query, &q))
        for (auto& kv : q) keys.push_back(kv.first);
      r.action = s3policy::resolve_action_and_resource(r.method, r.path, keys).first;
    }
    audit(c, r, r.auth_user, k.status, r.auth_role, r.auth_audit.empty() ? k.code : r.auth_audit);
  }
  return ok;
}

bool S3Front::standalone(Conn* c, Req& r, const uint8_t* body, uint64_t n, const std::string& why) {
  (void)n;
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.standalone_answers++;
    st_.standalone_reasons[why]++;
  }
  // a body this path did not read cannot be skipped reliably: the connection ends after the answer
  if (!body && (r.content_length > 0 || r.chunked)) r.keep_alive = false;
  if (!r.auth_kind.empty()) return auth_error(c, r);
  if (why == "metrics") {
    if (r.raw_path == "/health") {
      std::string h = "HTTP/1.1 200 OK\r\nContent-Type: text/plain; charset=utf-8\r\nContent-Length: 2\r\n" +
                      std::string(r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
      r.status = 200;
      return send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>("OK"), 2);
    }
    const std::string m = native_metrics();
    std::string h = "HTTP/1.1 200 OK\r\nContent-Type: text/plain; charset=utf-8\r\nContent-Length: " +
                    std::to_string(m.size()) + "\r\n" +
                    (r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n");
    r.status = 200;
    return send_head_body(c->io(), h, reinterpret_cast<const uint8_t*>(m.data()), m.size());
  }
  std::string p = r.path.size() > 1 ? r.path.substr(1) : "";
  const size_t slash = p.find('/');
  const std::string bucket = p.substr(0, slash), key = slash == std::string::npos ? "" : p.substr(slash + 1);
  std::map<std::string, std::string> q;
  decode_query(r.raw_query, &q);
  const std::string upload = q.count("uploadId") ? q["uploadId"] : "";
  if (!key.empty() && reserved_key(key))
    return s3_error(c, r, 400, "InvalidArgument", "object key " + py_repr(key) + " is reserved");
  if (why == "list-empty") return s3_error(c, r, 404, "NoSuchBucket", "The specified bucket does not exist", bucket);
  if (why == "missing" || why == "head-missing")
    return s3_error(c, r, 404, "NoSuchKey", "The specified key does not exist.", "/" + bucket + "/" + key);
  if (why == "copy-missing") {
    std::string src;
    const std::string* cs = r.get("x-amz-copy-source");
    if (!cs || !unquote(cs->substr(0, cs->find('?')), &src)) src.clear();
    if (src.empty() || src[0] != '/') src = "/" + src;
    return s3_error(c, r, 404, "NoSuchKey", "The specified key does not exist.", src);
  }
  if (why == "copy-args") return s3_error(c, r, 400, "InvalidArgument", "copy source is reserved");
  if (why == "no-upload" || why == "mpu-missing")
    return s3_error(c, r, 404, "NoSuchUpload", "The specified upload does not exist.", upload);
  if (why == "mpu-part" || why == "mpu-order")
    return s3_error(c, r, 400, why == "mpu-part" ? "InvalidPart" : "InvalidPartOrder",
                    "One or more of the specified parts could not be found or the specified entity tag might not "
                    "have matched.",
                    upload);
  if (why == "mpu-xml" || why == "delete-xml")
    return s3_error(c, r, 400, "MalformedXML", "The XML you provided was not well-formed");
  if (why == "part-args") {
    if (upload.empty() || upload.find('/') != std::string::npos || upload == "." || upload == "..")
      return s3_error(c, r, 400, "InvalidArgument", "bad uploadId");
    const std::string pn = q.count("partNumber") ? q["partNumber"] : "";
    if (!all_digits(pn)) return s3_error(c, r, 400, "InvalidArgument", "bad partNumber");
    return s3_error(c, r, 400, "InvalidArgument", "partNumber must be 1..10000");
  }
  if (why == "list-args") return s3_error(c, r, 400, "InvalidArgument", "max-keys must be an integer");
  if (why == "large")
    return s3_error(c, r, 400, "EntityTooLarge", "Your proposed upload exceeds the maximum allowed object size.");
  if (why == "method") return respond(c, r, 405, "");
  if (why == "uri") return s3_error(c, r, 400, "InvalidURI", "Couldn't parse the specified URI.");
  if (why == "route" || why == "query" || why == "put-form" || why == "body")
    return s3_error(c, r, 501, "NotImplemented", "A header or query you provided implies functionality that is not "
                                                 "implemented.");
  return s3_error(c, r, 500, "InternalError", "the gateway could not serve the request (" + why + ")",
                  r.raw_path);
}

// AssumeRoleWithWebIdentity (reference sts_handler.rs:65-395; tests/models/s3_gateway.py handle_sts): the
// web identity token validated against the OIDC issuer's JWKS, the role's trust policy
// evaluated on its claims, and a session token sealed with the STS key.
bool S3Front::native_sts(Conn* c, Req& r, std::map<std::string, std::string>& q) {
  TraceRange tr("dfs.s3.sts");
  std::map<std::string, std::string> params = q;
  const std::string* ct = r.get("content-type");
  if (r.method == "POST" && ct && lower(*ct).compare(0, 33, "application/x-www-form-urlencoded") == 0) {
    if (r.chunked || r.content_length > (1 << 20)) return standalone(c, r, nullptr, 0, "body");
    std::string body(static_cast<size_t>(std::max<int64_t>(r.content_length, 0)), '\0');
    if (r.expect_continue && !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) return false;
    if (!body.empty() && !read_body(c, reinterpret_cast<uint8_t*>(&body[0]), body.size())) return false;
    std::map<std::string, std::string> form;
    if (decode_query(body, &form))
      for (auto& kv : form) params[kv.first] = kv.second;
  }
  const std::string action = params.count("Action") ? params["Action"] : "Unknown";
  const std::string sts_res = "arn:dfs:sts:::*";
  auto fail = [&](int status, const std::string& code, const std::string& msg, const std::string& user = "anonymous",
                  const std::string& role = "") {
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.sts_results["failure|" + code]++;
    }
    const bool ok = respond(c, r, status,
                            "<ErrorResponse><Error>" + xel("Code", code) + xel("Message", msg) +
                                "</Error><RequestId></RequestId></ErrorResponse>");
    audit(c, r, user, status, role, code, action, sts_res);
    return ok;
  };
  if (action != "AssumeRoleWithWebIdentity") {
    {
      std::lock_guard<std::mutex> g(st_mu_);
      st_.sts_results["failure|InvalidAction"]++;
    }
    const bool ok = respond(c, r, 400, "", "Content-Length: 0\r\n");
    audit(c, r, "anonymous", 400, "", "InvalidAction", action, sts_res);
    return ok;
  }
  if (!oidc_) return fail(500, "OIDC_NOT_ENABLED", "OIDC validation is not enabled on this server.");
  if (sts_keys_.empty()) return fail(500, "STS_NOT_ENABLED", "STS is not enabled on this server.");
  if (!iam_) return fail(500, "IAM_NOT_ENABLED", "IAM policy evaluation is not enabled on this server.");
  const std::string token = params.count("WebIdentityToken") ? params["WebIdentityToken"] : "";
  if (token.empty()) return fail(400, "MissingToken", "WebIdentityToken is required");
  const std::string role_arn = params.count("RoleArn") ? params["RoleArn"] : "";
  if (role_arn.empty()) return fail(400, "MissingRole", "RoleArn is required");
  sts::Claims claims;
  std::string kind, detail;
  const bool valid = oidc_->validate(token, &claims, &kind, &detail);
  {
    std::lock_guard<std::mutex> g(st_mu_);
    st_.oidc_results[valid ? "success" : "failure"]++;
  }
  if (!valid) return fail(403, "InvalidIdentityToken", kind + (detail.empty() ? "" : ": " + detail), "anonymous", role_arn);
  s3policy::Context ctx;
  ctx.principal_id = claims.sub;
  ctx.groups = claims.groups;
  ctx.claims = {{"sub", claims.sub}, {"iss", claims.iss}};
  if (!iam_->can_assume_role(role_arn, ctx))
    return fail(403, "AccessDenied", "User is not authorized to assume this role.", claims.sub, role_arn);
  int64_t duration = 3600;
  if (params.count("DurationSeconds")) {
    const std::string& d = params["DurationSeconds"];
    const bool neg = !d.empty() && d[0] == '-';
    if (!all_digits(neg ? d.substr(1) : d))
      return fail(400, "ValidationError", "DurationSeconds must be an integer", claims.sub, role_arn);
    duration = neg ? -1 : std::stoll(d);
  }
  if (duration < 1 || duration > 43200)
    return fail(400, "ValidationError", "DurationSeconds must be in [1, 43200]", claims.sub, role_arn);
  const int64_t exp = static_cast<int64_t>(now_s()) + duration;
  auto k = sts_keys_.find(cfg_.sts_active_kid);
  if (k == sts_keys_.end())
    return fail(500, "InternalError", "internal: active KID " + std::to_string(cfg_.sts_active_kid) + " not found",
                claims.sub, role_arn);
  const std::string secret = sts::random_alnum(40);
  std::string akid = "ASIA" + uuid4().substr(0, 8) + uuid4().substr(9, 4) + uuid4().substr(14, 4);
  for (auto& ch : akid) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
  const std::string tok = sts::make_token(k->second, cfg_.sts_active_kid, role_arn, secret, exp, claims);
  std::string role_name = role_arn.substr(role_arn.rfind('/') == std::string::npos ? 0 : role_arn.rfind('/') + 1);
  if (role_name.empty()) role_name = "role";
  const std::string session = params.count("RoleSessionName") ? params["RoleSessionName"] : "session";
  char expiration[32];
  time_t et = static_cast<time_t>(exp);
  tm g{};
  gmtime_r(&et, &g);
  std::strftime(expiration, sizeof expiration, "%Y-%m-%dT%H:%M:%SZ", &g);
  {
    std::lock_guard<std::mutex> lg(st_mu_);
    st_.sts_results["success|none"]++;
    st_.sts_issued++;
  }
  const std::string x = "<AssumeRoleWithWebIdentityResponse><AssumeRoleWithWebIdentityResult><Credentials>" +
                        xel("AccessKeyId", akid) + xel("SecretAccessKey", secret) + xel("SessionToken", tok) +
                        xel("Expiration", expiration) + "</Credentials>" + xel("SubjectFromWebIdentityToken", claims.sub) +
                        "<AssumedRoleUser>" + xel("AssumedRoleId", role_name + ":" + session) +
                        xel("Arn", "arn:dfs:sts:::assumed-role/" + role_name + "/" + session) +
                        "</AssumedRoleUser></AssumeRoleWithWebIdentityResult></AssumeRoleWithWebIdentityResponse>";
  const bool ok = respond(c, r, 200, x);
  audit(c, r, claims.sub, 200, role_arn, "", action, sts_res);
  return ok;
}

// ---------------------------------------------------------------- hand-off to Python
int S3Front::backend_conn() {
  {
    std::lock_guard<std::mutex> g(be_mu_);
    if (!be_idle_.empty()) {
      int fd = be_idle_.back();
      be_idle_.pop_back();
      return fd;
    }
  }
  int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  sockaddr_un sa{};
  sa.sun_family = AF_UNIX;
  std::snprintf(sa.sun_path, sizeof sa.sun_path, "%s", cfg_.backend.c_str());
  if (::connect(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0) {
    ::close(fd);
    return -1;
  }
  timeval tv{300, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  return fd;
}

void S3Front::backend_done(int fd, bool reuse) {
  if (!reuse) {
    ::close(fd);
    return;
  }
  std::lock_guard<std::mutex> g(be_mu_);
  be_idle_.push_back(fd);
}

namespace {

// Copies one HTTP/1.1 chunked body from `src` (with `buf` holding bytes already read past
// `*pos`) to `dst`, raw. Returns false on any I/O or framing error.
bool relay_chunked(Io src, std::string& buf, size_t* pos, Io dst) {
  auto need = [&](size_t k) {
    char tmp[kRelayChunk];
    while (buf.size() - *pos < k) {
      long n = io_recv(src, tmp, sizeof tmp);
      if (n <= 0) return false;
      buf.append(tmp, static_cast<size_t>(n));
    }
    return true;
  };
  auto line = [&](std::string* out) {
    size_t e;
    while ((e = buf.find("\r\n", *pos)) == std::string::npos) {
      if (buf.size() - *pos > 8192 || !need(buf.size() - *pos + 1)) return false;
    }
    *out = buf.substr(*pos, e - *pos);
    if (!send_all(dst, buf.data() + *pos, e + 2 - *pos)) return false;
    *pos = e + 2;
    return true;
  };
  for (;;) {
    std::string l;
    if (!line(&l)) return false;
    size_t semi = l.find(';');
    std::string hex = trim(l.substr(0, semi));
    if (hex.empty() || hex.size() > 15) return false;
    uint64_t n = std::stoull(hex, nullptr, 16);
    if (n == 0) {
      for (;;) {  // trailers, then the empty line
        std::string t;
        if (!line(&t)) return false;
        if (t.empty()) return true;
      }
    }
    uint64_t left = n + 2;
    while (left) {
      if (*pos == buf.size()) {
        buf.clear();
        *pos = 0;
        if (!need(1)) return false;
      }
      size_t k = std::min<uint64_t>(left, buf.size() - *pos);
      if (!send_all(dst, buf.data() + *pos, k)) return false;
      *pos += k;
      left -= k;
    }
  }
}

bool relay_n(Io src, std::string& buf, size_t* pos, Io dst, uint64_t n) {
  uint64_t have = std::min<uint64_t>(n, buf.size() - *pos);
  if (have && !send_all(dst, buf.data() + *pos, have)) return false;
  *pos += have;
  n -= have;
  std::vector<char> tmp(kRelayChunk);
  while (n) {
    long k = io_recv(src, tmp.data(), std::min<uint64_t>(n, tmp.size()));
    if (k <= 0 || !send_all(dst, tmp.data(), static_cast<size_t>(k))) return false;
    n -= static_cast<uint64_t>(k);
  }
  return true;
}

}  // namespace

static bool read_body_fd(int fd, char* dst, uint64_t n) {
  uint64_t got = 0;
  while (got < n) {
    ssize_t k = ::recv(fd, dst + got, n - got, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    got += static_cast<uint64_t>(k);
  }
  return true;
}

std::string S3Front::native_metrics() {
  S3FrontStats s = stats();
  std::string o = "# HELP s3_native_requests_total S3 requests served by the native front end\n"
                  "# TYPE s3_native_requests_total counter\n";
  for (auto& kv : s.by_status) {
    size_t sp = kv.first.find(' ');
    o += "s3_native_requests_total{method=\"" + kv.first.substr(0, sp) + "\",status=\"" + kv.first.substr(sp + 1) +
         "\"} " + std::to_string(kv.second) + "\n";
  }
  o += "# HELP s3_native_handoffs_total S3 requests handed to the Python gateway, by reason\n"
       "# TYPE s3_native_handoffs_total counter\n";
  for (auto& kv : s.proxy_reasons)
    o += "s3_native_handoffs_total{reason=\"" + kv.first + "\"} " + std::to_string(kv.second) + "\n";
  if (cfg_.backend.empty()) {
    o += "# HELP s3_native_fallback_answers_total requests the executable gateway answered on its fallback path "
         "(errors, health, metrics), by reason\n# TYPE s3_native_fallback_answers_total counter\n";
    for (auto& kv : s.standalone_reasons)
      o += "s3_native_fallback_answers_total{reason=\"" + kv.first + "\"} " + std::to_string(kv.second) + "\n";
  }
  o += "# TYPE s3_native_store_fallbacks_total counter\ns3_native_store_fallbacks_total " +
       std::to_string(fc_->fallbacks()) + "\n";
  o += "# TYPE s3_native_bytes_in_total counter\ns3_native_bytes_in_total " + std::to_string(s.bytes_in) + "\n";
  o += "# TYPE s3_native_bytes_out_total counter\ns3_native_bytes_out_total " + std::to_string(s.bytes_out) + "\n";
  o += "# HELP s3_native_get_phase_seconds_total native GET time by phase (stat, read, send)\n"
       "# TYPE s3_native_get_phase_seconds_total counter\n";
  for (auto& kv : {std::make_pair("stat", s.get_stat_us), std::make_pair("read", s.get_read_us),
                   std::make_pair("send", s.get_send_us)})
    o += std::string("s3_native_get_phase_seconds_total{phase=\"") + kv.first + "\"} " +
         std::to_string(kv.second / 1e6) + "\n";
  o += "# TYPE s3_native_get_timed_total counter\ns3_native_get_timed_total " + std::to_string(s.get_timed) + "\n";
  if (cfg_.backend.empty()) {  // no Python workers: the IAM metrics they would export (tests/models/s3_gateway.py)
    auto split = [](const std::string& k) {
      size_t b = k.find('|');
      return std::make_pair(k.substr(0, b), b == std::string::npos ? std::string() : k.substr(b + 1));
    };
    o += "# HELP iam_auth_requests_total Total authentication attempts\n# TYPE iam_auth_requests_total counter\n";
    for (auto& kv : s.auth_results) {
      auto rt = split(kv.first);
      o += "iam_auth_requests_total{result=\"" + rt.first + "\",error_type=\"" + rt.second + "\"} " +
           std::to_string(kv.second) + "\n";
    }
    o += "# HELP iam_sts_requests_total STS requests\n# TYPE iam_sts_requests_total counter\n";
    for (auto& kv : s.sts_results) {
      auto rt = split(kv.first);
      o += "iam_sts_requests_total{result=\"" + rt.first + "\",error_type=\"" + rt.second + "\"} " +
           std::to_string(kv.second) + "\n";
    }
    o += "# HELP iam_policy_evaluations_total Policy evaluations\n# TYPE iam_policy_evaluations_total counter\n";
    for (auto& kv : s.policy_results) {
      auto rt = split(kv.first);
      o += "iam_policy_evaluations_total{result=\"" + rt.first + "\",action=\"" + rt.second + "\"} " +
           std::to_string(kv.second) + "\n";
    }
    o += "# HELP iam_oidc_validations_total Total OIDC token validations\n# TYPE iam_oidc_validations_total counter\n";
    for (auto& kv : s.oidc_results)
      o += "iam_oidc_validations_total{result=\"" + kv.first + "\"} " + std::to_string(kv.second) + "\n";
    if (oidc_) {
      o += "# TYPE iam_oidc_jwks_fetches_total counter\n";
      o += "iam_oidc_jwks_fetches_total{result=\"success\"} " + std::to_string(oidc_->fetches_ok()) + "\n";
      o += "iam_oidc_jwks_fetches_total{result=\"failure\"} " + std::to_string(oidc_->fetches_failed()) + "\n";
    }
  }
  return o;
}

bool S3Front::proxy(Conn* c, Req& r, const uint8_t* body, uint64_t body_len, const std::string& why) {
  if (cfg_.backend.empty()) return standalone(c, r, body, body_len, why);
  note_proxy(why);
  int be = backend_conn();
  auto bad_gateway = [&] {
    const char* m = "HTTP/1.1 502 Bad Gateway\r\nContent-Length: 0\r\nConnection: close\r\n\r\n";
    send_all(c->io(), m, std::strlen(m));
    return false;
  };
  if (be < 0) return bad_gateway();
  std::string head = r.method + " " + r.target + " HTTP/1.1\r\n";
  for (size_t i = 0; i < r.headers.size(); ++i) {
    const std::string& n = r.headers[i].first;
    if (n == "connection" || n == "keep-alive" || n == "expect" || n == "proxy-connection" || n == "x-real-ip" ||
        n == "x-forwarded-for" || n == "x-forwarded-proto")
      continue;
    head += r.names[i] + ": " + r.headers[i].second + "\r\n";
  }
  // the gateway's TLS requirement sees how the request really arrived (never the client's say)
  head += "X-Real-IP: " + c->ip + "\r\nX-Forwarded-For: " + c->ip + "\r\nX-Forwarded-Proto: " +
          (c->tls ? "https" : "http") + "\r\nConnection: keep-alive\r\n\r\n";
  if (!body && r.expect_continue && (r.content_length > 0 || r.chunked) &&
      !send_all(c->io(), "HTTP/1.1 100 Continue\r\n\r\n", 25)) {
    backend_done(be, false);
    return false;
  }
  bool ok = send_all(be, head.data(), head.size());
  if (ok && body) ok = send_all(be, body, body_len);
  else if (ok && r.chunked) ok = relay_chunked(c->io(), c->buf, &c->pos, Io{be});
  else if (ok && r.content_length > 0) ok = relay_n(c->io(), c->buf, &c->pos, Io{be}, static_cast<uint64_t>(r.content_length));
  if (!ok) {
    backend_done(be, false);
    return false;
  }
  // the response head
  std::string rb;
  size_t rp = 0, end;
  char tmp[16 << 10];
  while ((end = rb.find("\r\n\r\n")) == std::string::npos) {
    if (rb.size() > kMaxHead) {
      backend_done(be, false);
      return bad_gateway();
    }
    ssize_t n = ::recv(be, tmp, sizeof tmp, 0);
    if (n <= 0) {
      backend_done(be, false);
      return bad_gateway();
    }
    rb.append(tmp, static_cast<size_t>(n));
  }
  std::string rh = rb.substr(0, end);
  rp = end + 4;
  size_t le = rh.find("\r\n");
  std::string status_line = rh.substr(0, le);
  int status = 0;
  {
    size_t sp = status_line.find(' ');
    if (sp != std::string::npos) status = std::atoi(status_line.c_str() + sp + 1);
  }
  std::string out = status_line + "\r\n";
  int64_t clen = -1;
  bool chunked = false, be_close = false;
  for (size_t p = le == std::string::npos ? rh.size() : le + 2; p < rh.size();) {
    size_t e = rh.find("\r\n", p);
    if (e == std::string::npos) e = rh.size();
    std::string h = rh.substr(p, e - p);
    p = e + 2;
    size_t colon = h.find(':');
    if (colon == std::string::npos) continue;
    std::string n = lower(h.substr(0, colon)), v = trim(h.substr(colon + 1));
    if (n == "connection") {
      be_close = lower(v).find("close") != std::string::npos;
      continue;
    }
    if (n == "keep-alive") continue;
    if (n == "content-length" && all_digits(v)) clen = static_cast<int64_t>(std::stoull(v));
    if (n == "transfer-encoding" && lower(v).find("chunked") != std::string::npos) chunked = true;
    out += h + "\r\n";
  }
  const bool no_body = r.method == "HEAD" || status == 204 || status == 304 || (status >= 100 && status < 200);
  if (r.method == "GET" && r.raw_path == "/metrics" && status == 200 && !chunked && clen >= 0) {
    // the Python workers render their registry; the front appends its own counters
    std::string text(static_cast<size_t>(clen), '\0');
    uint64_t have = std::min<uint64_t>(clen, rb.size() - rp);
    std::memcpy(text.data(), rb.data() + rp, have);
    rp += have;
    if (have < static_cast<uint64_t>(clen) && !read_body_fd(be, text.data() + have, clen - have)) {
      backend_done(be, false);
      return bad_gateway();
    }
    text += native_metrics();
    std::string o2;
    for (size_t p = 0; p < out.size();) {  // drop the old Content-Length
      size_t e = out.find("\r\n", p);
      std::string h = out.substr(p, e - p);
      if (lower(h).compare(0, 15, "content-length:") != 0) o2 += h + "\r\n";
      p = e + 2;
    }
    o2 += "Content-Length: " + std::to_string(text.size()) + "\r\n";
    o2 += r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
    r.status = status;
    backend_done(be, !be_close && rp == rb.size());
    return send_head_body(c->io(), o2, reinterpret_cast<const uint8_t*>(text.data()), text.size());
  }
  const bool until_close = !no_body && !chunked && clen < 0;
  if (until_close) r.keep_alive = false;
  out += r.keep_alive ? "Connection: keep-alive\r\n\r\n" : "Connection: close\r\n\r\n";
  r.status = status;
  ok = send_all(c->io(), out.data(), out.size());
  if (ok && !no_body) {
    if (chunked) {
      ok = relay_chunked(Io{be}, rb, &rp, c->io());
    } else if (clen > 0) {
      ok = relay_n(Io{be}, rb, &rp, c->io(), static_cast<uint64_t>(clen));
    } else if (until_close) {
      if (rp < rb.size()) ok = send_all(c->io(), rb.data() + rp, rb.size() - rp);
      ssize_t n;
      while (ok && (n = ::recv(be, tmp, sizeof tmp, 0)) > 0) ok = send_all(c->io(), tmp, static_cast<size_t>(n));
      be_close = true;
    }
  }
  backend_done(be, ok && !be_close && rp == rb.size());
  return ok;
}

}  // namespace dfs
