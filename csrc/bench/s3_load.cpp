// s3_load: a native HTTP/1.1 load generator for the S3 gateway (config 5). One keep-alive
// connection per client thread, requests back to back — the shape of the Python `requests`
// load generator in bench_configs.py, without an interpreter on the client side, so the
// numbers describe the gateway rather than the client.
//
//   s3_load --host 127.0.0.1 --port 9000 --op put|get|range --bucket b --prefix p [--key k]
//           --count N --size BYTES --conc C [--range-size 65536] [--verify]
// Payload of object i: a xorshift stream seeded by i (`--verify` checks GET bodies against it).
// Prints one JSON object: ops, seconds, MB/s, req/s, p50/p99 latency, errors.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

void fill(std::vector<char>& b, uint64_t seed) {
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  for (size_t i = 0; i < b.size(); i += 8) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    std::memcpy(b.data() + i, &x, std::min<size_t>(8, b.size() - i));
  }
}

struct Conn {
  int fd = -1;
  std::string buf;
  bool open(const std::string& host, int port) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port));
    ::inet_pton(AF_INET, host.c_str(), &a.sin_addr);
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return ::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) == 0;
  }
  bool send_all(const char* p, size_t n) {
    while (n) {
      ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
      if (w <= 0) return false;
      p += w;
      n -= static_cast<size_t>(w);
    }
    return true;
  }
  // Reads one response; returns the status (-1 on error); body into *body (if non-null).
  int response(std::string* body, bool head_only = false) {
    size_t end;
    char tmp[1 << 16];
    while ((end = buf.find("\r\n\r\n")) == std::string::npos) {
      ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
      if (n <= 0) return -1;
      buf.append(tmp, static_cast<size_t>(n));
    }
    std::string head = buf.substr(0, end);
    buf.erase(0, end + 4);
    int status = std::atoi(head.c_str() + head.find(' ') + 1);
    size_t clen = 0;
    for (size_t p = 0; (p = head.find("\r\n", p)) != std::string::npos;) {
      p += 2;
      if (strncasecmp(head.c_str() + p, "content-length:", 15) == 0) clen = std::strtoull(head.c_str() + p + 15, nullptr, 10);
    }
    if (head_only) clen = 0;
    if (body) {
      body->resize(clen);
      size_t have = std::min(clen, buf.size());
      std::memcpy(body->data(), buf.data(), have);
      buf.erase(0, have);
      while (have < clen) {
        ssize_t n = ::recv(fd, body->data() + have, clen - have, 0);
        if (n <= 0) return -1;
        have += static_cast<size_t>(n);
      }
    } else {
      size_t have = std::min(clen, buf.size());
      buf.erase(0, have);
      while (have < clen) {
        ssize_t n = ::recv(fd, tmp, std::min(sizeof tmp, clen - have), 0);
        if (n <= 0) return -1;
        have += static_cast<size_t>(n);
      }
    }
    return status;
  }
};

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1", op = "get", bucket = "bench", prefix = "nat", fixed_key;
  int port = 9000, conc = 10;
  uint64_t count = 100, size = 1 << 20, rsize = 65536, keys = 0;
  bool verify = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto nxt = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--host") host = nxt();
    else if (a == "--port") port = std::atoi(nxt().c_str());
    else if (a == "--op") op = nxt();
    else if (a == "--bucket") bucket = nxt();
    else if (a == "--prefix") prefix = nxt();
    else if (a == "--key") fixed_key = nxt();  // every request on this one key (e.g. a multipart object)
    else if (a == "--count") count = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--size") size = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--conc") conc = std::atoi(nxt().c_str());
    else if (a == "--range-size") rsize = std::strtoull(nxt().c_str(), nullptr, 10);
    else if (a == "--verify") verify = true;
    else if (a == "--keys") keys = std::strtoull(nxt().c_str(), nullptr, 10);  // request i -> key i % keys
  }
  if (keys == 0) keys = count;
  // Payloads are generated before the clock starts (PUT bodies, and the expected bytes of a
  // verified GET): generating 1 MiB of xorshift per request inside the timed loop costs the
  // client ~0.5 ms, which would be measured as gateway latency. Falls back to per-request
  // generation when the key set is too large to hold.
  std::vector<std::vector<char>> cache;
  const bool need = op == "put" || (verify && fixed_key.empty());
  if (need && keys * size <= (4ull << 30)) {
    cache.resize(keys);
    for (uint64_t k = 0; k < keys; ++k) {
      cache[k].resize(size);
      fill(cache[k], k);
    }
  }
  std::vector<std::vector<double>> lat(conc);
  std::atomic<uint64_t> errors{0}, bytes{0};
  auto t0 = Clock::now();
  std::vector<std::thread> th;
  for (int t = 0; t < conc; ++t)
    th.emplace_back([&, t] {
      Conn c;
      if (!c.open(host, port)) {
        errors += count;
        return;
      }
      std::vector<char> payload(size);
      std::string body;
      for (uint64_t i = static_cast<uint64_t>(t); i < count; i += static_cast<uint64_t>(conc)) {
        char key[64];
        if (fixed_key.empty())
          std::snprintf(key, sizeof key, "%s_%05llu", prefix.c_str(), static_cast<unsigned long long>(i % keys));
        else
          std::snprintf(key, sizeof key, "%s", fixed_key.c_str());
        std::string req;
        auto s0 = Clock::now();
        int st;
        if (op == "put") {
          const char* body = payload.data();
          if (!cache.empty()) body = cache[i % keys].data();
          else fill(payload, i % keys);
          req = "PUT /" + bucket + "/" + key + " HTTP/1.1\r\nHost: " + host + "\r\nContent-Length: " +
                std::to_string(size) + "\r\n\r\n";
          st = c.send_all(req.data(), req.size()) && c.send_all(body, size) ? c.response(nullptr) : -1;
          if (st == 200) bytes += size;
        } else {
          uint64_t off = 0, want = size;
          req = "GET /" + bucket + "/" + key + " HTTP/1.1\r\nHost: " + host + "\r\n";
          if (op == "range") {
            off = (i * 7919 * 4096) % (size - rsize);
            want = rsize;
            req += "Range: bytes=" + std::to_string(off) + "-" + std::to_string(off + rsize - 1) + "\r\n";
          }
          req += "\r\n";
          st = c.send_all(req.data(), req.size()) ? c.response(&body) : -1;
          if ((st == 200 || st == 206) && body.size() == want) {
            bytes += want;
            if (verify && fixed_key.empty()) {
              const char* exp = payload.data();
              if (!cache.empty()) exp = cache[i % keys].data();
              else fill(payload, i % keys);
              if (std::memcmp(exp + off, body.data(), want) != 0) st = -2;
            }
          } else {
            st = -1;
          }
        }
        if (st != 200 && st != 206) errors++;
        lat[t].push_back(std::chrono::duration<double>(Clock::now() - s0).count());
      }
      ::close(c.fd);
    });
  for (auto& x : th) x.join();
  double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  std::vector<double> all;
  for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : 1e3 * all[std::min(all.size() - 1, size_t(all.size() * p))]; };
  std::printf("{\"op\": \"%s\", \"ops\": %zu, \"seconds\": %.4f, \"mb_per_s\": %.1f, \"req_per_s\": %.1f, "
              "\"p50_ms\": %.3f, \"p99_ms\": %.3f, \"errors\": %llu, \"concurrency\": %d, \"size\": %llu}\n",
              op.c_str(), all.size(), secs, bytes.load() / 1048576.0 / secs, all.size() / secs, pct(0.5), pct(0.99),
              static_cast<unsigned long long>(errors.load()), conc, static_cast<unsigned long long>(size));
  return errors.load() ? 1 : 0;
}
