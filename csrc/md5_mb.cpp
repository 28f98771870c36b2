// Multi-buffer MD5 (see md5_mb.h). RFC 1321's rounds, 16 messages per AVX-512 register.
#include "md5_mb.h"

#include <immintrin.h>
#include <openssl/evp.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "thread_name.h"

namespace dfs {

namespace {

constexpr uint32_t kK[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
constexpr uint32_t kIv[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};

// One 64-byte block on each of the 16 lanes: st = {a, b, c, d} (lane L of each is message
// L's state), ptrs[L] its block. The message words are gathered across the lanes (word w of
// lane L at ptrs[L] + 4w); F, G, H, I are each one vpternlogd on (d, b, c) (truth-table bit
// (d << 2 | b << 1 | c)):
//   F = b ? c : d -> 0xB8,  G = d ? b : c -> 0xCA,  H = b ^ c ^ d -> 0x96,  I = c ^ (b | ~d) -> 0x65.
__attribute__((target("avx512f"))) void md5_block16(uint32_t (*st)[16], const uint8_t* const* ptrs) {
  // the 16 blocks (one row of 16 words per lane) transposed into X[w] = word w of every lane:
  // 16 loads and 64 in-register shuffles instead of 32 gathers
  __m512i X[16], t[16];
  for (int i = 0; i < 16; ++i) X[i] = _mm512_loadu_si512(reinterpret_cast<const void*>(ptrs[i]));
  for (int i = 0; i < 8; ++i) {
    t[2 * i] = _mm512_unpacklo_epi32(X[2 * i], X[2 * i + 1]);
    t[2 * i + 1] = _mm512_unpackhi_epi32(X[2 * i], X[2 * i + 1]);
  }
  for (int i = 0; i < 4; ++i) {  // u[4i+j], 128-bit chunk k: word 4k+j of rows 4i..4i+3
    X[4 * i + 0] = _mm512_unpacklo_epi64(t[4 * i], t[4 * i + 2]);
    X[4 * i + 1] = _mm512_unpackhi_epi64(t[4 * i], t[4 * i + 2]);
    X[4 * i + 2] = _mm512_unpacklo_epi64(t[4 * i + 1], t[4 * i + 3]);
    X[4 * i + 3] = _mm512_unpackhi_epi64(t[4 * i + 1], t[4 * i + 3]);
  }
  for (int j = 0; j < 4; ++j) {
    const __m512i v0 = _mm512_shuffle_i32x4(X[j], X[4 + j], 0x88), v1 = _mm512_shuffle_i32x4(X[j], X[4 + j], 0xDD);
    const __m512i v2 = _mm512_shuffle_i32x4(X[8 + j], X[12 + j], 0x88),
                  v3 = _mm512_shuffle_i32x4(X[8 + j], X[12 + j], 0xDD);
    t[0 + j] = _mm512_shuffle_i32x4(v0, v2, 0x88);
    t[8 + j] = _mm512_shuffle_i32x4(v0, v2, 0xDD);
    t[4 + j] = _mm512_shuffle_i32x4(v1, v3, 0x88);
    t[12 + j] = _mm512_shuffle_i32x4(v1, v3, 0xDD);
  }
  for (int w = 0; w < 16; ++w) X[w] = t[w];
  __m512i a = _mm512_loadu_si512(st[0]), b = _mm512_loadu_si512(st[1]), c = _mm512_loadu_si512(st[2]),
          d = _mm512_loadu_si512(st[3]);
  const __m512i a0 = a, b0 = b, c0 = c, d0 = d;
  // The dependent chain of a step is f(b) -> +ak -> rol -> +b (4 ops): ak = a + X[g] + K[i]
  // only involves older values, and the empty asm keeps the compiler from reassociating K
  // back onto the chain; f's destructive operand is d (copied off the chain, b arrives last).
#define DFS_MD5_STEP(IMM, a, b, c, d, g, s, i)                                                    \
  do {                                                                                            \
    __m512i ak = _mm512_add_epi32(a, _mm512_add_epi32(X[g], _mm512_set1_epi32(static_cast<int>(kK[i])))); \
    __asm__("" : "+v"(ak));                                                                       \
    const __m512i f = _mm512_ternarylogic_epi32(d, b, c, IMM);                                    \
    a = _mm512_add_epi32(b, _mm512_rol_epi32(_mm512_add_epi32(ak, f), s));                       \
  } while (0)
  // round 1: g = i
  for (int i = 0; i < 16; i += 4) {
    DFS_MD5_STEP(0xB8, a, b, c, d, i + 0, 7, i + 0);
    DFS_MD5_STEP(0xB8, d, a, b, c, i + 1, 12, i + 1);
    DFS_MD5_STEP(0xB8, c, d, a, b, i + 2, 17, i + 2);
    DFS_MD5_STEP(0xB8, b, c, d, a, i + 3, 22, i + 3);
  }
  // round 2: g = (5i + 1) mod 16
  for (int i = 16; i < 32; i += 4) {
    DFS_MD5_STEP(0xCA, a, b, c, d, (5 * (i + 0) + 1) & 15, 5, i + 0);
    DFS_MD5_STEP(0xCA, d, a, b, c, (5 * (i + 1) + 1) & 15, 9, i + 1);
    DFS_MD5_STEP(0xCA, c, d, a, b, (5 * (i + 2) + 1) & 15, 14, i + 2);
    DFS_MD5_STEP(0xCA, b, c, d, a, (5 * (i + 3) + 1) & 15, 20, i + 3);
  }
  // round 3: g = (3i + 5) mod 16
  for (int i = 32; i < 48; i += 4) {
    DFS_MD5_STEP(0x96, a, b, c, d, (3 * (i + 0) + 5) & 15, 4, i + 0);
    DFS_MD5_STEP(0x96, d, a, b, c, (3 * (i + 1) + 5) & 15, 11, i + 1);
    DFS_MD5_STEP(0x96, c, d, a, b, (3 * (i + 2) + 5) & 15, 16, i + 2);
    DFS_MD5_STEP(0x96, b, c, d, a, (3 * (i + 3) + 5) & 15, 23, i + 3);
  }
  // round 4: g = 7i mod 16
  for (int i = 48; i < 64; i += 4) {
    DFS_MD5_STEP(0x65, a, b, c, d, (7 * (i + 0)) & 15, 6, i + 0);
    DFS_MD5_STEP(0x65, d, a, b, c, (7 * (i + 1)) & 15, 10, i + 1);
    DFS_MD5_STEP(0x65, c, d, a, b, (7 * (i + 2)) & 15, 15, i + 2);
    DFS_MD5_STEP(0x65, b, c, d, a, (7 * (i + 3)) & 15, 21, i + 3);
  }
#undef DFS_MD5_STEP
  _mm512_storeu_si512(st[0], _mm512_add_epi32(a, a0));
  _mm512_storeu_si512(st[1], _mm512_add_epi32(b, b0));
  _mm512_storeu_si512(st[2], _mm512_add_epi32(c, c0));
  _mm512_storeu_si512(st[3], _mm512_add_epi32(d, d0));
}

// K messages interleaved in one scalar instruction stream: K independent step chains of
// ~4.5 cycles each (a scalar MD5's latency), so one core hashes K messages at the speed of
// one. F and I are 2 dependent ops on b, G and H one; K[i] and the message word are added to
// the 4-steps-old `a` off the chain.
inline uint32_t rol32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

template <int K>
void md5_block_scalar(uint32_t (*st)[16], const uint8_t* const* ptrs) {
  uint32_t X[K][16], a[K], b[K], c[K], d[K], a0[K], b0[K], c0[K], d0[K];
  for (int l = 0; l < K; ++l) {
    std::memcpy(X[l], ptrs[l], 64);  // little-endian words (x86)
    a0[l] = a[l] = st[0][l];
    b0[l] = b[l] = st[1][l];
    c0[l] = c[l] = st[2][l];
    d0[l] = d[l] = st[3][l];
  }
  // (the empty asm pins t = a + X + K as one value, so the compiler cannot move those adds
  // back behind F onto the chain)
#define DFS_MD5_S(FN, A, B, C, D, g, s, i)                       \
  _Pragma("clang loop unroll(full)") for (int l = 0; l < K; ++l) { \
    uint32_t t = A[l] + X[l][g] + kK[i];                         \
    __asm__("" : "+r"(t));                                       \
    A[l] = B[l] + rol32(t + FN(B[l], C[l], D[l]), s);            \
  }
#define DFS_F(x, y, z) ((((y) ^ (z)) & (x)) ^ (z))
#define DFS_G(x, y, z) (((x) & (z)) + ((y) & ~(z)))
#define DFS_H(x, y, z) ((x) ^ (y) ^ (z))
#define DFS_I(x, y, z) ((y) ^ ((x) | ~(z)))
  _Pragma("clang loop unroll(full)") for (int i = 0; i < 16; i += 4) {
    DFS_MD5_S(DFS_F, a, b, c, d, i + 0, 7, i + 0)
    DFS_MD5_S(DFS_F, d, a, b, c, i + 1, 12, i + 1)
    DFS_MD5_S(DFS_F, c, d, a, b, i + 2, 17, i + 2)
    DFS_MD5_S(DFS_F, b, c, d, a, i + 3, 22, i + 3)
  }
  _Pragma("clang loop unroll(full)") for (int i = 16; i < 32; i += 4) {
    DFS_MD5_S(DFS_G, a, b, c, d, (5 * (i + 0) + 1) & 15, 5, i + 0)
    DFS_MD5_S(DFS_G, d, a, b, c, (5 * (i + 1) + 1) & 15, 9, i + 1)
    DFS_MD5_S(DFS_G, c, d, a, b, (5 * (i + 2) + 1) & 15, 14, i + 2)
    DFS_MD5_S(DFS_G, b, c, d, a, (5 * (i + 3) + 1) & 15, 20, i + 3)
  }
  _Pragma("clang loop unroll(full)") for (int i = 32; i < 48; i += 4) {
    DFS_MD5_S(DFS_H, a, b, c, d, (3 * (i + 0) + 5) & 15, 4, i + 0)
    DFS_MD5_S(DFS_H, d, a, b, c, (3 * (i + 1) + 5) & 15, 11, i + 1)
    DFS_MD5_S(DFS_H, c, d, a, b, (3 * (i + 2) + 5) & 15, 16, i + 2)
    DFS_MD5_S(DFS_H, b, c, d, a, (3 * (i + 3) + 5) & 15, 23, i + 3)
  }
  _Pragma("clang loop unroll(full)") for (int i = 48; i < 64; i += 4) {
    DFS_MD5_S(DFS_I, a, b, c, d, (7 * (i + 0)) & 15, 6, i + 0)
    DFS_MD5_S(DFS_I, d, a, b, c, (7 * (i + 1)) & 15, 10, i + 1)
    DFS_MD5_S(DFS_I, c, d, a, b, (7 * (i + 2)) & 15, 15, i + 2)
    DFS_MD5_S(DFS_I, b, c, d, a, (7 * (i + 3)) & 15, 21, i + 3)
  }
#undef DFS_MD5_S
#undef DFS_F
#undef DFS_G
#undef DFS_H
#undef DFS_I
  for (int l = 0; l < K; ++l) {
    st[0][l] = a[l] + a0[l];
    st[1][l] = b[l] + b0[l];
    st[2][l] = c[l] + c0[l];
    st[3][l] = d[l] + d0[l];
  }
}

std::string hex_of(const uint8_t d[16]) {
  static const char* hx = "0123456789abcdef";
  std::string o(32, '0');
  for (int i = 0; i < 16; ++i) {
    o[2 * i] = hx[d[i] >> 4];
    o[2 * i + 1] = hx[d[i] & 15];
  }
  return o;
}

}  // namespace

std::string md5_hex_scalar(const uint8_t* p, size_t n) {
  unsigned char d[EVP_MAX_MD_SIZE];
  unsigned int len = 0;
  EVP_Digest(p, n, d, &len, EVP_md5(), nullptr);
  return hex_of(d);
}

bool Md5MultiBuffer::available() {
  static const bool ok = [] {
#if defined(__HIP_DEVICE_COMPILE__)
    return false;  // (the device pass of hipcc parses host code too)
#else
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") != 0;
#endif
  }();
  return ok;
}

double Md5MultiBuffer::cores_per_rank() {
  double cores = static_cast<double>(std::max(1u, std::thread::hardware_concurrency()));
  auto read = [](const char* path) {
    std::string s;
    if (FILE* f = std::fopen(path, "r")) {
      char buf[128];
      size_t n = std::fread(buf, 1, sizeof buf - 1, f);
      std::fclose(f);
      s.assign(buf, n);
    }
    return s;
  };
  const std::string v2 = read("/sys/fs/cgroup/cpu.max");  // "<quota> <period>" or "max <period>"
  if (!v2.empty() && v2.compare(0, 3, "max") != 0) {
    double q = 0, p = 0;
    if (std::sscanf(v2.c_str(), "%lf %lf", &q, &p) == 2 && q > 0 && p > 0) cores = std::min(cores, q / p);
  } else if (v2.empty()) {
    const double q = std::atof(read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").c_str()),
                 p = std::atof(read("/sys/fs/cgroup/cpu/cpu.cfs_period_us").c_str());
    if (q > 0 && p > 0) cores = std::min(cores, q / p);
  }
  int ranks = 1;
  for (const char* k : {"DFS_RANKS_ON_NODE", "LOCAL_WORLD_SIZE"})
    if (const char* e = std::getenv(k)) {
      ranks = std::max(1, std::atoi(e));
      break;
    }
  return cores / ranks;
}

Md5MultiBuffer::Kind Md5MultiBuffer::wanted() {
  static const Kind k = [] {
    const char* e = std::getenv("DFS_MD5_MB");
    const std::string v = e ? e : "auto";
    if (v == "0" || v == "openssl") return Kind::None;
    if (v == "scalar") return Kind::Scalar;
    if (v == "1" || v == "avx512") return available() ? Kind::Avx512 : Kind::Scalar;
    // the cheapest engine that the rank's CPU budget calls for (profiles/r6/md5, Zen 5, 10
    // writes in flight): OpenSSL per message 0.99 ms on ~10 cores; 2 interleaved per thread
    // 1.01 ms on 5; AVX-512 lanes 1.9 ms on 1
    const double c = cores_per_rank();
    const char* hi = std::getenv("DFS_MD5_OPENSSL_MIN_CORES");
    const char* lo = std::getenv("DFS_MD5_MB_MIN_CORES");
    if (c >= (hi && *hi ? std::atof(hi) : 12.0)) return Kind::None;
    if (c >= (lo && *lo ? std::atof(lo) : 6.0) || !available()) return Kind::Scalar;
    return Kind::Avx512;
  }();
  return k;
}

Md5MultiBuffer::Md5MultiBuffer(int engines, Kind kind, int scalar_lanes)
    : kind_(kind), lanes_(kind == Kind::Avx512 ? kLanes : std::max(1, std::min(3, scalar_lanes))) {
  for (int i = 0; i < std::max(1, engines); ++i) {
    engines_.push_back(std::make_unique<Engine>());
    Engine* e = engines_.back().get();
    e->th = std::thread([this, e] { run(e); });
  }
}

Md5MultiBuffer::~Md5MultiBuffer() {
  for (auto& e : engines_) {
    {
      std::lock_guard<std::mutex> g(e->mu);
      e->stop = true;
    }
    e->cv.notify_all();
  }
  for (auto& e : engines_) e->th.join();
}

std::future<std::string> Md5MultiBuffer::submit(const uint8_t* p, size_t n) {
  // first fit: fill an engine's lanes before waking the next (a lane costs no latency, a
  // thread costs a core); all full: the least loaded one queues it
  Engine* best = nullptr;
  int load = 0;
  for (auto& e : engines_) {
    std::lock_guard<std::mutex> g(e->mu);
    if (e->load < lanes_) {
      best = e.get();
      break;
    }
    if (!best || e->load < load) {
      best = e.get();
      load = e->load;
    }
  }
  Job j{p, n, {}};
  std::future<std::string> f = j.done.get_future();
  {
    std::lock_guard<std::mutex> g(best->mu);
    best->q.push_back(std::move(j));
    best->load++;
    best->queued.fetch_add(1, std::memory_order_release);
  }
  best->cv.notify_one();
  return f;
}

uint64_t Md5MultiBuffer::messages() const {
  uint64_t s = 0;
  for (auto& e : engines_) {
    std::lock_guard<std::mutex> g(e->mu);
    s += e->messages;
  }
  return s;
}

uint64_t Md5MultiBuffer::blocks() const {
  uint64_t s = 0;
  for (auto& e : engines_) {
    std::lock_guard<std::mutex> g(e->mu);
    s += e->blocks;
  }
  return s;
}

uint64_t Md5MultiBuffer::rounds() const {
  uint64_t s = 0;
  for (auto& e : engines_) {
    std::lock_guard<std::mutex> g(e->mu);
    s += e->rounds;
  }
  return s;
}

void Md5MultiBuffer::run(Engine* e) {
  name_thread(kind_ == Kind::Avx512 ? "md5-avx512" : "md5-x");
  struct Lane {
    bool active = false;
    const uint8_t* p = nullptr;
    uint64_t full = 0;  // whole 64-byte blocks left at p
    int tail_blocks = 0, tail_i = 0;
    alignas(64) uint8_t tail[128];
    std::promise<std::string> done;
  };
  const int nl = lanes_;
  std::vector<Lane> lanes(nl);
  alignas(64) static const uint8_t zero_block[64] = {};
  alignas(64) uint32_t st[4][16];
  std::memset(st, 0, sizeof st);
  alignas(64) const uint8_t* ptrs[kLanes];
  int nactive = 0;
  uint64_t blocks = 0, rounds = 0, msgs = 0;
  for (;;) {
    // take queued messages into free lanes (checked every round: a message waits one block at
    // most; the lock only when something is queued)
    if (nactive == 0 || (nactive < nl && e->queued.load(std::memory_order_acquire) > 0)) {
      std::unique_lock<std::mutex> lk(e->mu);
      if (nactive == 0) {
        e->blocks += blocks;
        e->rounds += rounds;
        e->messages += msgs;
        blocks = rounds = msgs = 0;
        e->cv.wait(lk, [&] { return e->stop || !e->q.empty(); });
        if (e->stop && e->q.empty()) return;
      }
      for (int l = 0; l < nl && !e->q.empty(); ++l) {
        Lane& L = lanes[l];
        if (L.active) continue;
        Job j = std::move(e->q.front());
        e->q.pop_front();
        e->queued.fetch_sub(1, std::memory_order_relaxed);
        L.active = true;
        L.p = j.p;
        L.full = j.n / 64;
        const size_t rem = j.n % 64;
        std::memset(L.tail, 0, sizeof L.tail);
        if (rem) std::memcpy(L.tail, j.p + L.full * 64, rem);
        L.tail[rem] = 0x80;
        L.tail_blocks = rem + 9 <= 64 ? 1 : 2;
        const uint64_t bits = static_cast<uint64_t>(j.n) * 8;
        std::memcpy(L.tail + 64 * L.tail_blocks - 8, &bits, 8);  // little-endian bit length
        L.tail_i = 0;
        L.done = std::move(j.done);
        for (int k = 0; k < 4; ++k) st[k][l] = kIv[k];
        ++nactive;
      }
    }
    for (int l = 0; l < nl; ++l) {
      const Lane& L = lanes[l];
      ptrs[l] = !L.active ? zero_block : L.full ? L.p : L.tail + 64 * L.tail_i;
    }
    if (kind_ == Kind::Avx512) md5_block16(st, ptrs);
    else if (nl == 3) md5_block_scalar<3>(st, ptrs);
    else if (nl == 2) md5_block_scalar<2>(st, ptrs);
    else md5_block_scalar<1>(st, ptrs);
    ++rounds;
    bool finished = false;
    for (int l = 0; l < nl; ++l) {
      Lane& L = lanes[l];
      if (!L.active) continue;
      ++blocks;
      if (L.full) {
        L.p += 64;
        --L.full;
      } else if (++L.tail_i == L.tail_blocks) {
        finished = true;
      }
    }
    if (!finished) continue;
    for (int l = 0; l < nl; ++l) {
      Lane& L = lanes[l];
      if (!L.active || L.full || L.tail_i != L.tail_blocks) continue;
      uint8_t dg[16];
      for (int k = 0; k < 4; ++k) std::memcpy(dg + 4 * k, &st[k][l], 4);
      L.active = false;
      --nactive;
      ++msgs;
      std::promise<std::string> done = std::move(L.done);
      {
        std::lock_guard<std::mutex> g(e->mu);
        e->load--;
      }
      done.set_value(hex_of(dg));
    }
  }
}

}  // namespace dfs
