// Multi-buffer MD5 for the ETag of every write (reference dfs/client/src/mod.rs:426-430:
// CRC + MD5 per write; the MD5 is the S3 ETag, stored by CompleteFile).
//
// MD5 is one strictly sequential chain per message, ~1 ms per MiB on one core: with 10 writes
// in flight a client kept ~5 cores busy hashing (at 8 ranks the node's
// cores, not its GPUs or volume, would bind). Here one thread hashes up to 16 messages at
// once, one per 32-bit lane of AVX-512 registers: each MD5 step is a vpternlogd (F/G/H/I), a
// vprold and three vpaddd on all 16 lanes, the same dependent chain a scalar MD5 runs, so a
// message's latency stays a scalar hash's while the CPU cost is shared by every lane. A new
// message joins at the next 64-byte block (a few tens of ns); lanes finish independently.
//
// Needs AVX-512F (checked at run time); without it `available()` is false and callers hash
// with OpenSSL on their own workers as before.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <future>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dfs {

class Md5MultiBuffer {
 public:
  static constexpr int kLanes = 16;
  // Avx512: 16 lanes in zmm registers (a tenth of the cores, twice the latency on Zen 5);
  // Scalar: 2-3 messages interleaved in one scalar instruction stream (the latency of one
  // scalar hash on a half / a third of the cores); None: callers hash with OpenSSL.
  enum class Kind { None, Scalar, Avx512 };
  // `engines` threads of lanes each (kLanes, or `scalar_lanes` in 1..3); a message takes a
  // free lane of the first engine that has one.
  explicit Md5MultiBuffer(int engines = 1, Kind kind = Kind::Avx512, int scalar_lanes = 2);
  Kind kind() const { return kind_; }
  int lanes() const { return lanes_; }
  ~Md5MultiBuffer();
  Md5MultiBuffer(const Md5MultiBuffer&) = delete;

  static bool available();  // the CPU has AVX-512F (and the DFS_MD5_MB switch is not 0)
  // Which engine a client should hash its ETags on. On the MI355X hosts (Zen 5) an AVX-512
  // lane's step chain is twice a scalar core's (2-cycle vector integer latency,
  // profiles/r6/md5): ~1.9 ms per MiB against ~1.0 for a scalar hash. So the AVX-512 engine is
  // a CPU-budget choice made from the cores this process may use (the cgroup quota, else the
  // online CPUs, divided by the ranks sharing the node: LOCAL_WORLD_SIZE or DFS_RANKS_ON_NODE):
  // >= DFS_MD5_OPENSSL_MIN_CORES (12): OpenSSL per message (lowest latency, ~1 core per write
  // in flight); >= DFS_MD5_MB_MIN_CORES (6): the scalar engine, 2 messages per thread at a
  // scalar hash's latency; below: the AVX-512 lanes (one core for 16 messages).
  // The engine a client should use (DFS_MD5_MB: 0/openssl, scalar, 1/avx512, auto).
  static Kind wanted();
  static double cores_per_rank();
  // MD5 of p[0..n) as 32 lowercase hex digits. The caller keeps p alive until the future is ready.
  std::future<std::string> submit(const uint8_t* p, size_t n);

  uint64_t messages() const;
  uint64_t blocks() const;  // 64-byte blocks hashed (all lanes)
  uint64_t rounds() const;  // engine iterations (one block on every active lane)

 private:
  struct Job {
    const uint8_t* p;
    size_t n;
    std::promise<std::string> done;
  };
  struct Engine {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Job> q;
    int load = 0;  // active + queued (mu)
    std::atomic<int> queued{0};  // jobs in q: the engine takes the lock only when there are some
    bool stop = false;
    std::thread th;
    uint64_t messages = 0, blocks = 0, rounds = 0;  // (mu on read; the engine thread writes)
  };
  void run(Engine* e);
  const Kind kind_;
  const int lanes_;
  std::vector<std::unique_ptr<Engine>> engines_;
};

// One-shot helper: the multi-buffer engine when available, else OpenSSL on this thread.
std::string md5_hex_scalar(const uint8_t* p, size_t n);

}  // namespace dfs
