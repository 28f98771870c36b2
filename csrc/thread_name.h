// Names for the threads of a process (at most 15 characters, as the kernel keeps them), so
// /proc/<pid>/task/*/comm, and the per-thread CPU report built from it, say who spent what.
#pragma once
#include <pthread.h>
#include <sys/prctl.h>

#include <cstdio>
#include <cstring>
#include <dirent.h>
#include <map>
#include <string>
#include <unistd.h>

namespace dfs {

// Also sets the thread's timer slack to 1 us: the data path's short polls (a copy's event,
// a staged slice) sleep 5-10 us between checks, and the default 50 us slack stretched each
// such sleep to ~60 us, longer than the copy it waits for.
inline void name_thread(const char* name) {
  char buf[16];
  std::strncpy(buf, name, sizeof(buf) - 1);
  buf[sizeof(buf) - 1] = 0;
  (void)pthread_setname_np(pthread_self(), buf);
  (void)::prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
}

// CPU milliseconds (user + system) of this process's live threads, summed by thread name.
// Threads that already exited are not counted (their time shows in the process total only).
inline std::map<std::string, double> thread_cpu_ms() {
  std::map<std::string, double> out;
  const double tick_ms = 1000.0 / static_cast<double>(::sysconf(_SC_CLK_TCK));
  DIR* d = ::opendir("/proc/self/task");
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    if (e->d_name[0] == '.') continue;
    const std::string base = std::string("/proc/self/task/") + e->d_name;
    char stat[1024] = {0};
    FILE* f = std::fopen((base + "/stat").c_str(), "r");
    if (!f) continue;
    const size_t got = std::fread(stat, 1, sizeof(stat) - 1, f);
    std::fclose(f);
    stat[got] = 0;
    // "tid (comm) state ppid ..." : utime and stime are fields 14 and 15; comm may hold spaces
    const char* rp = std::strrchr(stat, ')');
    const char* lp = std::strchr(stat, '(');
    if (!rp || !lp || rp < lp) continue;
    std::string comm(lp + 1, rp);
    unsigned long long ut = 0, st = 0;
    // after ") " come fields 3.. : skip 11 of them (3..13) to reach utime
    if (std::sscanf(rp + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %llu %llu", &ut, &st) != 2) continue;
    out[comm] += static_cast<double>(ut + st) * tick_ms;
  }
  ::closedir(d);
  return out;
}

}  // namespace dfs
