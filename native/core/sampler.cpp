// Per-thread CPU-time sampler for the native threads (yoda-io, yoda-lane, yoda-engine).
//
// Python's samplers (scripts/profile_bench.py) see the interpreter thread only; the native
// threads that carry the headline burst were measured by /proc CPU totals alone. This is a
// flat profile of them: one POSIX timer per thread on that thread's own CPU clock
// (pthread_getcpuclockid via clock id of the tid), delivering SIGPROF to that thread only
// (SIGEV_THREAD_ID), whose handler stores the interrupted program counter in a fixed
// array with one atomic index bump. Nothing in the handler allocates or locks. The PCs are
// symbolised afterwards in Python (utils/native_prof.py: /proc/self/maps + addr2line).
//
// Samples count thread CPU time, so a thread blocked in epoll_wait or on a condition
// variable is not sampled: the profile answers "where does this thread's CPU go".
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <cstdio>
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <utility>
#include <vector>

namespace yoda_sampler {

namespace {
constexpr size_t kCap = 1 << 18;                 // samples kept
constexpr int kDepth = 8;                        // return addresses kept per sample
uintptr_t g_pc[kCap];
void* g_stack[kCap][kDepth];
int g_depth = 0;                                 // 0: the interrupted PC alone
int32_t g_tid[kCap];
std::atomic<size_t> g_n{0};
std::atomic<size_t> g_dropped{0};
std::vector<timer_t> g_timers;
struct sigaction g_old;
bool g_running = false;

void on_prof(int, siginfo_t* si, void* uc) {
  const size_t i = g_n.fetch_add(1, std::memory_order_relaxed);
  if (i >= kCap) {
    g_dropped.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  const ucontext_t* u = static_cast<const ucontext_t*>(uc);
  g_pc[i] = (uintptr_t)u->uc_mcontext.gregs[REG_RIP];
  // callers through the libgcc unwinder (opt-in: it is not async-signal-safe if the thread
  // is itself unwinding, which the sampled threads do not do on their hot paths). The first
  // frames are this handler and the signal trampoline; the Python side drops them.
  if (g_depth) {
    const int n = backtrace(g_stack[i], kDepth);
    for (int k = n; k < kDepth; ++k) g_stack[i][k] = nullptr;
  }
  // the kernel checks thread CPU timers at its tick: expiries since the last check arrive
  // as one signal with si_overrun set, so a sample weighs 1 + overrun periods
  g_tid[i] = (int32_t)syscall(SYS_gettid) | ((int32_t)std::min(si->si_overrun, 127) << 24);
}

// CPU-time clock of another thread of this process (the kernel's encoding behind
// pthread_getcpuclockid, usable with a bare tid): CPUCLOCK_SCHED | per-thread flag.
clockid_t thread_cpu_clock(pid_t tid) { return (clockid_t)((~(unsigned)tid << 3) | 6u); }
}  // namespace

// Start sampling the given threads every `period_us` of their own CPU time.
void start(const std::vector<int>& tids, int period_us, bool stacks) {
  if (g_running) throw std::runtime_error("sampler already running");
  if (stacks) {
    void* warm[2];
    backtrace(warm, 2);          // loads libgcc_s outside the handler
  }
  g_depth = stacks ? kDepth : 0;
  if (period_us < 50) period_us = 50;
  g_n.store(0);
  g_dropped.store(0);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, &g_old) != 0) throw std::runtime_error("sigaction(SIGPROF) failed");
  g_running = true;
  for (int tid : tids) {
    struct sigevent sev;
    std::memset(&sev, 0, sizeof sev);
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = tid;
    timer_t t;
    if (timer_create(thread_cpu_clock(tid), &sev, &t) != 0) continue;   // thread gone
    struct itimerspec its;
    its.it_interval.tv_sec = period_us / 1000000;
    its.it_interval.tv_nsec = (period_us % 1000000) * 1000L;
    its.it_value = its.it_interval;
    timer_settime(t, 0, &its, nullptr);
    g_timers.push_back(t);
  }
}

// Stop and return (pc, tid | (overrun << 24), [return addresses]) of every sample, plus the
// count dropped for lack of room.
std::pair<std::vector<std::tuple<uintptr_t, int, std::vector<uintptr_t>>>, size_t> stop() {
  for (timer_t t : g_timers) timer_delete(t);
  g_timers.clear();
  if (g_running) sigaction(SIGPROF, &g_old, nullptr);
  g_running = false;
  const size_t n = std::min(g_n.load(), kCap);
  std::vector<std::tuple<uintptr_t, int, std::vector<uintptr_t>>> out;
  out.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    std::vector<uintptr_t> st;
    for (int k = 0; k < g_depth && g_stack[i][k]; ++k) st.push_back((uintptr_t)g_stack[i][k]);
    out.emplace_back(g_pc[i], g_tid[i], std::move(st));
  }
  return {std::move(out), g_dropped.load()};
}

// Stop and write the samples to `path` (one "pc tid_w ret1 ret2 ..." hex line per sample)
// and this process's executable mappings to `path`.maps: for a process without Python
// (the fake apiserver), symbolised by utils/native_prof.py::load_dump.
bool dump(const std::string& path) {
  auto r = stop();
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return false;
  fprintf(f, "# dropped %zu\n", r.second);
  for (auto& [pc, tw, st] : r.first) {
    fprintf(f, "%lx %x", (unsigned long)pc, (unsigned)tw);
    for (uintptr_t a : st) fprintf(f, " %lx", (unsigned long)a);
    fputc('\n', f);
  }
  fclose(f);
  FILE* in = fopen("/proc/self/maps", "r");
  FILE* out = fopen((path + ".maps").c_str(), "w");
  if (in && out) {
    char buf[4096];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, in)) > 0) fwrite(buf, 1, n, out);
  }
  if (in) fclose(in);
  if (out) fclose(out);
  return true;
}

}  // namespace yoda_sampler
