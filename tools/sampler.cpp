// sampler.cpp -- a tiny in-process sampling profiler for the host stages (no
// perf in the image).  Every thread that exists at start() gets its own
// CLOCK_MONOTONIC timer delivering SIGPROF to that thread (SIGEV_THREAD_ID),
// so each thread is sampled in wall time, busy or waiting; the handler records
// the instruction pointer.  stop() writes "module offset count" lines (module
// from /proc/self/maps) for tools/sampler.py to symbolise with nm.
//   build: g++ -O2 -shared -fPIC tools/sampler.cpp -o tools/libsampler.so
#include <csignal>
#include <cstdint>
#include <dirent.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <sys/time.h>
#include <ucontext.h>
#include <vector>

namespace {
constexpr size_t kCap = 1 << 20;
constexpr int kDepth = 16;
uint64_t g_buf[kCap][kDepth];
volatile size_t g_n = 0;

void on_prof(int, siginfo_t *, void *ucv) {
    const size_t i = __atomic_fetch_add(&g_n, 1, __ATOMIC_RELAXED);
    if (i >= kCap) return;
    const ucontext_t *uc = (const ucontext_t *)ucv;
    uint64_t *o = g_buf[i];
    o[0] = (uint64_t)uc->uc_mcontext.gregs[REG_RIP];
    const uint64_t rsp = (uint64_t)uc->uc_mcontext.gregs[REG_RSP];
    uint64_t fp = (uint64_t)uc->uc_mcontext.gregs[REG_RBP];
    int d = 1;
    // walk only inside this thread's stack: fp above rsp, increasing, aligned
    while (d < kDepth && fp >= rsp && fp < rsp + (64u << 20) && (fp & 7) == 0) {
        const uint64_t *f = (const uint64_t *)fp;
        const uint64_t next = f[0], ret = f[1];
        if (ret < 4096) break;
        o[d++] = ret - 1;   // inside the call instruction
        if (next <= fp) break;
        fp = next;
    }
    if (d < kDepth) o[d] = 0;
}
}  // namespace

extern "C" {

std::vector<timer_t> g_timers;

int sampler_start(int hz) {
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGPROF, &sa, nullptr) != 0) return -1;
    g_n = 0;
    DIR *d = opendir("/proc/self/task");
    if (!d) return -1;
    while (dirent *e = readdir(d)) {
        if (e->d_name[0] == '.') continue;
        const int tid = std::atoi(e->d_name);
        struct sigevent sev;
        std::memset(&sev, 0, sizeof sev);
        sev.sigev_notify = SIGEV_THREAD_ID;
        sev.sigev_signo = SIGPROF;
        sev._sigev_un._tid = tid;
        timer_t t;
        if (timer_create(CLOCK_MONOTONIC, &sev, &t) != 0) continue;
        struct itimerspec its;
        its.it_interval.tv_sec = 0;
        its.it_interval.tv_nsec = 1000000000L / hz;
        its.it_value = its.it_interval;
        timer_settime(t, 0, &its, nullptr);
        g_timers.push_back(t);
    }
    closedir(d);
    return (int)g_timers.size();
}

int sampler_stop(const char *path) {
    for (timer_t t : g_timers) timer_delete(t);
    g_timers.clear();
    signal(SIGPROF, SIG_IGN);
    struct Map { uint64_t a, b, off; std::string name; };
    std::vector<Map> maps;
    if (FILE *f = std::fopen("/proc/self/maps", "r")) {
        char line[4096];
        while (std::fgets(line, sizeof line, f)) {
            unsigned long a, b, off;
            char perm[8], dev[16], name[3000] = {0};
            unsigned long ino;
            if (std::sscanf(line, "%lx-%lx %7s %lx %15s %lu %2999s", &a, &b, perm, &off, dev, &ino, name) >= 6)
                if (perm[2] == 'x') maps.push_back({a, b, off, name});
        }
        std::fclose(f);
    }
    std::map<std::pair<std::string, uint64_t>, uint64_t> hist;
    const size_t n = g_n < kCap ? g_n : kCap;
    auto locate = [&](uint64_t ip, std::string &mod, uint64_t &rel) {
        mod = "?";
        rel = ip;
        for (auto &m : maps)
            if (ip >= m.a && ip < m.b) { mod = m.name; rel = ip - m.a + m.off; return; }
    };
    std::string chains_path = std::string(path) + ".chains";
    FILE *ch = std::fopen(chains_path.c_str(), "w");
    for (size_t i = 0; i < n; ++i) {
        std::string mod;
        uint64_t rel;
        locate(g_buf[i][0], mod, rel);
        ++hist[{mod, rel}];
        if (!ch) continue;
        for (int d = 0; d < kDepth && g_buf[i][d]; ++d) {
            locate(g_buf[i][d], mod, rel);
            std::fprintf(ch, d ? " %s:%lx" : "%s:%lx", mod.c_str(), (unsigned long)rel);
        }
        std::fputc('\n', ch);
    }
    if (ch) std::fclose(ch);
    FILE *o = std::fopen(path, "w");
    if (!o) return -1;
    for (auto &kv : hist) std::fprintf(o, "%s %lx %lu\n", kv.first.first.c_str(), (unsigned long)kv.first.second, (unsigned long)kv.second);
    std::fclose(o);
    return (int)n;
}

}  // extern "C"
