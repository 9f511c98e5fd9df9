// post.cpp -- exact host restatement of the repeat post-processing
// (TandemRepeatFinder, bwt.py:3144-3944) over the raw strict hits.
//
// Work is organised per "fold unit": the contigs whose natural sort keys are
// equal (normally exactly one contig).  Every stage of the reference either
// groups by chromosome or folds over the globally sorted list with a
// same-chromosome test, so units are independent.  Inside a unit every stage
// is either data-parallel (nested-suppression queries, refine, restore) or a
// fold that is parallelised speculatively and then repaired to the exact
// sequential result (merge), so the output does not depend on thread count.
//
// Records travel as compact Items: a strict hit (bwt.py:1952-1993) is fully
// determined by (start, end, motif length, copies) -- its motif is a slice of
// the contig, confidence 0.95, mismatch 0, ... -- so only records produced by
// _recompute_repeat carry an Extra with their own fields.  actual_sequence is
// always the current frame's slice [start, end) (trimmed before
// _restore_reference_coordinates, full after), so it is never stored.
#include <algorithm>
#include <optional>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <string_view>
#include <thread>
#include <type_traits>
#include <vector>

#include <sched.h>

#include "common.h"

namespace bwtmi {

// CPUs this process may use: the affinity mask, capped by a cgroup CPU quota
static int cpus_visible() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::max(1u, std::thread::hardware_concurrency());
    long q = -1, per = -1;
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {   // cgroup v2: "max 100000" or "Q P"
        char a[32] = {0};
        long b = 0;
        if (std::fscanf(f, "%31s %ld", a, &b) == 2 && std::strcmp(a, "max") != 0) {
            q = std::atol(a);
            per = b;
        }
        std::fclose(f);
    } else if (FILE *g = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {   // cgroup v1
        if (std::fscanf(g, "%ld", &q) != 1) q = -1;
        std::fclose(g);
        if (FILE *h = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
            if (std::fscanf(h, "%ld", &per) != 1) per = -1;
            std::fclose(h);
        }
    }
    if (q > 0 && per > 0) n = std::min<int>(n, (int)std::max<long>(1, (q + per - 1) / per));
    return n;
}

int host_cpu_budget(int *visible, int *local_world) {
    static const int vis = cpus_visible();
    static const int lw = [] {
        const char *e = std::getenv("LOCAL_WORLD_SIZE");
        const int v = e ? std::atoi(e) : 1;
        return v > 0 ? v : 1;
    }();
    if (visible) *visible = vis;
    if (local_world) *local_world = lw;
    return std::max(1, std::min(16, vis / lw));   // 16 measured fastest per rank
}

int host_threads(const bwtmi_params &p) {
    if (p.threads > 0) return p.threads;
    return host_cpu_budget(nullptr, nullptr);
}

// ------------------------------------------------------------ NUMA placement
// The CPU set host work runs on (empty: unchanged).  Set once per process by
// bind_host_numa; the calling thread takes it at once, pool workers at the
// start of their next region (they may predate the binding).
namespace {
std::mutex g_bind_mu;
cpu_set_t g_bind_set;
std::atomic<int> g_bind_epoch{0};
thread_local int tl_bind_epoch = 0;
inline void apply_binding() {
    const int e = g_bind_epoch.load(std::memory_order_acquire);
    if (e == tl_bind_epoch) return;
    cpu_set_t cs;
    {
        std::lock_guard<std::mutex> lk(g_bind_mu);
        cs = g_bind_set;
    }
    (void)sched_setaffinity(0, sizeof cs, &cs);
    tl_bind_epoch = e;
}
}  // namespace

std::string cpulist_str(const cpu_set_t &cs) {
    std::string s;
    for (int c = 0; c < CPU_SETSIZE; ++c) {
        if (!CPU_ISSET(c, &cs)) continue;
        int e = c;
        while (e + 1 < CPU_SETSIZE && CPU_ISSET(e + 1, &cs)) ++e;
        if (!s.empty()) s += ',';
        s += std::to_string(c);
        if (e > c) s += '-' + std::to_string(e);
        c = e;
    }
    return s;
}
bool parse_cpulist(const char *txt, cpu_set_t &cs) {
    CPU_ZERO(&cs);
    for (const char *p = txt; p && *p && *p != '\n';) {
        char *e;
        const long a = std::strtol(p, &e, 10);
        if (e == p) return false;
        long b = a;
        p = e;
        if (*p == '-') {
            b = std::strtol(p + 1, &e, 10);
            if (e == p + 1) return false;
            p = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET((int)c, &cs);
        if (*p == ',') ++p;
    }
    return true;
}
namespace {
int read_int(const std::string &path, int def) {
    int v = def;
    if (FILE *f = std::fopen(path.c_str(), "r")) {
        if (std::fscanf(f, "%d", &v) != 1) v = def;
        std::fclose(f);
    }
    return v;
}
int g_bound_node = -1;   // the node host work is bound to (under g_bind_mu)
cpu_set_t g_orig_set;    // the affinity the first binding replaced
}  // namespace

// The NUMA node of a GPU from its PCI address ("0000:75:00.0"), -1 unknown
int gpu_numa_node(const char *sysroot, const char *pci) {
    std::string id(pci ? pci : "");
    for (auto &ch : id) ch = (char)std::tolower((unsigned char)ch);
    return read_int(std::string(sysroot) + "/bus/pci/devices/" + id + "/numa_node", -1);
}

// Pure planner (no affinity change; sysfs read under `sysroot`, "/sys" on a
// host, a faked tree in the tests).  Local rank r of the node drives the GPU
// at rank_pci[r]; this rank's GPU is rank_pci[local_rank].  The set: the
// `allowed` CPUs of this GPU's NUMA node; with one hardware thread per
// physical core when those cores can hold every local rank WHOSE GPU SITS ON
// THAT NODE with `threads` workers + 4 runtime threads each (two workers on
// the siblings of one core run the memory-bound host passes at well under
// half speed each; smt keeps the siblings).  False (no binding): unknown
// node, the process already runs inside the node, or fewer allowed CPUs there
// than `threads` (a small cpuset split over both nodes).
bool plan_host_binding(const char *sysroot, int local_rank, const std::vector<std::string> &rank_pci, int threads,
                       bool smt, const cpu_set_t &allowed, cpu_set_t &out, int *node_out, int *ranks_on_node) {
    if (local_rank < 0 || local_rank >= (int)rank_pci.size()) return false;
    const int node = gpu_numa_node(sysroot, rank_pci[(size_t)local_rank].c_str());
    if (node_out) *node_out = node;
    if (node < 0) return false;
    int peers = 0;
    for (const auto &p : rank_pci) peers += gpu_numa_node(sysroot, p.c_str()) == node;
    if (ranks_on_node) *ranks_on_node = peers;
    cpu_set_t want, both;
    FILE *f = std::fopen((std::string(sysroot) + "/devices/system/node/node" + std::to_string(node) + "/cpulist").c_str(), "r");
    if (!f) return false;
    char buf[4096];
    const bool ok = std::fgets(buf, sizeof buf, f) != nullptr;
    std::fclose(f);
    if (!ok || !parse_cpulist(buf, want)) return false;
    CPU_AND(&both, &want, &allowed);
    if (CPU_EQUAL(&both, &allowed) || CPU_COUNT(&both) < threads) return false;
    if (!smt) {
        cpu_set_t one;
        CPU_ZERO(&one);
        std::vector<std::pair<int, int>> seen;   // (package, core) taken
        for (int c = 0; c < CPU_SETSIZE; ++c) {
            if (!CPU_ISSET(c, &both)) continue;
            const std::string t = std::string(sysroot) + "/devices/system/cpu/cpu" + std::to_string(c) + "/topology/";
            const int pkg = read_int(t + "physical_package_id", -1), core = read_int(t + "core_id", -1);
            if (pkg < 0 || core < 0) { CPU_ZERO(&one); break; }   // no topology: keep the node set
            if (std::find(seen.begin(), seen.end(), std::make_pair(pkg, core)) != seen.end()) continue;
            seen.emplace_back(pkg, core);
            CPU_SET(c, &one);
        }
        if (CPU_COUNT(&one) >= peers * (threads + 4)) both = one;
    }
    out = both;
    return true;
}

bool bind_host_numa(int local_rank, const std::vector<std::string> &rank_pci) {
    cpu_set_t cur, want;
    if (sched_getaffinity(0, sizeof cur, &cur) != 0) return false;
    int node = -1;
    if (!plan_host_binding("/sys", local_rank, rank_pci, host_cpu_budget(nullptr, nullptr), knob(KN_NUMA_SMT) != 0, cur,
                           want, &node, nullptr))
        return false;
    {
        std::lock_guard<std::mutex> lk(g_bind_mu);
        if (g_bound_node >= 0 && g_bound_node != node) return false;   // contexts on two nodes: keep the first
        if (g_bound_node < 0) g_orig_set = cur;
        g_bound_node = node;
        g_bind_set = want;
    }
    g_bind_epoch.fetch_add(1, std::memory_order_acq_rel);
    apply_binding();
    return true;
}

bool unbind_host() {
    {
        std::lock_guard<std::mutex> lk(g_bind_mu);
        if (g_bound_node < 0) return false;
        g_bound_node = -1;
        g_bind_set = g_orig_set;
    }
    g_bind_epoch.fetch_add(1, std::memory_order_acq_rel);
    apply_binding();
    return true;
}

// Persistent worker pools: parallel regions reuse the same threads (and their
// thread-local DP scratch) instead of spawning per call.  The caller takes
// part as worker 0; a region started from inside a worker of the same pool
// runs inline.  Parallel regions go to the calling thread's current pool (the
// process-wide one unless the thread belongs to a unit group, postprocess).
namespace {
// Region hand-off: a region is published by bumping `agen`; workers that
// finished their last region may spin on it for a while (BWTMI_POOL_SPIN_US)
// before they block on the condition variable, and the caller spins on
// `apending` the same way before it blocks.  10 us catches the back-to-back
// regions of a step (r03aa/r03ab: C3 +4 %, W=8 shard step 8.0-8.1 vs 8.6-8.9
// ms), while a 60 us spin, also held through longer serial parts, cost the C3
// line ~7 % on another box (r03z).  Auto (-1, the default): 200 us while the
// calling job holds <= 32 Mbp (its regions are short and come back to back:
// W=8 shard 6.3-6.6 vs 6.8-7.3 ms at 10 us, r05gd), else 10 us (C3 within
// its run-to-run spread either way; round 6 tried 300 us: r06y favoured it,
// but interleaved after a warm-up run on one box, r06ar, 300 us 3582 / 3543 /
// 3679 vs 10 us 3447 / 3615 / 3767 Mbp/s -- no gain, more CPU).  0 = block at once.
std::atomic<int64_t> g_auto_spin_ns{10000};
inline int64_t pool_spin_ns() {
    const int64_t k = knob(KN_POOL_SPIN_US);
    return k >= 0 ? k * 1000 : g_auto_spin_ns.load(std::memory_order_relaxed);
}
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// spin until pred() or the spin window ends; true when pred() held
template <class P>
inline bool spin_until(P &&pred) {
    const int64_t lim = pool_spin_ns();
    if (lim <= 0) return pred();
    const int64_t t0 = now_ns();
    for (int k = 0;; ++k) {
        if (pred()) return true;
        __builtin_ia32_pause();
        if ((k & 63) == 63 && now_ns() - t0 > lim) return pred();
    }
}

class Pool {
public:
    static Pool &global() {
        static Pool p;
        return p;
    }
    static Pool &current() { return tl_pool ? *tl_pool : global(); }
    // f(w) for w in [0, nt)
    void run(int nt, const std::function<void(int)> &f) {
        if (nt <= 1 || worker_of == this) {
            for (int w = 0; w < nt; ++w) f(w);
            return;
        }
        std::unique_lock<std::mutex> region(region_mu);   // one region at a time
        grow(nt - 1);
        bool wake;
        {
            std::lock_guard<std::mutex> lk(mu);
            job = &f;
            want = nt - 1;
            err = nullptr;
            apending.store(nt - 1, std::memory_order_relaxed);
            agen.store(agen.load(std::memory_order_relaxed) + 1, std::memory_order_release);
            wake = sleepers > 0;
        }
        if (wake) cv.notify_all();
        Pool *const outer = worker_of;
        worker_of = this;
        try {
            f(0);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
        worker_of = outer;
        // every worker finishes before f (and what it references) goes out of scope
        if (!spin_until([&] { return apending.load(std::memory_order_acquire) == 0; })) {
            std::unique_lock<std::mutex> lk(mu);
            caller_waits = true;
            done.wait(lk, [&] { return apending.load(std::memory_order_acquire) == 0; });
            caller_waits = false;
        }
        std::lock_guard<std::mutex> lk(mu);
        job = nullptr;
        if (err) {
            std::exception_ptr e = err;
            err = nullptr;
            std::rethrow_exception(e);
        }
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            agen.store(agen.load(std::memory_order_relaxed) + 1, std::memory_order_release);
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
    static thread_local Pool *tl_pool;   // the pool this thread's regions go to (nullptr: global)

private:
    void grow(int n) {
        while ((int)th.size() < n) {
            const int id = (int)th.size();
            th.emplace_back([this, id] { loop(id); });
        }
    }
    void loop(int id) {
        worker_of = this;
        tl_pool = this;
        int64_t seen = 0;
        {
            std::lock_guard<std::mutex> lk(mu);
            seen = agen.load(std::memory_order_relaxed);   // a worker created for the current region still takes part in it
            if (job && id < want) seen -= 1;
        }
        for (;;) {
            const std::function<void(int)> *f;
            if (!spin_until([&] { return agen.load(std::memory_order_acquire) != seen; })) {
                std::unique_lock<std::mutex> lk(mu);
                ++sleepers;
                cv.wait(lk, [&] { return agen.load(std::memory_order_relaxed) != seen; });
                --sleepers;
            }
            {
                std::lock_guard<std::mutex> lk(mu);   // job / want / stop of the generation seen
                if (stop) return;
                seen = agen.load(std::memory_order_relaxed);
                if (id >= want) continue;
                f = job;
            }
            apply_binding();
            try {
                (*f)(id + 1);
            } catch (...) {   // reported to the caller of run(); never escapes the thread
                std::lock_guard<std::mutex> lk(mu);
                if (!err) err = std::current_exception();
            }
            if (apending.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu);   // after the decrement: no lost wake-up
                if (caller_waits) done.notify_one();
            }
        }
    }
    std::vector<std::thread> th;
    std::mutex mu, region_mu;
    std::condition_variable cv, done;
    const std::function<void(int)> *job = nullptr;
    std::exception_ptr err;
    int want = 0, sleepers = 0;
    bool caller_waits = false;
    std::atomic<int64_t> agen{0};
    std::atomic<int> apending{0};
    bool stop = false;
    static thread_local Pool *worker_of;   // the pool whose region this thread is running
};
thread_local Pool *Pool::worker_of = nullptr;
thread_local Pool *Pool::tl_pool = nullptr;
}  // namespace

void pool_spin_for_job(const Job &job) {
    int64_t bases = 0;
    for (size_t i = 0; i < job.contigs.size(); ++i)
        if (job.selected.empty() || (i < job.selected.size() && job.selected[i])) bases += job.contigs[i].trimmed_len();
    g_auto_spin_ns.store(bases <= 32000000 ? 200000 : 10000, std::memory_order_relaxed);
}

// fn(begin, end) over [0, n) in contiguous chunks
template <class F>
static void parallel_for(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (n + 1023) / 1024));
    if (nt <= 1) {
        fn((int64_t)0, n);
        return;
    }
    Pool::current().run(nt, [&](int t) { fn(n * t / nt, n * (t + 1) / nt); });
}

// dynamic scheduling: fn(item, worker)
template <class F>
static void parallel_items(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    std::atomic<int64_t> next{0};
    auto work = [&](int w) {
        for (;;) {
            const int64_t k = next.fetch_add(1, std::memory_order_relaxed);
            if (k >= n) break;
            fn(k, w);
        }
    };
    if (nt == 1) { work(0); return; }
    Pool::current().run(nt, work);
}

// static blocks: worker w takes items [n w / nt, n (w + 1) / nt) -- for the
// memory-bound passes over the fold's chunks, so that a chunk is read by the
// worker (and the core's cache) that wrote it in the pass before
template <class F>
static void parallel_blocks(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    auto work = [&](int w) {
        for (int64_t k = n * w / nt; k < n * (w + 1) / nt; ++k) fn(k, w);
    };
    if (nt == 1) { work(0); return; }
    Pool::current().run(nt, work);
}

void run_tasks(int64_t n, int nt, const std::function<void(int64_t)> &fn) {
    parallel_items(n, nt, [&](int64_t k, int) { fn(k); });
}

// ------------------------------------------------------------ natural key
std::vector<NatPart> natural_key(const std::string &s) {      // bwt.py:22-36
    std::vector<NatPart> out;
    size_t i = 0, n = s.size();
    while (i < n) {
        size_t j = i;
        const bool dig = s[i] >= '0' && s[i] <= '9';
        while (j < n && ((s[j] >= '0' && s[j] <= '9') == dig)) ++j;
        NatPart p;
        p.digit = dig;
        if (dig) {
            size_t k = i;
            while (k + 1 < j && s[k] == '0') ++k;  // int(part): strip leading zeros
            p.text = s.substr(k, j - k);
        } else {
            p.text = s.substr(i, j - i);
            for (auto &c : p.text)
                if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
        }
        out.push_back(std::move(p));
        i = j;
    }
    return out;
}

int natural_cmp(const std::vector<NatPart> &a, const std::vector<NatPart> &b) {
    const size_t n = std::min(a.size(), b.size());
    for (size_t i = 0; i < n; ++i) {
        const NatPart &x = a[i], &y = b[i];
        if (x.digit != y.digit) return x.digit ? -1 : 1;  // (0, int) < (1, str)
        if (x.digit && x.text.size() != y.text.size()) return x.text.size() < y.text.size() ? -1 : 1;
        const int c = x.text.compare(y.text);
        if (c) return c < 0 ? -1 : 1;
    }
    if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
    return 0;
}

void Job::assign_units() {
    natkeys.clear();
    for (auto &c : contigs) natkeys.push_back(natural_key(c.name));
    std::vector<int32_t> order(contigs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int32_t)i;
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return natural_cmp(natkeys[a], natkeys[b]) < 0; });
    nunits = 0;
    unit_rank.clear();
    for (size_t k = 0; k < order.size(); ++k) {
        if (k == 0 || natural_cmp(natkeys[order[k - 1]], natkeys[order[k]]) != 0) {
            unit_rank.push_back(nunits);
            ++nunits;
        }
        contigs[order[k]].unit = nunits - 1;   // unit ids are ranks by natural key
    }
}

std::vector<int32_t> shard_units(Job &job, int32_t world, int32_t rank) {
    job.assign_units();
    std::vector<int64_t> w((size_t)job.nunits, 0);
    for (auto &c : job.contigs) w[(size_t)c.unit] += c.weight;
    std::vector<int32_t> order((size_t)job.nunits);
    for (int32_t u = 0; u < job.nunits; ++u) order[(size_t)u] = u;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return w[(size_t)a] > w[(size_t)b]; });
    std::vector<int64_t> load((size_t)std::max(1, world), 0);
    std::vector<int32_t> owner((size_t)job.nunits, 0);
    for (int32_t u : order) {
        int32_t r = 0;
        for (int32_t x = 1; x < world; ++x)
            if (load[(size_t)x] < load[(size_t)r]) r = x;
        load[(size_t)r] += w[(size_t)u];
        owner[(size_t)u] = r;
    }
    std::vector<int32_t> out;
    for (size_t c = 0; c < job.contigs.size(); ++c)
        if (owner[(size_t)job.contigs[c].unit] == rank) out.push_back((int32_t)c);
    return out;
}

namespace {

// fields of a record produced by _recompute_repeat (bwt.py:3593-3614)
struct Extra {                  // trivially destructible: strings live in the Pools arena
    std::string_view motif;     // == consensus_motif
    std::string_view variations;  // ';'-joined, empty == None
    double copies = 0, confidence = 0, mm = 0, pmatch = 0, pindel = 0;
    int64_t max_mm = 0, n_eval = 0, score = 0;
    int64_t req_end = -1;       // the (clamped) end and motif length the recompute
    int32_t req_m = 0;          // was asked for
    int32_t tier = 2;
    char strand = '+';
    bool stats_none = false;    // Rec::stats_none
    // the DP walk stopped at a copy that failed (not at its safety limit):
    // where, and with which min_copies (1: min_copies, 2: the retry with 1).
    // A later call with the same start and motif length whose limit lies past
    // wk_stop walks the same windows (recompute's reuse; refine's calls)
    int8_t wk_phase = 0;
    int64_t wk_stop = -1;
};

static_assert(std::is_trivially_destructible<Extra>::value, "Extras live in raw arena blocks");

// 32 bytes: a strict hit (x == nullptr) is fully determined by its span and
// primitive motif length -- motif = sequence[start, start + mlen) of the frame,
// copies = (end - start) / mlen (bwt.py:1957-1961; also (end - i) / L when the
// unit is primitive), tier 2; every other record carries an Extra
struct Item {
    int64_t start, end;   // current frame (trimmed, then full after restore)
    // recomputed record (nullptr for a strict hit), tagged in bit 0 when its
    // mismatch rate is non-zero: the refine pass tests every fold output and
    // only those records, so it reads no Extra for the others (each read a
    // cache miss: the C3 assembly pass 6.0 -> ~2 ms)
    const Extra *xp;
    int32_t chrom, mlen;
    const Extra *x() const { return reinterpret_cast<const Extra *>(reinterpret_cast<uintptr_t>(xp) & ~uintptr_t(1)); }
    bool imperfect() const { return (reinterpret_cast<uintptr_t>(xp) & 1u) != 0; }
    void set_x(const Extra *e) {   // after e->mm is final
        xp = reinterpret_cast<const Extra *>(reinterpret_cast<uintptr_t>(e) | (e && e->mm != 0.0 ? 1u : 0u));
    }
};
static_assert(sizeof(Item) == 32, "fold items stay 32 bytes");

// vector storage without value-initialisation: large item arrays are written
// once in parallel, so the first touch happens in the filling threads
using ItemVec = std::vector<Item, NoInit<Item>>;

// per-worker bump arenas for Extras and their strings (pointer-stable; the
// blocks are cached huge-page blocks, mem.h)
struct Pools {
    struct Block {
        void *p = nullptr;
        size_t bytes = 0;
        Block(size_t b) : p(big_alloc(b)), bytes(b) {}
        Block(Block &&o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; }
        Block(const Block &) = delete;
        ~Block() { if (p) big_free(p, bytes); }
    };
    struct Arena {
        std::vector<Block> xb;
        size_t xn = 0;                                   // used in the last Extra block
        std::vector<Block> cb;
        size_t cn = 0, ccap = 0;                         // used / size of the last char block
        // the worker's DP scratch and summary (recompute)
        std::unique_ptr<AlignScratch, void (*)(AlignScratch *)> as{align_scratch_new(), align_scratch_free};
        AlignSummary sum;
        // the last maximal homopolymer run this worker walked: [hlo, hhi) of
        // byte hb in sequence hseq (sequences do not change while the pools live)
        const char *hseq = nullptr;
        int64_t hlo = 0, hhi = 0;
        char hb = 0;
        // the worker's last host recompute whose walk stopped at a copy that
        // failed (not at its safety limit): from the same start with the same
        // motif length, any call whose limit lies past that stop walks the same
        // windows -- a merge chain re-asks this for every record it absorbs
        bool wk_ok = false;
        const char *wk_seq = nullptr;
        int64_t wk_start = 0, wk_m = 0, wk_stop = 0;
        int wk_phase = 0;   // 1: the min_copies walk succeeded; 2: the min_copies = 1 retry
        Item wk_item{};
    };
    static constexpr size_t XB = 16384, CB = size_t(2) << 20;   // Extras are trivially destructible
    std::vector<Arena> a;
    explicit Pools(int n) : a((size_t)n) {}
    std::string_view str(Arena &A, std::string_view s) {
        if (s.empty()) return {};
        if (A.cb.empty() || A.cn + s.size() > A.ccap) {
            A.ccap = std::max(CB, s.size());
            A.cb.emplace_back(A.ccap);
            A.cn = 0;
        }
        char *d = (char *)A.cb.back().p + A.cn;
        std::memcpy(d, s.data(), s.size());
        A.cn += s.size();
        return std::string_view(d, s.size());
    }
    // motif already lives in static storage, no variations
    Extra *add_static(int w, const Extra &e, std::string_view motif) {
        Arena &A = a[(size_t)w];
        if (A.xb.empty() || A.xn == XB) {
            A.xb.emplace_back(XB * sizeof(Extra));
            A.xn = 0;
        }
        Extra *x = (Extra *)A.xb.back().p + A.xn++;
        ::new ((void *)x) Extra(e);
        x->motif = motif;
        x->variations = {};
        return x;
    }
    // a copy of e sharing its strings (the arena keeps them)
    Extra *clone(int w, const Extra &e) {
        Arena &A = a[(size_t)w];
        if (A.xb.empty() || A.xn == XB) {
            A.xb.emplace_back(XB * sizeof(Extra));
            A.xn = 0;
        }
        Extra *x = (Extra *)A.xb.back().p + A.xn++;
        ::new ((void *)x) Extra(e);
        return x;
    }
    Extra *add(int w, const Extra &e, std::string_view motif, std::string_view variations) {
        Arena &A = a[(size_t)w];
        if (A.xb.empty() || A.xn == XB) {
            A.xb.emplace_back(XB * sizeof(Extra));
            A.xn = 0;
        }
        Extra *x = (Extra *)A.xb.back().p + A.xn++;
        ::new ((void *)x) Extra(e);
        x->motif = str(A, motif);
        x->variations = str(A, variations);
        return x;
    }
};

struct UnitCtx {
    const Job *job;
    int64_t min_copies;
    bool restored = false;        // items are in full-sequence coordinates (multi-offset units)
};

inline std::string_view motif_of(const UnitCtx &u, const Item &it) {
    if (it.xp) return it.x()->motif;
    const Contig &c = u.job->contigs[(size_t)it.chrom];
    return std::string_view((u.restored ? c.full.data() : c.trimmed()) + it.start, (size_t)it.mlen);
}
inline int64_t strict_copies(const Item &it) { return (it.end - it.start) / it.mlen; }
inline int32_t tier_of(const Item &it) { return it.xp ? it.x()->tier : 2; }
inline double copies_of(const Item &it) { return it.xp ? it.x()->copies : (double)strict_copies(it); }
inline double mm_of(const Item &it) { return it.xp ? it.x()->mm : 0.0; }
inline double conf_of(const Item &it) { return it.xp ? it.x()->confidence : 0.95; }

// stable sort of items by (start, end)
void sort_by_pos(ItemVec &v, int nt) {
    const size_t n = v.size();
    if (n < 2) return;
    // order checks in parallel chunks (each chunk also checks the pair across its left edge)
    const int C = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt * 4, n / 32768 + 1));
    std::vector<uint8_t> c_sorted((size_t)C, 1), c_start((size_t)C, 1);
    parallel_items(C, nt, [&](int64_t t, int) {
        const size_t a = std::max<size_t>(1, n * (size_t)t / (size_t)C), b = n * (size_t)(t + 1) / (size_t)C;
        bool so = true, bs = true;
        for (size_t i = a; i < b && bs; ++i) {
            bs = v[i - 1].start <= v[i].start;
            so = so && (v[i - 1].start < v[i].start || v[i - 1].end <= v[i].end);
        }
        c_sorted[(size_t)t] = so;
        c_start[(size_t)t] = bs;
    });
    bool sorted = true, by_start = true;
    for (int t = 0; t < C; ++t) {
        sorted = sorted && c_sorted[(size_t)t];
        by_start = by_start && c_start[(size_t)t];
    }
    if (sorted && by_start) return;
    if (by_start) {   // the usual case after merge/refine: only equal-start runs need ordering by end
        // chunk t orders the runs that begin inside it
        parallel_items(C, nt, [&](int64_t t, int) {
            size_t i = n * (size_t)t / (size_t)C;
            const size_t b = n * (size_t)(t + 1) / (size_t)C;
            while (i > 0 && i < b && v[i - 1].start == v[i].start) ++i;
            while (i < b) {
                size_t j = i + 1;
                while (j < n && v[j].start == v[i].start) ++j;
                if (j - i > 1)
                    std::stable_sort(v.begin() + (std::ptrdiff_t)i, v.begin() + (std::ptrdiff_t)j,
                                     [](const Item &x, const Item &y) { return x.end < y.end; });
                i = j;
            }
        });
        return;
    }
    auto lt = [](const Item &a, const Item &b) {
        if (a.start != b.start) return a.start < b.start;
        return a.end < b.end;
    };
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, n / 65536 + 1));
    if (T == 1) {
        std::stable_sort(v.begin(), v.end(), lt);
        return;
    }
    std::vector<size_t> cut((size_t)T + 1);
    for (int t = 0; t <= T; ++t) cut[(size_t)t] = n * (size_t)t / (size_t)T;
    parallel_items(T, T, [&](int64_t t, int) { std::stable_sort(v.begin() + cut[(size_t)t], v.begin() + cut[(size_t)t + 1], lt); });
    for (int w = 1; w < T; w *= 2) {    // pairwise stable merges, one level at a time
        std::vector<std::array<size_t, 3>> jobs;
        for (int t = 0; t + w < T; t += 2 * w) jobs.push_back({cut[(size_t)t], cut[(size_t)(t + w)], cut[(size_t)std::min(T, t + 2 * w)]});
        parallel_items((int64_t)jobs.size(), nt, [&](int64_t q, int) {
            auto &j = jobs[(size_t)q];
            std::inplace_merge(v.begin() + j[0], v.begin() + j[1], v.begin() + j[2], lt);
        });
    }
}

// ---------------------------------------------------- nested suppression
// bwt.py:3402-3497.  A repeat is tested only against kept spans of a strictly
// longer motif; the stable sort by (mismatch_rate > 0, -len(motif)) places
// every such span of its class (and the whole perfect class) before it, and
// repeats of equal motif length never test each other.  So each (class,
// length) group is screened -- in parallel, against a frozen grid of the
// spans kept so far -- and its survivors are appended as a whole.  The
// predicate is the reference's, division for division.
ItemVec suppress_nested(const ItemVec &rs, double thr, int nt) {
    const size_t n = rs.size();
    int32_t maxlen = 0;
    for (auto &r : rs) maxlen = std::max(maxlen, r.mlen);
    const size_t nb = 2 * ((size_t)maxlen + 1);
    auto bucket = [&](const Item &r) {
        return (mm_of(r) > 0 ? (size_t)maxlen + 1 : 0) + (size_t)(maxlen - r.mlen);
    };
    std::vector<uint32_t> cnt(nb + 1, 0), order(n);
    for (auto &r : rs) ++cnt[bucket(r) + 1];
    for (size_t b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
    std::vector<uint32_t> groups(cnt.begin(), cnt.end());
    for (size_t i = 0; i < n; ++i) order[cnt[bucket(rs[i])]++] = (uint32_t)i;

    int64_t maxpos = 1;
    for (auto &r : rs) maxpos = std::max(maxpos, r.end + 1);
    const int64_t B = 256;
    struct Span { int64_t s, e, M; };
    std::vector<std::vector<Span>> grid((size_t)(maxpos / B + 2));
    std::vector<uint8_t> keep(n, 0);
    ItemVec kept;
    kept.reserve(n);
    for (size_t g = 0; g < nb; ++g) {
        const size_t g0 = groups[g], g1 = groups[g + 1];
        if (g0 == g1) continue;
        const bool any_kept = !kept.empty();
        parallel_for((int64_t)(g1 - g0), any_kept ? nt : 1, [&](int64_t a, int64_t b) {
            for (int64_t q = a; q < b; ++q) {
                const Item &r = rs[order[g0 + (size_t)q]];
                const int64_t s0 = r.start, e0 = r.end, m = r.mlen;
                const int64_t rl = e0 - s0;
                bool nested = false;
                if (any_kept && e0 > s0) {
                    const int64_t b0 = std::max<int64_t>(0, s0) / B, b1 = std::max<int64_t>(0, e0 - 1) / B;
                    for (int64_t bk = b0; bk <= b1 && !nested && bk < (int64_t)grid.size(); ++bk) {
                        for (const Span &sp : grid[(size_t)bk]) {
                            if (sp.M <= m) continue;
                            const int64_t ov = std::max<int64_t>(0, std::min(e0, sp.e) - std::max(s0, sp.s));
                            if (ov == 0) continue;
                            const double ratio = (double)sp.M / (double)m;
                            const double frac = (double)ov / (double)rl;
                            if (m == 1 && sp.M > 1 && frac >= 0.8) { nested = true; break; }
                            const double t = ratio >= 10 ? 0.1 : (ratio >= 5 ? 0.3 : thr);
                            if (frac >= t) { nested = true; break; }
                        }
                    }
                }
                keep[order[g0 + (size_t)q]] = !nested;
            }
        });
        for (size_t q = g0; q < g1; ++q) {
            const uint32_t idx = order[q];
            if (!keep[idx]) continue;
            const Item &r = rs[idx];
            if (r.end > r.start) {
                const Span sp{r.start, r.end, (int64_t)r.mlen};
                const int64_t b0 = std::max<int64_t>(0, r.start) / B, b1 = std::max<int64_t>(0, r.end - 1) / B;
                for (int64_t bk = b0; bk <= b1 && bk < (int64_t)grid.size(); ++bk) grid[(size_t)bk].push_back(sp);
            }
            kept.push_back(r);
        }
    }
    return kept;
}

// every byte value as a one-character string (motifs of one-base recomputes)
const struct ByteChars {
    char c[256];
    ByteChars() { for (int i = 0; i < 256; ++i) c[i] = (char)i; }
    const char &operator[](size_t i) const { return c[i]; }
} kByteChars;

inline char comp_of(char c) {   // bwt.py:688-691
    switch (c) {
        case 'A': return 'T';
        case 'T': return 'A';
        case 'C': return 'G';
        case 'G': return 'C';
        default: return c;
    }
}

std::atomic<int64_t> g_recomputes{0}, g_recompute_ns{0}, g_merges{0}, g_canons{0}, g_tests{0}, g_same{0}, g_walk_reuse{0};
// BWTMI_STATS=1: stage timers; =2: also per-recompute / per-test counters (slow)
const char *const g_dump = std::getenv("BWTMI_DUMP_RECOMPUTE");
std::atomic<int64_t> g_hist_n[8][8], g_hist_ns[8][8];
std::atomic<int64_t> g_fresh_tests{0}, g_chain_tests{0}, g_fresh_merges{0}, g_chain_merges{0};   // [log4 motif len][log4 region len]
inline int lg4(int64_t v) { int k = 0; while (v >= 4 && k < 7) { v >>= 2; ++k; } return k; }

// align_repeat_region's result as _recompute_repeat reads it (a host AlignSummary)
struct RcView {
    bool ok = false;
    int64_t consumed = 0, copies = 0, motif_len = 0, max_err = 0, tot_ins = 0, tot_del = 0;
    double mm = 0.0;
    std::string_view consensus, var;
};
Item item_of_alignment(const UnitCtx &u, Pools &pools, int w, int32_t chrom, int64_t start, int64_t end, int64_t m,
                       int32_t tier, std::string_view tmpl, const RcView &v);

// bwt.py:3515-3614 (on the trimmed sequence, before coordinate restore)
// prev (optional): an earlier record from the same start (refine passes the
// record it refines) -- reused when its walk stopped at a failing copy inside
// this call's limit
Item recompute(const UnitCtx &u, Pools &pools, int w, int32_t chrom, int64_t start, int64_t end,
               int64_t motif_len, int32_t tier, const Item *prev = nullptr) {
    struct Tick {   // BWTMI_STATS=2 only
        int a, b;
        std::chrono::steady_clock::time_point t;
        Tick(int a_, int b_) : a(a_), b(b_) { if (stats_on(2)) t = std::chrono::steady_clock::now(); }
        ~Tick() {
            if (!stats_on(2)) return;
            const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t).count();
            g_recomputes.fetch_add(1, std::memory_order_relaxed);
            g_recompute_ns.fetch_add(ns, std::memory_order_relaxed);
            g_hist_n[a][b].fetch_add(1, std::memory_order_relaxed);
            g_hist_ns[a][b].fetch_add(ns, std::memory_order_relaxed);
        }
    } tick{lg4(motif_len), lg4(end - start)};
    const Contig &c = u.job->contigs[(size_t)chrom];
    const char *seq = c.trimmed();
    const int64_t L = c.trimmed_len();
    const int64_t m = std::max<int64_t>(1, motif_len);
    start = std::max<int64_t>(0, start);
    end = end > 0 ? std::min(L, end) : L;
    if (end <= start) end = std::min(L, start + m);
    const int64_t req_end = end;
    if (m == 1 && start < L) {
        // One-base motif (~75 % of the recomputes): align_repeat_region's closed
        // form (motif.cpp) without building any strings.  The template is
        // seq[start]; the walk is the run of that base up to its limit, first
        // with min_copies, then (bwt.py:3530-3534) with min_copies 1, which
        // always succeeds (the run holds the template itself).
        const char b = seq[start];
        const int64_t mc = std::max<int64_t>(1, u.min_copies);
        // the maximal run of b through start: a merge chain over one long run
        // (an assembly gap's N run yields a hit per unit length, ~1000 of them,
        // each merge recomputing the union) walks it once per worker
        Pools::Arena &HA = pools.a[(size_t)w];
        if (!(HA.hseq == seq && HA.hb == b && HA.hlo <= start && start < HA.hhi)) {
            HA.hseq = seq;
            HA.hb = b;
            HA.hlo = start;
            HA.hhi = run_end(seq, start, L, b);
        }
        const int64_t hhi = HA.hhi;
        auto run_to = [&](int64_t limit) { return std::min(hhi, limit) - start; };
        int64_t run = run_to(std::min<int64_t>(L, std::max<int64_t>(end, start + mc) + 4));
        if (run < mc) run = run_to(std::min<int64_t>(L, std::max<int64_t>(end, start + 1) + 4));
        Extra x;
        x.copies = (double)run;        // tl / 1 is integral
        x.confidence = 1.0;            // max(0.3, 1 - 0)
        x.mm = 0.0;
        x.n_eval = std::max<int64_t>(1, run);
        x.max_mm = 0;
        const char rc = comp_of(b);
        x.strand = (unsigned char)b <= (unsigned char)rc ? '+' : '-';   // get_canonical_motif_stranded
        x.pmatch = 100.0;
        x.pindel = 0.0;
        x.score = trf_score(run, 0.0);
        x.tier = tier;
        x.req_end = req_end;
        x.req_m = (int32_t)m;
        Item it{};
        it.start = start;
        it.end = start + run;
        it.chrom = chrom;
        it.mlen = 1;
        it.set_x(pools.add_static(w, x, std::string_view(&kByteChars[(uint8_t)b], 1)));
        return it;
    }
    if (g_dump) {   // BWTMI_DUMP_RECOMPUTE=path: the DP recomputes' arguments (tools/recompute_bench.cpp)
        static std::mutex mu;
        std::lock_guard<std::mutex> lk(mu);
        static FILE *df = std::fopen(g_dump, "w");
        if (df) std::fprintf(df, "%lld %lld %lld %lld\n", (long long)start, (long long)end, (long long)m,
                             (long long)std::max<int64_t>(1, u.min_copies));
    }
    auto slice = [&](int64_t a, int64_t b) {   // Python seq[a:b], a,b >= 0
        a = std::min(a, L);
        b = std::min(b, L);
        return b > a ? std::string(seq + a, (size_t)(b - a)) : std::string();
    };
    Pools::Arena &A = pools.a[(size_t)w];
    const int64_t mc = std::max<int64_t>(1, u.min_copies);
    // the walk's safety limit for a min_copies (motif.cpp align_repeat_region, bwt.py:1033)
    const int64_t mi = std::max<int64_t>(1, std::min<int64_t>(10, m >= 4 ? m / 2 : 1));
    auto walk_limit = [&](int64_t mcx) {
        const int64_t e2 = std::min(L, end > start ? end : L);
        return std::min(L, std::max(e2, start + m * mcx) + std::max(m * 3, mi * 4));
    };
    if (prev && prev->xp && prev->start == start && prev->chrom == chrom) {
        const Extra &px = *prev->x();
        if (px.wk_stop >= 0 && px.req_m == m && px.wk_stop < walk_limit(px.wk_phase == 1 ? mc : 1)) {
            if (stats_on(2)) g_walk_reuse.fetch_add(1, std::memory_order_relaxed);
            Extra *x = pools.clone(w, px);
            x->req_end = req_end;
            x->tier = tier;
            Item it = *prev;
            it.set_x(x);
            return it;
        }
    }
    if (A.wk_ok && A.wk_seq == seq && A.wk_start == start && A.wk_m == m &&
        A.wk_stop < walk_limit(A.wk_phase == 1 ? mc : 1)) {
        // the same windows up to the same failing copy: the same record, but
        // for what depends on the call itself (the requested end, the tier)
        if (stats_on(2)) g_walk_reuse.fetch_add(1, std::memory_order_relaxed);
        Extra *x = pools.clone(w, *A.wk_item.x());
        x->req_end = req_end;
        x->tier = tier;
        Item it = A.wk_item;
        it.set_x(x);
        return it;
    }
    std::string tmpl = slice(start, start + m);
    if (tmpl.empty()) {
        const int64_t a = std::max<int64_t>(0, start - m);
        tmpl = slice(a, a + m);
    }
    if (tmpl.empty()) tmpl.assign((size_t)m, 'N');
    AlignSummary &s = A.sum;
    s.want_copies = false;
    int phase = 1;
    // resume: a chain of merges recomputes a growing region from one start,
    // and each walk that stopped at its limit goes on from where it stopped
    constexpr bool resume = true;
    bool ok = align_repeat_region(seq, L, start, end, tmpl, mc, s, 0.1, -1, A.as.get(), resume);
    if (!ok) {
        phase = 2;
        ok = align_repeat_region(seq, L, start, end, tmpl, 1, s, 0.1, -1, A.as.get(), resume);
    }
    RcView v;
    v.ok = ok;
    if (ok) {
        v.consumed = s.consumed;
        v.copies = s.copies;
        v.motif_len = s.motif_len;
        v.max_err = s.max_errors;
        v.tot_ins = s.tot_ins;
        v.tot_del = s.tot_del;
        v.mm = s.mismatch_rate;
        v.consensus = s.consensus;
        if (s.any_variation) v.var = s.variations;
    }
    Item it = item_of_alignment(u, pools, w, chrom, start, end, m, tier, tmpl, v);
    A.wk_ok = ok && !s.at_limit;
    if (A.wk_ok) {   // this worker's new Extra: the record carries its walk's stop for later calls
        Extra *xe = const_cast<Extra *>(it.x());
        xe->wk_stop = start + s.consumed;
        xe->wk_phase = (int8_t)phase;
    }
    if (A.wk_ok) {
        A.wk_seq = seq;
        A.wk_start = start;
        A.wk_m = m;
        A.wk_stop = start + s.consumed;
        A.wk_phase = phase;
        A.wk_item = it;
    }
    return it;
}

// the record _recompute_repeat builds from an alignment (bwt.py:3536-3614)
Item item_of_alignment(const UnitCtx &u, Pools &pools, int w, int32_t chrom, int64_t start, int64_t end, int64_t m,
                       int32_t tier, std::string_view tmpl, const RcView &v) {
    const Contig &c = u.job->contigs[(size_t)chrom];
    const int64_t L = c.trimmed_len();
    const int64_t req_end = end;
    Extra x;
    int64_t consumed, cint;
    double mm, pind;
    std::string_view motif_s = tmpl;   // never empty
    std::string_view var_s;
    if (!v.ok) {
        consumed = std::min(L - start, std::max(m, end - start));
        cint = std::max<int64_t>(1, consumed / m);
        mm = 0.0;
        x.max_mm = 0;
        pind = 0.0;
    } else {
        consumed = v.consumed;
        cint = v.copies;
        if (!v.consensus.empty()) motif_s = v.consensus;
        mm = v.mm;
        const int64_t tb = v.copies * v.motif_len;
        const double ir = tb > 0 ? (double)(v.tot_ins + v.tot_del) / (double)tb : 0.0;
        pind = ir * 100.0;
        x.max_mm = v.max_err;
        var_s = v.var;
    }
    // actual_sequence = sequence[start:start+consumed]
    const int64_t a0 = std::min(start, L), a1 = std::max(a0, std::min(start + consumed, L));
    const int64_t tl = a1 - a0;
    const int64_t mle = (int64_t)motif_s.size();
    double cf = (double)cint;
    if (tl > 0 && mle > 0) {
        const double fr = (double)tl / (double)mle;
        const double rr = std::nearbyint(fr);  // Python round(): half to even
        cf = std::fabs(fr - rr) < 1e-6 ? rr : fr;
    }
    x.copies = cf;
    x.confidence = std::max(0.3, 1.0 - mm);
    x.mm = mm;
    x.n_eval = std::max<int64_t>(1, cint);
    x.strand = canonical_strand(motif_s.data(), (int64_t)motif_s.size());
    x.pmatch = std::max(0.0, 100.0 - mm * 100.0);
    x.pindel = pind;
    x.score = trf_score(tl, mm);
    x.tier = tier;
    x.req_end = req_end;
    x.req_m = (int32_t)m;
    Item it{};
    it.start = start;
    it.end = start + tl;
    it.chrom = chrom;
    it.mlen = (int32_t)motif_s.size();
    it.set_x(pools.add(w, x, motif_s, var_s));
    return it;
}

// ------------------------------------------------------------ merge fold
// bwt.py:3222-3289.  should_merge needs a recompute only for same-canonical
// neighbours within min_len + 1; when it accepts and len(cur.motif) equals the
// min_len it used, _merge_repeats' recompute has identical arguments and that
// result is reused.  Canonical motifs are computed lazily: most neighbours
// fail the distance test first.
struct Canon {
    std::string s;     // canonical string (motifs that do not pack)
    unsigned __int128 key = 0;  // packed canonical word of an ACGT motif <= 64 bases
    int32_t len = -1;  // motif length; -1 = not computed yet
    bool packed = false;
    bool ok = false;
};

// the canonical form of an item's motif, computed once per fold position:
// for ACGT motifs <= 32 bases the least of the packed rotations of the motif
// and of its reverse complement (the packed word orders like the string)
inline void canon_fill(const UnitCtx &u, const Item &it, Canon &c) {
    if (c.ok) return;
    if (stats_on(2)) g_canons.fetch_add(1, std::memory_order_relaxed);
    const std::string_view mv = motif_of(u, it);
    c.len = (int32_t)mv.size();
    uint64_t x;
    c.packed = mv.size() <= 32 && pack2_acgt(mv.data(), (int64_t)mv.size(), x);
    if (c.packed) {
        c.key = canon2(x, (int64_t)mv.size());
    } else if (mv.size() > 32 && mv.size() <= 64 && canon_key128(mv.data(), (int64_t)mv.size(), c.key)) {
        c.packed = true;   // same length on both sides (same_canonical), so the 64- and 128-bit keys never meet
    } else {
        thread_local std::string tmp;
        tmp.assign(mv.data(), mv.size());
        char st;
        canonical_stranded(tmp, c.s, st);
    }
    c.ok = true;
}

// get_canonical_motif_stranded(m1)[0] == ...(m2)[0] (bwt.py:694-716): equal
// canonical forms.  A motif that packs (ACGT only) and one that does not never
// share a canonical form (rotations and the reverse complement keep non-ACGT
// symbols), so mixed pairs are unequal without building strings.
// the canonical form of a one-base motif, by byte (canonical_stranded of that
// byte, computed once per value): at C3 ~3/4 of the merge tests are between
// one-base runs
inline uint8_t canon_base(uint8_t b) {
    static const std::array<uint8_t, 256> t = [] {
        std::array<uint8_t, 256> a{};
        for (int c = 0; c < 256; ++c) {
            std::string cs;
            char st;
            canonical_stranded(std::string(1, (char)c), cs, st);
            a[(size_t)c] = cs.size() == 1 ? (uint8_t)cs[0] : (uint8_t)c;
        }
        return a;
    }();
    return t[b];
}

inline bool same_canonical(const UnitCtx &u, const Item &r1, Canon &c1, const Item &r2, Canon &c2) {
    const int64_t m1 = r1.xp ? (int64_t)r1.x()->motif.size() : r1.mlen, m2 = r2.xp ? (int64_t)r2.x()->motif.size() : r2.mlen;
    if (m1 != m2) return false;
    if (m1 == 0) return true;
    if (m1 == 1)
        return canon_base((uint8_t)motif_of(u, r1)[0]) == canon_base((uint8_t)motif_of(u, r2)[0]);
    canon_fill(u, r1, c1);
    canon_fill(u, r2, c2);
    if (c1.packed != c2.packed) return false;
    return c1.packed ? c1.key == c2.key : c1.s == c2.s;
}


bool try_merge(const UnitCtx &u, Pools &pools, int w, const Item &r1, Canon &c1, const Item &r2, Canon &c2,
               Item &merged) {
    if (r1.chrom != r2.chrom) return false;
    if (r1.mlen == 0 || r2.mlen == 0) return false;
    const int64_t ml = std::min(r1.mlen, r2.mlen);
    if (std::max<int64_t>(0, r2.start - r1.end) > ml + 1) return false;   // cheap test first
    if (stats_on(2)) g_tests.fetch_add(1, std::memory_order_relaxed);
    if (!same_canonical(u, r1, c1, r2, c2)) return false;
    if (stats_on(2)) g_same.fetch_add(1, std::memory_order_relaxed);
    const int64_t s = std::min(r1.start, r2.start), e = std::max(r1.end, r2.end);
    const int32_t tier = std::min(tier_of(r1), tier_of(r2));
    Item mg = recompute(u, pools, w, r1.chrom, s, e, std::max<int64_t>(1, ml), tier);
    if (mg.x()->copies < (double)u.min_copies) return false;
    const double base = std::max(std::max(mm_of(r1), mm_of(r2)), 0.01);
    if (!(mg.x()->mm <= base + 0.2)) return false;
    if (stats_on(2)) g_merges.fetch_add(1, std::memory_order_relaxed);
    if ((int64_t)r1.mlen == std::max<int64_t>(1, ml)) merged = mg;   // len(r1.consensus_motif)
    else merged = recompute(u, pools, w, r1.chrom, s, e, r1.mlen, tier);
    return true;
}

// Output of a speculative run, compactly: most records leave the fold
// unchanged, so an emitted record is its index in R (>= 0), or ~k for side[k],
// a merged record with the index of its run's first item.  The step at which
// entry q was emitted is the first index of the next run (entry q + 1, or the
// pending run).
struct SpecOut {
    struct Side {
        int64_t j;
        Item it;
    };
    std::vector<int64_t, BigAlloc<int64_t>> emitted;
    std::vector<Side> side;
    Item pending;
    int64_t pending_j = 0;
    Canon pending_canon;
    int64_t start(size_t q) const {
        if (q >= emitted.size()) return pending_j;
        const int64_t e = emitted[q];
        return e >= 0 ? e : side[(size_t)~e].j;
    }
    const Item &record(const ItemVec &R, size_t q) const {
        const int64_t e = emitted[q];
        return e >= 0 ? R[(size_t)e] : side[(size_t)~e].it;
    }
};

// speculative run over [b, e): starts with cur = R[b] as if fresh at b
void spec_run(const UnitCtx &u, Pools &pools, int w, const ItemVec &R, int64_t b, int64_t e,
              std::vector<uint8_t, BigAlloc<uint8_t>> &fresh, SpecOut &o) {
    Item cur = R[(size_t)b];
    int64_t cur_j = b;
    bool merged = false;
    Canon cb[2];   // canonical forms of cur and of the next record; roles swap by index
    int ci_cur = 0;
    fresh[(size_t)b] = 1;
    Item mg;
    o.emitted.reserve((size_t)(e - b));
    for (int64_t i = b + 1; i < e; ++i) {
        Canon &cc = cb[ci_cur], &ci = cb[ci_cur ^ 1];
        ci.ok = false;
        if (stats_on(2)) (merged ? g_chain_tests : g_fresh_tests).fetch_add(1, std::memory_order_relaxed);
        if (try_merge(u, pools, w, cur, cc, R[(size_t)i], ci, mg)) {
            if (stats_on(2)) (merged ? g_chain_merges : g_fresh_merges).fetch_add(1, std::memory_order_relaxed);
            cur = mg;
            merged = true;
            cc.ok = false;
            fresh[(size_t)i] = 0;
        } else {
            if (merged) {
                o.emitted.push_back(~(int64_t)o.side.size());
                o.side.push_back({cur_j, cur});
            } else {
                o.emitted.push_back(cur_j);
            }
            cur = R[(size_t)i];
            cur_j = i;
            merged = false;
            ci_cur ^= 1;
            fresh[(size_t)i] = 1;
        }
    }
    o.pending = cur;
    o.pending_j = cur_j;
    o.pending_canon = std::move(cb[ci_cur]);
}

// _refine_repeats (bwt.py:3291-3314) for one record: only recomputed records
// can carry mismatches; a record whose recompute already covered exactly
// [start, end) with this motif length would be recomputed with the same
// arguments (same result)
inline void refine_one(const UnitCtx &u, Pools &pools, int w, Item &r) {
    if (!r.imperfect()) return;   // a strict hit, or mismatch rate 0
    if (r.mlen > 0 && r.mlen == r.x()->req_m && r.x()->req_end == r.end) return;
    int64_t m = r.mlen;
    if (m <= 0) {
        const int64_t rc = (int64_t)std::nearbyint(copies_of(r));
        m = std::max<int64_t>(1, (r.end - r.start) / std::max<int64_t>(1, rc ? rc : 1));
    }
    r = recompute(u, pools, w, r.chrom, r.start, r.end, m, tier_of(r), &r);
}

// the fold's output, refined (the refine pass runs inside the parallel
// assembly: records are independent there)
// chunks of the fold's output for the collapse pass: [cut[k], cut[k+1]) with
// cmax[k] >= the largest end in it (exact unless an equal-start run was
// reordered across the chunk's edge: then an upper bound, which only moves the
// collapse's independent cuts later)
struct OutChunks {
    std::vector<int64_t> cut, cmax;
};

// fill (optional): writes R[a, b) -- the records are converted by the
// speculative task that reads them first (device-screened hits), not by a pass
// of their own
ItemVec merge_fold(const UnitCtx &u0, Pools &pools, const ItemVec &R, int nt, OutChunks *oc = nullptr,
                   const std::function<void(int64_t, int64_t)> *fill = nullptr) {
    const int64_t n = (int64_t)R.size();
    if (n == 0) return {};
    const UnitCtx &u = u0;
    const int64_t K = std::max<int64_t>(1, std::min<int64_t>((int64_t)nt * 8, n / 2048 + 1));
    std::vector<int64_t> cut((size_t)K + 1);
    for (int64_t k = 0; k <= K; ++k) cut[(size_t)k] = n * k / K;
    std::vector<uint8_t, BigAlloc<uint8_t>> fresh((size_t)n, 0);
    std::vector<SpecOut> spec((size_t)K);
    auto ts0 = std::chrono::steady_clock::now();
    std::vector<double> cms(stats_on() ? (size_t)K : 0);
    // test hook: BWTMI_FAIL_MERGE_CHUNK=k throws inside worker task k (-2: the last
    // task) -- the pool must hand the error back through the C ABI (tests/test_host.py)
    const int64_t inj_k = knob(KN_FAIL_MERGE_CHUNK);
    const int64_t inj = inj_k == -1 ? -1 : inj_k < 0 ? K - 1 : inj_k;
    auto spec_task = [&](int64_t k, int w) {
        if (k == inj) fail(BWTMI_E_STATE, "injected failure in merge task %lld", (long long)k);
        auto a = std::chrono::steady_clock::now();
        if (fill) (*fill)(cut[(size_t)k], cut[(size_t)k + 1]);
        spec_run(u, pools, w, R, cut[(size_t)k], cut[(size_t)k + 1], fresh, spec[(size_t)k]);
        if (stats_on()) cms[(size_t)k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
    };
    parallel_items(K, nt, spec_task);   // dynamic: the chunks' costs are uneven (r04ze: static blocks no better)
    auto ts1 = std::chrono::steady_clock::now();
    if (stats_on()) {
        double sum = 0, mx = 0;
        for (double v : cms) { sum += v; mx = std::max(mx, v); }
        std::fprintf(stderr, "  merge spec %.1f ms (K=%lld, chunk sum %.1f max %.1f ms)\n",
                     std::chrono::duration<double, std::milli>(ts1 - ts0).count(), (long long)K, sum, mx);
    }
    // repair: chunk 0 is exact; a later chunk's speculative results hold from
    // the first index where the true run restarts (non-merge) at an index
    // where the speculative run restarted too
    // The serial part only walks each chunk up to its sync point; the output
    // is then assembled in parallel: chunk k contributes rep[k] (records the
    // true run emitted before syncing) and its speculative entries from[k] on.
    std::vector<ItemVec> rep((size_t)K);
    std::vector<size_t> from((size_t)K, 0);
    std::vector<uint8_t> synced((size_t)K, 0);
    synced[0] = 1;
    Item cur = spec[0].pending;
    Canon cb[2];
    int ci_cur = 0;
    cb[0] = std::move(spec[0].pending_canon);
    Item mg;
    for (int64_t k = 1; k < K; ++k) {
        const int64_t b = cut[(size_t)k], e = cut[(size_t)k + 1];
        SpecOut &sp = spec[(size_t)k];
        int64_t sync = -1;
        for (int64_t i = b; i < e; ++i) {
            Canon &cc = cb[ci_cur], &ci = cb[ci_cur ^ 1];
            ci.ok = false;
            if (try_merge(u, pools, 0, cur, cc, R[(size_t)i], ci, mg)) {
                cur = mg;
                cc.ok = false;
            } else {
                rep[(size_t)k].push_back(cur);
                cur = R[(size_t)i];
                ci_cur ^= 1;
                if (fresh[(size_t)i]) { sync = i; break; }
            }
        }
        if (sync < 0) continue;   // never re-synchronised: `cur` carries into chunk k+1
        size_t q = 0;             // the speculative entry of the run starting at sync
        while (q < sp.emitted.size() && sp.start(q + 1) <= sync) ++q;
        from[(size_t)k] = q;
        synced[(size_t)k] = 1;
        cur = sp.pending;
        cb[ci_cur] = std::move(sp.pending_canon);
    }
    auto ts2 = std::chrono::steady_clock::now();
    std::vector<size_t> at((size_t)K + 1, 0);
    for (int64_t k = 0; k < K; ++k) {
        const SpecOut &sp = spec[(size_t)k];
        at[(size_t)k + 1] = at[(size_t)k] + rep[(size_t)k].size() +
                            (synced[(size_t)k] ? sp.emitted.size() - from[(size_t)k] : 0);
    }
    ItemVec out(at[(size_t)K] + 1);
    // assembly, refine, and the (start, end) order of the result: the fold's
    // output is ordered by start (a merged record starts where its run did);
    // refine only moves ends, so only runs of equal start need ordering by end
    // -- done here per chunk, then for the runs that cross a chunk edge
    std::vector<uint8_t> by_start((size_t)K, 1);
    std::vector<int64_t> cm((size_t)K + 1, INT64_MIN);
    auto by_end = [](const Item &x, const Item &y) { return x.end < y.end; };
    // a chunk's largest end, its order check and its equal-start runs ordered by end
    auto finish_chunk = [&](int64_t k) {
        Item *const d0 = out.data() + at[(size_t)k], *const dst = out.data() + at[(size_t)k + 1];
        int64_t mx = INT64_MIN;
        for (Item *it = d0; it < dst; ++it) mx = std::max(mx, it->end);
        cm[(size_t)k] = mx;
        for (Item *it = d0 + 1; it < dst; ++it)
            if (it[-1].start > it->start) { by_start[(size_t)k] = 0; return; }
        for (Item *i = d0; i < dst;) {
            Item *j = i + 1;
            while (j < dst && j->start == i->start) ++j;
            if (j - i > 1) std::stable_sort(i, j, by_end);
            i = j;
        }
    };
    // The imperfect records (the only ones refine recomputes) are few and
    // clustered along the contig: refined inside the assembly, a chunk holding
    // hundreds of them held its worker for milliseconds while the others idled
    // (20 Mbp: 4.5k imperfect of 767k, 2.6k recomputes; the pass 3-6 ms, 1.5-2
    // without them).  So the assembly copies and lists them, they are refined
    // as one dynamic task list, and only the chunks holding them are finished
    // after that.
    std::vector<std::vector<int64_t>> imp((size_t)K);
    parallel_items(K, nt, [&](int64_t k, int) {
        const SpecOut &sp = spec[(size_t)k];
        Item *const d0 = out.data() + at[(size_t)k];
        Item *dst = d0;
        const ItemVec &rp = rep[(size_t)k];
        dst = std::copy(rp.begin(), rp.end(), dst);
        if (synced[(size_t)k])
            for (size_t q = from[(size_t)k]; q < sp.emitted.size(); ++q) *dst++ = sp.record(R, q);
        for (Item *it = d0; it < dst; ++it)
            if (it->imperfect()) imp[(size_t)k].push_back(it - out.data());
        if (imp[(size_t)k].empty()) finish_chunk(k);
    });
    std::vector<int64_t> todo;
    for (auto &v : imp) todo.insert(todo.end(), v.begin(), v.end());
    if (!todo.empty()) {
        constexpr int64_t kPer = 8;   // records per task
        parallel_items(((int64_t)todo.size() + kPer - 1) / kPer, nt, [&](int64_t q, int w) {
            const int64_t a = q * kPer, b = std::min<int64_t>((int64_t)todo.size(), a + kPer);
            for (int64_t i = a; i < b; ++i) refine_one(u, pools, w, out[(size_t)todo[(size_t)i]]);
        });
        parallel_items(K, nt, [&](int64_t k, int) {
            if (!imp[(size_t)k].empty()) finish_chunk(k);
        });
    }
    out[at[(size_t)K]] = cur;
    refine_one(u, pools, 0, out[at[(size_t)K]]);
    cm[(size_t)K] = out[at[(size_t)K]].end;   // the last record is chunk K of its own
    bool ordered = true;
    for (int64_t k = 0; k < K; ++k) ordered = ordered && by_start[(size_t)k];
    const size_t N = out.size();
    for (int64_t k = 1; k <= K && ordered; ++k) {   // chunk edges (the last edge precedes `cur`)
        const size_t b = at[(size_t)k];
        if (b == 0 || b >= N) continue;
        if (out[b - 1].start > out[b].start) { ordered = false; break; }
        if (out[b - 1].start < out[b].start || out[b - 1].end <= out[b].end) continue;
        size_t i = b - 1, j = b + 1;   // the equal-start run across the edge
        while (i > 0 && out[i - 1].start == out[b].start) --i;
        while (j < N && out[j].start == out[b].start) ++j;
        std::stable_sort(out.begin() + (std::ptrdiff_t)i, out.begin() + (std::ptrdiff_t)j, by_end);
        // the chunks the run touches share one bound
        size_t k0 = (size_t)k, k1 = (size_t)k;
        while (k0 > 0 && at[k0] > i) --k0;
        while (k1 < (size_t)K && at[k1 + 1] < j) ++k1;
        int64_t m = INT64_MIN;
        for (size_t q = k0; q <= k1; ++q) m = std::max(m, cm[q]);
        for (size_t q = k0; q <= k1; ++q) cm[q] = m;
    }
    if (!ordered) sort_by_pos(out, nt);   // not expected: the general stable sort
    if (oc && ordered) {
        oc->cut.assign(at.begin(), at.end());
        oc->cut.push_back((int64_t)N);
        oc->cmax.assign(cm.begin(), cm.end());
    }
    if (stats_on()) {
        auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "  merge: repair %.1f assemble %.1f ms\n", d(ts1, ts2),
                     d(ts2, std::chrono::steady_clock::now()));
    }
    return out;
}

// bwt.py:3327-3354
bool should_collapse(const UnitCtx &u, const Item &r1, const Item &r2) {
    if (r1.chrom != r2.chrom) return false;
    const int64_t ov = std::min(r1.end, r2.end) - std::max(r1.start, r2.start);
    if (ov <= 0) return false;
    const int64_t sh = std::min(r1.end - r1.start, r2.end - r2.start);
    if (sh <= 0) return false;
    const double f = (double)ov / (double)sh;
    if (f < 0.8) return false;
    {
        Canon c1, c2;
        if (same_canonical(u, r1, c1, r2, c2)) return true;
    }
    if ((r1.mlen == 1 || r2.mlen == 1) && f >= 0.95) return true;
    if (r1.mlen == r2.mlen && f >= 0.9) return std::fabs(mm_of(r1) - mm_of(r2)) >= 0.2;
    return false;
}

// bwt.py:3356-3400 -> true when r1 is preferred
bool prefer_first(const UnitCtx &u, const Item &r1, const Item &r2) {
    const std::string_view m1 = motif_of(u, r1), m2 = motif_of(u, r2);
    const size_t l1 = m1.size(), l2 = m2.size();
    if (l1 != l2) {
        if (l1 == 1 && l2 > 1) return false;
        if (l2 == 1 && l1 > 1) return true;
        const std::string_view sh = l1 < l2 ? m1 : m2, lo = l1 < l2 ? m2 : m1;
        if (lo.size() % sh.size() == 0) {
            bool rep = true;
            for (size_t i = 0; i < lo.size() && rep; ++i) rep = lo[i] == sh[i % sh.size()];
            if (rep) return l1 < l2;
        }
        return l1 > l2;
    }
    if (mm_of(r1) != mm_of(r2)) return mm_of(r1) < mm_of(r2);
    if (conf_of(r1) != conf_of(r2)) return conf_of(r1) > conf_of(r2);
    const int64_t len1 = r1.end - r1.start, len2 = r2.end - r2.start;
    if (len1 != len2) return len1 >= len2;
    return true;
}

// bwt.py:3189-3220.  After the (start, end) sort, equal keys (chrom, start,
// end, motif) sit inside runs of equal (start, end); the first occurrence
// keeps its position and takes the preferred content.
void dedup_sorted(const UnitCtx &u, ItemVec &recs) {
    ItemVec d;
    d.reserve(recs.size());
    size_t i = 0;
    const size_t n = recs.size();
    while (i < n) {
        size_t j = i + 1;
        while (j < n && recs[j].start == recs[i].start && recs[j].end == recs[i].end) ++j;
        const size_t first_out = d.size();
        for (size_t q = i; q < j; ++q) {
            const Item &r = recs[q];
            size_t hit = SIZE_MAX;
            for (size_t x = first_out; x < d.size(); ++x)
                if (d[x].chrom == r.chrom && d[x].mlen == r.mlen && motif_of(u, d[x]) == motif_of(u, r)) {
                    hit = x;
                    break;
                }
            if (hit == SIZE_MAX) { d.push_back(r); continue; }
            const Item &ex = d[hit];
            bool repl = false;
            if (conf_of(r) > conf_of(ex)) repl = true;
            else if (conf_of(r) == conf_of(ex)) {
                if (mm_of(r) < mm_of(ex)) repl = true;
                else if (mm_of(r) == mm_of(ex) && tier_of(r) < tier_of(ex)) repl = true;
            }
            if (repl) d[hit] = r;
        }
        i = j;
    }
    recs.swap(d);
}

// an input record that is not a strict hit (Tier 3): every field carried in an Extra
Item item_of_rec(Pools &pools, const Rec &r) {
    Extra x;
    x.copies = r.copies;
    x.confidence = r.confidence;
    x.mm = r.mismatch_rate;
    x.pmatch = r.pmatch;
    x.pindel = r.pindel;
    x.max_mm = r.max_mm;
    x.n_eval = r.n_eval;
    x.score = r.score;
    x.strand = r.strand;
    x.stats_none = r.stats_none;
    x.tier = r.tier;
    Item it{};
    it.start = r.start;
    it.end = r.end;
    it.chrom = r.chrom;
    it.mlen = (int32_t)r.motif.size();
    it.set_x(pools.add(0, x, r.motif, r.variations));
    return it;
}

// final Rec of an item (after restore): strict fields per bwt.py:1972-1993
void materialize(const UnitCtx &u, const Item &it, int64_t shift, Rec &r) {   // r: a fresh Rec
    const Contig &c = u.job->contigs[(size_t)it.chrom];
    r.chrom = it.chrom;
    r.tier = tier_of(it);
    r.start = it.start + shift;
    r.end = it.end + shift;
    r.length = it.end - it.start;
    if (it.xp) {
        const Extra &x = *it.x();
        r.motif = x.motif;
        r.copies = x.copies;
        r.confidence = x.confidence;
        r.mismatch_rate = x.mm;
        r.max_mm = x.max_mm;
        r.n_eval = x.n_eval;
        r.strand = x.strand;
        r.pmatch = x.pmatch;
        r.pindel = x.pindel;
        r.score = x.score;
        r.variations = x.variations;
        r.stats_none = x.stats_none;
    } else {
        r.motif.assign(c.trimmed() + (it.start - (u.restored ? c.trim_left : 0)), (size_t)it.mlen);
        const int64_t count = strict_copies(it);
        r.copies = (double)count;
        r.confidence = 0.95;
        r.mismatch_rate = 0.0;
        r.max_mm = 0;
        r.n_eval = count;
        r.strand = '+';
        r.pmatch = (1.0 - 0.0) * 100.0;
        r.pindel = 0.0;
        r.score = trf_score(r.length, 0.0);
    }
    // actual_sequence = full_sequence[start:end] after restore (bwt.py:3323-3325)
    if (!c.full.empty()) {
        const int64_t L = (int64_t)c.full.size();
        const int64_t a = std::min(r.start, L), b = std::max(a, std::min(r.end, L));
        r.act_kind = ACT_FULL;
        r.act_off = a;
        r.act_len = b - a;
    }
}

void process_unit(const Job &job, const std::vector<int32_t> &chroms, std::vector<HitVec> &raw,
                  std::vector<ScreenedVec> &shits, RecVec &out, double *ms, int nt) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    UnitCtx u{&job, job.params.min_copies};
    Pools pools(std::max(1, nt));
    // 1. nested suppression per chromosome (bwt.py:3928), concatenated in
    //    chromosome order, stable-sorted by (start, end).
    //    Hits the device already screened (nested.hip) arrive kept, sorted and
    //    deduplicated per chromosome; a one-chromosome unit then skips 1-2.
    ItemVec recs;
    bool presorted = chroms.size() == 1;
    // one device-screened contig (the usual unit): its compact hits become
    // records inside the merge fold's speculative tasks, chunk by chunk
    std::function<void(int64_t, int64_t)> fill_fn;
    if (chroms.size() == 1) {
        const int32_t c = chroms[0];
        const bool scr = (size_t)c < job.screened.size() && job.screened[(size_t)c] && (size_t)c < shits.size();
        const bool mine = job.selected.empty() || ((size_t)c < job.selected.size() && job.selected[(size_t)c]);
        const bool t3 = mine && (size_t)c < job.t3.size() && !job.t3[(size_t)c].empty();
        if (scr && !t3) {
            const ScreenedVec &sh = shits[(size_t)c];
            recs.resize(sh.size());   // NoInit: filled by fill_fn
            fill_fn = [&recs, &sh, c](int64_t a, int64_t b) {
                sh.wait(b);   // the scan's download of these hits may still be landing
                for (int64_t k = a; k < b; ++k) {
                    int64_t s0, len, prim;
                    sh.get(k, s0, len, prim);
                    recs[(size_t)k] = Item{s0, s0 + len, nullptr, c, (int32_t)prim};
                }
            };
        }
    }
    for (int32_t c : chroms) {
        if (fill_fn) break;   // the fused path above
        auto &h = raw[(size_t)c];
        const bool scr = (size_t)c < job.screened.size() && job.screened[(size_t)c];
        presorted = presorted && scr;
        ItemVec items;
        if (scr && (size_t)c < shits.size()) {   // device-screened: compact records
            auto &sh = shits[(size_t)c];
            items.resize(sh.size());
            sh.wait(sh.size());
            parallel_for((int64_t)sh.size(), nt, [&](int64_t a, int64_t b) {
                for (int64_t k = a; k < b; ++k) {
                    int64_t s0, len, prim;
                    sh.get(k, s0, len, prim);
                    items[(size_t)k] = Item{s0, s0 + len, nullptr, c, (int32_t)prim};
                }
            });
            ScreenedVec().swap(sh);
        } else {
            items.resize(h.size());
            parallel_for((int64_t)h.size(), nt, [&](int64_t a, int64_t b) {
                for (int64_t k = a; k < b; ++k) {
                    const bwtmi_hit &x = h[(size_t)k];
                    items[(size_t)k] = Item{x.start, x.end, nullptr, c, x.prim_len};
                }
            });
        }
        HitVec().swap(h);
        // Tier 3 records of this chromosome come after all worker records (bwt.py:3918-3924)
        const bool mine = job.selected.empty() || ((size_t)c < job.selected.size() && job.selected[(size_t)c]);
        if (mine && (size_t)c < job.t3.size() && !job.t3[(size_t)c].empty()) {
            if (scr) fail(BWTMI_E_STATE, "contig %d holds device-screened hits and Tier 3 records", (int)c);
            for (const Rec &r : job.t3[(size_t)c]) items.push_back(item_of_rec(pools, r));
        }
        if (!scr) items = suppress_nested(items, 0.5, nt);
        if (recs.empty()) recs.swap(items);
        else recs.insert(recs.end(), items.begin(), items.end());
    }
    if (!presorted) sort_by_pos(recs, nt);
    auto t1 = clk::now();
    // 2. dedup (bwt.py:3189-3220)
    if (!presorted) dedup_sorted(u, recs);
    auto t2 = clk::now();
    // 3. merge adjacent (bwt.py:3222-3289)
    OutChunks oc;
    {
        BWTMI_STAGE("bwtmi:merge");
        recs = merge_fold(u, pools, recs, nt, &oc, fill_fn ? &fill_fn : nullptr);
    }
    if (fill_fn) {
        ScreenedVec().swap(shits[(size_t)chroms[0]]);
        HitVec().swap(raw[(size_t)chroms[0]]);
    }
    auto t3 = clk::now();
    std::optional<StageRange> rf;
    rf.emplace("bwtmi:refine..filter");
    // 4. refine (bwt.py:3291-3314): done inside merge_fold's assembly
    auto r1 = clk::now();   // merge_fold returns its records in (start, end) order
    auto r2 = clk::now();
    // 5. restore coordinates (bwt.py:3316-3325); actual_sequence is the frame slice.
    //    With one trim offset for the whole unit the (start, end) order is unchanged.
    //    Collapse only compares overlaps, lengths and motifs, all shift-invariant,
    //    so one common offset is added when the records are materialised.
    bool one_offset = true;
    for (int32_t c : chroms) one_offset = one_offset && job.contigs[(size_t)c].trim_left == job.contigs[(size_t)chroms[0]].trim_left;
    const int64_t shift = one_offset && !chroms.empty() ? job.contigs[(size_t)chroms[0]].trim_left : 0;
    if (!one_offset)
        parallel_for((int64_t)recs.size(), nt, [&](int64_t a, int64_t b) {
            for (int64_t k = a; k < b; ++k) {
                Item &r = recs[(size_t)k];
                const int64_t off = job.contigs[(size_t)r.chrom].trim_left;
                r.start += off;
                r.end += off;
            }
        });
    if (!one_offset) u.restored = true;
    // 6. collapse (bwt.py:3499-3513)
    if (!one_offset) sort_by_pos(recs, nt);
    auto r3 = clk::now();
    const size_t n_before_collapse = recs.size();
    clk::time_point t_collapse;
    // collapsed list as indices into recs (the slot takes the preferred record).
    // The fold only ever compares with the last kept record, and a collapse
    // needs an overlap, so an index whose start is >= every earlier end always
    // starts fresh: chunks cut at such indices fold independently.  Each chunk
    // then counts its records that pass the final filter (bwt.py:3940-3944),
    // and every chunk materialises its passing records at its offset.
    const double mc = (double)job.params.min_copies;
    auto pass = [&](uint32_t i) { return copies_of(recs[i]) >= mc && recs[i].end - recs[i].start >= 6; };
    size_t n_collapsed = 0;
    {
        const int64_t N = (int64_t)recs.size();
        // nominal chunks and the largest end in each: the merge fold's output
        // chunks (it tracked their ends while assembling), else one pass here
        std::vector<int64_t> nom, cmax;
        if (one_offset && !oc.cut.empty() && oc.cut.back() == N) {
            nom = std::move(oc.cut);
            cmax = std::move(oc.cmax);
        } else {
            const int C0 = N > 8192 ? 4 * std::max(1, nt) : 1;
            nom.resize((size_t)C0 + 1);
            for (int t = 0; t <= C0; ++t) nom[(size_t)t] = N * t / C0;
            cmax.assign((size_t)C0, INT64_MIN);
            parallel_items(C0, nt, [&](int64_t t, int) {
                int64_t m = INT64_MIN;
                for (int64_t k = nom[(size_t)t]; k < nom[(size_t)t + 1]; ++k) m = std::max(m, recs[(size_t)k].end);
                cmax[(size_t)t] = m;
            });
        }
        const int C = (int)cmax.size();
        std::vector<int64_t> sb((size_t)C + 1, N);
        std::vector<int64_t> pre((size_t)C, INT64_MIN);   // max end before nominal chunk t
        for (int t = 1; t < C; ++t) pre[(size_t)t] = std::max(pre[(size_t)t - 1], cmax[(size_t)t - 1]);
        sb[0] = 0;
        parallel_blocks(C - 1, nt, [&](int64_t q, int) {
            const int64_t t = q + 1;
            int64_t i = nom[(size_t)t], m = pre[(size_t)t];
            while (i < N && recs[(size_t)i].start < m) m = std::max(m, recs[(size_t)i++].end);
            sb[(size_t)t] = i;
        });
        for (int t = 1; t <= C; ++t) sb[(size_t)t] = std::max(sb[(size_t)t], sb[(size_t)t - 1]);
        std::vector<std::vector<uint32_t>> part((size_t)C);
        std::vector<int64_t> cnt((size_t)C + 1, 0);
        parallel_blocks(C, nt, [&](int64_t t, int) {
            auto &pc = part[(size_t)t];
            pc.reserve((size_t)(sb[(size_t)t + 1] - sb[(size_t)t]) + 1);   // nearly every record stays
            int64_t c = 0;   // records passing the final filter, counted as each slot is settled
            for (int64_t k = sb[(size_t)t]; k < sb[(size_t)t + 1]; ++k) {
                if (!pc.empty() && should_collapse(u, recs[pc.back()], recs[(size_t)k])) {
                    if (!prefer_first(u, recs[pc.back()], recs[(size_t)k])) pc.back() = (uint32_t)k;
                } else {
                    if (!pc.empty()) c += pass(pc.back());
                    pc.push_back((uint32_t)k);
                }
            }
            if (!pc.empty()) c += pass(pc.back());
            cnt[(size_t)t + 1] = c;
        });
        for (int t = 0; t < C; ++t) {
            cnt[(size_t)t + 1] += cnt[(size_t)t];
            n_collapsed += part[(size_t)t].size();
        }
        t_collapse = clk::now();
        {
            DeferConstruct raw;   // constructed below, in parallel
            out.resize((size_t)cnt[(size_t)C]);
        }
        // each chunk constructs its slots and materialises them in one pass (the
        // record is still in cache).  Every slot is constructed whatever throws:
        // a chunk whose materialize throws constructs the rest of its slots
        // before it reports, and the chunks after it only construct theirs, so
        // the vector's destructor never meets a raw slot.
        static_assert(std::is_nothrow_default_constructible<Rec>::value, "Rec() must not throw");
        std::atomic<bool> failed{false};
        std::exception_ptr err;
        std::mutex err_mu;
        parallel_blocks(C, nt, [&](int64_t t, int) {
            const int64_t q0 = cnt[(size_t)t], q1 = cnt[(size_t)t + 1];
            int64_t o = q0;   // slots [q0, o) are constructed
            if (!failed.load(std::memory_order_relaxed)) {
                try {
                    const std::vector<uint32_t> &pt = part[(size_t)t];
                    for (size_t j = 0; j < pt.size(); ++j) {
                        if (j + 8 < pt.size()) {   // the record data of a later slot (written by other workers)
                            const Item &ahead = recs[pt[j + 8]];
                            if (ahead.xp) __builtin_prefetch(ahead.x());
                        }
                        const uint32_t i = pt[j];
                        if (pass(i)) {
                            ::new ((void *)&out[(size_t)o]) Rec();
                            ++o;
                            materialize(u, recs[i], shift, out[(size_t)o - 1]);
                        }
                    }
                } catch (...) {
                    failed.store(true, std::memory_order_relaxed);
                    std::lock_guard<std::mutex> lk(err_mu);
                    if (!err) err = std::current_exception();
                }
            }
            for (; o < q1; ++o) ::new ((void *)&out[(size_t)o]) Rec();
        });
        if (err) std::rethrow_exception(err);
    }
    auto t4 = clk::now();
    rf.reset();
    if (stats_on()) {
        auto d = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "  merge %.1f (-> %zu) refine %.1f sort %.1f restore+sort %.1f collapse %.1f (%zu -> %zu) filter+mat %.1f ms\n",
                     d(t2, t3), n_before_collapse, d(t3, r1), d(r1, r2), d(r2, r3), d(r3, t_collapse), n_before_collapse,
                     n_collapsed, d(t_collapse, t4));
    }
    if (ms) {
        ms[0] += std::chrono::duration<double, std::milli>(t1 - t0).count();
        ms[1] += std::chrono::duration<double, std::milli>(t2 - t1).count();
        ms[2] += std::chrono::duration<double, std::milli>(t3 - t2).count();
        ms[3] += std::chrono::duration<double, std::milli>(t4 - t3).count();
    }
}

}  // namespace

void postprocess(Job &job) {
    job.assign_units();
    std::vector<std::vector<int32_t>> units((size_t)job.nunits);
    for (size_t c = 0; c < job.contigs.size(); ++c) units[(size_t)job.contigs[c].unit].push_back((int32_t)c);
    if (job.hits.size() < job.contigs.size()) job.hits.resize(job.contigs.size());
    std::vector<RecVec> res((size_t)job.nunits);
    std::vector<double> ms((size_t)job.nunits * 4, 0.0);
    const int T = host_threads(job.params);
    // many small units: one thread per unit; few large units: all threads inside each
    int64_t busy = 0;
    for (size_t c = 0; c < job.hits.size(); ++c)
        busy += (job.hits[c].empty() && (c >= job.shits.size() || job.shits[c].empty())) ? 0 : 1;
    // a few units and threads to spare: G groups of T / G threads, each its own
    // pool, take units longest first (a unit's parallel regions carry serial
    // parts and joins that one 16-thread region per unit paid unit by unit)
    const int kGroupThreads = (int)std::max<int64_t>(1, knob(KN_UNIT_GROUP_THREADS));
    const int G = (int)std::min<int64_t>(busy, T / kGroupThreads);
    if (busy >= T) {
        parallel_items(job.nunits, T, [&](int64_t k, int) {
            process_unit(job, units[(size_t)k], job.hits, job.shits, res[(size_t)k], &ms[(size_t)k * 4], 1);
        });
    } else if (G >= 2 && job.nunits >= 2) {
        static std::vector<std::unique_ptr<Pool>> groups;   // persistent, like the global pool
        while ((int)groups.size() < G) groups.push_back(std::make_unique<Pool>());
        std::vector<int32_t> order((size_t)job.nunits);
        std::vector<int64_t> work((size_t)job.nunits, 0);
        for (int32_t k = 0; k < job.nunits; ++k) {
            order[(size_t)k] = k;
            for (int32_t ci : units[(size_t)k]) {
                const size_t c = (size_t)ci;
                work[(size_t)k] += (c < job.hits.size() ? (int64_t)job.hits[c].size() : 0) +
                                   (c < job.shits.size() ? (int64_t)job.shits[c].size() : 0);
            }
        }
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return work[(size_t)a] > work[(size_t)b]; });
        std::atomic<int64_t> next{0};
        const int per = T / G;
        parallel_items(G, G, [&](int64_t g, int) {
            Pool *const prev = Pool::tl_pool;
            Pool::tl_pool = groups[(size_t)g].get();
            try {
                for (;;) {
                    const int64_t q = next.fetch_add(1, std::memory_order_relaxed);
                    if (q >= job.nunits) break;
                    const size_t k = (size_t)order[(size_t)q];
                    process_unit(job, units[k], job.hits, job.shits, res[k], &ms[k * 4], per);
                }
            } catch (...) {
                Pool::tl_pool = prev;
                throw;
            }
            Pool::tl_pool = prev;
        });
    } else {
        for (int32_t k = 0; k < job.nunits; ++k) {
            auto a = std::chrono::steady_clock::now();
            process_unit(job, units[(size_t)k], job.hits, job.shits, res[(size_t)k], &ms[(size_t)k * 4], T);
            if (stats_on())
                std::fprintf(stderr, "  unit %d: %.1f ms total\n", k,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count());
        }
    }
    job.final_recs.clear();
    size_t tot = 0, nonempty = 0, last = 0;
    for (size_t k = 0; k < res.size(); ++k)
        if (!res[k].empty()) {
            tot += res[k].size();
            ++nonempty;
            last = k;
        }
    if (nonempty <= 1) {   // one unit with records (one contig, or this rank's only one): no copy
        if (nonempty) job.final_recs.swap(res[last]);
    } else {   // the units' records moved into place in parallel
        std::vector<size_t> at(res.size() + 1, 0);
        for (size_t k = 0; k < res.size(); ++k) at[k + 1] = at[k] + res[k].size();
        {
            DeferConstruct raw;   // move-constructed below, in parallel
            job.final_recs.resize(tot);
        }
        static_assert(std::is_nothrow_move_constructible<Rec>::value, "the parallel moves must not throw");
        run_tasks((int64_t)res.size(), T, [&](int64_t k) {
            Rec *d = job.final_recs.data() + at[(size_t)k];
            for (Rec &r : res[(size_t)k]) ::new ((void *)d++) Rec(std::move(r));
        });
    }
    // the units' emptied vectors are released behind the next stage
    {
        auto old = std::make_shared<std::vector<RecVec>>(std::move(res));
        defer([old] { old->clear(); });
    }
    for (int s = 0; s < 4; ++s) {
        job.stage_ms[2 + s] = 0;
        for (int32_t k = 0; k < job.nunits; ++k) job.stage_ms[2 + s] += ms[(size_t)k * 4 + s];
    }
    if (stats_on(2))
        std::fprintf(stderr, "[bwtmi] recomputes=%lld (%.1f ms thread-summed; %lld reused walks) merges=%lld canons=%lld "
                     "final=%zu\n", (long long)g_recomputes.exchange(0), g_recompute_ns.exchange(0) / 1e6,
                     (long long)g_walk_reuse.exchange(0), (long long)g_merges.exchange(0),
                     (long long)g_canons.exchange(0), job.final_recs.size());
    if (stats_on(2))
        std::fprintf(stderr, "[bwtmi] merge tests past the gap test=%lld, same canonical=%lld\n",
                     (long long)g_tests.exchange(0), (long long)g_same.exchange(0));
    if (stats_on(2))
        std::fprintf(stderr, "[bwtmi] fold steps with a fresh current record=%lld (merged %lld), with a merged one=%lld (merged %lld)\n",
                     (long long)g_fresh_tests.exchange(0), (long long)g_fresh_merges.exchange(0),
                     (long long)g_chain_tests.exchange(0), (long long)g_chain_merges.exchange(0));
    if (stats_on(2))
        for (int a = 0; a < 8; ++a)
            for (int b = 0; b < 8; ++b)
                if (int64_t c = g_hist_n[a][b].exchange(0))
                    std::fprintf(stderr, "  m~4^%d len~4^%d: n=%lld %.1f ms (%.2f us)\n", a, b, (long long)c,
                                 g_hist_ns[a][b].load() / 1e6, g_hist_ns[a][b].exchange(0) / 1e3 / (double)c);
    job.postprocessed = true;
}

}  // namespace bwtmi
