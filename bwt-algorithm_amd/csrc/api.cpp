// api.cpp -- the extern "C" boundary of libbwtmi.so (include/bwtmi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <condition_variable>
#include <cstring>
#include <exception>
#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "device.h"

namespace bwtmi {

static thread_local std::string g_err;

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

void fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    throw Error{code, buf};
}

template <class F>
static int guard(F &&f) {
    try {
        f();
        return BWTMI_OK;
    } catch (const Error &e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::bad_alloc &) {
        g_err = "out of host memory";
        return BWTMI_E_NOMEM;
    } catch (const std::exception &e) {
        g_err = e.what();
        return BWTMI_E_STATE;
    }
}

// device copy of one contig's trimmed sequence, padded for vector loads
struct DevContig {
    DBuf buf;
    int64_t n = -1;
    uint64_t gen = 0;   // Contig::gen of the uploaded content
};

// Host blocks of contig bases (mem.h cached blocks) are registered for DMA the
// first time they are uploaded and stay registered while the block lives
// (cached blocks keep it); the unmap hook drops the registration.
std::mutex g_reg_mu;
std::unordered_map<void *, size_t> g_registered;

void unregister_block(void *p, size_t) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = g_registered.find(p);
    if (it == g_registered.end()) return;
    (void)hipHostUnregister(p);
    g_registered.erase(it);
}

// true when [p, p+n) lies in a registered (pinned) block
bool ensure_pinned(const void *base, const void *p, size_t n) {
    const size_t sz = big_block_size(base);
    if (!sz || (const char *)p + n > (const char *)base + sz) return false;
    static std::once_flag hook;
    std::call_once(hook, [] { big_set_unmap_hook(unregister_block); });
    std::lock_guard<std::mutex> lk(g_reg_mu);
    if (g_registered.count(const_cast<void *>(base))) return true;
    if (hipHostRegister(const_cast<void *>(base), sz, hipHostRegisterDefault) != hipSuccess) {
        (void)hipGetLastError();
        return false;   // pageable copy
    }
    g_registered.emplace(const_cast<void *>(base), sz);
    return true;
}

struct JobDev {
    int device = -1;
    std::vector<DevContig> seqs;
    Ctx *bg_ctx = nullptr;   // context whose background work reads these buffers (cleared by its join)
};

// every entry point that touches a context: join its background work, select the device
static Ctx &use(Ctx &c) {
    ctx_wait(c);
    c.activate();
    return c;
}

// Output file descriptor: closed on every path; when the write fails part-way
// (an exception or a short write) the file is cut to 0 bytes rather than left
// holding a mix of old and new rows.
struct OutFd {
    int fd = -1;
    bool ok = false;
    explicit OutFd(const char *path) : fd(::open(path, O_WRONLY | O_CREAT, 0644)) {
        if (fd < 0) fail(BWTMI_E_IO, "cannot open %s for writing", path);
    }
    ~OutFd() {
        if (fd < 0) return;
        if (!ok) (void)::ftruncate(fd, 0);
        (void)::close(fd);
    }
    // cut to `size` (when whole) and close; false on error
    bool finish(bool whole, size_t size) {
        bool good = !whole || ::ftruncate(fd, (off_t)size) == 0;
        ok = good;
        good = (::close(fd) == 0) && good;
        fd = -1;
        return good;
    }
};

// Buffers [p[k], p[k] + n[k]) written back to back at byte offset `at` of fd,
// IOV_MAX at a time: one writer with large pwritev calls.  Buffered writes to
// one file serialise on its inode lock, so parallel writers only contend: on
// the box host a 55 MB file took 2.8-3.1 ms as one pwrite and 4.3-4.8 ms from
// 16 threads (tools/write_bench.cpp, profiles/r06/write_bench_r06g.txt).
// False on a short write.
static bool pwrite_run(int fd, const char *const *p, const size_t *n, size_t cnt, size_t at) {
    constexpr size_t kIov = 1024;
    iovec v[kIov];
    size_t k = 0, skip = 0;   // next buffer, bytes of it already written
    while (k < cnt) {
        size_t m = 0;
        for (size_t j = k; j < cnt && m < kIov; ++j) {
            const size_t off = j == k ? skip : 0;
            if (n[j] <= off) continue;
            v[m].iov_base = const_cast<char *>(p[j] + off);
            v[m].iov_len = n[j] - off;
            ++m;
        }
        if (m == 0) break;
        const ssize_t w = ::pwritev(fd, v, (int)m, (off_t)at);
        if (w <= 0) return false;
        at += (size_t)w;
        size_t left = (size_t)w;   // advance (k, skip) past the bytes written
        while (k < cnt && left >= n[k] - skip) {
            left -= n[k] - skip;
            skip = 0;
            ++k;
        }
        skip += left;
    }
    return true;
}

// parts[k] lands at byte offset at[k] of `path` (one writer, consecutive parts
// in one pwritev).  `whole`: the parts are the whole file -- it is overwritten
// in place and cut to at.back() bytes afterwards (the content is that of
// open(path, 'w') + write; rewriting a file of the same size reuses its
// page-cache pages).
static void pwrite_parts(const char *path, bool whole, const std::vector<Text> &parts,
                         const std::vector<size_t> &at, int threads) {
    (void)threads;
    OutFd out(path);
    const int fd = out.fd;
    std::vector<const char *> p;
    std::vector<size_t> n;
    bool good = true;
    for (size_t k = 0; k < parts.size() && good;) {   // runs of parts that are consecutive in the file
        size_t j = k, end = at[k];
        p.clear();
        n.clear();
        while (j < parts.size() && at[j] == end) {
            p.push_back(parts[j].data());
            n.push_back(parts[j].size());
            end += parts[j].size();
            ++j;
        }
        good = pwrite_run(fd, p.data(), n.data(), p.size(), at[k]);
        k = j;
    }
    if (!good) fail(BWTMI_E_IO, "short write to %s", path);   // ~OutFd cuts a whole-file write
    if (!out.finish(whole, at.back())) fail(BWTMI_E_IO, "short write to %s", path);
}

// One output file written by its own writer thread while the rows are being
// formatted (bwtmi_job_write, bwtmi_job_write_async).  The formatting tasks
// mark their part done; the writer pwritev's every run of consecutive done
// parts in file order, the header first -- ONE writer, since buffered writes
// to one file serialise on its inode lock (pwrite_run).  The content is that
// of one open(path, 'w') + write: the file is overwritten in place and cut to
// its size at the end (a short write or an error cuts it to 0).
struct FileWrite {
    OutFd out;
    std::string path;
    Rendered R;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint8_t> done;
    size_t next = 0, off = 0;
    bool started = false, rendered = false, aborted = false, header_done = false, bad = false;
    std::thread th;
    explicit FileWrite(const char *p) : out(p), path(p) {}
    ~FileWrite() {
        if (th.joinable()) {
            abort();
            th.join();
        }
    }
    void part_done(size_t k) {   // (render_rows sized R.parts before the first part)
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!started) {
                done.assign(R.parts.size(), 0);
                started = true;
            }
            done[k] = 1;
        }
        cv.notify_one();
    }
    void render_done() {
        {
            std::lock_guard<std::mutex> lk(mu);
            rendered = true;
        }
        cv.notify_one();
    }
    void abort() {
        {
            std::lock_guard<std::mutex> lk(mu);
            rendered = aborted = true;
        }
        cv.notify_one();
    }
    void run() {
        std::unique_lock<std::mutex> lk(mu);
        std::vector<const char *> wp;
        std::vector<size_t> wn;
        auto ready = [&] { return started && next < done.size() && done[next]; };
        for (;;) {
            cv.wait(lk, [&] { return aborted || rendered || (started && !header_done) || ready(); });
            if (aborted) return;
            if (!header_done) {   // the header exists once a part or the whole render is done
                header_done = true;
                const char *hp = R.header.data();
                const size_t hn = R.header.size();
                off = hn;
                lk.unlock();
                if (!pwrite_run(out.fd, &hp, &hn, 1, 0)) bad = true;
                lk.lock();
                continue;
            }
            if (ready()) {
                const size_t at = off;
                wp.clear();
                wn.clear();
                while (ready()) {
                    wp.push_back(R.parts[next].data());
                    wn.push_back(R.parts[next].size());
                    off += R.parts[next].size();
                    ++next;
                }
                lk.unlock();
                if (!pwrite_run(out.fd, wp.data(), wn.data(), wp.size(), at)) bad = true;
                lk.lock();
                continue;
            }
            if (rendered) return;   // every part is done and written
        }
    }
    // wait for the writer, cut the file to its size and close it; false on a short write
    bool finish() {
        if (th.joinable()) th.join();
        return !bad && !aborted && out.finish(true, off);
    }
};

}  // namespace bwtmi

using namespace bwtmi;

struct bwtmi_ctx {
    Ctx c;
};
struct bwtmi_index {
    DeviceIndex *d = nullptr;
    bwtmi_ctx *ctx = nullptr;
};
struct bwtmi_job {
    Job j;
    JobDev dev;
    std::unique_ptr<FileWrite> wr;   // a file still being written (bwtmi_job_write_async)
    std::thread units_wr;            // rendered units still being written (bwtmi_job_write_units_async)
    std::exception_ptr units_err;
};

namespace {
// the job's file write in flight, if any: wait for it and report its error
void write_join(bwtmi_job *job) {
    if (job->units_wr.joinable()) job->units_wr.join();
    if (job->units_err) {
        std::exception_ptr e = job->units_err;
        job->units_err = nullptr;
        std::rethrow_exception(e);
    }
    if (!job->wr) return;
    std::unique_ptr<FileWrite> w = std::move(job->wr);
    if (!w->finish()) fail(BWTMI_E_IO, "short write to %s", w->path.c_str());
}
// format the job's rows into `path`, the writer thread writing behind the
// formatting; returns with the writer still running (job->wr)
void write_start(bwtmi_job *job, int fmt, const char *path) {
    pool_spin_for_job(job->j);
    job->j.text_join();
    auto w = std::make_unique<FileWrite>(path);
    FileWrite *f = w.get();
    f->th = std::thread([f] { f->run(); });
    const std::function<void(size_t)> on_part = [f](size_t k) { f->part_done(k); };
    render_rows(job->j, fmt, nullptr, f->R, &on_part);   // (throws: ~FileWrite stops the writer, cuts the file)
    f->render_done();
    job->wr = std::move(w);
}
}  // namespace

// readers of contig bytes join a deferred host pass first (bwtmi_job_load_fasta_dev)
#define TEXT_JOIN(job) const_cast<bwtmi_job *>(job)->j.text_join()

#define CHECK_ARG(cond, msg)                     \
    do {                                         \
        if (!(cond)) fail(BWTMI_E_ARG, "%s", msg); \
    } while (0)

extern "C" {

const char *bwtmi_last_error(void) { return g_err.c_str(); }
// sha256 of the sources the library was built from (csrc/*.cpp *.h *.hip and
// include/bwtmi.h in path order; generated by the Makefile into build/srchash.c)
extern "C" const char bwtmi_src_sha256[];
const char *bwtmi_source_hash(void) { return bwtmi_src_sha256; }
const char *bwtmi_version(void) {
    static const std::string v = std::string("bwtmi 0.5 (gfx950) src ") + bwtmi_src_sha256;
    return v.c_str();
}
void bwtmi_free(void *p) { std::free(p); }

int bwtmi_device_count(int *count) {
    return guard([&] {
        CHECK_ARG(count, "null count");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *count = (e == hipSuccess) ? n : 0;
    });
}

// Host threads next to the GPU: a process free to run on both sockets of a
// box spread its 16 threads (and their first-touch pages) over both, and the
// W = 8 shard step came out at 8.0 or 9.0 ms from run to run; pinned to either
// node every run took 7.5-8.3 ms (r04x/r04y).  Local rank r drives device
// r mod (visible devices) -- LOCAL_RANK / LOCAL_WORLD_SIZE of the launcher --
// so the ranks sharing this GPU's node are counted from their own GPUs.
static bool bind_host_for(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return false;
    }
    const char *lw_e = std::getenv("LOCAL_WORLD_SIZE");
    const char *lr_e = std::getenv("LOCAL_RANK");
    const int lw = std::max(1, lw_e ? std::atoi(lw_e) : 1);
    int lr = lr_e ? std::atoi(lr_e) : device;
    if (lr < 0 || lr >= lw) lr = 0;
    std::vector<std::string> pci((size_t)lw);
    for (int r = 0; r < lw; ++r) {
        const int d = r == lr ? device : r % ndev;
        char bus[64] = {0};
        if (hipDeviceGetPCIBusId(bus, (int)sizeof bus, d) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        pci[(size_t)r] = bus;
    }
    return bind_host_numa(lr, pci);
}

int bwtmi_open(int device, bwtmi_ctx **out) {
    return guard([&] {
        CHECK_ARG(out, "null out");
        *out = nullptr;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
            fail(BWTMI_E_NODEVICE, "no HIP device available (libbwtmi has no CPU fallback)");
        if (device < 0 || device >= n) fail(BWTMI_E_NODEVICE, "device %d out of range (%d devices)", device, n);
        hipDeviceProp_t prop;
        HIPCHECK(hipGetDeviceProperties(&prop, device));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            fail(BWTMI_E_NODEVICE, "device %d is %s; libbwtmi is built for gfx950 only", device, prop.gcnArchName);
        auto *ctx = new bwtmi_ctx();
        ctx->c.device = device;
        HIPCHECK(hipSetDevice(device));
        // host threads next to the GPU only when asked for (bwtmi_bind_host, or
        // BWTMI_NUMA_BIND=1 here): a library call never changes the caller's
        // affinity on its own
        if (knob(KN_NUMA_BIND)) bind_host_for(device);
        // how a host thread waits for the device: the background index build
        // waits on the device while every host thread post-processes, so a
        // spinning wait would take a core from them -- blocking waits (r02az, C3:
        // 1949 vs 1895 Mbp/s over 3 runs each); the scan's short waits poll
        // (scan_wait)
        if (hipSetDeviceFlags(hipDeviceScheduleBlockingSync) != hipSuccess) (void)hipGetLastError();
        HIPCHECK(hipStreamCreateWithFlags(&ctx->c.stream, hipStreamNonBlocking));
        HIPCHECK(hipEventCreate(&ctx->c.ev0));
        HIPCHECK(hipEventCreate(&ctx->c.ev1));
        *out = ctx;
    });
}

static void ctx_release(Ctx &c) {
    (void)hipStreamSynchronize(c.stream);
    for (auto &l : c.lanes) ctx_release(*l);
    c.lanes.clear();
    if (c.scratch_index) index_free(c.scratch_index);
    c.scratch_index = nullptr;
    for (auto &s : c.slot) s.release();
    c.lb_ticket.release();
    for (auto &h : c.host) h.release();
    c.mbox.release();
    for (hipEvent_t e : c.evpool) (void)hipEventDestroy(e);
    c.evpool.clear();
    (void)hipEventDestroy(c.ev0);
    (void)hipEventDestroy(c.ev1);
    (void)hipStreamDestroy(c.stream);
}

// lane k of c (k >= 1): a context of its own on c's device, created on first use
static Ctx &scan_lane(Ctx &c, size_t k) {
    while (c.lanes.size() < k) {
        auto l = std::make_unique<Ctx>();
        l->device = c.device;
        HIPCHECK(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
        HIPCHECK(hipEventCreate(&l->ev0));
        HIPCHECK(hipEventCreate(&l->ev1));
        c.lanes.push_back(std::move(l));
    }
    Ctx &l = *c.lanes[k - 1];
    l.ktiming = c.ktiming;
    l.kfilter = c.kfilter;
    l.timing = c.timing;
    return l;
}

int bwtmi_bind_host(bwtmi_ctx *ctx, int on, int *changed) {
    return guard([&] {
        CHECK_ARG(ctx, "null argument");
        const bool b = on ? bind_host_for(ctx->c.device) : unbind_host();
        if (changed) *changed = b ? 1 : 0;
    });
}

int bwtmi_host_binding_plan(const char *sysroot, int local_rank, const char *rank_pci, int threads, int smt,
                            const char *allowed, char *out, int64_t cap, int *node, int *ranks_on_node) {
    return guard([&] {
        CHECK_ARG(sysroot && rank_pci && allowed && out && cap > 0, "null argument");
        std::vector<std::string> pci;
        for (const char *p = rank_pci; *p;) {
            const char *e = std::strchr(p, ',');
            pci.emplace_back(p, e ? (size_t)(e - p) : std::strlen(p));
            p = e ? e + 1 : p + std::strlen(p);
        }
        cpu_set_t al, cs;
        if (!parse_cpulist(allowed, al)) fail(BWTMI_E_ARG, "bad cpulist '%s'", allowed);
        int nd = -1, peers = 0;
        const bool b = plan_host_binding(sysroot, local_rank, pci, threads, smt != 0, al, cs, &nd, &peers);
        const std::string str = b ? cpulist_str(cs) : std::string();
        if ((int64_t)str.size() + 1 > cap) fail(BWTMI_E_ARG, "output buffer too small");
        std::memcpy(out, str.c_str(), str.size() + 1);
        if (node) *node = nd;
        if (ranks_on_node) *ranks_on_node = peers;
    });
}

int bwtmi_close(bwtmi_ctx *ctx) {
    return guard([&] {
        if (!ctx) return;
        ctx_join(ctx->c);   // a background error dies with the context
        ctx->c.activate();
        ctx_release(ctx->c);
        delete ctx;
    });
}

int bwtmi_last_timing(bwtmi_ctx *ctx, double *out3) {
    return guard([&] {
        CHECK_ARG(ctx && out3, "null argument");
        ctx_wait(ctx->c);
        out3[0] = ctx->c.last_total_ms;
        out3[1] = ctx->c.last_dom_ms;
        out3[2] = ctx->c.last_dom_launches;
    });
}

int bwtmi_kernel_stats_filter(bwtmi_ctx *ctx, const char *name) {
    return guard([&] {
        CHECK_ARG(ctx, "null ctx");
        ctx_wait(ctx->c);
        ctx->c.kfilter = name ? name : "";
    });
}

int bwtmi_kernel_stats(bwtmi_ctx *ctx, int enable, int reset, char *out, int64_t cap) {
    return guard([&] {
        CHECK_ARG(ctx, "null ctx");
        Ctx &c = ctx->c;
        ctx_wait(c);
        if (!c.pending.empty()) {   // launches of calls that end without resolving their timers
            HIPCHECK(hipStreamSynchronize(c.stream));
            c.kresolve();
        }
        std::string s;
        char line[160];
        for (auto &k : c.kstats) {
            snprintf(line, sizeof line, "%s %.6f %lld %.0f\n", k.first.c_str(), k.second.ms,
                     (long long)k.second.launches, k.second.bytes);
            s += line;
        }
        if (out && cap > 0) {
            const size_t m = std::min<size_t>((size_t)cap - 1, s.size());
            std::memcpy(out, s.data(), m);
            out[m] = 0;
        }
        if (reset) c.kstats.clear();
        c.ktiming = enable != 0;
    });
}

// ------------------------------------------------------------ strict scan
static void upload_text(Ctx &c, DBuf &buf, const uint8_t *seq, int64_t n) {
    buf.ensure((size_t)n + 128);
    HIPCHECK(hipMemsetAsync((uint8_t *)buf.p + n, 0, 128, c.stream));
    if (n) HIPCHECK(hipMemcpyAsync(buf.p, seq, (size_t)n, hipMemcpyHostToDevice, c.stream));
}

int bwtmi_strict_scan(bwtmi_ctx *ctx, const uint8_t *seq, int64_t n, int32_t min_unit, int32_t max_unit,
                      int32_t max_mismatch, int32_t min_copies, bwtmi_hit **hits, int64_t *nhits) {
    return guard([&] {
        CHECK_ARG(ctx && hits && nhits && (seq || n == 0) && n >= 0, "bad argument");
        CHECK_ARG(max_mismatch >= 0, "max_mismatch must be >= 0");
        *hits = nullptr;
        *nhits = 0;
        if (n > 0 && seq[n - 1] == '$') --n;   // bwt.py:1915-1916
        Ctx &c = ctx->c;
        use(c);
        upload_text(c, c.slot[S_TEXT], seq, n);
        ScanResult r;
        if (max_mismatch > 0)   // Hamming-tolerant adjacency (library calls)
            strict_scan_mm_device(c, c.slot[S_TEXT].as<uint8_t>(), n, min_unit, max_unit, max_mismatch, min_copies,
                                  r.hits);
        else
            strict_scan_device(c, c.slot[S_TEXT].as<uint8_t>(), n, min_unit, max_unit, min_copies, r);
        *nhits = (int64_t)r.hits.size();
        auto *out = (bwtmi_hit *)std::malloc(std::max<size_t>(1, r.hits.size()) * sizeof(bwtmi_hit));
        if (!out) fail(BWTMI_E_NOMEM, "malloc");
        if (!r.hits.empty()) std::memcpy(out, r.hits.data(), r.hits.size() * sizeof(bwtmi_hit));
        *hits = out;
    });
}

// ------------------------------------------------------------ index
int bwtmi_index_build(bwtmi_ctx *ctx, const uint8_t *text, int64_t n, int32_t sa_sample, int32_t occ_sample,
                      uint32_t flags, bwtmi_index **out) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:index");
        CHECK_ARG(ctx && out && (text || n == 0) && n >= 0 && sa_sample > 0 && occ_sample > 0, "bad argument");
        *out = nullptr;
        Ctx &c = ctx->c;
        use(c);
        upload_text(c, c.slot[S_TEXT], text, n);
        auto *idx = new bwtmi_index();
        idx->ctx = ctx;
        try {
            idx->d = index_build_device(c, c.slot[S_TEXT].as<uint8_t>(), n, sa_sample, occ_sample, flags);
        } catch (...) {
            delete idx;
            throw;
        }
        *out = idx;
    });
}

int bwtmi_index_free(bwtmi_index *idx) {
    return guard([&] {
        if (!idx) return;
        use(idx->ctx->c);
        index_free(idx->d);
        delete idx;
    });
}

int64_t bwtmi_index_size(const bwtmi_index *idx) { return idx ? index_n(idx->d) : -1; }
int64_t bwtmi_index_occ_len(const bwtmi_index *idx) { return idx ? index_occ_len(idx->d) : -1; }
int64_t bwtmi_index_sampled_len(const bwtmi_index *idx) { return idx ? index_sampled_len(idx->d) : -1; }
int64_t bwtmi_index_kmer_count(const bwtmi_index *idx) { return idx ? index_kmer_count(idx->d) : -1; }

int bwtmi_index_get_sa(const bwtmi_index *idx, int32_t *sa) {
    return guard([&] { CHECK_ARG(idx && sa, "null"); index_get_sa(use(idx->ctx->c), idx->d, sa); });
}
int bwtmi_index_get_bwt(const bwtmi_index *idx, uint8_t *bwt) {
    return guard([&] { CHECK_ARG(idx && bwt, "null"); index_get_bwt(use(idx->ctx->c), idx->d, bwt); });
}
int bwtmi_index_get_counts(const bwtmi_index *idx, int64_t *totals, int64_t *C) {
    return guard([&] { CHECK_ARG(idx && totals && C, "null"); index_get_counts(idx->d, totals, C); });
}
int bwtmi_index_get_occ(const bwtmi_index *idx, uint8_t code, int32_t *cp) {
    return guard([&] { CHECK_ARG(idx && cp, "null"); index_get_occ(use(idx->ctx->c), idx->d, code, cp); });
}
int bwtmi_index_get_sampled(const bwtmi_index *idx, int32_t *vals) {
    return guard([&] { CHECK_ARG(idx && vals, "null"); index_get_sampled(use(idx->ctx->c), idx->d, vals); });
}
int bwtmi_index_get_kmer(const bwtmi_index *idx, int64_t *offsets, int32_t *positions) {
    return guard([&] {
        CHECK_ARG(idx && offsets && positions, "null");
        index_get_kmer(use(idx->ctx->c), idx->d, offsets, positions);
    });
}
int bwtmi_index_lcp(bwtmi_ctx *ctx, bwtmi_index *idx, int32_t *lcp) {
    return guard([&] {
        CHECK_ARG(ctx && idx && lcp, "null");
        use(ctx->c);
        index_lcp(ctx->c, idx->d, lcp);
    });
}
int bwtmi_backward_search_batch(bwtmi_ctx *ctx, bwtmi_index *idx, const uint8_t *pats, const int64_t *off,
                                int64_t npat, int64_t *sp_ep) {
    return guard([&] {
        CHECK_ARG(ctx && idx && off && sp_ep && npat >= 0, "bad argument");
        use(ctx->c);
        index_backward_search(ctx->c, idx->d, pats, off, npat, sp_ep);
    });
}

static LibParams lib_params(const bwtmi_lib_params *p) {
    LibParams q;
    if (p) {
        q.min_period = p->min_period;
        q.max_period = p->max_period;
        q.max_short_motif = p->max_short_motif;
        q.min_copies = p->min_copies;
        q.min_array_length = p->min_array_length;
        q.allow_mismatches = p->allow_mismatches;
        q.min_entropy = p->min_entropy;
    }
    return q;
}

int bwtmi_index_lcp_plateaus(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p, int64_t **out,
                             int64_t *n) {
    return guard([&] {
        CHECK_ARG(ctx && idx && out && n, "null argument");
        *out = nullptr;
        *n = 0;
        use(ctx->c);
        std::vector<int64_t> v;
        lcp_plateaus_device(ctx->c, idx->d, lib_params(p), v);
        auto *o = (int64_t *)std::malloc(std::max<size_t>(1, v.size()) * sizeof(int64_t));
        if (!o) fail(BWTMI_E_NOMEM, "malloc");
        if (!v.empty()) std::memcpy(o, v.data(), v.size() * sizeof(int64_t));
        *out = o;
        *n = (int64_t)(v.size() / 3);
    });
}

int bwtmi_index_short_imperfect(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p, const int64_t *seen,
                                int64_t nseen, bwtmi_job *job, int32_t contig_id) {
    return guard([&] {
        CHECK_ARG(ctx && idx && job && (seen || nseen == 0) && nseen >= 0, "bad argument");
        CHECK_ARG(contig_id >= 0 && contig_id < (int32_t)job->j.contigs.size(), "bad contig id");
        CHECK_ARG((int64_t)job->j.contigs[(size_t)contig_id].full.size() == index_n(idx->d),
                  "the job contig must hold the index text");
        use(ctx->c);
        std::vector<int64_t> sp(seen, seen + 2 * nseen);
        short_imperfect_device(ctx->c, idx->d, lib_params(p), sp, contig_id, job->j.final_recs);
        job->j.postprocessed = true;
    });
}

int bwtmi_index_tier3(bwtmi_ctx *ctx, bwtmi_index *idx, const uint8_t *reads, const int64_t *read_off,
                      int64_t nreads, bwtmi_job *job, int32_t contig_id, int32_t as_input) {
    return guard([&] {
        CHECK_ARG(ctx && idx && job && nreads >= 0 && (read_off || nreads == 0), "bad argument");
        CHECK_ARG(contig_id >= 0 && contig_id < (int32_t)job->j.contigs.size(), "bad contig id");
        if (nreads > 0) {
            CHECK_ARG(read_off[0] == 0 && (reads || read_off[nreads] == 0), "bad read offsets");
            for (int64_t r = 0; r < nreads; ++r) CHECK_ARG(read_off[r + 1] >= read_off[r], "bad read offsets");
        }
        use(ctx->c);
        RecVec recs;
        tier3_device(ctx->c, idx->d, reads, read_off, nreads, contig_id, recs);
        Job &J = job->j;
        if (as_input) {
            if (J.t3.size() < J.contigs.size()) J.t3.resize(J.contigs.size());
            auto &dst = J.t3[(size_t)contig_id];
            for (auto &r : recs) dst.push_back(std::move(r));
        } else {
            for (auto &r : recs) J.final_recs.push_back(std::move(r));
            J.postprocessed = true;
        }
    });
}

int bwtmi_index_long_repeats(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p, const int64_t *seen,
                             int64_t nseen, bwtmi_job *job, int32_t contig_id) {
    return guard([&] {
        CHECK_ARG(ctx && idx && job && (seen || nseen == 0) && nseen >= 0, "bad argument");
        CHECK_ARG(contig_id >= 0 && contig_id < (int32_t)job->j.contigs.size(), "bad contig id");
        CHECK_ARG(p->min_copies >= 0 && p->min_array_length >= 0, "bad parameters");
        use(ctx->c);
        std::vector<int64_t> sp(seen, seen + 2 * nseen);
        simple_scan_device(ctx->c, idx->d, lib_params(p), sp, contig_id, job->j.final_recs);
        job->j.postprocessed = true;
    });
}

int bwtmi_job_tier1(bwtmi_ctx *ctx, bwtmi_job *job, int32_t contig_id, int32_t max_motif_length) {
    return guard([&] {
        CHECK_ARG(ctx && job, "null argument");
        TEXT_JOIN(job);
        CHECK_ARG(contig_id >= 0 && contig_id < (int32_t)job->j.contigs.size(), "bad contig id");
        Ctx &c = ctx->c;
        use(c);
        const Seq &full = job->j.contigs[(size_t)contig_id].full;
        const int64_t n = (int64_t)full.size();
        upload_text(c, c.slot[S_TEXT], (const uint8_t *)full.data(), n);
        tier1_device(c, c.slot[S_TEXT].as<uint8_t>(), (const uint8_t *)full.data(), n, max_motif_length, contig_id,
                     job->j.final_recs);
        job->j.postprocessed = true;
    });
}

// ------------------------------------------------------------ job
int bwtmi_job_create(const bwtmi_params *params, bwtmi_job **out) {
    return guard([&] {
        CHECK_ARG(params && out, "null argument");
        auto *j = new bwtmi_job();
        j->j.params = *params;
        if (j->j.params.sa_sample <= 0) j->j.params.sa_sample = 32;
        *out = j;
    });
}

int bwtmi_job_free(bwtmi_job *job) {
    return guard([&] {
        if (!job) return;
        if (job->j.text_th.joinable()) job->j.text_th.join();   // its error dies with the job
        if (job->wr) (void)job->wr->finish();   // a file still being written is finished (its error dies too)
        if (job->units_wr.joinable()) job->units_wr.join();
        if (job->dev.bg_ctx) ctx_join(*job->dev.bg_ctx);   // its error stays for the ctx's next call
        if (job->dev.device >= 0) (void)hipSetDevice(job->dev.device);
        for (auto &d : job->dev.seqs) d.buf.release();
        delete job;
    });
}

int bwtmi_job_add_contig(bwtmi_job *job, const char *name, const uint8_t *full, int64_t full_len,
                         int64_t trim_left, int64_t trim_right, int32_t *contig_id) {
    return guard([&] {
        CHECK_ARG(job && name && (full || full_len == 0) && full_len >= 0, "bad argument");
        TEXT_JOIN(job);
        CHECK_ARG(trim_left >= 0 && trim_right >= 0 && trim_left + trim_right <= full_len, "bad trim");
        Contig c;
        c.name = name;
        c.full.assign((const char *)full, (size_t)full_len);
        c.trim_left = trim_left;
        c.trim_right = trim_right;
        c.weight = full_len - trim_left - trim_right;
        c.gen = next_contig_gen();
        job->j.contigs.push_back(std::move(c));
        if (contig_id) *contig_id = (int32_t)job->j.contigs.size() - 1;
    });
}

int bwtmi_job_load_fasta(bwtmi_job *job, const char *path, int32_t flank_trim) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(job && path, "null argument");
        TEXT_JOIN(job);
        load_fasta(job->j, path, flank_trim);
        pool_spin_for_job(job->j);
    });
}

// bwtmi_job_load_fasta_dev: the loader's device placement (common.h FastaDev).
// The file image goes up right after the read (pinned, overlapping the host's
// first pass), the plain chunks are rebuilt from it on the device
// (fasta_dev.hip), the host-written pieces follow, and the host pass over the
// plain chunks runs behind all of it (joined by the scan or any reader).
namespace {
struct DevLoad final : FastaDev {
    Ctx &c;
    bwtmi_job *job;
    DevLoad(Ctx &c_, bwtmi_job *j) : c(c_), job(j) {}
    const char *img = nullptr;
    bool preloaded = false;   // the image is the pass-1 part already queued to S_FASTA
    void image(const char *p, int64_t n) override {
        img = p;
        const Job &J = job->j;
        preloaded = J.part_dev_tag != 0 && c.fasta_tag == J.part_dev_tag && p == J.part.data() &&
                    n <= (int64_t)J.part.size();
        if (!preloaded) c.fasta_tag = 0;   // S_FASTA gets other bytes
        if (n <= 0 || preloaded) return;
        ensure_pinned(p, p, (size_t)n);
        c.slot[S_FASTA].ensure((size_t)n + 64);
    }
    void image_part(int64_t off, int64_t n) override {   // from the reading threads
        if (preloaded) return;
        HIPCHECK(hipSetDevice(c.device));
        HIPCHECK(hipMemcpyAsync(c.slot[S_FASTA].as<char>() + off, img + off, (size_t)n, hipMemcpyHostToDevice,
                                c.stream));
    }
    void contigs() override {
        JobDev &d = job->dev;
        const Job &J = job->j;
        if (d.device >= 0 && d.device != c.device) {
            for (auto &s : d.seqs) s.buf.release();
            d.seqs.clear();
        }
        d.device = c.device;
        d.seqs.resize(J.contigs.size());
        for (size_t i = 0; i < J.contigs.size(); ++i) {
            const Contig &ct = J.contigs[i];
            DevContig &dc = d.seqs[i];
            if (!J.selected.empty() && (i >= J.selected.size() || !J.selected[i])) continue;   // another rank's contig
            const int64_t tn = ct.trimmed_len();
            if (dc.n == tn && dc.gen == ct.gen) continue;   // on the device already (not in this file)
            if (!ct.full.empty()) ensure_pinned(ct.full.data(), ct.full.data(), ct.full.size());
            dc.buf.ensure((size_t)tn + 128);
            HIPCHECK(hipMemsetAsync(dc.buf.as<uint8_t>() + tn, 0, 128, c.stream));
            dc.n = tn;
            dc.gen = ct.gen;
        }
    }
    void plain(const std::vector<FastaPiece> &ps) override {
        std::vector<FastaDevPiece> v;
        v.reserve(ps.size());
        for (const FastaPiece &p : ps) {
            const Contig &ct = job->j.contigs[(size_t)p.cid];
            v.push_back(FastaDevPiece{p.a, p.b, p.off, ct.trim_left, ct.trimmed_len(),
                                      job->dev.seqs[(size_t)p.cid].buf.as<char>()});
        }
        fasta_build_device(c, c.slot[S_FASTA].as<uint8_t>(), v.data(), (int64_t)v.size());
    }
    void piece(int32_t cid, int64_t off, const char *host, int64_t n) override {
        const Contig &ct = job->j.contigs[(size_t)cid];
        const int64_t tl = ct.trim_left, tn = ct.trimmed_len();
        const int64_t lo = std::max(off, tl), hi = std::min(off + n, tl + tn);
        if (hi <= lo) return;
        HIPCHECK(hipMemcpyAsync(job->dev.seqs[(size_t)cid].buf.as<char>() + (lo - tl), host + (lo - off),
                                (size_t)(hi - lo), hipMemcpyHostToDevice, c.stream));
    }
    void defer(std::function<void()> fn, std::shared_ptr<void> hold) override {
        hipEvent_t ev;   // every copy out of `hold` (the image) is queued before it
        HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(ev, c.stream));
        const int dev = c.device;
        job->j.text_defer([fn = std::move(fn), hold = std::move(hold), ev, dev]() mutable {
            struct Done {   // also when fn throws: the image outlives its copy
                hipEvent_t ev;
                int dev;
                std::shared_ptr<void> &hold;
                ~Done() {
                    (void)hipSetDevice(dev);
                    (void)hipEventSynchronize(ev);
                    (void)hipEventDestroy(ev);
                    hold.reset();
                }
            } done{ev, dev, hold};
            fn();
        });
    }
};
}  // namespace

int bwtmi_job_load_fasta_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t flank_trim) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(ctx && job && path, "null argument");
        Ctx &c = ctx->c;
        job->j.text_join();
        if (job->dev.bg_ctx && job->dev.bg_ctx != &c) ctx_wait(*job->dev.bg_ctx);   // it reads the old buffers
        use(c);
        device_wake(c);
        DevLoad dl(c, job);
        load_fasta(job->j, path, flank_trim, 1, 0, &dl);
        pool_spin_for_job(job->j);
    });
}

int bwtmi_job_device_text(bwtmi_ctx *ctx, bwtmi_job *job, int32_t id, uint8_t *dst) {
    return guard([&] {
        CHECK_ARG(ctx && job && dst && id >= 0 && id < (int32_t)job->j.contigs.size(), "bad argument");
        Ctx &c = use(ctx->c);
        const JobDev &d = job->dev;
        CHECK_ARG(d.device == c.device && (size_t)id < d.seqs.size() && d.seqs[(size_t)id].n >= 0 &&
                      d.seqs[(size_t)id].gen == job->j.contigs[(size_t)id].gen,
                  "contig not resident on this device");
        const DevContig &dc = d.seqs[(size_t)id];
        if (dc.n) HIPCHECK(hipMemcpyAsync(dst, dc.buf.p, (size_t)dc.n, hipMemcpyDeviceToHost, c.stream));
        HIPCHECK(hipStreamSynchronize(c.stream));
    });
}

int bwtmi_job_load_fasta_shard(bwtmi_job *job, const char *path, int32_t flank_trim, int32_t world, int32_t rank) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(job && path && world >= 1 && rank >= 0 && rank < world, "bad argument");
        TEXT_JOIN(job);
        load_fasta(job->j, path, flank_trim, world, rank);
        pool_spin_for_job(job->j);
    });
}

int bwtmi_job_fasta_scan_part(bwtmi_job *job, const char *path, int32_t world, int32_t rank, int64_t **blob,
                              int64_t *nwords) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(job && path && blob && nwords && world >= 1 && rank >= 0 && rank < world, "bad argument");
        TEXT_JOIN(job);
        std::vector<int64_t> v;
        fasta_scan_part(job->j, path, world, rank, v);
        auto *o = (int64_t *)std::malloc(std::max<size_t>(1, v.size()) * sizeof(int64_t));
        if (!o) fail(BWTMI_E_NOMEM, "malloc");
        std::memcpy(o, v.data(), v.size() * sizeof(int64_t));
        *blob = o;
        *nwords = (int64_t)v.size();
    });
}

// pass 1 as above, and the part's bytes queued to ctx's FASTA image slot right
// away: when this rank's contigs lie inside its part (equal contigs, one per
// rank), pass 2 (bwtmi_job_load_fasta_parts_dev on the same ctx) finds its
// image on the device and the copy has overlapped the part-table exchange
int bwtmi_job_fasta_scan_part_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t world, int32_t rank,
                                  int64_t **blob, int64_t *nwords) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(ctx && job && path && blob && nwords && world >= 1 && rank >= 0 && rank < world, "bad argument");
        TEXT_JOIN(job);
        Ctx &c = ctx->c;
        if (job->dev.bg_ctx && job->dev.bg_ctx != &c) ctx_wait(*job->dev.bg_ctx);
        use(c);
        // the previous part's copy (if any, on whichever context) has left
        // job->j.part before pass 1 overwrites it (fasta_scan_part settles it)
        std::vector<int64_t> v;
        fasta_scan_part(job->j, path, world, rank, v);
        const Seq &part = job->j.part;
        if (!part.empty()) {
            static std::atomic<uint64_t> tags{0};
            const uint64_t tag = ++tags;
            ensure_pinned(part.data(), part.data(), part.size());
            c.slot[S_FASTA].ensure(part.size() + 64);
            HIPCHECK(hipMemcpyAsync(c.slot[S_FASTA].p, part.data(), part.size(), hipMemcpyHostToDevice, c.stream));
            hipEvent_t ev;
            HIPCHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            HIPCHECK(hipEventRecord(ev, c.stream));
            job->j.part_inflight = [ev] {   // an event wait needs no current device
                (void)hipEventSynchronize(ev);
                (void)hipEventDestroy(ev);
            };
            c.fasta_tag = tag;
            job->j.part_dev_tag = tag;
        }
        auto *o = (int64_t *)std::malloc(std::max<size_t>(1, v.size()) * sizeof(int64_t));
        if (!o) fail(BWTMI_E_NOMEM, "malloc");
        std::memcpy(o, v.data(), v.size() * sizeof(int64_t));
        *blob = o;
        *nwords = (int64_t)v.size();
    });
}

int64_t bwtmi_fasta_count_records(const char *path, int64_t limit) {
    if (!path || limit < 0) return -1;
    try {
        return fasta_count_records(path, limit);
    } catch (...) {
        return -1;
    }
}

int bwtmi_job_load_fasta_parts_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t flank_trim,
                                   int32_t world, int32_t rank, const int64_t *blob, int64_t nwords) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(ctx && job && path && blob && nwords >= 6 && world >= 1 && rank >= 0 && rank < world,
                  "bad argument");
        Ctx &c = ctx->c;
        job->j.text_join();
        if (job->dev.bg_ctx && job->dev.bg_ctx != &c) ctx_wait(*job->dev.bg_ctx);
        use(c);
        device_wake(c);
        DevLoad dl(c, job);
        fasta_load_parts(job->j, path, flank_trim, world, rank, blob, nwords, &dl);
        pool_spin_for_job(job->j);
    });
}

int bwtmi_job_load_fasta_parts(bwtmi_job *job, const char *path, int32_t flank_trim, int32_t world, int32_t rank,
                               const int64_t *blob, int64_t nwords) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:load");
        CHECK_ARG(job && path && blob && nwords >= 6 && world >= 1 && rank >= 0 && rank < world, "bad argument");
        TEXT_JOIN(job);
        fasta_load_parts(job->j, path, flank_trim, world, rank, blob, nwords);
        pool_spin_for_job(job->j);
    });
}

int bwtmi_job_select_shard(bwtmi_job *job, int32_t world, int32_t rank, int32_t *ids, int32_t *n) {
    return guard([&] {
        CHECK_ARG(job && world >= 1 && rank >= 0 && rank < world, "bad argument");
        TEXT_JOIN(job);
        std::vector<int32_t> v = shard_units(job->j, world, rank);
        Job &J = job->j;
        J.selected.assign(J.contigs.size(), 0);
        for (int32_t c : v) J.selected[(size_t)c] = 1;
        if (n) *n = (int32_t)v.size();
        if (ids) std::copy(v.begin(), v.end(), ids);
    });
}

int bwtmi_host_info(int32_t *cpus_visible, int32_t *local_world, int32_t *threads) {
    return guard([&] {
        int v = 0, lw = 0;
        const int t = host_cpu_budget(&v, &lw);
        if (cpus_visible) *cpus_visible = v;
        if (local_world) *local_world = lw;
        if (threads) *threads = t;
    });
}

int32_t bwtmi_job_contig_count(const bwtmi_job *job) { return job ? (int32_t)job->j.contigs.size() : -1; }

int64_t bwtmi_job_contig_weight(const bwtmi_job *job, int32_t id) {
    if (!job || id < 0 || id >= (int32_t)job->j.contigs.size()) return -1;
    return job->j.contigs[(size_t)id].weight;
}

int64_t bwtmi_job_contig_info(const bwtmi_job *job, int32_t id, char *name, int64_t cap, int64_t *full_len,
                              int64_t *trim_left, int64_t *trim_right) {
    if (!job || id < 0 || id >= (int32_t)job->j.contigs.size()) return -1;
    const Contig &c = job->j.contigs[(size_t)id];
    if (name && cap > 0) {
        const size_t k = std::min<size_t>((size_t)cap - 1, c.name.size());
        std::memcpy(name, c.name.data(), k);
        name[k] = 0;
    }
    if (full_len) *full_len = (int64_t)c.full.size();
    if (trim_left) *trim_left = c.trim_left;
    if (trim_right) *trim_right = c.trim_right;
    return (int64_t)c.name.size();
}

int bwtmi_job_contig_seq(const bwtmi_job *job, int32_t id, uint8_t *dst) {
    return guard([&] {
        CHECK_ARG(job && dst && id >= 0 && id < (int32_t)job->j.contigs.size(), "bad argument");
        TEXT_JOIN(job);
        const Contig &c = job->j.contigs[(size_t)id];
        std::memcpy(dst, c.full.data(), c.full.size());
    });
}

static void job_upload(bwtmi_ctx *ctx, bwtmi_job *job) {
    Ctx &c = ctx->c;
    if (job->dev.bg_ctx && job->dev.bg_ctx != &c) ctx_wait(*job->dev.bg_ctx);
    use(c);
    JobDev &d = job->dev;
    if (d.device >= 0 && d.device != c.device) {
        for (auto &s : d.seqs) s.buf.release();
        d.seqs.clear();
    }
    d.device = c.device;
    d.seqs.resize(job->j.contigs.size());
    for (size_t i = 0; i < job->j.contigs.size(); ++i) {
        const Contig &ct = job->j.contigs[i];
        DevContig &dc = d.seqs[i];
        if (!job->j.selected.empty() && !job->j.selected[i]) continue;   // another rank's shard
        if (dc.n == ct.trimmed_len() && dc.gen == ct.gen) continue;
        job->j.text_join();   // host bytes are read below
        ensure_pinned(ct.full.data(), ct.trimmed(), (size_t)ct.trimmed_len());
        upload_text(c, dc.buf, (const uint8_t *)ct.trimmed(), ct.trimmed_len());
        dc.n = ct.trimmed_len();
        dc.gen = ct.gen;
    }
    HIPCHECK(hipStreamSynchronize(c.stream));
}

int bwtmi_job_upload(bwtmi_ctx *ctx, bwtmi_job *job) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:upload");
        CHECK_ARG(ctx && job, "null argument");
        job_upload(ctx, job);
    });
}

int bwtmi_job_reset(bwtmi_job *job) {
    return guard([&] {
        CHECK_ARG(job, "null argument");
        job->j.hits.clear();
        job->j.screened.clear();
        job->j.shits.clear();
        job->j.raw_n.clear();
        {   // the last records are released on the background reaper thread,
            // behind the next step's device phase
            auto old = std::make_shared<RecVec>();
            old->swap(job->j.final_recs);
            defer([old] { RecVec().swap(*old); });
        }
        job->j.t3.clear();
        job->j.postprocessed = false;
    });
}

int bwtmi_job_set_params(bwtmi_job *job, const bwtmi_params *params) {
    return guard([&] {
        CHECK_ARG(job && params, "null argument");
        job->j.params = *params;
        if (job->j.params.sa_sample <= 0) job->j.params.sa_sample = 32;
    });
}

int bwtmi_job_select(bwtmi_job *job, const int32_t *ids, int32_t n) {
    return guard([&] {
        CHECK_ARG(job && (ids || n <= 0), "bad argument");
        Job &J = job->j;
        J.selected.clear();
        if (n < 0) return;
        J.selected.assign(J.contigs.size(), 0);
        for (int32_t k = 0; k < n; ++k) {
            CHECK_ARG(ids[k] >= 0 && ids[k] < (int32_t)J.contigs.size(), "bad contig id");
            J.selected[(size_t)ids[k]] = 1;
        }
    });
}

int bwtmi_job_scan(bwtmi_ctx *ctx, bwtmi_job *job) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:scan");
        CHECK_ARG(ctx && job, "null argument");
        pool_spin_for_job(job->j);
        auto t0 = std::chrono::steady_clock::now();
        job_upload(ctx, job);
        Job &J = job->j;
        Ctx &c = ctx->c;
        J.hits.assign(J.contigs.size(), {});
        J.screened.assign(J.contigs.size(), 0);
        J.shits.assign(J.contigs.size(), {});
        J.raw_n.assign(J.contigs.size(), 0);
        J.errors.assign(J.contigs.size(), std::string());
        const char *fail_contig = std::getenv("BWTMI_FAIL_CONTIG");   // test hook: this contig's worker fails
        const char *fail_kind = std::getenv("BWTMI_FAIL_KIND");       // "hip": as a device fault
        // nested suppression + sort + dedup on the device (BWTMI_HOST_SCREEN=1: on the host)
        const bool screen = knob(KN_HOST_SCREEN) == 0;
        J.final_recs.clear();
        J.postprocessed = false;
        const bwtmi_params &P = J.params;
        std::vector<std::pair<const uint8_t *, int64_t>> to_index;
        std::vector<size_t> todo;   // contigs to scan
        for (size_t i = 0; i < J.contigs.size(); ++i) {
            const Contig &ct = J.contigs[i];
            const int64_t len = ct.trimmed_len();
            if (!J.selected.empty() && !J.selected[i]) continue;   // another rank's shard
            if (P.build_index) to_index.push_back({job->dev.seqs[i].buf.as<uint8_t>(), len});
            if (!P.tier2) continue;                                  // bwt.py:3068
            if (len > 50000000 && !P.show_progress) continue;        // bwt.py:3070
            if (P.min_copies <= 0) continue;                         // worker raises -> [] (bwt.py:3137)
            todo.push_back(i);
        }
        // the screen drops hits only the final filter would see (nested.hip) for a
        // contig that is a fold unit of its own: in a unit of several contigs the
        // records interleave by position, and another contig's record between two
        // breaks their merge chain (bwt.py:3222-3289)
        J.assign_units();
        std::vector<int32_t> unit_size((size_t)std::max<int32_t>(1, J.nunits), 0);
        for (const Contig &ct : J.contigs) ++unit_size[(size_t)ct.unit];
        auto scan_one = [&](Ctx &lc, size_t i) {
            const Contig &ct = J.contigs[i];
            const int64_t len = ct.trimmed_len();
            const int64_t U = std::max<int64_t>(P.max_unit_len, std::min<int64_t>(len / P.min_copies, 1000));
            // a contig with Tier 3 records is screened on the host, together with them
            const bool t3 = i < J.t3.size() && !J.t3[i].empty();
            ScanResult r;
            // a failing contig yields no records and an error message, the others go on
            // (the worker's `except Exception: print(...); return []`, bwt.py:3137-3141)
            // A device fault (BWTMI_E_HIP: a failed launch, copy or synchronisation) is
            // not contig-local -- the lanes share one device, and a sticky fault fails
            // every later contig -- and the reference has no such failure: the scan
            // stops and the call returns the error, so the run fails instead of
            // writing a partial repeat.tab.
            try {
                if (fail_contig && ct.name == fail_contig)
                    fail(fail_kind && !std::strcmp(fail_kind, "hip") ? BWTMI_E_HIP : BWTMI_E_STATE,
                         "injected failure (BWTMI_FAIL_CONTIG)");
                strict_scan_device(lc, job->dev.seqs[i].buf.as<uint8_t>(), len, 1,
                                   (int32_t)std::min<int64_t>(U, INT32_MAX), P.min_copies, r,
                                   screen && !t3 && len < (int64_t)UINT32_MAX,   // 32-bit hit lengths
                                   unit_size[(size_t)ct.unit] == 1 ? P.min_copies : 0);
            } catch (const Error &e) {
                if (e.code == BWTMI_E_HIP) throw;
                J.errors[i] = e.msg;
                (void)hipGetLastError();
                (void)hipStreamSynchronize(lc.stream);
                return;
            } catch (const std::bad_alloc &) {
                J.errors[i] = "out of host memory";
                return;
            }
            J.hits[i].swap(r.hits);   // Rule 1 (bwt.py:3118-3130) never fires on strict hits
            J.shits[i].swap(r.shits);
            J.screened[i] = r.screened ? 1 : 0;
            J.raw_n[i] = r.raw;
        };
        // several contigs: up to kLanes scans in flight, each lane a context with
        // its own stream and scratch driven by its own host thread (a contig's
        // scan is a chain of small dependent launches and host reads, so one
        // stream leaves the device idle between them); contigs go to lanes
        // longest first, each to the least loaded lane
        const int kLanes = (int)std::max<int64_t>(1, std::min<int64_t>(8, knob(KN_SCAN_LANES)));
        const size_t nl = std::min<size_t>((size_t)kLanes, todo.size());
        if (nl <= 1) {
            for (size_t i : todo) scan_one(c, i);
        } else {
            std::vector<size_t> ord(todo);
            std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) {
                return J.contigs[x].trimmed_len() > J.contigs[y].trimmed_len();
            });
            std::vector<std::vector<size_t>> part(nl);
            std::vector<int64_t> load(nl, 0);
            for (size_t i : ord) {
                const size_t k = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
                part[k].push_back(i);
                load[k] += J.contigs[i].trimmed_len();
            }
            std::vector<Ctx *> lc(nl);
            lc[0] = &c;
            for (size_t k = 1; k < nl; ++k) lc[k] = &scan_lane(c, k);
            std::vector<std::exception_ptr> ex(nl);
            std::vector<std::thread> th;
            for (size_t k = 1; k < nl; ++k)
                th.emplace_back([&, k] {
                    try {
                        lc[k]->activate();
                        for (size_t i : part[k]) scan_one(*lc[k], i);
                    } catch (...) {
                        ex[k] = std::current_exception();
                    }
                });
            try {
                for (size_t i : part[0]) scan_one(c, i);
            } catch (...) {
                ex[0] = std::current_exception();
            }
            for (auto &t : th) t.join();
            for (size_t k = 1; k < nl; ++k) c.absorb_kstats(*lc[k]);
            for (auto &e : ex)
                if (e) std::rethrow_exception(e);
        }
        J.text_join();   // the host copies written behind this scan (bwtmi_job_load_fasta_dev)
        J.stage_ms[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        J.stage_ms[1] = 0;
        if (to_index.empty()) return;
        // BWTCore(seq + '$') of the worker (bwt.py:3053-3054). The worker never consumes
        // it, so the builds run on a background thread behind the host
        // post-processing; every later use of this ctx (or of this job's device
        // buffers) joins them first. The scratch index keeps its buffers between builds.
        const int32_t sa_sample = P.sa_sample;
        c.bg_ms = 0;
        job->dev.bg_ctx = &c;
        c.bg_link = &job->dev.bg_ctx;
        c.bg = std::thread([&c, sa_sample, to_index] {
            BWTMI_STAGE("bwtmi:index");
            auto ti = std::chrono::steady_clock::now();
            try {
                c.activate();
                // one build on context x (its own stream, slots and scratch index)
                auto build = [sa_sample](Ctx &x, const std::pair<const uint8_t *, int64_t> &tx) {
                    const int64_t len = tx.second;
                    // (S_CAND_K2 is free after the scan; index_build_device uses the MISC/IDX slots)
                    DBuf &tb = x.slot[S_CAND_K2];
                    tb.ensure((size_t)len + 1 + 128);
                    HIPCHECK(hipMemcpyAsync(tb.p, tx.first, (size_t)len, hipMemcpyDeviceToDevice, x.stream));
                    HIPCHECK(hipMemsetAsync(tb.as<uint8_t>() + len, '$', 1, x.stream));
                    HIPCHECK(hipMemsetAsync(tb.as<uint8_t>() + len + 1, 0, 127, x.stream));
                    x.scratch_index = index_build_device(x, tb.as<uint8_t>(), len + 1, sa_sample, 128, 0u,
                                                         x.scratch_index);
                };
                // several contigs: the builds go to the scan lanes (longest first, each
                // to the least loaded lane), each lane's builds on its own stream and
                // host thread -- a 12.5 Mbp build is a chain of small launches and host
                // reads that leaves the device mostly idle, and eight of them in a row
                // outlasted the host stages of the 8-contig step (C4: 35 ms, r04final)
                const int kIndexLanes = (int)std::max<int64_t>(1, std::min<int64_t>(8, knob(KN_INDEX_LANES)));
                const size_t nl = std::min<size_t>((size_t)kIndexLanes, to_index.size());
                if (nl <= 1) {
                    for (const auto &tx : to_index) build(c, tx);
                    HIPCHECK(hipStreamSynchronize(c.stream));
                } else {
                    std::vector<size_t> ord(to_index.size());
                    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
                    std::stable_sort(ord.begin(), ord.end(),
                                     [&](size_t x, size_t y) { return to_index[x].second > to_index[y].second; });
                    std::vector<std::vector<size_t>> part(nl);
                    std::vector<int64_t> load(nl, 0);
                    for (size_t i : ord) {
                        const size_t k = (size_t)(std::min_element(load.begin(), load.end()) - load.begin());
                        part[k].push_back(i);
                        load[k] += to_index[i].second;
                    }
                    std::vector<Ctx *> lc(nl);
                    lc[0] = &c;
                    for (size_t k = 1; k < nl; ++k) lc[k] = &scan_lane(c, k);
                    std::vector<std::exception_ptr> ex(nl);
                    auto run = [&](size_t k) {
                        try {
                            if (k) lc[k]->activate();
                            for (size_t i : part[k]) build(*lc[k], to_index[i]);
                            HIPCHECK(hipStreamSynchronize(lc[k]->stream));
                        } catch (...) {
                            ex[k] = std::current_exception();
                        }
                    };
                    std::vector<std::thread> th;
                    for (size_t k = 1; k < nl; ++k) th.emplace_back(run, k);
                    run(0);
                    for (auto &t : th) t.join();
                    for (size_t k = 1; k < nl; ++k) c.absorb_kstats(*lc[k]);
                    for (auto &e : ex)
                        if (e) std::rethrow_exception(e);
                }
            } catch (const Error &e) {
                c.bg_code = e.code;
                c.bg_err = "background index build: " + e.msg;
            } catch (const std::bad_alloc &) {
                c.bg_code = BWTMI_E_NOMEM;
                c.bg_err = "background index build: out of host memory";
            } catch (const std::exception &e) {
                c.bg_code = BWTMI_E_STATE;
                c.bg_err = std::string("background index build: ") + e.what();
            }
            c.bg_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ti).count();
        });
    });
}

int bwtmi_job_wait(bwtmi_ctx *ctx, bwtmi_job *job) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:index_wait");
        CHECK_ARG(ctx && job, "null argument");
        const bool ran = ctx->c.bg.joinable();
        ctx_wait(ctx->c);
        if (ran) job->j.stage_ms[1] = ctx->c.bg_ms;
    });
}

int bwtmi_job_add_hits(bwtmi_job *job, int32_t contig_id, const bwtmi_hit *hits, int64_t n) {
    return guard([&] {
        CHECK_ARG(job && (hits || n == 0) && n >= 0, "bad argument");
        TEXT_JOIN(job);
        Job &J = job->j;
        CHECK_ARG(contig_id >= 0 && contig_id < (int32_t)J.contigs.size(), "bad contig id");
        if (J.hits.size() < J.contigs.size()) J.hits.resize(J.contigs.size());
        if (J.screened.size() < J.contigs.size()) J.screened.resize(J.contigs.size(), 0);
        if (J.raw_n.size() < J.contigs.size()) J.raw_n.resize(J.contigs.size(), 0);
        CHECK_ARG(!J.screened[(size_t)contig_id] || n == 0,
                  "contig holds device-screened hits; reset the job before adding raw hits");
        J.hits[(size_t)contig_id].insert(J.hits[(size_t)contig_id].end(), hits, hits + n);
        J.raw_n[(size_t)contig_id] += n;
    });
}

int64_t bwtmi_job_raw_count(const bwtmi_job *job) {
    if (!job) return -1;
    int64_t n = 0;
    for (auto v : job->j.raw_n) n += v;
    return n;
}

int bwtmi_job_postprocess(bwtmi_job *job) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:postprocess");
        CHECK_ARG(job, "null argument");
        pool_spin_for_job(job->j);
        TEXT_JOIN(job);
        Job &J = job->j;
        postprocess(J);
    });
}

int64_t bwtmi_job_count(const bwtmi_job *job) { return job ? (int64_t)job->j.final_recs.size() : -1; }

int bwtmi_job_render(bwtmi_job *job, int fmt, char **out, int64_t *len) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && out && len, "null argument");
        pool_spin_for_job(job->j);
        TEXT_JOIN(job);
        const std::vector<Text> parts = render_parts(job->j, fmt);
        std::vector<size_t> at(parts.size() + 1, 0);
        for (size_t k = 0; k < parts.size(); ++k) at[k + 1] = at[k] + parts[k].size();
        const size_t tot = at.back();
        char *p = (char *)std::malloc(tot + 1);
        if (!p) fail(BWTMI_E_NOMEM, "malloc");
        run_tasks((int64_t)parts.size(), host_threads(job->j.params), [&](int64_t k) {
            std::memcpy(p + at[(size_t)k], parts[(size_t)k].data(), parts[(size_t)k].size());
        });
        p[tot] = 0;
        *out = p;
        *len = (int64_t)tot;
    });
}

// The file is written while it is being formatted (FileWrite): a part whose
// predecessors are all formatted has a known offset, and the writer thread
// writes each run of such parts as it completes.
int bwtmi_job_write(bwtmi_job *job, int fmt, const char *path) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && path, "null argument");
        write_join(job);
        write_start(job, fmt, path);
        write_join(job);
    });
}

// The same, returning once every row is formatted: the writer finishes the
// file behind the caller.  bwtmi_job_write_join waits for it and returns its
// error; every later write of the job, and bwtmi_job_free, joins it first.
int bwtmi_job_write_async(bwtmi_job *job, int fmt, const char *path) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && path, "null argument");
        write_join(job);
        write_start(job, fmt, path);
    });
}

int bwtmi_job_write_join(bwtmi_job *job) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write_join");
        CHECK_ARG(job, "null argument");
        write_join(job);
    });
}

int32_t bwtmi_job_unit_count(bwtmi_job *job) {
    if (!job) return -1;
    job->j.assign_units();
    return job->j.nunits;
}

int bwtmi_job_unit_rows(bwtmi_job *job, int64_t *unit_rows) {
    return guard([&] {
        CHECK_ARG(job && unit_rows, "null argument");
        TEXT_JOIN(job);
        Job &J = job->j;
        J.assign_units();
        for (int32_t u = 0; u < J.nunits; ++u) unit_rows[u] = 0;
        for (const Rec &r : J.final_recs) ++unit_rows[J.contigs[(size_t)r.chrom].unit];
    });
}

int bwtmi_job_render_units(bwtmi_job *job, int fmt, const int64_t *row_base, int64_t *bytes) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && bytes, "null argument");
        pool_spin_for_job(job->j);
        TEXT_JOIN(job);
        Job &J = job->j;
        render_rows(J, fmt, row_base, J.rendered);
        for (int32_t u = 0; u <= J.nunits; ++u) bytes[u] = 0;
        bytes[0] = (int64_t)J.rendered.header.size();
        for (size_t k = 0; k < J.rendered.parts.size(); ++k)
            bytes[1 + J.rendered.part_unit[k]] += (int64_t)J.rendered.parts[k].size();
    });
}

namespace {
// the rendered units (bwtmi_job_render_units) as parts at their file offsets;
// the job's rendering is handed over to them
void units_parts(bwtmi_job *job, const int64_t *offsets, int write_header, std::vector<Text> &parts,
                 std::vector<size_t> &at) {
    Job &J = job->j;
    Rendered &R = J.rendered;
    std::vector<int64_t> fill((size_t)J.nunits, 0);
    if (write_header && !R.header.empty()) {
        parts.emplace_back(R.header.data(), R.header.size());
        at.push_back((size_t)offsets[0]);
    }
    for (size_t k = 0; k < R.parts.size(); ++k) {
        const int32_t u = R.part_unit[k];
        at.push_back((size_t)(offsets[1 + u] + fill[(size_t)u]));
        fill[(size_t)u] += (int64_t)R.parts[k].size();
        parts.push_back(std::move(R.parts[k]));
    }
    R = Rendered();
}
}  // namespace

int bwtmi_job_write_units(bwtmi_job *job, const char *path, const int64_t *offsets, int write_header) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && path && offsets, "null argument");
        pool_spin_for_job(job->j);
        TEXT_JOIN(job);
        write_join(job);
        std::vector<Text> parts;
        std::vector<size_t> at;
        units_parts(job, offsets, write_header, parts, at);
        pwrite_parts(path, false, parts, at, host_threads(job->j.params));
    });
}

// The same behind the caller: the parts are written by the job's own thread;
// bwtmi_job_write_join waits for it and returns its error (the job's next
// write and bwtmi_job_free join it first).
int bwtmi_job_write_units_async(bwtmi_job *job, const char *path, const int64_t *offsets, int write_header) {
    return guard([&] {
        BWTMI_STAGE("bwtmi:write");
        CHECK_ARG(job && path && offsets, "null argument");
        TEXT_JOIN(job);
        write_join(job);
        std::vector<Text> parts;
        std::vector<size_t> at;
        units_parts(job, offsets, write_header, parts, at);
        const int nt = host_threads(job->j.params);
        job->units_wr = std::thread([job, p = std::string(path), parts = std::move(parts), at = std::move(at), nt] {
            try {
                pwrite_parts(p.c_str(), false, parts, at, nt);
            } catch (...) {
                job->units_err = std::current_exception();
            }
        });
    });
}

int bwtmi_job_get_records(bwtmi_job *job, int64_t *ints9, double *dbls5) {
    return guard([&] {
        CHECK_ARG(job && ints9 && dbls5, "null argument");
        TEXT_JOIN(job);
        size_t k = 0;
        for (const Rec &r : job->j.final_recs) {
            int64_t *I = ints9 + 9 * k;
            double *D = dbls5 + 5 * k;
            I[0] = r.start; I[1] = r.end; I[2] = r.length; I[3] = r.tier; I[4] = r.n_eval; I[5] = r.max_mm;
            I[6] = r.score; I[7] = (r.stats_none ? 1 : 0) | (r.kmer_stats ? 2 : 0); I[8] = r.chrom;
            D[0] = r.copies; D[1] = r.mismatch_rate; D[2] = r.confidence; D[3] = r.pmatch; D[4] = r.pindel;
            ++k;
        }
    });
}

namespace {
// string `which` of a record (bwtmi_job_get_string); false for an unknown `which`
bool rec_string(const bwtmi_job *job, const Rec &r, int which, std::string_view &s) {
    switch (which) {
        case 0: case 1: s = r.motif; return true;
        case 2: s = r.variations; return true;
        case 3:
            s = {};
            if (r.act_kind != ACT_NONE) {
                const Contig &c = job->j.contigs[(size_t)r.chrom];
                const char *p = (r.act_kind == ACT_FULL ? c.full.data() : c.trimmed()) + r.act_off;
                s = std::string_view(p, (size_t)r.act_len);
            }
            return true;
        case 4: s = std::string_view(&r.strand, 1); return true;
        default: return false;
    }
}
}  // namespace

int64_t bwtmi_job_get_string(bwtmi_job *job, int64_t i, int which, char *buf, int64_t cap) {
    if (!job || i < 0 || i >= (int64_t)job->j.final_recs.size()) return -1;
    std::string_view s;
    if (!rec_string(job, job->j.final_recs[(size_t)i], which, s)) return -1;
    if (buf && cap > 0) std::memcpy(buf, s.data(), std::min<size_t>((size_t)cap, s.size()));
    return (int64_t)s.size();
}

int64_t bwtmi_job_get_strings(bwtmi_job *job, int which, char *buf, int64_t cap, int64_t *offsets) {
    if (!job || which < 0 || which > 4) return -1;
    int64_t tot = 0;
    std::string_view s;
    const auto &recs = job->j.final_recs;
    for (size_t i = 0; i < recs.size(); ++i) {
        if (offsets) offsets[i] = tot;
        rec_string(job, recs[i], which, s);
        tot += (int64_t)s.size();
    }
    if (offsets) offsets[recs.size()] = tot;
    if (buf && cap >= tot) {
        char *w = buf;
        for (const Rec &r : recs) {
            rec_string(job, r, which, s);
            std::memcpy(w, s.data(), s.size());
            w += s.size();
        }
    }
    return tot;
}

// record wire format for the multi-GPU gather: POD header + strings
struct WireRec {
    int32_t chrom, tier;
    int64_t start, end, length, max_mm, n_eval, score, act_off, act_len;
    double copies, confidence, mismatch_rate, pmatch, pindel;
    int8_t act_kind, strand, is_compound, kmer_stats, stats_none;
    int32_t motif_len, var_len;
};

int bwtmi_job_export(bwtmi_job *job, uint8_t **buf, int64_t *len) {
    return guard([&] {
        CHECK_ARG(job && buf && len, "null argument");
        TEXT_JOIN(job);
        std::string s;
        const int64_t n = (int64_t)job->j.final_recs.size();
        s.append((const char *)&n, sizeof n);
        for (const Rec &r : job->j.final_recs) {
            WireRec w{};
            w.chrom = r.chrom; w.tier = r.tier; w.start = r.start; w.end = r.end; w.length = r.length;
            w.max_mm = r.max_mm; w.n_eval = r.n_eval; w.score = r.score; w.act_off = r.act_off; w.act_len = r.act_len;
            w.copies = r.copies; w.confidence = r.confidence; w.mismatch_rate = r.mismatch_rate;
            w.pmatch = r.pmatch; w.pindel = r.pindel; w.act_kind = r.act_kind; w.strand = r.strand;
            w.is_compound = r.is_compound; w.kmer_stats = r.kmer_stats; w.stats_none = r.stats_none;
            w.motif_len = (int32_t)r.motif.size(); w.var_len = (int32_t)r.variations.size();
            s.append((const char *)&w, sizeof w);
            s.append(r.motif);
            s.append(r.variations);
        }
        auto *p = (uint8_t *)std::malloc(s.size());
        if (!p) fail(BWTMI_E_NOMEM, "malloc");
        std::memcpy(p, s.data(), s.size());
        *buf = p;
        *len = (int64_t)s.size();
    });
}

static void import_wire(bwtmi_job *job, const uint8_t *buf, int64_t len) {
    CHECK_ARG(job && buf && len >= 8, "bad argument");
    int64_t n;
    std::memcpy(&n, buf, 8);
    int64_t o = 8;
    for (int64_t k = 0; k < n; ++k) {
        CHECK_ARG(o + (int64_t)sizeof(WireRec) <= len, "truncated record buffer");
        WireRec w;
        std::memcpy(&w, buf + o, sizeof w);
        o += sizeof w;
        CHECK_ARG(w.motif_len >= 0 && w.var_len >= 0 && o + w.motif_len + w.var_len <= len, "truncated record strings");
        CHECK_ARG(w.chrom >= 0 && w.chrom < (int32_t)job->j.contigs.size(), "record for unknown contig");
        if (w.act_kind != ACT_NONE) {
            const Contig &c = job->j.contigs[(size_t)w.chrom];
            const int64_t L = w.act_kind == ACT_FULL ? (int64_t)c.full.size() : c.trimmed_len();
            CHECK_ARG(w.act_off >= 0 && w.act_len >= 0 && w.act_off + w.act_len <= L, "actual_sequence outside its contig");
        }
        Rec r;
        r.chrom = w.chrom; r.tier = w.tier; r.start = w.start; r.end = w.end; r.length = w.length;
        r.max_mm = w.max_mm; r.n_eval = w.n_eval; r.score = w.score; r.act_off = w.act_off; r.act_len = w.act_len;
        r.copies = w.copies; r.confidence = w.confidence; r.mismatch_rate = w.mismatch_rate;
        r.pmatch = w.pmatch; r.pindel = w.pindel; r.act_kind = w.act_kind; r.strand = (char)w.strand;
        r.is_compound = w.is_compound; r.kmer_stats = w.kmer_stats; r.stats_none = w.stats_none;
        r.motif.assign((const char *)buf + o, (size_t)w.motif_len);
        o += w.motif_len;
        r.variations.assign((const char *)buf + o, (size_t)w.var_len);
        o += w.var_len;
        job->j.final_recs.push_back(std::move(r));
    }
    // keep the reference's global order (natural chrom, start, end; stable,
    // bwt.py:3184-3187, 4147): every unit arrives whole, in order
    Job &J = job->j;
    J.assign_units();
    std::stable_sort(J.final_recs.begin(), J.final_recs.end(), [&](const Rec &a, const Rec &b) {
        const int32_t ua = J.contigs[(size_t)a.chrom].unit, ub = J.contigs[(size_t)b.chrom].unit;
        if (ua != ub) return ua < ub;
        if (a.start != b.start) return a.start < b.start;
        return a.end < b.end;
    });
    J.postprocessed = true;
}

int bwtmi_job_import(bwtmi_job *job, const uint8_t *buf, int64_t len) {
    return guard([&] { import_wire(job, buf, len); });
}

int bwtmi_job_set_records(bwtmi_job *job, const uint8_t *buf, int64_t len) {
    return guard([&] {
        CHECK_ARG(job, "null argument");
        TEXT_JOIN(job);
        job->j.final_recs.clear();
        import_wire(job, buf, len);
    });
}

int bwtmi_wire_record_size(void) { return (int)sizeof(WireRec); }

int64_t bwtmi_job_contig_error(const bwtmi_job *job, int32_t id, char *buf, int64_t cap) {
    if (!job || id < 0 || id >= (int32_t)job->j.contigs.size()) return -1;
    if ((size_t)id >= job->j.errors.size()) return 0;
    const std::string &e = job->j.errors[(size_t)id];
    if (buf && cap > 0) {
        const size_t m = std::min<size_t>((size_t)cap - 1, e.size());
        std::memcpy(buf, e.data(), m);
        buf[m] = 0;
    }
    return (int64_t)e.size();
}

int bwtmi_job_stage_ms(const bwtmi_job *job, double *out8) {
    return guard([&] {
        CHECK_ARG(job && out8, "null argument");
        for (int i = 0; i < 8; ++i) out8[i] = job->j.stage_ms[i];
    });
}

int bwtmi_align_region(const char *seq, int64_t seq_len, int64_t start, int64_t end, const char *tmpl,
                       int64_t tmpl_len, double frac, int64_t max_indel, int64_t min_copies, int64_t *ints8,
                       double *mismatch_rate, char *consensus, char **variations, int64_t **copy_len,
                       int64_t **copy_err) {
    int found = 0;
    int rc = guard([&] {
        CHECK_ARG((seq || seq_len == 0) && (tmpl || tmpl_len == 0) && ints8 && mismatch_rate && consensus &&
                      variations && copy_len && copy_err, "null argument");
        *variations = nullptr;
        *copy_len = *copy_err = nullptr;
        AlignSummary s;
        std::string t(tmpl ? tmpl : "", (size_t)tmpl_len);
        if (!align_repeat_region(seq, seq_len, start, end, t, min_copies, s, frac, max_indel)) return;
        found = 1;
        ints8[0] = s.copies; ints8[1] = s.motif_len; ints8[2] = s.consumed; ints8[3] = s.max_errors;
        ints8[4] = s.tot_ins; ints8[5] = s.tot_del; ints8[6] = ints8[7] = 0;
        *mismatch_rate = s.mismatch_rate;
        std::memcpy(consensus, s.consensus.data(), s.consensus.size());
        char *v = (char *)std::malloc(s.variations.size() + 1);
        std::memcpy(v, s.variations.data(), s.variations.size());
        v[s.variations.size()] = 0;
        *variations = v;
        auto *cl = (int64_t *)std::malloc(std::max<size_t>(1, s.copy_len.size()) * 8);
        auto *ce = (int64_t *)std::malloc(std::max<size_t>(1, s.copy_err.size()) * 8);
        for (size_t i = 0; i < s.copy_len.size(); ++i) { cl[i] = s.copy_len[i]; ce[i] = s.copy_err[i]; }
        *copy_len = cl;
        *copy_err = ce;
    });
    return rc ? rc : found;
}

}  // extern "C"
