// device.h -- HIP context, device buffers and the device-primitive entry points.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace bwtmi {

#define HIPCHECK(expr)                                                                  \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            ::bwtmi::fail(BWTMI_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                          __FILE__, __LINE__);                                          \
    } while (0)

// growable device allocation
struct DBuf {
    void *p = nullptr;
    size_t bytes = 0;
    void ensure(size_t n) {
        if (n <= bytes) return;
        if (p) {
            HIPCHECK(hipDeviceSynchronize());  // queued kernels may still use the old block
            HIPCHECK(hipFree(p));
        }
        size_t cap = n + n / 8 + 256;
        HIPCHECK(hipMalloc(&p, cap));
        bytes = cap;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

struct HBuf {  // pinned host staging
    void *p = nullptr;
    size_t bytes = 0;
    // async copies still reading the buffer: arm() after queueing them, and
    // every writer (and ensure / release) settles first
    hipEvent_t inflight = nullptr;
    void settle() {
        if (inflight) HIPCHECK(hipEventSynchronize(inflight));
    }
    void arm(hipStream_t st) {
        if (!inflight) HIPCHECK(hipEventCreateWithFlags(&inflight, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(inflight, st));
    }
    void ensure(size_t n) {
        settle();
        if (n <= bytes) return;
        if (p) HIPCHECK(hipHostFree(p));
        size_t cap = n + n / 8 + 256;
        HIPCHECK(hipHostMalloc(&p, cap, hipHostMallocDefault));
        bytes = cap;
    }
    void release() {
        if (inflight) {
            (void)hipEventSynchronize(inflight);
            (void)hipEventDestroy(inflight);
            inflight = nullptr;
        }
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

enum Slot {
    S_TEXT = 0, S_PACK, S_CAND_K, S_CAND_V, S_CAND_K2, S_CAND_V2, S_FLAG, S_SCAN, S_HITS, S_COUNTS,
    S_SORT_TMP0, S_SORT_TMP1, S_SORT_HIST, S_SCAN_TMP, S_MISC0, S_MISC1, S_MISC2, S_MISC3,
    S_IDX0, S_IDX1, S_IDX2, S_IDX3, S_IDX4, S_IDX5, S_IDX6, S_IDX7, S_IDX8, S_IDX9, S_IDX10, S_IDX11, S_IDX12,
    S_FASTA,   // a whole-file load's FASTA image (fasta_dev.hip)
    S_SORT_DIG,   // the next pass's digit of every key, written by a radix pass (radix.hip)
    S_LB,         // look-back granules of the single-pass scans and radix histograms (radix.hip)
    S_NSLOTS
};

struct KernelTimer {
    hipEvent_t a = nullptr, b = nullptr;
    double total_ms = 0;
    int launches = 0;
};

struct KStat {
    double ms = 0;
    int64_t launches = 0;
    double bytes = 0;   // algorithmic bytes (compulsory reads + writes) of those launches
};

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // per-kernel HIP-event timing (on the ctx stream), enabled by bwtmi_kernel_stats
    bool ktiming = [] {   // BWTMI_KTRACE=path: every launch of every call, timed from the start
        const char *e = std::getenv("BWTMI_KTRACE");
        return e && *e;
    }();
    struct Pend {
        std::string name;
        hipEvent_t a, b;
        double bytes;
    };
    std::vector<Pend> pending;
    std::vector<size_t> open;   // kbegin/kend nest (a stage timer around primitive timers)
    // bwtmi_kernel_stats_filter: time only the launches of this name ("" = every
    // launch); the others get no events, so they run back to back as untimed
    std::string kfilter;
    std::vector<std::pair<std::string, KStat>> kstats;
    std::vector<hipEvent_t> evpool;   // reused across kresolve calls
    size_t evused = 0;
    hipEvent_t pooled_event() {
        if (evused == evpool.size()) {
            hipEvent_t e;
            HIPCHECK(hipEventCreate(&e));
            evpool.push_back(e);
        }
        return evpool[evused++];
    }
    // BWTMI_KTRACE=path (timing on): one line per launch (name, ms, idle ms
    // since the previous launch ended) and the drivers' notes, appended to path
    static FILE *ktrace_file() {
        static FILE *f = [] {
            const char *e = std::getenv("BWTMI_KTRACE");
            return e && *e ? std::fopen(e, "a") : (FILE *)nullptr;
        }();
        return f;
    }
    // every kernel launch is a leaf timer (KLAUNCH); kbegin/kend must not nest
    void kbegin(const char *name, double alg_bytes = 0) {
        if (!ktiming) return;
        if (!kfilter.empty() && kfilter != name) {
            open.push_back(SIZE_MAX);   // (kend pops it without an event)
            return;
        }
        hipEvent_t a = pooled_event(), b = pooled_event();
        HIPCHECK(hipEventRecord(a, stream));
        open.push_back(pending.size());
        pending.push_back({name, a, b, alg_bytes});
    }
    void kend() {
        if (!ktiming || open.empty()) return;
        const size_t i = open.back();
        open.pop_back();
        if (i != SIZE_MAX) HIPCHECK(hipEventRecord(pending[i].b, stream));
    }
    void kresolve() {   // after a stream sync
        FILE *trace = ktrace_file();
        for (size_t i = 0; i < pending.size(); ++i) {
            auto &p = pending[i];
            float ms = 0;
            if (hipEventElapsedTime(&ms, p.a, p.b) != hipSuccess) {
                ms = 0;
                (void)hipGetLastError();   // do not leave a sticky error for the next check
            }
            if (trace) {
                float gap = 0;
                if (i && hipEventElapsedTime(&gap, pending[i - 1].b, p.a) != hipSuccess) {
                    gap = -1;
                    (void)hipGetLastError();
                }
                std::fprintf(trace, "%s %.4f %.4f\n", p.name.c_str(), ms, gap);
            }
            bool found = false;
            for (auto &k : kstats)
                if (k.first == p.name) {
                    k.second.ms += ms;
                    ++k.second.launches;
                    k.second.bytes += p.bytes;
                    found = true;
                    break;
                }
            if (!found) kstats.push_back({p.name, KStat{ms, 1, p.bytes}});
        }
        if (trace) {
            std::fprintf(trace, "-- resolve\n");
            std::fflush(trace);
        }
        pending.clear();
        open.clear();
        evused = 0;
    }
    DBuf slot[S_NSLOTS];
    // BWTMI_DEVICE_CHECKS=1: the radix passes and the suffix sort's kernels test
    // the bounds of their tickets, list slots and scattered writes, skip a
    // store that would leave its array and set a bit here (kChk*); the host
    // reads the word at the sort's stream waits (checks_verify) and fails
    // naming what was hit.  Off (nullptr): nothing is tested.
    DBuf chk;
    uint32_t *checks() {
        if (!knob(KN_DEVICE_CHECKS)) return nullptr;
        if (!chk.p) {
            chk.ensure(64);
            HIPCHECK(hipMemsetAsync(chk.p, 0, 64, stream));
        }
        return chk.as<uint32_t>();
    }
    void checks_verify(const char *where);   // after a wait on `stream` (radix.hip)
    DBuf lb_ticket;          // the look-back launches' tile ticket (radix.hip)
    uint64_t fasta_tag = 0;  // what S_FASTA holds: a split loader's pass-1 part (its job's tag), 0 anything else
    uint32_t lb_epoch = 0;   // the last look-back launch's epoch
    HBuf host[4];
    // pinned mailbox of the scan's small device->host reads: the reads of one
    // step are queued into it and share one stream wait (a copy into pageable
    // memory is staged synchronously -- one host round trip per value, ~20 us)
    HBuf mbox;
    template <class T>
    T *mailbox(size_t n) {
        mbox.ensure(std::max<size_t>(n * sizeof(T), 4096));
        return mbox.as<T>();
    }
    struct DeviceIndex *scratch_index = nullptr;   // reused by the worker-path index builds
    // device work that runs behind host work (the worker-path index builds):
    // every entry point that uses this context joins it first (ctx_wait)
    std::thread bg;
    int bg_code = 0;
    std::string bg_err;
    double bg_ms = 0;                 // wall time of the last background index builds
    Ctx **bg_link = nullptr;          // the job field naming this ctx while bg reads its buffers
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double last_total_ms = 0, last_dom_ms = 0;
    int last_dom_launches = 0;
    std::string dom_name;
    bool timing = true;
    // scan lanes: extra contexts (own stream and scratch) on the same device, so
    // the strict scans of several contigs overlap (api.cpp bwtmi_job_scan)
    std::vector<std::unique_ptr<Ctx>> lanes;
    void activate() const { HIPCHECK(hipSetDevice(device)); }
    // per-kernel statistics of another context (a lane) folded into this one
    void absorb_kstats(Ctx &o) {
        for (auto &k : o.kstats) {
            bool found = false;
            for (auto &m : kstats)
                if (m.first == k.first) {
                    m.second.ms += k.second.ms;
                    m.second.launches += k.second.launches;
                    m.second.bytes += k.second.bytes;
                    found = true;
                    break;
                }
            if (!found) kstats.push_back(k);
        }
        o.kstats.clear();
    }
};

// A kernel launch on ctx `c`'s stream `st`, timed as `name` (algorithmic bytes
// `bytes`, 0 when not modelled) when kernel statistics are on.
#define KLAUNCH(name, bytes, kern, grid, block, shm, st, ...)                  \
    do {                                                                       \
        c.kbegin(name, bytes);                                                 \
        hipLaunchKernelGGL(kern, grid, block, shm, st, __VA_ARGS__);           \
        c.kend();                                                              \
    } while (0)

// join the context's background device work; rethrows its error
// The scan's host reads (candidate counts, key widths, hit counts) wait on the
// stream by polling: a blocking wait (hipDeviceScheduleBlockingSync, kept for
// the long waits behind host work) sleeps the thread, and its wake-up delays
// the next dependent launch.
inline void scan_wait(hipStream_t st) {
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return;
        if (e != hipErrorNotReady) HIPCHECK(e);
        __builtin_ia32_pause();
    }
}

inline void ctx_join(Ctx &c) {
    if (c.bg.joinable()) c.bg.join();
    if (c.bg_link) *c.bg_link = nullptr;
    c.bg_link = nullptr;
}
inline void ctx_wait(Ctx &c) {
    ctx_join(c);
    if (c.bg_code) {
        const int code = c.bg_code;
        c.bg_code = 0;
        fail(code, "%s", c.bg_err.c_str());
    }
}

// device check bits (Ctx::checks)
constexpr uint32_t kChkHistTicket = 1;   // a histogram workgroup drew a ticket >= its launch's workgroups
constexpr uint32_t kChkScatter = 2;      // a radix scatter slot outside [0, n)
constexpr uint32_t kChkRankPut = 4;      // a first-rank position outside [0, n)
constexpr uint32_t kChkShortFix = 8;     // the end fix-up: a group or a short suffix not where it must be
constexpr uint32_t kChkRunList = 16;     // more runs of >= 16 equal symbols than the run list holds
constexpr uint32_t kChkRunEnd = 32;      // a run end / run-end block outside the text
constexpr uint32_t kChkDeepEnd = 64;     // a deep suffix whose run end is not inside the text

// ----- primitives (radix.hip)
template <class T>
void exclusive_scan(Ctx &c, const T *in, T *out, int64_t n);   // out may alias in
// `rows` independent scans of n uint32 each, row r at in / out + r * stride, in one launch
void exclusive_scan_rows(Ctx &c, const uint32_t *in, uint32_t *out, int64_t n, int rows, int64_t stride);
void radix_sort_pairs(Ctx &c, uint64_t *keys, uint64_t *vals, int64_t n, int bit0, int bit1);
void radix_sort_pairs32(Ctx &c, uint64_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1);
void radix_sort_pairs_k32(Ctx &c, uint32_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1);
void radix_sort_pairs_k16(Ctx &c, uint16_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1);
// XCD-aware tile order: blocks b and b + 8 share an XCD (and its L2) under the
// observed round-robin placement, so each group of blocks b % 8 takes one
// contiguous range of tiles and neighbouring tiles run on one L2 at about the
// same time (their writes to a shared 128-B line merge there before HBM).
// Bijective for any ntiles; speed only, never correctness.
__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t ntiles) {
    const int64_t q = ntiles / 8, r = ntiles % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// one stable 8-bit pass at `shift` from (kin, vin) into (kout, vout)
void radix_pass_k32(Ctx &c, const uint32_t *kin, const uint32_t *vin, uint32_t *kout, uint32_t *vout, int64_t n,
                    int shift);

// ----- a FASTA file's plain chunks rebuilt on the device (fasta_dev.hip):
// image bytes [a, b) minus their newlines, upper-cased, land at content offset
// `off` of a contig whose trimmed window [tl, tl + tn) is at dst (device)
struct FastaDevPiece {
    int64_t a, b, off, tl, tn;
    char *dst;
};
void fasta_build_device(Ctx &c, const uint8_t *d_img, const FastaDevPiece *pieces, int64_t npieces);
// An empty kernel queued (not waited for) ahead of host work that precedes the
// first device work of a job: after tens of ms without device work the first
// operation on the box pays ~5 ms (a 4-byte download 4.5-5.4 ms, the next
// ones 0.03 ms; r04r), which then elapses behind the host work instead.

void device_wake(Ctx &c);

// ----- strict scan (strict_scan.hip)
struct ScanResult {
    HitVec hits;                   // raw hits in worker order (screen = false)
    ScreenedVec shits;             // screened hits (screen = true)
    double kernel_ms = 0;
    int64_t candidates = 0;
    int64_t raw = 0;               // raw strict hits found
    bool screened = false;
};
// d_text: device copy of the trimmed contig (n bytes, padded by >= 64 bytes).
// screen: also run nested suppression + (start, end) sort + dedup on the
// device (nested.hip) and return only the survivors, in that order.
// drop_min_copies: passed to the screen (screen_hits_device)
void strict_scan_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t min_unit, int32_t max_unit,
                        int32_t min_copies, ScanResult &out, bool screen = false, int32_t drop_min_copies = 0);
// max_mismatch > 0: hits in emission order (host vector)
void strict_scan_mm_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t min_unit, int32_t max_unit,
                           int32_t max_mismatch, int32_t min_copies, HitVec &hits);

// ----- nested suppression / sort / dedup of one contig's strict hits (nested.hip)
// maxlen: the hits' longest span, when the caller knows it (the strict scan's
// compaction reduces it and reads it with the hit count); -1: reduced here
// drop_min_copies > 0: also drop the kept hits the post-processing would only
// carry to its final filter (k_drop_flags; the job's min_copies)
void screen_hits_device(Ctx &c, const bwtmi_hit *d_hits, int64_t n, int64_t text_len, int32_t lmax,
                        ScreenedVec &out, int64_t maxlen = -1, int32_t drop_min_copies = 0);

// ----- suffix array + BWT of ACGT* '$' texts (sa_dna.hip)
bool sa_dna_eligible(uint8_t last, int64_t n, const int64_t *totals);
// also writes the sampled SA (bwt.py:328-333): sampled[j] = SA[j * sample] for j < ceil(n / sample)
bool sa_dna_device(Ctx &c, const uint8_t *t, int64_t n, uint32_t *SA, uint8_t *BWT, int32_t *sampled, int32_t sample);
// texts whose non-'$' symbols are at most 7 bytes above '$' (ACGT with N runs,
// IUPAC codes): the symbol count (lut: byte -> code 0..6, sym: code -> byte,
// sym[7] = '$'), else 0
int sa_small_alphabet(uint8_t last, int64_t n, const int64_t *totals, uint8_t *lut, uint8_t *sym);
bool sa_small_device(Ctx &c, const uint8_t *t, int64_t n, uint32_t *SA, uint8_t *BWT, int32_t *sampled, int32_t sample,
                     const uint8_t *lut, const uint8_t *sym);

// ----- index (index.hip)
// true when [p, p+n) lies in a host block of mem.h that is (now) registered
// for DMA (api.cpp); the block stays registered while it is cached
bool ensure_pinned(const void *base, const void *p, size_t n);

struct DeviceIndex;
// d_text: device text incl. sentinel, n bytes (padded by >= 64 bytes)
DeviceIndex *index_build_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t sa_sample,
                                int32_t occ_sample, uint32_t flags, DeviceIndex *reuse = nullptr);
void index_free(DeviceIndex *);
int64_t index_n(const DeviceIndex *);
int64_t index_occ_len(const DeviceIndex *);
int64_t index_sampled_len(const DeviceIndex *);
int64_t index_kmer_count(const DeviceIndex *);
void index_get_sa(Ctx &c, const DeviceIndex *, int32_t *out);
void index_get_bwt(Ctx &c, const DeviceIndex *, uint8_t *out);
void index_get_counts(const DeviceIndex *, int64_t *totals, int64_t *C);
void index_get_occ(Ctx &c, const DeviceIndex *, uint8_t code, int32_t *out);
void index_get_sampled(Ctx &c, const DeviceIndex *, int32_t *out);
void index_get_kmer(Ctx &c, const DeviceIndex *, int64_t *offsets, int32_t *pos);
void index_lcp(Ctx &c, DeviceIndex *, int32_t *out);
const int32_t *index_lcp_device(Ctx &c, DeviceIndex *);   // in the S_MISC1 slot
const uint8_t *index_text_device(const DeviceIndex *);
const uint32_t *index_sa_device(const DeviceIndex *);
void index_get_text(Ctx &c, const DeviceIndex *, uint8_t *out);

// ----- library finders off the CLI path (library.hip)
struct LibParams {
    int32_t min_period = 1, max_period = 1000, max_short_motif = 9, min_copies = 3;
    int32_t min_array_length = 6, allow_mismatches = 1;
    double min_entropy = 1.0;
};
// Tier2LCPFinder._detect_lcp_plateaus (bwt.py:2118-2145, 2500-2560): (start, copies, period) in order
void lcp_plateaus_device(Ctx &c, DeviceIndex *ix, const LibParams &p, std::vector<int64_t> &out);
// Tier2LCPFinder.find_short_imperfect_repeats (bwt.py:2027-2095, 2562-2825); records appended
// to `out` with chrom = `chrom`; `seen` = (start, end) pairs already found (tier1_seen)
void short_imperfect_device(Ctx &c, DeviceIndex *ix, const LibParams &p, const std::vector<int64_t> &seen,
                            int32_t chrom, RecVec &out);
// Tier1STRFinder.find_strs (bwt.py:1426-1538) over text t (host) / d_text (device copy, n bytes)
void tier1_device(Ctx &c, const uint8_t *d_text, const uint8_t *t, int64_t n, int32_t max_motif_length,
                  int32_t chrom, RecVec &out);
void index_backward_search(Ctx &c, DeviceIndex *, const uint8_t *pats, const int64_t *off, int64_t npat,
                           int64_t *sp_ep);
void index_sa_rows(Ctx &c, const DeviceIndex *, const int64_t *rows, int64_t k, int64_t *out);
// Tier2LCPFinder.find_long_repeats -> _find_repeats_simple (bwt.py:2097-2106, 2177-2498)
void simple_scan_device(Ctx &c, DeviceIndex *ix, const LibParams &p, const std::vector<int64_t> &seen_pairs,
                        int32_t chrom, RecVec &out);
// Tier3LongReadFinder.find_very_long_repeats (bwt.py:2837-3036) of `reads` (concatenated,
// read_off[nreads + 1]) against the index; consolidated records with chrom = `chrom`
void tier3_device(Ctx &c, DeviceIndex *ix, const uint8_t *reads, const int64_t *read_off, int64_t nreads,
                  int32_t chrom, RecVec &out);

}  // namespace bwtmi
