// common.h -- internal declarations shared by the libbwtmi translation units.
#pragma once

#include <sched.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/bwtmi.h"
#include "mem.h"

namespace bwtmi {

// ---------------------------------------------------------------- errors
void set_error(const char *fmt, ...);
struct Error {   // the message travels with the exception (it may cross threads)
    int code;
    std::string msg;
};
[[noreturn]] void fail(int code, const char *fmt, ...);

// vector storage without value-initialisation, large arrays from the cached
// huge-page blocks of mem.h: arrays that are written once (device downloads,
// parallel fills) skip a serial zero fill and, from the second step on, the
// page faults
template <class T>
using NoInit = BigAlloc<T>;
using HitVec = std::vector<bwtmi_hit, NoInit<bwtmi_hit>>;

// a device-screened strict hit is [start, start + len) with primitive motif
// length prim, and its copies are len / prim (count after primitive
// reduction, bwt.py:1957-1961; (end-i)/L otherwise, as end = i + count*L).
// Downloaded as one 64-bit word per hit -- start | len << 32 | prim << (32 +
// lbits), lbits = the bits of the longest span -- when len and prim fit the
// high half (32 B per hit on the device, 8 B over PCIe), else as two words
// {start, len | prim << 32}.
// a device download still landing in host memory (nested.hip): wait(k) returns
// once hits [0, k) are there; the destructor waits for all of it
struct Landing {
    virtual ~Landing() = default;
    virtual void wait(int64_t k) = 0;
};

struct ScreenedVec {
    std::vector<uint64_t, NoInit<uint64_t>> w;
    int32_t lbits = -1;   // one word per hit when >= 0
    // the download into w, when it is still in flight: declared after w, so it
    // is destroyed (and waited for) before w is freed
    std::shared_ptr<Landing> landing;
    int64_t size() const { return lbits >= 0 ? (int64_t)w.size() : (int64_t)w.size() / 2; }
    bool empty() const { return w.empty(); }
    // hits [0, k) readable
    void wait(int64_t k) const {
        if (landing) landing->wait(k);
    }
    void clear() {
        landing.reset();
        w.clear();
        lbits = -1;
    }
    void swap(ScreenedVec &o) noexcept {
        w.swap(o.w);
        std::swap(lbits, o.lbits);
        landing.swap(o.landing);
    }
    // hit k: start, length, primitive motif length
    void get(int64_t k, int64_t &start, int64_t &len, int64_t &prim) const {
        if (lbits >= 0) {
            const uint64_t x = w[(size_t)k];
            start = (int64_t)(uint32_t)x;
            len = (int64_t)((x >> 32) & ((uint64_t(1) << lbits) - 1));
            prim = (int64_t)(x >> (32 + lbits));
        } else {
            start = (int64_t)w[2 * (size_t)k];
            const uint64_t y = w[2 * (size_t)k + 1];
            len = (int64_t)(uint32_t)y;
            prim = (int64_t)(y >> 32);
        }
    }
};

// ---------------------------------------------------------------- contigs
// contig bases live in cached huge-page blocks (mem.h); the device layer pins
// those blocks once for DMA (api.cpp), so re-loading a FASTA of the same shape
// reuses already-faulted, already-registered memory
class Seq {
public:
    Seq() = default;
    Seq(const Seq &o) { assign(o.data(), o.size()); }
    Seq(Seq &&o) noexcept { swap(o); }
    Seq &operator=(const Seq &o) {
        if (this != &o) assign(o.data(), o.size());
        return *this;
    }
    Seq &operator=(Seq &&o) noexcept {
        swap(o);
        return *this;
    }
    ~Seq() { release(); }
    const char *data() const { return p_ ? p_ : ""; }
    char *data() { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    char operator[](size_t i) const { return p_[i]; }
    void swap(Seq &o) noexcept {
        std::swap(p_, o.p_);
        std::swap(n_, o.n_);
        std::swap(cap_, o.cap_);
    }
    void clear() { release(); }
    // n bytes of unspecified content (written by the caller)
    char *resize_uninit(size_t n) {
        if (n > cap_) {
            release();
            p_ = (char *)(n >= kBigMin ? big_alloc(n) : ::operator new(n));
            cap_ = n;
        }
        n_ = n;
        return p_;
    }
    void assign(const char *s, size_t n) {
        char *d = resize_uninit(n);
        if (n) std::memcpy(d, s, n);
    }

private:
    void release() {
        if (p_) {
            if (cap_ >= kBigMin) big_free(p_, cap_);
            else ::operator delete(p_);
        }
        p_ = nullptr;
        n_ = cap_ = 0;
    }
    char *p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};
uint64_t next_contig_gen();   // fresh content id (device copies are keyed by it)

struct Contig {
    std::string name;
    Seq full;               // untrimmed, upper-cased (bwt.py:3739); empty for another rank's contig
    int64_t trim_left = 0;  // trim_offsets[name] (bwt.py:3733)
    int64_t trim_right = 0;
    int64_t weight = 0;     // analysed length (shard weight), also for contigs not loaded here
    uint64_t gen = 0;       // content id of `full`
    int32_t unit = 0;       // fold unit (contigs with equal natural sort key)
    const char *trimmed() const { return full.data() + trim_left; }
    int64_t trimmed_len() const { return (int64_t)full.size() - trim_left - trim_right; }
};

// natural sort key (bwt.py:22-36) and its comparison
struct NatPart {
    bool digit;
    std::string text;  // digits with leading zeros stripped, or lower-cased text
};
std::vector<NatPart> natural_key(const std::string &s);
int natural_cmp(const std::vector<NatPart> &a, const std::vector<NatPart> &b);

// ---------------------------------------------------------------- records
// Field-for-field counterpart of TandemRepeat (bwt.py:429-452) as it occurs
// on the CLI path.  On that path consensus_motif == motif for every record
// (strict hits bwt.py:1981, recomputes 3602, compound pieces 4077/4086), so
// one string carries both.
enum ActKind : int8_t { ACT_NONE = 0, ACT_TRIMMED = 1, ACT_FULL = 2 };

struct Rec {
    int32_t chrom = 0;
    int32_t tier = 2;
    int64_t start = 0, end = 0, length = 0;
    std::string motif;
    double copies = 0.0;
    double confidence = 1.0;
    double mismatch_rate = 0.0;
    int64_t max_mm = 0;
    int64_t n_eval = 0;
    char strand = '+';
    double pmatch = 0.0, pindel = 0.0;
    int64_t score = 0;
    int8_t act_kind = ACT_NONE;  // actual_sequence = slice of trimmed/full contig
    int64_t act_off = 0, act_len = 0;
    std::string variations;      // ';'-joined; empty == None
    int32_t partner = -1;        // compound partner index in the owning pool, -1 = none
    bool is_compound = false;
    bool kmer_stats = false;     // compound-stage pieces: score 100.0, zero composition,
                                 // entropy 1.5 (bwt.py:3980-3987, 4074-4091)
    bool stats_none = false;     // composition None, entropy 0.0: records built without
                                 // statistics (consolidated Tier 3 calls, bwt.py:3021-3030)
};

using RecVec = std::vector<Rec, BigAlloc<Rec>>;

// motif utilities (MotifUtils, bwt.py:675-1381)
std::string min_rotation(const std::string &s);
void canonical_stranded(const std::string &s, std::string &canon, char &strand);
char canonical_strand(const char *s, int64_t n);   // the strand of canonical_stranded only
// ACGT strings of <= 32 bases as 2-bit codes (A0 C1 G2 T3, first base high):
// rotations compare as integers, rc2 = reverse complement, min_rot2 = least rotation
bool pack2_acgt(const char *s, int64_t n, uint64_t &x);
uint64_t rc2(uint64_t x, int64_t n);
uint64_t min_rot2(uint64_t x, int64_t n);
// min(min_rot2(x, n), min_rot2(rc2(x, n), n)): the canonical word of a packed
// ACGT motif; n <= 8 from a table built once (4^n entries per length)
uint64_t canon2(uint64_t x, int64_t n);
// canonical word (min over rotations of the motif and its reverse complement)
// of an ACGT motif of 33..64 bases; false if it has another symbol
bool canon_key128(const char *s, int64_t n, unsigned __int128 &key);
int64_t smallest_period(const char *s, int64_t n);
double entropy_of(const char *s, int64_t n);
void composition_of(const char *s, int64_t n, double out[4]);
int64_t trf_score(int64_t length, double mm);

struct AlignSummary {
    bool want_copies = true;                  // fill copy_len / copy_err (bwtmi_align_region)
    std::vector<int64_t> copy_len, copy_err;  // per copy: consumed bases, errors
    std::string consensus;
    int64_t motif_len = 0, copies = 0, consumed = 0, max_errors = 0, tot_ins = 0, tot_del = 0, tot_err = 0;
    double mismatch_rate = 0.0;
    std::string variations;  // ';'-joined
    bool any_variation = false;
    // the walk ended because it reached its safety limit (bwt.py:1033), not at
    // a copy that failed to align or a window too short: only then can a
    // larger `end` change the result
    bool at_limit = false;
};
// first position >= pos and < lim whose byte differs from b (lim if none):
// the end of a homopolymer run, 32 bytes per step (assembly gaps hold N runs
// of up to megabases, and a run is walked by every recompute merging into it)
int64_t run_end(const char *s, int64_t pos, int64_t lim, char b);
// MotifUtils.align_repeat_region (bwt.py:998-1102), max_indel=None, frac=0.1
bool align_repeat_region(const char *seq, int64_t seq_len, int64_t start, int64_t end,
                         const std::string &tmpl, int64_t min_copies, AlignSummary &out,
                         double frac = 0.1, int64_t max_indel_arg = -1);
// the same with caller-owned DP scratch (one per worker: no thread-local
// lookups on the hot path -- __tls_get_addr was 14 % of a recompute)
struct AlignScratch;
AlignScratch *align_scratch_new();
void align_scratch_free(AlignScratch *);
// resume: a walk of the same region start and template that this scratch saw
// stop at its limit goes on from there when this call's limit is not smaller
// (and this call's walk is kept in turn when it stops at its limit)
bool align_repeat_region(const char *seq, int64_t seq_len, int64_t start, int64_t end,
                         const std::string &tmpl, int64_t min_copies, AlignSummary &out, double frac,
                         int64_t max_indel_arg, AlignScratch *ws, bool resume = false);


// ---------------------------------------------------------------- job
// formatted text in cached huge-page blocks (mem.h); the formatters write
// through a raw cursor into capacity they reserved, so growing never
// zero-fills (a std::string resize wrote every reserved byte once more)
class Text {
public:
    Text() = default;
    Text(const char *s, size_t n) {
        grow(n);
        if (n) std::memcpy(p_, s, n);
        n_ = n;
    }
    Text(Text &&o) noexcept { swap(o); }
    Text &operator=(Text &&o) noexcept {
        swap(o);
        return *this;
    }
    Text(const Text &) = delete;
    Text &operator=(const Text &) = delete;
    ~Text() { release(); }
    const char *data() const { return p_ ? p_ : ""; }
    char *data() { return p_; }
    size_t size() const { return n_; }
    size_t capacity() const { return cap_; }
    // capacity >= cap, content [0, size) kept
    void grow(size_t cap) {
        if (cap <= cap_) return;
        char *q = (char *)(cap >= kBigMin ? big_alloc(cap) : ::operator new(cap));
        if (n_) std::memcpy(q, p_, n_);
        release_keep_size();
        p_ = q;
        cap_ = cap;
    }
    void set_size(size_t n) { n_ = n; }   // n <= capacity(), bytes written by the caller
    void swap(Text &o) noexcept {
        std::swap(p_, o.p_);
        std::swap(n_, o.n_);
        std::swap(cap_, o.cap_);
    }

private:
    void release_keep_size() {
        if (p_) {
            if (cap_ >= kBigMin) big_free(p_, cap_);
            else ::operator delete(p_);
        }
        p_ = nullptr;
        cap_ = 0;
    }
    void release() {
        release_keep_size();
        n_ = 0;
    }
    char *p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};

// formatted output: header + parts of consecutive rows, each inside one fold unit
struct Rendered {
    std::string header;
    std::vector<Text> parts;
    std::vector<int32_t> part_unit;
};

struct Job {
    bwtmi_params params{};
    std::vector<Contig> contigs;
    std::vector<std::vector<NatPart>> natkeys;
    int32_t nunits = 0;
    std::vector<int32_t> unit_rank;                  // unit id -> rank by natural key
    std::vector<HitVec> hits;                        // per contig strict hits: raw (worker order), or
    std::vector<uint8_t> screened;                   // screened[c]: nested-suppressed, sorted by
                                                     // (start, end, m desc, worker order) and deduped
    std::vector<ScreenedVec> shits;                  // per contig: those screened hits (hits[c] empty)
    std::vector<int64_t> raw_n;                      // raw strict hits per contig
    std::vector<std::string> errors;                 // per contig: the worker's error (empty = none)
    RecVec final_recs;                               // after bwt.py:3940-3944
    std::vector<RecVec> t3;                          // per contig: Tier 3 records (bwt.py:3918-3924), joined
                                                     // after the contig's strict hits before nested suppression
    std::vector<uint8_t> selected;                   // scan only these contigs (empty = all)
    bool postprocessed = false;
    Rendered rendered;                               // last bwtmi_job_render_units result
    double stage_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // the split loader's pass-1 bytes (file range [part_a, part_b) of part_path,
    // read at the file's size/mtime part_stamp), reused by pass 2 for the own
    // contigs that lie inside it
    Seq part;
    std::string part_path;
    int64_t part_a = 0, part_b = 0, part_stamp[2] = {-1, -1};
    // pass 1 with a device (bwtmi_job_fasta_scan_part_dev): the part's bytes
    // were queued to that context's FASTA image slot under this tag (0: not),
    // and part_inflight waits for that copy; every path that rewrites or frees
    // `part` settles first (a host pass 1 on another file or rank
    // kept the tag, and the copy could still be reading the old bytes)
    uint64_t part_dev_tag = 0;
    std::function<void()> part_inflight;
    void part_settle() {
        part_dev_tag = 0;
        if (part_inflight) {
            std::function<void()> f = std::move(part_inflight);
            part_inflight = nullptr;
            f();
        }
    }
    void assign_units();
    // host text written behind the device work (a whole-file load with device
    // placement, bwtmi_job_load_fasta_dev): every reader of contig bytes joins it
    std::thread text_th;
    std::exception_ptr text_err;
    void text_defer(std::function<void()> fn) {
        text_join();
        text_th = std::thread([this, fn = std::move(fn)] {
            try {
                fn();
            } catch (...) {
                text_err = std::current_exception();
            }
        });
    }
    void text_join() {
        if (text_th.joinable()) text_th.join();
        if (text_err) {
            std::exception_ptr e = text_err;
            text_err = nullptr;
            std::rethrow_exception(e);
        }
    }
    Job() = default;
    Job(const Job &) = delete;
    Job &operator=(const Job &) = delete;
    ~Job() {
        if (text_th.joinable()) text_th.join();
        part_settle();   // `part` is freed with the job
    }
};

// Device placement of a whole-file load (api.cpp): the loader hands over the
// file image right after the read, the plain chunks' pieces (file bytes [a, b)
// minus their newlines, upper-cased, at content offset `off` of contig cid),
// and the pieces it wrote on the host; defer runs the host pass over the plain
// chunks behind the device work and keeps `hold` until the copies are done.
struct FastaPiece {
    int64_t a, b, off;
    int32_t cid;
};
struct FastaDev {
    virtual ~FastaDev() = default;
    virtual void image(const char *img, int64_t n) = 0;         // the image buffer (before the read)
    virtual void image_part(int64_t off, int64_t n) = 0;         // bytes [off, off + n) are read (any thread)
    virtual void contigs() = 0;   // names, trims and host buffers are settled
    virtual void plain(const std::vector<FastaPiece> &pieces) = 0;
    virtual void piece(int32_t cid, int64_t off, const char *host, int64_t n) = 0;
    virtual void defer(std::function<void()> fn, std::shared_ptr<void> hold) = 0;
};

// post.cpp
void postprocess(Job &job);
// render.cpp: the output as consecutive parts (formatted in parallel).
// row_base (per fold unit, may be null): global VCF row id of the unit's first row.
// on_part (may be null): called from the formatting thread as soon as part k is complete.
void render_rows(Job &job, int fmt, const int64_t *row_base, Rendered &out,
                 const std::function<void(size_t)> *on_part = nullptr);
std::vector<Text> render_parts(Job &job, int fmt);
std::string render(Job &job, int fmt);
// fasta.cpp: load_reference; with world > 1 only this rank's shard (fold units by
// longest-processing-time over the analysed lengths, shard_units) gets its bases
void load_fasta(Job &job, const char *path, int32_t flank_trim, int32_t world = 1, int32_t rank = 0,
                FastaDev *dev = nullptr);
// split multi-rank load: pass 1 over this rank's 1/world of the file -> part
// table; all ranks' tables (rank order) -> contigs, shard, own bases only
void fasta_scan_part(Job &job, const char *path, int32_t world, int32_t rank, std::vector<int64_t> &blob);
void fasta_load_parts(Job &job, const char *path, int32_t flank_trim, int32_t world, int32_t rank,
                      const int64_t *blob, int64_t nwords, FastaDev *dev = nullptr);
// fold units -> ranks by longest-processing-time greedy (deterministic; same as
// bwtmi.dist.assign): returns the contig ids owned by `rank`
std::vector<int32_t> shard_units(Job &job, int32_t world, int32_t rank);

// host threads of one process: params.threads, else this process's share of
// the CPUs it may run on (affinity mask and cgroup quota, divided among the
// LOCAL_WORLD_SIZE ranks of the node), at most 16
int host_threads(const bwtmi_params &p);
int host_cpu_budget(int *cpus_visible, int *local_world);
// Host work (the calling thread now, the worker pools from their next region)
// moves onto the CPUs of the NUMA node of local rank `local_rank`'s GPU
// (rank r drives the GPU at PCI address rank_pci[r]); asked for explicitly
// (bwtmi_bind_host: the CLI, bench and rank launcher), never by bwtmi_open.
// False when nothing changed (see plan_host_binding, post.cpp).
bool bind_host_numa(int local_rank, const std::vector<std::string> &rank_pci);
bool unbind_host();   // back to the affinity the binding replaced (calling thread now, workers at their next region)
int gpu_numa_node(const char *sysroot, const char *pci);
bool plan_host_binding(const char *sysroot, int local_rank, const std::vector<std::string> &rank_pci, int threads,
                       bool smt, const cpu_set_t &allowed, cpu_set_t &out, int *node_out, int *ranks_on_node);
std::string cpulist_str(const cpu_set_t &cs);
bool parse_cpulist(const char *txt, cpu_set_t &cs);

// ----- run-time switches (knobs.cpp): BWTMI_<NAME> read once from the
// environment, changeable in-process through bwtmi_knob_set
enum Knob {
    KN_RUNS_DENSE, KN_RUNS_UNTILED, KN_SA_SMALL, KN_SEG_LEVELS, KN_SCREEN_WIDE, KN_FM_BYTES, KN_LS_CAP,
    KN_HOST_SCREEN, KN_NO_PLAIN, KN_INDEX_LANES, KN_SCAN_LANES, KN_NO_AVX512, KN_POOL_SPIN_US,
    KN_UNIT_GROUP_THREADS, KN_STATS, KN_NUMA_BIND, KN_NUMA_SMT, KN_FAIL_MERGE_CHUNK, KN_HIST_S, KN_DEVICE_CHECKS,
    KN_SCREEN_DROP, KN_COUNT
};
// a roctx range for the lifetime of the object (trace.cpp); names "bwtmi:<stage>"
struct StageRange {
    explicit StageRange(const char *name);
    ~StageRange();
    StageRange(const StageRange &) = delete;
    StageRange &operator=(const StageRange &) = delete;
};
#define BWTMI_STAGE(name) ::bwtmi::StageRange bwtmi_stage_range_(name)

extern std::atomic<int64_t> g_knobs[KN_COUNT];
inline int64_t knob(Knob k) { return g_knobs[k].load(std::memory_order_relaxed); }
inline bool stats_on(int level = 1) { return knob(KN_STATS) >= level; }
// the pool's spin window when BWTMI_POOL_SPIN_US is -1 (auto), set from the
// size of the job that calls in (post.cpp): short regions with short serial
// gaps between them (a shard) keep their workers spinning longer
void pool_spin_for_job(const Job &job);
int64_t fasta_count_records(const char *path, int64_t limit);   // fasta.cpp
// fn(task) for task in [0, n) on up to nt threads (dynamic scheduling)
void run_tasks(int64_t n, int nt, const std::function<void(int64_t)> &fn);

}  // namespace bwtmi
