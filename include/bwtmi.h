/*
 * bwtmi.h -- C ABI of libbwtmi.so, the MI355X-native (gfx950) BWT/FM-index and
 * tandem-repeat engine behind the `bwt.py` drop-in surface.
 *
 * The reference (wyim-pgl/bwt-algorithm, bwt.py) is pure Python and has no
 * FFI; its "interface" is the Python names listed below.  Each entry point
 * here replaces the body of one of those names; the Python host
 * (bwt-algorithm_amd/bwtmi) keeps the names and binds these symbols with
 * ctypes.
 *
 * Conventions
 *   - every function returns 0 on success, a negative BWTMI_E* code on error;
 *     bwtmi_last_error() returns the thread-local message of the last error.
 *   - inputs are caller-owned and only borrowed for the duration of a call;
 *     outputs allocated by the library are released with bwtmi_free() or the
 *     matching *_free().
 *   - one bwtmi_ctx per device; calls on one ctx are serialised by the caller.
 *     HIP is not fork-safe: never fork() after bwtmi_open().
 *   - there is no CPU fallback: without a usable gfx950 device bwtmi_open()
 *     fails with BWTMI_E_NODEVICE.
 */
#ifndef BWTMI_H
#define BWTMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BWTMI_OK 0
#define BWTMI_E_ARG (-1)
#define BWTMI_E_NODEVICE (-2)
#define BWTMI_E_HIP (-3)
#define BWTMI_E_NOMEM (-4)
#define BWTMI_E_STATE (-5)
#define BWTMI_E_IO (-6)

typedef struct bwtmi_ctx bwtmi_ctx;
typedef struct bwtmi_index bwtmi_index;
typedef struct bwtmi_job bwtmi_job;

/* ------------------------------------------------------------ context */
const char *bwtmi_last_error(void);
/* "bwtmi 0.5 (gfx950) src <sha256>": the sources the library was built from */
const char *bwtmi_version(void);
/* sha256 (hex) of the csrc sources (.cpp, .h, .hip) and include/bwtmi.h, concatenated in
 * byte order of their paths, computed by the Makefile at build time: a test
 * or launcher compares it with the tree it runs from (bwtmi._lib.check_build) */
const char *bwtmi_source_hash(void);
int bwtmi_device_count(int *count);
int bwtmi_open(int device, bwtmi_ctx **out);
int bwtmi_close(bwtmi_ctx *ctx);
/* Host placement, asked for explicitly (the CLI, bench.py and the rank
 * launcher do; bwtmi_open never does unless BWTMI_NUMA_BIND=1): on=1 moves
 * this process's host work -- the calling thread now, the library's worker
 * threads at their next parallel region -- onto the CPUs of the NUMA node of
 * ctx's GPU; on=0 restores the affinity the binding replaced.  *changed = 1
 * when the placement changed.  Local rank r (LOCAL_RANK / LOCAL_WORLD_SIZE)
 * drives device r mod (visible devices); the ranks whose GPUs share this
 * node decide whether one hardware thread per core is taken.  A second
 * context on another node leaves the first binding in place. */
int bwtmi_bind_host(bwtmi_ctx *ctx, int on, int *changed);
/* The CPU set bwtmi_bind_host would choose, without changing anything: sysfs
 * read under `sysroot` ("/sys" on a host; a faked tree in the tests), local
 * rank `local_rank` of the ranks whose GPUs have the comma-separated PCI
 * addresses `rank_pci` (rank order), `threads` host threads per rank, `smt`
 * = keep sibling hardware threads, `allowed` = the process's affinity as a
 * cpulist.  out = the chosen cpulist ("" = no binding); *node = this GPU's
 * NUMA node, *ranks_on_node = local ranks whose GPUs sit on it. */
int bwtmi_host_binding_plan(const char *sysroot, int local_rank, const char *rank_pci, int threads, int smt,
                            const char *allowed, char *out, int64_t cap, int *node, int *ranks_on_node);
/* Run-time switches (INTEGRATION.md "Run-time switches"): BWTMI_<NAME> read
 * once from the environment; get/set in-process by NAME (with or without the
 * BWTMI_ prefix).  Unknown names: BWTMI_E_ARG.  bwtmi_knob_names(): all names,
 * comma-separated. */
/* roctx ranges (rocprofv3 --marker-trace): the library opens "bwtmi:<stage>"
 * around load, upload, scan, index, merge, refine..filter, compounds, format,
 * write and index_wait; a host application can nest its own with these. */
int bwtmi_trace_push(const char *name);
int bwtmi_trace_pop(void);
int bwtmi_knob_set(const char *name, int64_t value);
int bwtmi_knob_get(const char *name, int64_t *value);
int bwtmi_knob_default(const char *name, int64_t *value);
const char *bwtmi_knob_names(void);
void bwtmi_free(void *p);
/* time (ms) of the kernels of the last call on ctx, measured with HIP events
 * on the ctx stream: [0]=total device, [1]=dominant kernel, [2]=its launches */
int bwtmi_last_timing(bwtmi_ctx *ctx, double *out3);

/* per-kernel HIP-event timing on the ctx stream: enable=1 starts collecting,
 * the call writes "name ms launches\n" lines of everything collected so far
 * into out (cap bytes, NUL-terminated) and resets when reset=1 */
int bwtmi_kernel_stats(bwtmi_ctx *ctx, int enable, int reset, char *out, int64_t cap);
/* time only the launches named `name` (NULL or "": every launch); the others
 * then run without event records between them */
int bwtmi_kernel_stats_filter(bwtmi_ctx *ctx, const char *name);

/* ------------------------------------------------------------ strict scan
 * Replaces Tier2LCPFinder.find_long_unit_repeats_strict (bwt.py:1891-2001),
 * as called by _process_chromosome_worker (bwt.py:3103-3106).
 * seq: ASCII bases of one (trimmed) contig; a single trailing '$' is ignored
 * (bwt.py:1915-1916).  Hits come out in the reference's emission order
 * (unit_len descending, start ascending).  prim_len = smallest_period_str of
 * the first unit (bwt.py:1956); copies = count after primitive reduction
 * (bwt.py:1957-1961).  max_mismatch 0 is the CLI value; > 0 compares adjacent
 * L-blocks by Hamming distance <= max_mismatch (bwt.py:1929-1944, library calls). */
typedef struct {
    int64_t start;
    int64_t end;
    int32_t unit_len;
    int32_t prim_len;
    int64_t copies;
} bwtmi_hit;

int bwtmi_strict_scan(bwtmi_ctx *ctx, const uint8_t *seq, int64_t n, int32_t min_unit,
                      int32_t max_unit, int32_t max_mismatch, int32_t min_copies,
                      bwtmi_hit **hits, int64_t *nhits);

/* ------------------------------------------------------------ FM index
 * Replaces BWTCore.__init__ (bwt.py:106-136): suffix array (212-264), BWT
 * (266-274), C table (276-286), Occ checkpoints (288-326), sampled SA
 * (328-333) and the 8-mer hash (138-171).  text includes the sentinel, exactly
 * as the reference receives it (seq + '$'). */
#define BWTMI_INDEX_NO_KMER 1u

int bwtmi_index_build(bwtmi_ctx *ctx, const uint8_t *text, int64_t n, int32_t sa_sample,
                      int32_t occ_sample, uint32_t flags, bwtmi_index **out);
int bwtmi_index_free(bwtmi_index *idx);
int64_t bwtmi_index_size(const bwtmi_index *idx);
int bwtmi_index_get_sa(const bwtmi_index *idx, int32_t *sa /* n */);
int bwtmi_index_get_bwt(const bwtmi_index *idx, uint8_t *bwt /* n */);
/* totals[256] and cumulative C[256] over byte values (absent bytes: total 0) */
int bwtmi_index_get_counts(const bwtmi_index *idx, int64_t *totals, int64_t *C);
/* checkpoints of one byte code; length = 1 + n/occ + (n%occ != 0) */
int64_t bwtmi_index_occ_len(const bwtmi_index *idx);
int bwtmi_index_get_occ(const bwtmi_index *idx, uint8_t code, int32_t *cp);
/* sampled SA (bwt.py:328-333): values SA[i] for i = 0, s, 2s, ... */
int64_t bwtmi_index_sampled_len(const bwtmi_index *idx);
int bwtmi_index_get_sampled(const bwtmi_index *idx, int32_t *vals);
/* 8-mer hash as CSR: offsets[65537], positions[offsets[65536]] */
int64_t bwtmi_index_kmer_count(const bwtmi_index *idx);
int bwtmi_index_get_kmer(const bwtmi_index *idx, int64_t *offsets, int32_t *positions);
/* Kasai LCP over the index text (bwt.py:56-95, 2108-2116), int32[n] */
int bwtmi_index_lcp(bwtmi_ctx *ctx, bwtmi_index *idx, int32_t *lcp);
/* Library finders of Tier2LCPFinder over an index (not on the CLI path). */
typedef struct {
    int32_t min_period;        /* Tier2LCPFinder(min_period=1, max_period=1000, max_short_motif=9) */
    int32_t max_period;
    int32_t max_short_motif;
    int32_t min_copies;        /* self.min_copies = 3 (bwt.py:1880) */
    int32_t min_array_length;  /* 6 (bwt.py:1881) */
    int32_t allow_mismatches;
    double min_entropy;        /* 1.0 (bwt.py:1882) */
} bwtmi_lib_params;
/* _detect_lcp_plateaus over the index's Kasai LCP (bwt.py:2118-2145, 2500-2560):
 * *out = (start, copies, period) triples in the reference's order (free with bwtmi_free) */
int bwtmi_index_lcp_plateaus(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p, int64_t **out,
                             int64_t *n);
/* find_short_imperfect_repeats(chromosome, tier1_seen) (bwt.py:2027-2095, 2562-2825): the
 * records are appended to job's final records with contig contig_id, whose sequence must be
 * the index text; seen = nseen (start, end) pairs (tier1_seen) */
int bwtmi_index_short_imperfect(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p,
                                const int64_t *seen, int64_t nseen, bwtmi_job *job, int32_t contig_id);
/* find_long_repeats(chromosome, tier1_seen) -> _find_repeats_simple (bwt.py:2097-2106,
 * 2177-2498): adaptive period/position scan with majority-vote extension; records appended to
 * job's final records with contig contig_id (the reference's extra 30 s wall-clock stop,
 * bwt.py:2238-2257, is not reproduced; its 100,000-iteration cap is) */
int bwtmi_index_long_repeats(bwtmi_ctx *ctx, bwtmi_index *idx, const bwtmi_lib_params *p,
                             const int64_t *seen, int64_t nseen, bwtmi_job *job, int32_t contig_id);
/* Tier1STRFinder(text_arr, max_motif_length).find_strs (bwt.py:1426-1538) over the full
 * sequence of the job's contig contig_id; records appended to the job's final records */
int bwtmi_job_tier1(bwtmi_ctx *ctx, bwtmi_job *job, int32_t contig_id, int32_t max_motif_length);
/* Tier3LongReadFinder(bwt_core).find_very_long_repeats(long_reads, chromosome) (bwt.py:2837-3036)
 * over the index (built over seq + '$'): reads = the reads' bytes back to back, read_off[nreads + 1]
 * their offsets (read_off[0] = 0).  The consolidated records get contig contig_id and go
 *   as_input = 0: to the job's final records (the library call's return value);
 *   as_input = 1: to the job's Tier 3 input of that contig, which bwtmi_job_postprocess joins after
 *                 the contig's strict hits before nested suppression (find_tandem_repeats_parallel,
 *                 bwt.py:3917-3924); call after bwtmi_job_reset and before bwtmi_job_scan. */
int bwtmi_index_tier3(bwtmi_ctx *ctx, bwtmi_index *idx, const uint8_t *reads, const int64_t *read_off,
                      int64_t nreads, bwtmi_job *job, int32_t contig_id, int32_t as_input);
/* BWTCore.backward_search (bwt.py:359-389) for npat patterns packed in pats,
 * pattern p = pats[off[p] .. off[p+1]).  Writes sp_ep[2p], sp_ep[2p+1]
 * (inclusive interval, or -1,-1). */
int bwtmi_backward_search_batch(bwtmi_ctx *ctx, bwtmi_index *idx, const uint8_t *pats,
                                const int64_t *off, int64_t npat, int64_t *sp_ep);

/* ------------------------------------------------------------ repeat job
 * Replaces the per-contig worker result handling and the post-processing of
 * TandemRepeatFinder (bwt.py:3040-3141, 3402-3944) and save_results with
 * compound detection and the five writers (bwt.py:454-641, 3995-4198). */
typedef struct {
    int32_t min_copies;     /* --min-copies (default 3) */
    int32_t max_unit_len;   /* --max-unit-len (default 120) */
    int32_t show_progress;  /* --progress: lifts the >50 Mbp Tier-2 gate (bwt.py:3070) */
    int32_t tier2;          /* 0 when --tier1 (bwt.py:4257-4259) */
    int32_t threads;        /* host threads for post-processing (0 = auto) */
    int32_t build_index;    /* also build the FM index per contig in bwtmi_job_scan, as the
                               reference worker does (bwt.py:3053-3054); 0 = skip */
    int32_t sa_sample;      /* --sa-sample (default 32) */
    int32_t reserved;
} bwtmi_params;

#define BWTMI_FMT_STRFINDER 0
#define BWTMI_FMT_BED 1
#define BWTMI_FMT_VCF 2
#define BWTMI_FMT_TRF_TABLE 3
#define BWTMI_FMT_TRF_DAT 4

int bwtmi_job_create(const bwtmi_params *params, bwtmi_job **out);
int bwtmi_job_free(bwtmi_job *job);
/* register a contig: name, the full (untrimmed, upper-cased) sequence and the
 * trim offset; the analysed sequence is full[trim : full_len - trim_right]. */
int bwtmi_job_add_contig(bwtmi_job *job, const char *name, const uint8_t *full, int64_t full_len,
                         int64_t trim_left, int64_t trim_right, int32_t *contig_id);
/* run the worker on every registered contig on ctx's device (strict scan,
 * gates, Rule-1 filter) -- equivalent to find_tandem_repeats(_parallel) up to
 * all_repeats (bwt.py:3792-3822, 3850-3915) */
int bwtmi_job_scan(bwtmi_ctx *ctx, bwtmi_job *job);
/* the FM index builds of bwtmi_job_scan (build_index) run on the device behind
 * the host post-processing; this joins them (every other call on ctx, and
 * bwtmi_job_free, joins them too) and returns their error, if any */
int bwtmi_job_wait(bwtmi_ctx *ctx, bwtmi_job *job);
/* copy every contig to device memory now (bwtmi_job_scan does it on first use);
 * later scans reuse the resident copies */
int bwtmi_job_upload(bwtmi_ctx *ctx, bwtmi_job *job);
/* drop raw / final records so the job can be scanned again */
int bwtmi_job_reset(bwtmi_job *job);
int bwtmi_job_set_params(bwtmi_job *job, const bwtmi_params *params);
/* restrict bwtmi_job_scan to the listed contigs (this rank's shard); n < 0 = all */
int bwtmi_job_select(bwtmi_job *job, const int32_t *ids, int32_t n);
/* alternatively feed raw hits computed elsewhere (one contig at a time) */
int bwtmi_job_add_hits(bwtmi_job *job, int32_t contig_id, const bwtmi_hit *hits, int64_t n);
int64_t bwtmi_job_raw_count(const bwtmi_job *job);
/* nested suppression .. final filter (bwt.py:3926-3944) */
int bwtmi_job_postprocess(bwtmi_job *job);
int64_t bwtmi_job_count(const bwtmi_job *job);
/* render a format into a malloc'd buffer (free with bwtmi_free) or a file */
int bwtmi_job_render(bwtmi_job *job, int fmt, char **out, int64_t *len);
int bwtmi_job_write(bwtmi_job *job, int fmt, const char *path);
/* bwtmi_job_write returning once every row is formatted: the job's writer
 * thread finishes the file behind the caller (the header and each run of
 * formatted rows are written as they complete, in file order).
 * bwtmi_job_write_join waits for it and returns its error (BWTMI_E_IO: the file
 * is cut to 0 bytes); the job's next write or write_async, and bwtmi_job_free,
 * join it first (free drops the error).  Not in the reference: a caller that
 * writes one file per job (bwt.py:4141-4198) can overlap the file's tail with
 * its next job's load and scan. */
int bwtmi_job_write_async(bwtmi_job *job, int fmt, const char *path);
int bwtmi_job_write_join(bwtmi_job *job);
/* Sharded output (one process per GPU, each owning whole fold units = contigs
 * with equal natural sort keys, bwt.py:22-36): the file is the concatenation,
 * in unit order, of every unit's rows (bwt.py:4147-4150), so each rank writes
 * its own units at offsets from an exchange of sizes -- no record gather.
 *   unit_count              number of fold units (same on every rank)
 *   unit_rows[u]            local final records of unit u (VCF row ids)
 *   render_units            format the local units; bytes[0] = header size,
 *                           bytes[1 + u] = size of unit u (0 if not local);
 *                           row_base[u] = global VCF id of unit u's first row
 *                           (NULL: local numbering)
 *   write_units             pwrite the rendered units into `path` (opened
 *                           without truncation) at offsets[1 + u]; the header
 *                           at offsets[0] when write_header */
int32_t bwtmi_job_unit_count(bwtmi_job *job);
int bwtmi_job_unit_rows(bwtmi_job *job, int64_t *unit_rows);
int bwtmi_job_render_units(bwtmi_job *job, int fmt, const int64_t *row_base, int64_t *bytes);
int bwtmi_job_write_units(bwtmi_job *job, const char *path, const int64_t *offsets, int write_header);
/* the same behind the caller (the job's thread pwrites the rendered units);
 * bwtmi_job_write_join waits for it and returns its error */
int bwtmi_job_write_units_async(bwtmi_job *job, const char *path, const int64_t *offsets, int write_header);
/* final records as rows of int64: start, end, length, tier, n_copies_eval,
 * max_mm, score, flags (1: composition None / entropy 0.0, 2: k-mer scan piece),
 * chrom_id and doubles: copies, mismatch_rate, confidence, percent_matches,
 * percent_indels (for tests / the Python record view) */
int bwtmi_job_get_records(bwtmi_job *job, int64_t *ints9, double *dbls5);
/* strings of record i: which = 0 motif, 1 consensus, 2 variations(';'-joined),
 * 3 actual_sequence, 4 strand; returns length, copies up to cap bytes */
int64_t bwtmi_job_get_string(bwtmi_job *job, int64_t i, int which, char *buf, int64_t cap);
/* string `which` of every record, concatenated: offsets[0..count] (count + 1
 * entries, when offsets != NULL) and the bytes into buf when buf != NULL and
 * cap >= the total; returns the total byte count (-1: bad argument).  One
 * call per column for the Python record view instead of one per record. */
int64_t bwtmi_job_get_strings(bwtmi_job *job, int which, char *buf, int64_t cap, int64_t *offsets);
/* serialise final records for a gather to another rank; import appends them */
int bwtmi_job_export(bwtmi_job *job, uint8_t **buf, int64_t *len);
int bwtmi_job_import(bwtmi_job *job, const uint8_t *buf, int64_t len);
/* replace the final records by a serialised list (bwtmi_job_export's format;
 * save_results over a caller-built list of records, bwt.py:4141-4198);
 * bwtmi_wire_record_size = size of one fixed record header in that format */
int bwtmi_job_set_records(bwtmi_job *job, const uint8_t *buf, int64_t len);
int bwtmi_wire_record_size(void);
/* the worker's error of contig id in the last bwtmi_job_scan (0 = none): a
 * failing contig yields no records and the others go on, as the reference's
 * `except Exception: print("ERROR processing chromosome ..."); return []`
 * (bwt.py:3137-3141); copies the message, returns its length */
int64_t bwtmi_job_contig_error(const bwtmi_job *job, int32_t id, char *buf, int64_t cap);
/* per-stage wall times (ms) of the last scan/postprocess/render calls */
int bwtmi_job_stage_ms(const bwtmi_job *job, double *out8);

/* Shard layout over ranks (replaces the Pool over contigs, bwt.py:3850-3912):
 * fold units (contigs with equal natural sort keys, bwt.py:22-36) go to ranks
 * by longest-processing-time greedy over their analysed lengths (ties: lower
 * unit, then lower rank).  Restricts the job to rank's contigs; ids (may be
 * NULL, else room for every contig) receives them ascending, n their count. */
int bwtmi_job_select_shard(bwtmi_job *job, int32_t world, int32_t rank, int32_t *ids, int32_t *n);

/* host CPUs this process may use (affinity mask, cgroup quota), the ranks on
 * this node (LOCAL_WORLD_SIZE) and the post-processing threads per rank that
 * follow from them (threads = 0 in bwtmi_params) */
int bwtmi_host_info(int32_t *cpus_visible, int32_t *local_world, int32_t *threads);

/* ------------------------------------------------------------ collective
 * The multi-GPU path's only exchange: RCCL (over xGMI) all-reduce of small
 * host vectors -- per-unit row / byte counts for the sharded output file and
 * the step time.  librccl is loaded on first use.  The 128-byte id comes from
 * bwtmi_comm_unique_id on one rank and reaches the others out of band
 * (bwtmi/comm.py: a TCP rendezvous next to MASTER_ADDR:MASTER_PORT). */
typedef struct bwtmi_comm bwtmi_comm;
int bwtmi_comm_unique_id(uint8_t *id /* 128 bytes */);
int bwtmi_comm_init(int32_t device, int32_t world, int32_t rank, const uint8_t *id, bwtmi_comm **out);
/* in place over `count` host values; dtype 0 = int64, 1 = float64; op 0 = sum, 1 = max */
int bwtmi_comm_allreduce(bwtmi_comm *comm, void *vals, int64_t count, int32_t dtype, int32_t op);
int bwtmi_comm_free(bwtmi_comm *comm);
/* hipDeviceSynchronize on device (bench step brackets) */
int bwtmi_device_sync(int32_t device);

/* ------------------------------------------------------------ helpers
 * MotifUtils.align_repeat_region (bwt.py:998-1102) -- the banded per-copy
 * alignment used by merge/refine; exposed for the Python MotifUtils mirror.
 * max_indel < 0 means None.  Returns 1 with a summary, 0 for None.
 * ints8: copies, motif_len, consumed, max_errors, tot_ins, tot_del, 0, 0;
 * mismatch_rate; consensus (motif_len bytes) and variations (';'-joined,
 * malloc'd, free with bwtmi_free); copy_len/copy_err (malloc'd int64[copies]). */
int bwtmi_align_region(const char *seq, int64_t seq_len, int64_t start, int64_t end, const char *tmpl,
                       int64_t tmpl_len, double frac, int64_t max_indel, int64_t min_copies,
                       int64_t *ints8, double *mismatch_rate, char *consensus, char **variations,
                       int64_t **copy_len, int64_t **copy_err);
/* ------------------------------------------------------------ FASTA
 * TandemRepeatFinder.load_reference (bwt.py:3713-3756) natively: strip,
 * '>' headers (name = first whitespace token), upper-case sequence lines,
 * blank lines skipped, duplicate names overwrite in place.  Registers every
 * contig in job (trim = flank_trim if len > 2*flank_trim). */
int bwtmi_job_load_fasta(bwtmi_job *job, const char *path, int32_t flank_trim);
/* bwtmi_job_load_fasta + bwtmi_job_upload for a whole file, with the analysed
 * sequences built on ctx's device from the file image: its copy to the device
 * overlaps the loader's first pass, the plain chunks (whole lines of
 * 0x21..0x7f bytes other than '>') are rebuilt there (fasta_dev.hip), and the
 * host copies of those chunks are written behind the device work -- complete
 * when the next bwtmi_job_scan returns, or when any other call on the job
 * reads contig bytes (bwtmi_job_contig_seq, postprocess, render, ...).
 * Replaces the same load_reference (bwt.py:3713-3756) as bwtmi_job_load_fasta. */
int bwtmi_job_load_fasta_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t flank_trim);
/* the device copy of contig `id`'s analysed (trimmed) sequence into dst
 * (trimmed_len bytes); fails when it is not resident on ctx's device */
int bwtmi_job_device_text(bwtmi_ctx *ctx, bwtmi_job *job, int32_t id, uint8_t *dst);
/* the same for rank `rank` of `world` processes: every contig is registered
 * (names and analysed lengths, for the shard layout), but only the fold units
 * this rank owns (bwtmi_job_select_shard) get their bases, and the job is
 * restricted to them */
int bwtmi_job_load_fasta_shard(bwtmi_job *job, const char *path, int32_t flank_trim, int32_t world,
                               int32_t rank);
/* Split multi-rank load (no rank reads the whole file): rank r runs the
 * loader's first pass over its 1/world of the file and returns a part table
 * (int64 words, freed with bwtmi_free); the ranks exchange the tables (an
 * all-gather, bwtmi.comm); bwtmi_job_load_fasta_parts takes all of them in
 * rank order, builds the contig table (names, lengths, trims, fold units --
 * identical on every rank), restricts the job to this rank's shard and reads
 * only those contigs' bytes.  A non-ASCII byte anywhere fails every rank.
 * Replaces load_reference (bwt.py:3713-3756) + the contig split of 3850-3912. */
int bwtmi_job_fasta_scan_part(bwtmi_job *job, const char *path, int32_t world, int32_t rank, int64_t **blob,
                              int64_t *nwords);
/* the same, and the part's bytes go up to ctx's device at once: a following
 * bwtmi_job_load_fasta_parts_dev on that ctx whose contigs lie inside the part
 * skips their copy (it overlapped the part-table exchange) */
int bwtmi_job_fasta_scan_part_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t world, int32_t rank,
                                  int64_t **blob, int64_t *nwords);
/* header lines of a FASTA file ('>' at the start or after a line break),
 * counted up to limit; -1 if it cannot be read.  Host only (no device is
 * touched): the CLI's decision to launch one rank per GPU (bwt.py:3863-3864's
 * Pool size) before anything initialises a GPU */
int64_t bwtmi_fasta_count_records(const char *path, int64_t limit);
int bwtmi_job_load_fasta_parts(bwtmi_job *job, const char *path, int32_t flank_trim, int32_t world, int32_t rank,
                               const int64_t *blob, int64_t nwords);
/* the same with this rank's analysed sequences built on ctx's device
 * (bwtmi_job_load_fasta_dev's placement: plain chunks rebuilt there from the
 * own contigs' bytes, host copies written behind the next scan) */
int bwtmi_job_load_fasta_parts_dev(bwtmi_ctx *ctx, bwtmi_job *job, const char *path, int32_t flank_trim,
                                   int32_t world, int32_t rank, const int64_t *blob, int64_t nwords);
int32_t bwtmi_job_contig_count(const bwtmi_job *job);
/* analysed length of contig id (its shard weight), also for contigs whose bases
 * live on another rank */
int64_t bwtmi_job_contig_weight(const bwtmi_job *job, int32_t id);
int64_t bwtmi_job_contig_info(const bwtmi_job *job, int32_t id, char *name, int64_t cap,
                              int64_t *full_len, int64_t *trim_left, int64_t *trim_right);
int bwtmi_job_contig_seq(const bwtmi_job *job, int32_t id, uint8_t *dst /* full_len */);

#ifdef __cplusplus
}
#endif
#endif /* BWTMI_H */
