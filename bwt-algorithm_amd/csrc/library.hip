// library.hip -- the reference's library finders that are not on the CLI path
// (SURVEY.md §8(a) A2-9 and A2-10), over a device FM index.
//
// LCP plateaus (Tier2LCPFinder._detect_lcp_plateaus, bwt.py:2118-2145, with
// _analyze_sa_interval_for_tandems 2500-2549 and _validate_periodicity_arr
// 2551-2560): device Kasai LCP -> run flags at thr = max(min_period,
// min(max_period, max LCP, 20)) -> one stable radix sort of (run, SA value)
// keys gives every run's sorted positions in run order -> one thread per
// position counts its arithmetic progression of step thr and validates the
// periodicity of text[p, p + copies*thr) -> compaction in that order.
//
// Short imperfect repeats (Tier2LCPFinder.find_short_imperfect_repeats,
// bwt.py:2027-2095 -> _find_tandems_fm_with_mismatches 2562-2695 ->
// _extend_tandem_fm 2697-2805).  The extension of a candidate depends only on
// (candidate start, unit length): k_extend computes it for EVERY start and
// every unit length 1..9 at once (inputs are <= 1 Mbp), keeping per-column
// symbol counts so each added copy costs O(unit) instead of re-voting all
// copies (majority vote = np.unique + argmax: smallest byte among the most
// frequent; Hamming total and transversions follow from the counts).  The
// order-dependent part -- seeds from the k-mer table / FM locate per motif in
// enumerate_motifs order, the seen-region test, best-shift choice, primitive
// reduction (whose motif_len persists for later seeds, as in the reference),
// maximality, match-rate filter, variations -- runs on the host over that table.
#include <hip/hip_runtime.h>

#include <chrono>
#include <mutex>

#include <algorithm>
#include <array>
#include <map>
#include <memory>
#include <set>
#include <tuple>
#include <unordered_map>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kB = 256;
constexpr int kMaxUnit = 9;   // enumerate_motifs range ends at 9 (bwt.py:2052)

inline unsigned blocks(int64_t n) { return (unsigned)((n + kB - 1) / kB); }

// ------------------------------------------------------------- LCP plateaus
__global__ void k_max_i32(const int32_t *__restrict__ a, int64_t n, int *__restrict__ out) {
    int v = 0;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) v = max(v, a[i]);
    __shared__ int red[kB];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = kB / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(out, red[0]);
}

__global__ void k_plateau_flags(const int32_t *__restrict__ lcp, int64_t n, int32_t thr, uint32_t *__restrict__ inrun,
                                uint32_t *__restrict__ head) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const bool in = lcp[i] >= thr;
    inrun[i] = in ? 1u : 0u;
    head[i] = (in && (i == 0 || lcp[i - 1] < thr)) ? 1u : 0u;
}

__global__ void k_plateau_keys(const uint32_t *__restrict__ sa, const uint32_t *__restrict__ inrun,
                               const uint32_t *__restrict__ head, const uint32_t *__restrict__ hscan,
                               const uint32_t *__restrict__ cpos, int64_t n, uint64_t *__restrict__ keys) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n || !inrun[i]) return;
    const uint64_t run = (uint64_t)(hscan[i] + head[i] - 1);
    keys[cpos[i]] = (run << 32) | (uint64_t)sa[i];
}

// one sorted position of one run: progression length and periodicity test
__global__ void k_plateau_eval(const uint64_t *__restrict__ keys, int64_t m, const uint8_t *__restrict__ t, int64_t n,
                               int64_t thr, int64_t mc, uint32_t *__restrict__ flag, int64_t *__restrict__ copies) {
    const int64_t a = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (a >= m) return;
    const uint64_t run = keys[a] >> 32;
    const int64_t sp = (int64_t)(keys[a] & 0xffffffffull);
    int64_t c = 1;
    for (int64_t b = a + 1; b < m && (keys[b] >> 32) == run && (int64_t)(keys[b] & 0xffffffffull) == sp + c * thr; ++b)
        ++c;
    bool ok = false;
    if (c >= mc && sp + thr <= n) {
        const int64_t len = min(c * thr, n - sp);   // text[sp : sp + copies*thr]
        if (len >= 2 * thr) {
            int64_t match = 0;
            for (int64_t q = 0; q < len; ++q) match += t[sp + q] == t[sp + q % thr];
            ok = (double)match / (double)len >= 0.8;
        }
    }
    flag[a] = ok ? 1u : 0u;
    copies[a] = c;
}

__global__ void k_plateau_out(const uint64_t *__restrict__ keys, const uint32_t *__restrict__ flag,
                              const uint32_t *__restrict__ pos, const int64_t *__restrict__ copies, int64_t m,
                              int64_t thr, int64_t *__restrict__ out) {
    const int64_t a = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (a >= m || !flag[a]) return;
    int64_t *o = out + 3 * (int64_t)pos[a];
    o[0] = (int64_t)(keys[a] & 0xffffffffull);
    o[1] = copies[a];
    o[2] = thr;
}

// --------------------------------------------------------- seed extension
__device__ __host__ inline bool transversion(uint8_t a, uint8_t b) {   // count_transversions_array, 781-800
    if (a == b) return false;
    const uint8_t x = (a >= 65 && a <= 84) ? a : (uint8_t)'N', y = (b >= 65 && b <= 84) ? b : (uint8_t)'N';
    if (x == y) return false;   // is_transition(c, c) is True
    if ((x == 'A' && y == 'G') || (x == 'G' && y == 'A') || (x == 'C' && y == 'T') || (x == 'T' && y == 'C'))
        return false;
    return true;
}

__device__ __host__ inline int64_t max_mm_for_array(int64_t L, int64_t copies) {   // bwt.py:2003-2025
    const int64_t total = L * copies;
    if (L == 1) return 0;
    if (L <= 6) return max((int64_t)1, (int64_t)ceil(0.05 * (double)total));
    return max((int64_t)1, (int64_t)ceil(0.08 * (double)total));
}

// _extend_tandem_fm(text, cs, text[cs:cs+L], L) for every cs and L = 1..Lmax,
// with every column's symbol counts in registers: 5 bins
// per column in byte order (A C G N T, so a strict > scan over the bins keeps
// the smallest byte among the most frequent -- np.unique + argmax), and the
// copy's mismatches / transversions from the counts alone: a column with
// majority count b adds tc - b mismatches and the counts of the bins that are
// transversions of its consensus (count_transversions_array: A<->G and C<->T
// are transitions, every other pair of distinct symbols in 65..84 -- N
// included -- is not).  A copy costs O(L), never a re-vote of earlier copies,
// and nothing spills to scratch.  Any other byte (e.g. the final '$') sends
// the entry to the host's scalar extension.
//
// Output per (start cs, unit L), entry q = (L - 1) n + cs: one 32-bit word =
// copies added on the left | copies added on the right << 16; 0xffffffff =
// no extension (cs + L > n); a count past 0xfffe (long homopolymers) or an
// unbinned symbol writes 0xfffffffe and appends (q, left, right, unbinned) to
// a side list.  The host reads 4 bytes per entry instead of 13.
constexpr uint32_t kExtNone = 0xffffffffu, kExtSide = 0xfffffffeu;
struct ExtSide {
    int64_t q;
    uint32_t left, right;
    uint32_t unbinned, pad;
};

__device__ __forceinline__ int ext_bin(uint8_t b) {
    switch (b) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'N': return 3;
        case 'T': return 4;
        default: return -1;
    }
}

__global__ __launch_bounds__(256) void k_extend_cols(const uint8_t *__restrict__ t, int64_t n, int Lmax,
                                                     uint32_t *__restrict__ word, ExtSide *__restrict__ side,
                                                     unsigned long long *__restrict__ nside, int64_t side_cap) {
    // bins of the transversions of consensus bin x (A C G N T)
    constexpr uint32_t kTv[5] = {0x1au, 0x0du, 0x1au, 0x17u, 0x0du};
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (int64_t)Lmax * n) return;
    const int L = (int)(tid / n) + 1;
    const int64_t cs = tid - (int64_t)(L - 1) * n;
    if (cs + L > n) {
        word[tid] = kExtNone;
        return;
    }
    uint32_t cnt[kMaxUnit][5];
    bool ok = true;
#pragma unroll
    for (int p = 0; p < kMaxUnit; ++p) {
#pragma unroll
        for (int b = 0; b < 5; ++b) cnt[p][b] = 0;
        if (p < L) {
            const int b = ext_bin(t[cs + p]);
            if (b < 0) ok = false;
#pragma unroll
            for (int q = 0; q < 5; ++q) cnt[p][q] = q == b ? 1u : 0u;   // no dynamic index: registers only
        }
    }
    // try copy at `at`: add it, evaluate, keep or take it back
    auto try_copy = [&](int64_t at, uint32_t tc) -> bool {
        int bins[kMaxUnit];
        bool homo = L > 1;
        const uint8_t c0 = t[at];
#pragma unroll
        for (int p = 0; p < kMaxUnit; ++p) {
            bins[p] = 0;
            if (p < L) {
                const uint8_t c = t[at + p];
                homo = homo && c == c0;
                bins[p] = ext_bin(c);
            }
        }
        if (homo) return false;   // the next copy is a homopolymer
        int64_t mm = 0, tv = 0;
#pragma unroll
        for (int p = 0; p < kMaxUnit; ++p) {
            if (p < L) {
                if (bins[p] < 0) {
                    ok = false;
                    return false;
                }
#pragma unroll
                for (int b = 0; b < 5; ++b) cnt[p][b] += b == bins[p] ? 1u : 0u;
                uint32_t best = 0;
                int cb = 0;
#pragma unroll
                for (int b = 0; b < 5; ++b)
                    if (cnt[p][b] > best) {
                        best = cnt[p][b];
                        cb = b;
                    }
                mm += (int64_t)(tc - best);
#pragma unroll
                for (int b = 0; b < 5; ++b)
                    if ((kTv[cb] >> b) & 1u) tv += cnt[p][b];
            }
        }
        if (mm <= max_mm_for_array(L, tc) && tv == 0) return true;
#pragma unroll
        for (int p = 0; p < kMaxUnit; ++p)
            if (p < L) {
#pragma unroll
                for (int b = 0; b < 5; ++b) cnt[p][b] -= b == bins[p] ? 1u : 0u;
            }
        return false;
    };
    uint32_t copies = 1, right = 0, left = 0;
    int64_t start = cs, end = cs + L;
    if (ok) {
        while (end + L <= n && try_copy(end, copies + 1)) {
            ++copies;
            ++right;
            end += L;
        }
    }
    if (ok) {
        while (start - L >= 0 && try_copy(start - L, copies + 1)) {
            ++copies;
            ++left;
            start -= L;
        }
    }
    if (ok && left < 0xffffu && right < 0xffffu) {
        word[tid] = left | (right << 16);
        return;
    }
    word[tid] = kExtSide;
    const unsigned long long k = atomicAdd(nside, 1ull);
    if ((int64_t)k < side_cap) side[k] = ExtSide{tid, left, right, ok ? 0u : 1u, 0u};
}

// Which seeds can still yield a record (A2-10's parallel pass): seed s with
// unit L passes the copies / array-length test when the best extension over
// its shifts cs = s - sh (sh < min(L, s + 1)) does.  Every such window covers
// s, an entry's span is copies x L, and the best has the most copies, so the
// test holds iff some window has copies >= thr[L - 1] (= max(min_copies,
// ceil(min_array_length / L))).  Side entries (the host's own extension)
// are flagged unconditionally, so the flags are a superset of the passing
// seeds.  One bit per (L, s): bits[(L - 1) nw + s / 64], nw = ceil(n / 64).
struct SeedThr {
    uint32_t c[kMaxUnit];
};
__global__ __launch_bounds__(256) void k_seed_flags(const uint32_t *__restrict__ word, int64_t n, int Lmax, SeedThr thr,
                                                    uint64_t *__restrict__ bits, int64_t nw) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = nw * 64;
    const int L = (int)(tid / per) + 1;   // uniform over a wave: per is a multiple of 64
    if (L > Lmax) return;
    const int64_t s = tid - (int64_t)(L - 1) * per;
    bool f = false;
    if (s + L <= n) {
        const uint32_t *w = word + (int64_t)(L - 1) * n;
        const int64_t lo = s - min<int64_t>((int64_t)L, s + 1) + 1;
        const uint32_t need = thr.c[L - 1];
        for (int64_t cs = s; cs >= lo && !f; --cs) {
            const uint32_t x = w[cs];
            f = x == kExtSide || (x != kExtNone && 1u + (x & 0xffffu) + (x >> 16) >= need);
        }
    }
    const uint64_t b = __ballot(f);
    if ((threadIdx.x & 63) == 0) bits[tid >> 6] = b;
}

// -------------------------------------------------------------- Tier 1
// Tier1STRFinder._find_simple_tandems_kmer (bwt.py:1426-1532), one unit length:
// does the walk STOP at q (record a repeat) if it visits q?  Depends only on q
// and the positions marked by longer units.  Copies are counted up to the
// point where both length tests are settled (3 copies, and >= 10 bp when the
// motif's entropy is < 1; the closest entropy to 1.0 among motifs <= 9 bp is
// 0.009 away, so the device log2 cannot flip that test).
__global__ void k_t1_flags(const uint8_t *__restrict__ t, int64_t n, int L, const uint8_t *__restrict__ seen,
                           uint32_t *__restrict__ flag) {
    const int64_t q = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (q >= n) return;
    flag[q] = 0;
    if (q >= n - L || seen[q]) return;                     // while i < n - motif_len; seen_mask[i]
    uint8_t cnt[4] = {0, 0, 0, 0};
    for (int p = 0; p < L; ++p) {
        const uint8_t c = t[q + p];
        const int b = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : c == 'T' ? 3 : -1;
        if (b < 0) return;                                 // motif with N / non-ACGT
        ++cnt[b];
    }
    const int cap = max(3, (10 + L - 1) / L);
    int copies = 1;
    for (int64_t cp = q + L; copies < cap && cp + L <= n; cp += L) {
        bool eq = true;
        for (int p = 0; p < L && eq; ++p) eq = t[cp + p] == t[q + p];
        if (!eq) break;
        ++copies;
    }
    if (copies < 3) return;
    const int length = copies * L;                         // exact unless capped (then >= 10)
    double ent = 0.0;
    for (int b = 0; b < 4; ++b)
        if (cnt[b]) {
            const double pr = (double)cnt[b] / (double)L;
            ent -= pr * log2(pr);
        }
    if (ent < 1.0 && length < 10) return;
    if (length < 6) return;
    flag[q] = 1;
}

__global__ void k_t1_compact(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos, int64_t n,
                             int64_t *__restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (q < n && flag[q]) out[pos[q]] = q;
}

__global__ void k_t1_mark(const int64_t *__restrict__ ranges, int64_t nr, uint8_t *__restrict__ seen) {
    const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (r >= nr) return;
    for (int64_t x = ranges[2 * r]; x < ranges[2 * r + 1]; ++x) seen[x] = 1;
}

// ------------------------------------------------------------- Tier 3
// Tier3LongReadFinder._detect_repetitive_structure (bwt.py:2948-2984) for one
// 500-byte window per wave: for period p = 10..165 the score is
// #{i < 500 : w[i] == w[i % p]} / 500 (_score_periodicity: motif = w[:p], so
// every position counts); the first period with the highest score > 0.7 wins.
// Scores share the denominator, so "higher score" is "more matches"; the
// 0.7 test is done on the double quotient, as in the reference.
constexpr int kT3Win = 500, kT3Pmin = 10, kT3Pend = kT3Win / 3;   // range(10, len // 3)

__global__ __launch_bounds__(256) void k_t3_windows(const uint8_t *__restrict__ reads, const int64_t *__restrict__ wpos,
                                                    int64_t nwin, int32_t *__restrict__ best) {
    __shared__ uint8_t win[4][512];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + wv;
    const bool live = w < nwin;
    uint8_t c[8];
    if (live) {
        const uint8_t *src = reads + wpos[w];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = lane + 64 * k;
            c[k] = i < kT3Win ? src[i] : 0;
            if (i < kT3Win) win[wv][i] = c[k];
        }
    }
    __syncthreads();
    if (!live) return;
    int bp = 0, bm = 0;
    for (int p = kT3Pmin; p < kT3Pend; ++p) {
        int m = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = lane + 64 * k;
            const bool eq = i < kT3Win && c[k] == win[wv][i % p];
            m += __popcll(__ballot(eq));
        }
        if (m > bm && (double)m / (double)kT3Win > 0.7) {
            bm = m;
            bp = p;
        }
    }
    if (lane == 0) best[w] = bp ? (bp << 16) | bm : 0;
}

// --------------------------------------------------- simple period scan
// Tier2LCPFinder._extend_with_mismatches (bwt.py:2392-2498) for a batch of
// (start, period) candidates, one wave per candidate, lane l owning motif
// columns l, l + 64, l + 128, l + 192 (period <= 256).  Each column keeps up
// to kSimSyms (symbol, count) pairs, so adding or retracting a copy is O(1)
// per column; the array's mismatches against the majority consensus are
// sum over columns of (copies - max count), reduced across the wave.  The
// majority symbol is the smallest byte among the most frequent (np.unique +
// argmax).  A column needing more symbols marks the candidate for the host.
constexpr int kSimCols = 4, kSimSyms = 6, kSimMaxP = 64 * kSimCols;

__device__ __forceinline__ int64_t max_mm_for_array_dev(int64_t L, int64_t c) {   // bwt.py:2003-2025
    const int64_t tot = L * c;
    if (L == 1) return 0;
    const double f = L <= 6 ? 0.05 : 0.08;
    const int64_t m = (int64_t)ceil(f * (double)tot);
    return m > 1 ? m : 1;
}

// Wave reductions return a scalar (readfirstlane): loops and branches that
// exit on them are uniform by construction, never a per-lane copy the compiler
// could treat as divergent (the r02al-r02ap hang).
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

struct SimCol {
    uint8_t s[kSimSyms];
    uint32_t c[kSimSyms];
    int nd;
};

__device__ __forceinline__ void simcol_add(SimCol &k, uint8_t b, int d, bool &ovf) {
#pragma unroll
    for (int q = 0; q < kSimSyms; ++q)
        if (q < k.nd && k.s[q] == b) { k.c[q] += d; return; }
    if (k.nd < kSimSyms) {
#pragma unroll
        for (int q = 0; q < kSimSyms; ++q)
            if (q == k.nd) { k.s[q] = b; k.c[q] = (uint32_t)d; }
        ++k.nd;
    } else {
        ovf = true;
    }
}
// max count and the smallest symbol holding it
__device__ __forceinline__ void simcol_major(const SimCol &k, uint32_t &mx, uint8_t &sym) {
    mx = 0;
    sym = 255;
#pragma unroll
    for (int q = 0; q < kSimSyms; ++q)
        if (q < k.nd && (k.c[q] > mx || (k.c[q] == mx && k.c[q] > 0 && k.s[q] < sym))) { mx = k.c[q]; sym = k.s[q]; }
}

// out[5*j] = (array_start, array_end, copies, full_start, full_end); ovf[j] = 1: redo on the host
__global__ __launch_bounds__(256) void k_simple_extend(const uint8_t *__restrict__ t, int64_t n,
                                                       const int64_t *__restrict__ cand, int64_t ncand,
                                                       int64_t *__restrict__ out, uint8_t *__restrict__ ovf_out) {
    const int lane = threadIdx.x & 63;
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (j >= ncand) return;   // wave-uniform
    const int64_t s0 = cand[2 * j];
    const int64_t pw = cand[2 * j + 1];
    const int64_t p = pw & 0xFFFF;
    const bool allow = (pw >> 16) & 1;
    SimCol col[kSimCols];
    uint8_t cons[kSimCols];
    bool ovf = false;
#pragma unroll
    for (int k = 0; k < kSimCols; ++k) {
        const int64_t c = lane + 64 * k;
        col[k].nd = 0;
        cons[k] = 0;
        if (c < p) {
            cons[k] = t[s0 + c];
            simcol_add(col[k], cons[k], 1, ovf);
        }
    }
    int64_t start = s0, end = s0 + p, copies = 1;
    // extend right, then left, by whole copies (bwt.py:2417-2475)
    for (int dir = 0; dir < 2; ++dir) {
        for (;;) {
            const int64_t at = dir == 0 ? end : start - p;
            if (dir == 0 ? (end + p > n) : (start - p < 0)) break;
            const int64_t tc = copies + 1;
            int mm = 0;
#pragma unroll
            for (int k = 0; k < kSimCols; ++k) {
                const int64_t c = lane + 64 * k;
                if (c < p) {
                    simcol_add(col[k], t[at + c], 1, ovf);
                    uint32_t mx;
                    uint8_t sy;
                    simcol_major(col[k], mx, sy);
                    mm += (int)(tc - mx);
                }
            }
            const int64_t tot = wave_sum_i(mm);
            const int64_t lim = allow ? max_mm_for_array_dev(p, tc) : 0;
            if (tot <= lim) {
                copies = tc;
                if (dir == 0) end += p;
                else start -= p;
#pragma unroll
                for (int k = 0; k < kSimCols; ++k) {
                    const int64_t c = lane + 64 * k;
                    if (c < p) {
                        uint32_t mx;
                        uint8_t sy;
                        simcol_major(col[k], mx, sy);
                        cons[k] = sy;
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < kSimCols; ++k) {
                    const int64_t c = lane + 64 * k;
                    if (c < p) simcol_add(col[k], t[at + c], -1, ovf);
                }
                break;
            }
        }
    }
    // partial copies, exact matches only (bwt.py:2480-2496): first failing offset
    int pr = (int)p, pl = (int)p;
#pragma unroll
    for (int k = 0; k < kSimCols; ++k) {
        const int64_t c = lane + 64 * k;
        if (c < p) {
            if (!(end + c < n && t[end + c] == cons[k])) pr = min(pr, (int)c);
            const int64_t kk = p - 1 - c;                       // left offset whose consensus column is c
            if (!(start - kk - 1 >= 0 && t[start - kk - 1] == cons[k])) pl = min(pl, (int)kk);
        }
    }
    pr = wave_min_i(pr);
    pl = wave_min_i(pl);
    const int any_ovf = wave_sum_i(ovf ? 1 : 0);
    if (lane == 0) {
        out[5 * j] = start - pl;
        out[5 * j + 1] = end + pr;
        out[5 * j + 2] = copies;
        out[5 * j + 3] = start;
        out[5 * j + 4] = end;
        ovf_out[j] = any_ovf ? 1 : 0;
    }
}

// --------------------------------------------------- host-side exact helpers
// majority vote of n_copies copies from `start` (np.unique + argmax)
static void majority(const uint8_t *t, int64_t n, int64_t start, int64_t L, int64_t n_copies, std::string &cons,
                     int64_t &used) {
    cons.assign((size_t)L, '\0');
    used = 0;
    while (used < n_copies && start + (used + 1) * L <= n) ++used;
    for (int64_t p = 0; p < L; ++p) {
        int32_t cnt[256] = {0};
        for (int64_t i = 0; i < used; ++i) ++cnt[t[start + i * L + p]];
        int best = -1, bv = 0;
        for (int b = 0; b < 256; ++b)
            if (cnt[b] > bv) { bv = cnt[b]; best = b; }
        cons[(size_t)p] = (char)(best < 0 ? 0 : best);
    }
}

// scalar _extend_tandem_fm for a column with more than kD symbols
static void extend_host(const uint8_t *t, int64_t n, int64_t cs, int64_t L, int64_t &s, int64_t &e, int64_t &c) {
    s = cs;
    e = cs + L;
    c = 1;
    std::string cons;
    int64_t used;
    auto score = [&](int64_t from, int64_t tc, int64_t &mm, int64_t &tv) {
        majority(t, n, from, L, tc, cons, used);
        mm = tv = 0;
        for (int64_t i = 0; i < tc; ++i) {
            const int64_t a = from + i * L;
            if (a + L > n) continue;
            for (int64_t p = 0; p < L; ++p) {
                const uint8_t x = t[a + p], y = (uint8_t)cons[(size_t)p];
                if (x != y) {
                    ++mm;
                    if (transversion(x, y)) ++tv;
                }
            }
        }
    };
    auto homo = [&](int64_t a) {
        for (int64_t p = 1; p < L; ++p)
            if (t[a + p] != t[a]) return false;
        return true;
    };
    while (e + L <= n) {
        if (L > 1 && homo(e)) break;
        int64_t mm, tv;
        score(s, c + 1, mm, tv);
        if (mm <= max_mm_for_array(L, c + 1) && tv == 0) { ++c; e += L; }
        else break;
    }
    while (s - L >= 0) {
        if (L > 1 && homo(s - L)) break;
        int64_t mm, tv;
        score(s - L, c + 1, mm, tv);
        if (mm <= max_mm_for_array(L, c + 1) && tv == 0) { ++c; s -= L; }
        else break;
    }
}

// build_consensus_motif_array (bwt.py:1208-1256)
static bool consensus_array(const uint8_t *t, int64_t n, int64_t start, int64_t L, int64_t n_copies, std::string &cons,
                            double &mm_rate, int64_t &max_mm) {
    if (n_copies == 0 || L == 0) return false;
    int64_t used;
    majority(t, n, start, L, n_copies, cons, used);
    if (used == 0) return false;
    int64_t tot = 0;
    max_mm = 0;
    for (int64_t i = 0; i < used; ++i) {
        int64_t h = 0;
        for (int64_t p = 0; p < L; ++p) h += t[start + i * L + p] != (uint8_t)cons[(size_t)p];
        tot += h;
        max_mm = std::max(max_mm, h);
    }
    mm_rate = (double)tot / (double)(used * L);
    return true;
}

// canonical (least rotation, forward only) primitive ACGT strings of length k, product order
static void enumerate_motifs_build(int k, std::vector<std::string> &out) {
    out.clear();
    static const char A[4] = {'A', 'C', 'G', 'T'};
    const int64_t total = (int64_t)1 << (2 * k);
    std::string s((size_t)k, 'A');
    for (int64_t code = 0; code < total; ++code) {
        for (int j = 0; j < k; ++j) s[(size_t)j] = A[(code >> (2 * (k - 1 - j))) & 3];
        bool keep = true;
        for (int r = 1; r < k && keep; ++r) {
            int cmp = 0;
            for (int q = 0; q < k && !cmp; ++q) {
                const char x = s[(size_t)((q + r) % k)], y = s[(size_t)q];
                cmp = x < y ? -1 : (x > y ? 1 : 0);
            }
            keep = cmp > 0;   // a smaller rotation: not canonical; an equal one: not primitive
        }
        if (keep) out.push_back(s);
    }
}

// the same sets, built once per process (k <= 10: they never change)
static const std::vector<std::string> &motif_set(int k) {
    static std::vector<std::string> sets[11];
    static std::once_flag once[11];
    std::call_once(once[k], [k] { enumerate_motifs_build(k, sets[k]); });
    return sets[k];
}
// entropy_of of every motif of motif_set(k), in its order
static const std::vector<double> &motif_entropy(int k) {
    static std::vector<double> ent[11];
    static std::once_flag once[11];
    std::call_once(once[k], [k] {
        for (const std::string &m : motif_set(k)) ent[k].push_back(entropy_of(m.data(), (int64_t)m.size()));
    });
    return ent[k];
}

// A2-10's motifs in the reference's order (k ascending, enumerate_motifs
// order, entropy filter, bwt.py:2053-2095), each with its first locate
// pattern; the patterns that go through locate (k > 8, or no k-mer table):
// every rotation of the motif and of its reverse complement.  They depend on
// the parameters only, so they are built once per process per parameter set.
struct MotifTask {
    int k;
    const std::string *m;
    size_t pat;
};
struct SiPlan {
    std::vector<MotifTask> tasks;
    size_t npats = 0;
    std::string blob;
    std::vector<int64_t> off;
};
char comp_base(char c);
const SiPlan &si_plan(int kmin, int kend, double min_entropy, bool kmer_table) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, double, bool>, std::unique_ptr<SiPlan>> cache;
    std::lock_guard<std::mutex> lk(mu);
    std::unique_ptr<SiPlan> &slot = cache[std::make_tuple(kmin, kend, min_entropy, kmer_table)];
    if (slot) return *slot;
    auto pl = std::make_unique<SiPlan>();
    for (int k = kmin; k < kend; ++k) {
        const bool use_hash = k <= 8 && kmer_table;
        const std::vector<std::string> &ms = motif_set(k);
        const std::vector<double> &me = motif_entropy(k);
        for (size_t i = 0; i < ms.size(); ++i) {
            if (me[i] < min_entropy) continue;   // bwt.py:2058-2060
            pl->tasks.push_back({k, &ms[i], pl->npats});
            if (!use_hash) pl->npats += 2 * (size_t)k;
        }
    }
    pl->off.assign(pl->npats + 1, 0);
    if (pl->npats) {
        std::vector<size_t> at(pl->tasks.size(), 0);
        size_t bytes = 0;
        for (size_t ti = 0; ti < pl->tasks.size(); ++ti)
            if (!(pl->tasks[ti].k <= 8 && kmer_table)) {
                at[ti] = bytes;
                bytes += 2 * (size_t)pl->tasks[ti].k * (size_t)pl->tasks[ti].k;
            }
        pl->blob.resize(bytes);
        for (size_t ti = 0; ti < pl->tasks.size(); ++ti) {
            const MotifTask &mt = pl->tasks[ti];
            const int k = mt.k;
            if (k <= 8 && kmer_table) continue;
            const std::string &m = *mt.m;
            char rc[16];
            for (int x = 0; x < k; ++x) rc[x] = comp_base(m[(size_t)(k - 1 - x)]);
            char *w = &pl->blob[at[ti]];
            size_t q = mt.pat;
            for (int r = 0; r < k; ++r) {
                for (int x = 0; x < k; ++x) *w++ = m[(size_t)((r + x) % k)];
                pl->off[++q] = (int64_t)(at[ti] + (size_t)(2 * r + 1) * (size_t)k);
                for (int x = 0; x < k; ++x) *w++ = rc[(r + x) % k];
                pl->off[++q] = (int64_t)(at[ti] + (size_t)(2 * r + 2) * (size_t)k);
            }
        }
    }
    slot = std::move(pl);
    return *slot;
}

char comp_base(char c) {
    switch (c) {
        case 'A': return 'T';
        case 'T': return 'A';
        case 'C': return 'G';
        case 'G': return 'C';
        default: return c;
    }
}

}  // namespace

void lcp_plateaus_device(Ctx &c, DeviceIndex *ix, const LibParams &p, std::vector<int64_t> &out) {
    out.clear();
    const int64_t n = index_n(ix);
    if (n == 0) return;
    hipStream_t st = c.stream;
    const int32_t *lcp = index_lcp_device(c, ix);
    c.slot[S_COUNTS].ensure(64);
    int *d_max = c.slot[S_COUNTS].as<int>();
    HIPCHECK(hipMemsetAsync(d_max, 0, 4, st));
    KLAUNCH("k_max_i32", 0.0, k_max_i32, dim3((unsigned)std::min<int64_t>(1024, blocks(n))), dim3(kB), 0, st, lcp, n, d_max);
    int lmax = 0;
    HIPCHECK(hipMemcpyAsync(&lmax, d_max, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (lmax < p.min_period) return;
    const int64_t thr = std::max<int64_t>(p.min_period, std::min<int64_t>(std::min<int64_t>(p.max_period, lmax), 20));
    c.slot[S_IDX1].ensure((size_t)(n + 1) * 4);
    c.slot[S_IDX2].ensure((size_t)(n + 1) * 4);
    c.slot[S_IDX3].ensure((size_t)(n + 1) * 4);
    c.slot[S_IDX4].ensure((size_t)(n + 1) * 4);
    uint32_t *inrun = c.slot[S_IDX1].as<uint32_t>(), *head = c.slot[S_IDX2].as<uint32_t>();
    uint32_t *hscan = c.slot[S_IDX3].as<uint32_t>(), *cpos = c.slot[S_IDX4].as<uint32_t>();
    KLAUNCH("k_plateau_flags", 12.0 * (double)n, k_plateau_flags, dim3(blocks(n)), dim3(kB), 0, st, lcp, n, (int32_t)thr, inrun, head);
    HIPCHECK(hipMemsetAsync(inrun + n, 0, 4, st));
    HIPCHECK(hipMemsetAsync(head + n, 0, 4, st));
    exclusive_scan<uint32_t>(c, head, hscan, n + 1);
    exclusive_scan<uint32_t>(c, inrun, cpos, n + 1);
    uint32_t m32 = 0, runs = 0;
    HIPCHECK(hipMemcpyAsync(&m32, cpos + n, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(&runs, hscan + n, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    const int64_t m = m32;
    if (m == 0) return;
    c.slot[S_IDX0].ensure((size_t)m * 8);
    c.slot[S_IDX5].ensure((size_t)m * 8);
    c.slot[S_IDX6].ensure((size_t)(m + 1) * 4);
    c.slot[S_IDX7].ensure((size_t)(m + 1) * 4);
    uint64_t *keys = c.slot[S_IDX0].as<uint64_t>();
    int64_t *copies = c.slot[S_IDX5].as<int64_t>();
    uint32_t *flag = c.slot[S_IDX6].as<uint32_t>(), *pos = c.slot[S_IDX7].as<uint32_t>();
    KLAUNCH("k_plateau_keys", 0.0, k_plateau_keys, dim3(blocks(n)), dim3(kB), 0, st, index_sa_device(ix), inrun, head, hscan, cpos,
                       n, keys);
    int rb = 0;
    while (rb < 32 && ((uint64_t)runs >> rb)) ++rb;
    radix_sort_pairs32(c, keys, nullptr, m, 0, ((32 + rb + 7) / 8) * 8);
    KLAUNCH("k_plateau_eval", 0.0, k_plateau_eval, dim3(blocks(m)), dim3(kB), 0, st, keys, m, index_text_device(ix), n, thr,
                       (int64_t)p.min_copies, flag, copies);
    HIPCHECK(hipMemsetAsync(flag + m, 0, 4, st));
    exclusive_scan<uint32_t>(c, flag, pos, m + 1);
    uint32_t k32 = 0;
    HIPCHECK(hipMemcpyAsync(&k32, pos + m, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    if (k32 == 0) return;
    c.slot[S_MISC2].ensure((size_t)k32 * 24);
    KLAUNCH("k_plateau_out", 0.0, k_plateau_out, dim3(blocks(m)), dim3(kB), 0, st, keys, flag, pos, copies, m, thr,
                       c.slot[S_MISC2].as<int64_t>());
    HIPCHECK(hipGetLastError());
    out.resize((size_t)k32 * 3);
    HIPCHECK(hipMemcpyAsync(out.data(), c.slot[S_MISC2].p, (size_t)k32 * 24, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
}

void tier1_device(Ctx &c, const uint8_t *d_text, const uint8_t *t, int64_t n, int32_t max_motif_length,
                  int32_t chrom, RecVec &out) {
    if (n <= 0) return;
    hipStream_t st = c.stream;
    const int64_t step = n > 10000000 ? 50 : (n > 5000000 ? 20 : 1);   // bwt.py:1440-1447
    c.slot[S_MISC0].ensure((size_t)n + 64);
    c.slot[S_MISC1].ensure((size_t)(n + 1) * 4);
    c.slot[S_MISC2].ensure((size_t)(n + 1) * 4);
    uint8_t *seen = c.slot[S_MISC0].as<uint8_t>();
    uint32_t *flag = c.slot[S_MISC1].as<uint32_t>(), *pos = c.slot[S_MISC2].as<uint32_t>();
    HIPCHECK(hipMemsetAsync(seen, 0, (size_t)n, st));
    std::vector<int64_t> cand, ranges;
    for (int L = std::min(max_motif_length, 9); L >= 1; --L) {   // longest unit first (bwt.py:1451)
        KLAUNCH("k_t1_flags", 6.0 * (double)n, k_t1_flags, dim3(blocks(n)), dim3(kB), 0, st, d_text, n, L, seen, flag);
        HIPCHECK(hipMemsetAsync(flag + n, 0, 4, st));
        exclusive_scan<uint32_t>(c, flag, pos, n + 1);
        uint32_t m = 0;
        HIPCHECK(hipMemcpyAsync(&m, pos + n, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if (m == 0) continue;
        c.slot[S_MISC3].ensure((size_t)m * 8);
        KLAUNCH("k_t1_compact", 0.0, k_t1_compact, dim3(blocks(n)), dim3(kB), 0, st, flag, pos, n, c.slot[S_MISC3].as<int64_t>());
        HIPCHECK(hipGetLastError());
        cand.resize(m);
        HIPCHECK(hipMemcpyAsync(cand.data(), c.slot[S_MISC3].p, (size_t)m * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        // the walk visits ptr, ptr + step, ... and stops at the first stopping position
        ranges.clear();
        int64_t ptr = 0;
        for (int64_t q : cand) {
            if (q < ptr || (q - ptr) % step) continue;
            int64_t copies = 1, cp = q + L;
            while (cp + L <= n && std::memcmp(t + cp, t + q, (size_t)L) == 0) {
                ++copies;
                cp += L;
            }
            const int64_t end = q + copies * L;
            Rec r;
            r.chrom = chrom;
            r.tier = 1;
            r.start = q;
            r.end = end;
            r.length = end - q;
            r.motif.assign((const char *)t + q, (size_t)L);
            r.copies = (double)copies;
            r.confidence = 1.0;
            r.mismatch_rate = 0.0;
            r.max_mm = 0;
            r.n_eval = copies;
            r.strand = '+';
            r.pmatch = 100.0;
            r.pindel = 0.0;
            r.score = trf_score(end - q, 0.0);
            r.act_kind = ACT_FULL;
            r.act_off = q;
            r.act_len = end - q;
            out.push_back(std::move(r));
            ranges.push_back(q);
            ranges.push_back(end);
            ptr = end;
        }
        if (ranges.empty()) continue;
        const int64_t nr = (int64_t)ranges.size() / 2;
        c.slot[S_MISC3].ensure(ranges.size() * 8);
        HIPCHECK(hipMemcpyAsync(c.slot[S_MISC3].p, ranges.data(), ranges.size() * 8, hipMemcpyHostToDevice, st));
        KLAUNCH("k_t1_mark", 0.0, k_t1_mark, dim3(blocks(nr)), dim3(kB), 0, st, c.slot[S_MISC3].as<int64_t>(), nr, seen);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipStreamSynchronize(st));
    }
}

void short_imperfect_device(Ctx &c, DeviceIndex *ix, const LibParams &p, const std::vector<int64_t> &seen_pairs,
                            int32_t chrom, RecVec &out) {
    const int64_t n = index_n(ix);
    if (n > 1000000 || n == 0) return;                    // bwt.py:2048
    using clk = std::chrono::steady_clock;
    const bool stats = stats_on();
    const auto T0 = clk::now();
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const int kmin = std::max(1, p.min_period), kend = std::min(p.max_short_motif + 1, 10);
    hipStream_t st = c.stream;
    // the text through the context's pinned staging buffer
    HBuf &text_buf = c.host[1];
    text_buf.ensure((size_t)n);
    HIPCHECK(hipMemcpyAsync(text_buf.p, index_text_device(ix), (size_t)n, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    std::vector<uint8_t> text(text_buf.as<uint8_t>(), text_buf.as<uint8_t>() + n);
    const uint8_t *t = text.data();
    if (stats) std::fprintf(stderr, "    text down %.1f ms\n", ms_since(T0));

    // extension table for every start and unit length 1..9 (k_extend_cols)
    const int Lmax = kMaxUnit;
    const int64_t tot = (int64_t)Lmax * n;
    c.slot[S_IDX0].ensure((size_t)tot * 4);
    c.slot[S_COUNTS].ensure(256 * 8);
    // the table comes down into the context's pinned staging buffer (kept between calls)
    HBuf &ext_buf = c.host[2];
    ext_buf.ensure((size_t)tot * 4);
    uint32_t *const ext_word = ext_buf.as<uint32_t>();
    std::unordered_map<int64_t, std::array<int64_t, 3>> ext_side;   // q -> (start, end, copies)
    const int64_t nw = (n + 63) / 64;
    std::vector<uint64_t> seed_bits((size_t)Lmax * (size_t)nw);   // k_seed_flags
    c.slot[S_IDX2].ensure(seed_bits.size() * 8);
    for (int64_t cap = 1 << 16;;) {
        c.slot[S_IDX1].ensure((size_t)cap * sizeof(ExtSide));
        HIPCHECK(hipMemsetAsync(c.slot[S_COUNTS].p, 0, 8, st));
        KLAUNCH("k_extend", 9.0 * (double)n + 4.0 * (double)tot, k_extend_cols, dim3(blocks(tot)), dim3(kB), 0, st,
                index_text_device(ix), n, Lmax, c.slot[S_IDX0].as<uint32_t>(), c.slot[S_IDX1].as<ExtSide>(),
                c.slot[S_COUNTS].as<unsigned long long>(), cap);
        HIPCHECK(hipGetLastError());
        unsigned long long ns = 0;
        HIPCHECK(hipMemcpyAsync(&ns, c.slot[S_COUNTS].p, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if ((int64_t)ns > cap) {   // the side list overflowed: again with room for all of it
            cap = (int64_t)ns;
            continue;
        }
        std::vector<ExtSide> side((size_t)ns);
        if (stats) std::fprintf(stderr, "    text + extension kernel %.1f ms\n", ms_since(T0));
        SeedThr thr{};
        for (int L = 1; L <= Lmax; ++L) {
            const int64_t by_len = (std::max<int64_t>(0, p.min_array_length) + L - 1) / L;
            thr.c[L - 1] = (uint32_t)std::min<int64_t>(0xffffffffLL, std::max<int64_t>({(int64_t)0, (int64_t)p.min_copies, by_len}));
        }
        KLAUNCH("k_seed_flags", 4.0 * (double)tot + (double)Lmax * (double)nw * 8.0, k_seed_flags,
                dim3((unsigned)(((int64_t)Lmax * nw * 64 + kB - 1) / kB)), dim3(kB), 0, st, c.slot[S_IDX0].as<uint32_t>(), n,
                Lmax, thr, c.slot[S_IDX2].as<uint64_t>(), nw);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(seed_bits.data(), c.slot[S_IDX2].p, seed_bits.size() * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(ext_word, c.slot[S_IDX0].p, (size_t)tot * 4, hipMemcpyDeviceToHost, st));
        if (ns) HIPCHECK(hipMemcpyAsync(side.data(), c.slot[S_IDX1].p, (size_t)ns * sizeof(ExtSide),
                                        hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        for (const ExtSide &x : side) {
            const int64_t L = x.q / n + 1, cs = x.q % n;
            int64_t s0, e0, c0;
            if (x.unbinned) {   // a symbol outside A C G N T: the scalar extension
                extend_host(t, n, cs, L, s0, e0, c0);
            } else {
                s0 = cs - (int64_t)x.left * L;
                e0 = cs + L + (int64_t)x.right * L;
                c0 = 1 + (int64_t)x.left + (int64_t)x.right;
            }
            ext_side[x.q] = {s0, e0, c0};
        }
        break;
    }
    // (start, end, copies) of entry q (cs + L <= n)
    auto ext_of = [&](int64_t q, int64_t L, int64_t cs, int64_t &s0, int64_t &e0, int64_t &c0) {
        const uint32_t w = ext_word[(size_t)q];
        if (w == kExtSide) {
            const auto &v = ext_side.at(q);
            s0 = v[0];
            e0 = v[1];
            c0 = v[2];
            return;
        }
        const int64_t lf = w & 0xffffu, rt = w >> 16;
        s0 = cs - lf * L;
        e0 = cs + L + rt * L;
        c0 = 1 + lf + rt;
    };

    const double t_ext = ms_since(T0);
    // seeds: k-mer table (with the reference's short-k lookup, bwt.py:173-193) or FM locate
    std::vector<int64_t> koff;
    std::vector<int32_t> kpos;
    const int64_t kcount = index_kmer_count(ix);
    if (kcount > 0) {
        koff.resize(65537);
        kpos.resize((size_t)kcount);
        index_get_kmer(c, ix, koff.data(), kpos.data());
        if (stats) std::fprintf(stderr, "    kmer table down %.1f ms\n", ms_since(T0) - t_ext);
    }
    const SiPlan &plan = si_plan(kmin, kend, p.min_entropy, kcount > 0);
    const std::vector<MotifTask> &tasks = plan.tasks;
    const size_t npats = plan.npats;
    const std::string &blob = plan.blob;
    const std::vector<int64_t> &off = plan.off;
    const int nt = std::max(1, host_cpu_budget(nullptr, nullptr));
    std::vector<int64_t> spep;
    std::vector<int32_t> sa;
    if (npats) {
        spep.resize(npats * 2);
        if (stats) std::fprintf(stderr, "    motifs + %zu patterns %.1f ms\n", npats, ms_since(T0) - t_ext);
        index_backward_search(c, ix, (const uint8_t *)blob.data(), off.data(), (int64_t)npats, spep.data());
        if (stats) std::fprintf(stderr, "    backward search %.1f ms\n", ms_since(T0) - t_ext);
        sa.resize((size_t)n);
        index_get_sa(c, ix, sa.data());
    }

    std::vector<uint8_t> seen((size_t)n + 1, 0);
    for (size_t q = 0; q + 1 < seen_pairs.size(); q += 2)
        for (int64_t x = std::max<int64_t>(0, seen_pairs[q]); x < std::min<int64_t>(n, seen_pairs[q + 1]); ++x)
            seen[(size_t)x] = 1;
    const std::string seq((const char *)t, (size_t)n);

    // Seed positions of a motif: every rotation of it and of its reverse
    // complement, through the k-mer table (the reference's short-k lookup) or
    // the FM interval's SA rows -- restricted to the seeds k_seed_flags marks,
    // sorted.  Returns the number of unique seeds (flagged or not): distinct
    // 8-mer keys hold disjoint positions and distinct patterns of one length
    // disjoint SA intervals, so the count is a sum over the distinct ones.
    // A seed is kept when it is flagged for some unit length in [1, lmax] (the
    // parallel pass asks for exactly k: lmin = k).
    auto seeds_flagged = [&](const MotifTask &mt, int lmin, int lmax, std::vector<int64_t> &positions) -> int64_t {
        positions.clear();
        const int k = mt.k;
        auto flagged = [&](int64_t s) {
            uint64_t f = 0;
            for (int L = lmin; L <= lmax; ++L) f |= seed_bits[(size_t)(L - 1) * (size_t)nw + (size_t)(s >> 6)];
            return (f >> (s & 63)) & 1u;
        };
        const std::string &m = *mt.m;
        int64_t total = 0;
        if (k <= 8 && kcount > 0) {
            int64_t keys[16];
            int nk = 0;
            int64_t fw = 0, rw = 0;   // packed motif and reverse complement
            for (int x = 0; x < k; ++x) {
                const char ch = m[(size_t)x];
                fw = (fw << 2) | (ch == 'C' ? 1 : ch == 'G' ? 2 : ch == 'T' ? 3 : 0);
                const char rc = comp_base(m[(size_t)(k - 1 - x)]);
                rw = (rw << 2) | (rc == 'C' ? 1 : rc == 'G' ? 2 : rc == 'T' ? 3 : 0);
            }
            const int64_t mask = (int64_t(1) << (2 * k)) - 1;
            for (int r = 0; r < k; ++r) {   // rotation r: the word rotated left by r bases
                const int sh = 2 * (k - r);
                keys[nk++] = r ? (((fw << (2 * r)) | (fw >> sh)) & mask) : fw;
                keys[nk++] = r ? (((rw << (2 * r)) | (rw >> sh)) & mask) : rw;
            }
            std::sort(keys, keys + nk);
            nk = (int)(std::unique(keys, keys + nk) - keys);
            for (int i = 0; i < nk; ++i) {
                const int64_t a = koff[(size_t)keys[i]], b = koff[(size_t)keys[i] + 1];
                total += b - a;
                for (int64_t q = a; q < b; ++q)
                    if (flagged(kpos[(size_t)q])) positions.push_back(kpos[(size_t)q]);
            }
        } else {
            std::pair<int64_t, int64_t> iv[2 * kMaxUnit];
            int ni = 0;
            for (int r = 0; r < 2 * k; ++r) {
                const int64_t sp = spep[2 * (mt.pat + (size_t)r)], ep = spep[2 * (mt.pat + (size_t)r) + 1];
                if (sp >= 0) iv[ni++] = {sp, ep};
            }
            std::sort(iv, iv + ni);
            ni = (int)(std::unique(iv, iv + ni) - iv);
            for (int i = 0; i < ni; ++i) {
                total += iv[i].second - iv[i].first + 1;
                for (int64_t q = iv[i].first; q <= iv[i].second; ++q)
                    if (flagged(sa[(size_t)q])) positions.push_back(sa[(size_t)q]);
            }
        }
        std::sort(positions.begin(), positions.end());
        return total;
    };
    // the best extension through seed over the shifts whose start is not seen
    // (seen == nullptr: all shifts) -- most copies, then the leftmost start
    auto best_of = [&](int64_t seed, int64_t motif_len, const uint8_t *sn, int64_t &bs, int64_t &be, int64_t &bc) {
        bs = be = -1;
        bc = 0;
        const int64_t shifts = std::min<int64_t>(motif_len, seed + 1);
        for (int64_t sh = 0; sh < shifts; ++sh) {
            const int64_t cs = seed - sh;
            if (cs < 0 || cs + motif_len > n || (sn && sn[(size_t)cs])) continue;
            const int64_t q = (motif_len - 1) * n + cs;
            int64_t s0, e0, cc;
            ext_of(q, motif_len, cs, s0, e0, cc);
            if (!(s0 <= seed && seed < e0)) continue;
            if (cc > bc || (cc == bc && (bs < 0 || s0 < bs))) { bs = s0; be = e0; bc = cc; }
        }
    };
    // Parallel pass, per motif: its seeds, and the ones that can still become
    // a record.  `seen` only grows and removes shifts, and a subset's best has
    // no more copies (and span = copies x unit), so a seed whose best over all
    // shifts fails min_copies / min_array_length fails in the serial walk too.
    // The serial walk below then replays the order-dependent state (seen, the
    // motif length carried from one seed to the next, bwt.py:2655) over the
    // survivors only -- the consensus, periodicity and maximality work stays there.
    // The record a seed yields from its extension (start, end, copies) with
    // motif length L (bwt.py:2641-2690 after the extension): the majority-vote
    // consensus, the primitive reduction (the new motif length persists for
    // the motif's later seeds), maximality and the %match floor.  A pure
    // function of its arguments and the text.
    struct Decision {
        int64_t start = 0, end = 0, copies = 0, len_after = 0;   // len_after: the motif length for later seeds
        bool emit = false;
        std::string cons;
        double mm = 0;
        int64_t maxmm = 0;
    };
    auto decide = [&](int64_t start, int64_t end, int64_t copies, int64_t L, Decision &d) {
        d.emit = false;
        d.len_after = L;
        d.cons.clear();
        if (!consensus_array(t, n, start, L, copies, d.cons, d.mm, d.maxmm)) return;
        const int64_t prim = smallest_period(d.cons.data(), (int64_t)d.cons.size());
        if (prim < (int64_t)d.cons.size()) {
            L = prim;
            d.len_after = prim;                   // persists for the later seeds (as in the reference)
            copies = std::max<int64_t>(1, (end - start) / L);
            end = start + copies * L;
            if (!consensus_array(t, n, start, L, copies, d.cons, d.mm, d.maxmm)) return;
        }
        if (start > 0 && t[start - 1] == (uint8_t)d.cons[(size_t)L - 1]) return;   // _is_maximal_fm
        if (end < n && t[end] == (uint8_t)d.cons[0]) return;
        if ((1.0 - d.mm) * 100.0 < (L <= 6 ? 90.0 : 85.0)) return;
        d.start = start;
        d.end = end;
        d.copies = copies;
        d.emit = true;
    };
    struct Cand {
        int64_t seed, bs, be, bc;   // the best extension over all shifts
        Decision d;                 // what it yields with the motif's own length
    };
    struct TaskOut {
        bool skip = true;           // fewer than min_copies seeds, or no mismatch search
        std::vector<Cand> keep;     // candidate seeds, ascending
    };
    std::vector<TaskOut> tout(tasks.size());
    const double t_prep = ms_since(T0);
    run_tasks((int64_t)tasks.size(), nt, [&](int64_t ti) {
        thread_local std::vector<int64_t> positions;
        const MotifTask &mt = tasks[(size_t)ti];
        const int64_t total = seeds_flagged(mt, mt.k, mt.k, positions);
        TaskOut &o = tout[(size_t)ti];
        if (total < p.min_copies || !p.allow_mismatches) return;
        o.skip = false;
        for (int64_t seed : positions) {
            if (seed + mt.k > n) continue;
            Cand cd;
            best_of(seed, mt.k, nullptr, cd.bs, cd.be, cd.bc);
            if (cd.bs < 0 || !(cd.bc >= p.min_copies && cd.be - cd.bs >= p.min_array_length)) continue;
            cd.seed = seed;
            decide(cd.bs, cd.be, cd.bc, mt.k, cd.d);
            o.keep.push_back(std::move(cd));
        }
    });
    const double t_par = ms_since(T0);
    size_t nkeep = 0;
    for (const TaskOut &o : tout) nkeep += o.keep.size();
    const size_t first_new = out.size();
    struct Report {
        bool on;
        clk::time_point t0;
        double a, b, c;
        size_t tasks, keep;
        const RecVec &out;
        ~Report() {
            if (on)
                std::fprintf(stderr, "  short_imperfect: extension table %.1f, seeds/patterns %.1f, parallel seeds %.1f, "
                             "serial walk + variations %.1f ms (%zu motifs, %zu candidate seeds, %zu records)\n", a,
                             b - a, c - b, std::chrono::duration<double, std::milli>(clk::now() - t0).count() - c,
                             tasks, keep, out.size());
        }
    } report{stats, T0, t_ext, t_prep, t_par, tasks.size(), nkeep, out};
    // _find_tandems_fm_with_mismatches (bwt.py:2562-2695) in the reference's
    // order: only the seen test, the extension over the unseen shifts and the
    // motif length carried between seeds are order-dependent; a candidate
    // whose extension is the precomputed one takes its precomputed decision
    std::vector<int64_t> all;
    Decision dd;
    size_t nfull = 0;
    for (size_t ti = 0; ti < tasks.size(); ++ti) {
        TaskOut &o = tout[ti];
        if (o.skip) continue;
        const MotifTask &mt = tasks[ti];
        int64_t motif_len = mt.k;
        bool full = false;   // walking every seed (after a motif length change)
        const size_t cnt = o.keep.size();
        for (size_t si = 0; si < (full ? all.size() : cnt); ++si) {
            const int64_t seed = full ? all[si] : o.keep[si].seed;
            if (seen[(size_t)seed]) continue;
            if (seed + motif_len > n) continue;
            int64_t bs, be, bc;
            best_of(seed, motif_len, seen.data(), bs, be, bc);
            if (bs < 0) continue;
            if (!(bc >= p.min_copies && be - bs >= p.min_array_length)) continue;
            const Decision *d;
            if (!full && motif_len == mt.k && bs == o.keep[si].bs && be == o.keep[si].be && bc == o.keep[si].bc) {
                d = &o.keep[si].d;
            } else {
                decide(bs, be, bc, motif_len, dd);
                d = &dd;
            }
            const int64_t len_before = motif_len;
            motif_len = d->len_after;
            if (d->emit) {
                Rec r;
                r.chrom = chrom;
                r.tier = 2;
                r.start = d->start;
                r.end = d->end;
                r.length = d->end - d->start;
                r.motif = d->cons;
                r.copies = (double)d->copies;
                r.confidence = std::max(0.5, 1.0 - d->mm);
                r.mismatch_rate = d->mm;
                r.max_mm = d->maxmm;
                r.n_eval = d->copies;
                r.pmatch = (1.0 - d->mm) * 100.0;
                r.pindel = 0.0;
                r.score = trf_score(d->end - d->start, d->mm);
                r.act_kind = ACT_FULL;
                r.act_off = std::min(d->start, n);
                r.act_len = std::max<int64_t>(0, std::min(d->end, n) - r.act_off);
                for (int64_t x = d->start; x < std::min(d->end, n); ++x) seen[(size_t)x] = 1;
                out.push_back(std::move(r));
            }
            // a changed motif length changes every later seed's extension: the
            // candidates of the parallel pass (found with the motif's own length)
            // no longer cover them, so the walk goes on over all of its seeds
            if (motif_len != len_before && !full) {
                // the motif length only shrinks (a primitive period of the consensus),
                // and a seed that can pass with some length is flagged for it
                seeds_flagged(mt, 1, (int)motif_len, all);
                all.erase(all.begin(), std::upper_bound(all.begin(), all.end(), seed));
                full = true;
                ++nfull;
                si = (size_t)-1;   // ++ -> 0
            }
        }
    }
    if (stats) std::fprintf(stderr, "    serial walk %.1f ms (%zu motifs walked over all seeds)\n", ms_since(T0) - t_par, nfull);
    // per record, independent of the walk: the strand of the canonical motif
    // and the variations (summarize_variations_array -> align_repeat_region
    // with min_copies 1, bwt.py:1259-1287)
    run_tasks((int64_t)(out.size() - first_new), nt, [&](int64_t q) {
        thread_local AlignSummary summ;
        Rec &r = out[first_new + (size_t)q];
        std::string canon;
        char strand = '+';
        canonical_stranded(r.motif, canon, strand);
        r.strand = strand;
        if (align_repeat_region(seq.data(), n, r.start, r.end, r.motif, 1, summ) && summ.any_variation)
            r.variations = summ.variations;
    });
}


// Tier3LongReadFinder.find_very_long_repeats (bwt.py:2837-2850): every read of
// >= 1000 bytes, windows of 500 every 100 bytes (2852-2946).  The periodicity
// scan runs on the device (k_t3_windows); the anchors of repetitive windows
// (read[start-50:start], mapped only when located exactly once,
// _map_read_to_reference 2986-3001) go through the device backward search and
// SA; records are built and consolidated (3003-3036) on the host, in read and
// window order.
void tier3_device(Ctx &c, DeviceIndex *ix, const uint8_t *reads, const int64_t *read_off, int64_t nreads,
                  int32_t chrom, RecVec &out) {
    const int64_t n = index_n(ix);
    std::vector<int64_t> wpos;   // window starts (offsets into reads)
    std::vector<int64_t> wread;  // read of each window
    for (int64_t r = 0; r < nreads; ++r) {
        const int64_t a = read_off[r], len = read_off[r + 1] - read_off[r];
        if (len < 1000) continue;                                     // min_read_length (2833, 2842)
        for (int64_t s = 0; s < len - kT3Win; s += 100) {             // range(0, len - 500, 100)
            wpos.push_back(a + s);
            wread.push_back(r);
        }
    }
    const int64_t nwin = (int64_t)wpos.size();
    if (nwin == 0 || n == 0) return;
    hipStream_t st = c.stream;
    const int64_t rbytes = read_off[nreads];
    c.slot[S_IDX0].ensure((size_t)rbytes + 64);
    c.slot[S_IDX1].ensure((size_t)nwin * 8);
    c.slot[S_IDX2].ensure((size_t)nwin * 4);
    HIPCHECK(hipMemcpyAsync(c.slot[S_IDX0].p, reads, (size_t)rbytes, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(c.slot[S_IDX1].p, wpos.data(), (size_t)nwin * 8, hipMemcpyHostToDevice, st));
    KLAUNCH("k_t3_windows", 0.0, k_t3_windows, dim3((unsigned)((nwin + 3) / 4)), dim3(256), 0, st, c.slot[S_IDX0].as<uint8_t>(),
                       c.slot[S_IDX1].as<int64_t>(), nwin, c.slot[S_IDX2].as<int32_t>());
    HIPCHECK(hipGetLastError());
    std::vector<int32_t> best((size_t)nwin);
    HIPCHECK(hipMemcpyAsync(best.data(), c.slot[S_IDX2].p, (size_t)nwin * 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));

    // anchors of the repetitive windows: read[max(0, s-50):s], used when >= 20 bytes
    std::vector<int64_t> cand;        // window ids with an anchor
    std::vector<uint8_t> pats;
    std::vector<int64_t> poff(1, 0);
    for (int64_t w = 0; w < nwin; ++w) {
        if (!best[(size_t)w]) continue;
        const int64_t s = wpos[(size_t)w] - read_off[wread[(size_t)w]];
        const int64_t as = std::max<int64_t>(0, s - 50);
        if (s - as < 20) continue;
        cand.push_back(w);
        pats.insert(pats.end(), reads + read_off[wread[(size_t)w]] + as, reads + wpos[(size_t)w]);
        poff.push_back((int64_t)pats.size());
    }
    const int64_t na = (int64_t)cand.size();
    if (na == 0) return;
    std::vector<int64_t> spep((size_t)na * 2);
    index_backward_search(c, ix, pats.data(), poff.data(), na, spep.data());
    std::vector<int64_t> rows, hitw;
    for (int64_t q = 0; q < na; ++q)
        if (spep[2 * q] >= 0 && spep[2 * q] == spep[2 * q + 1]) {   // len(positions) == 1
            rows.push_back(spep[2 * q]);
            hitw.push_back(q);
        }
    if (rows.empty()) return;
    std::vector<int64_t> pos(rows.size());
    index_sa_rows(c, ix, rows.data(), (int64_t)rows.size(), pos.data());
    std::vector<uint8_t> text((size_t)n);
    index_get_text(c, ix, text.data());
    const uint8_t *t = text.data();
    const int64_t max_len = (n > 0 && t[n - 1] == '$') ? n - 1 : n;   // 2877-2880
    RecVec recs;
    AlignSummary summ;
    for (size_t h = 0; h < rows.size(); ++h) {
        const int64_t q = hitw[h], w = cand[(size_t)q];
        const int64_t s = wpos[(size_t)w] - read_off[wread[(size_t)w]];
        const int64_t as = std::max<int64_t>(0, s - 50);
        const int64_t ref_start = pos[h] + (s - as);
        const int64_t p = best[(size_t)w] >> 16, matches = best[(size_t)w] & 0xFFFF;
        int64_t motif_len = p;
        if (ref_start >= max_len) continue;
        const int64_t avail = std::max<int64_t>((max_len - ref_start) / motif_len, 0);
        if (avail == 0) continue;
        const int64_t copies_int = std::max<int64_t>(1, std::min<int64_t>(kT3Win / p, avail));
        const int64_t ref_end = ref_start + motif_len * copies_int;
        std::string cons((const char *)reads + wpos[(size_t)w], (size_t)p);   // motif = window[:p]
        double mm = 0.0;
        int64_t maxmm = 0;
        Rec r;
        r.pmatch = 100.0;
        r.score = 0;
        std::string cc;
        if (consensus_array(t, n, ref_start, motif_len, copies_int, cc, mm, maxmm)) {
            cons = cc;
            motif_len = (int64_t)cons.size();
        }
        // calculate_trf_statistics (1336-1366): ref_end <= max_len always holds here
        r.pmatch = (1.0 - mm) * 100.0;
        r.pindel = 0.0;
        r.score = trf_score(ref_end - ref_start, mm);
        std::string canon;
        canonical_stranded(cons, canon, r.strand);
        // summarize_variations_array over the index text (incl. '$'), min_copies = 1 (1259-1287)
        if (align_repeat_region((const char *)t, n, ref_start, std::min(ref_end, n), cons, 1, summ) &&
            summ.any_variation)
            r.variations = summ.variations;
        r.chrom = chrom;
        r.tier = 3;
        r.start = ref_start;
        r.end = ref_end;
        r.length = ref_end - ref_start;
        r.motif = cons;
        r.copies = (double)copies_int;
        r.confidence = (double)matches / (double)kT3Win;
        r.mismatch_rate = mm;
        r.max_mm = maxmm;
        r.n_eval = copies_int;
        r.act_kind = ACT_FULL;   // actual_sequence = text_arr[ref_start:ref_end] (1345-1346)
        r.act_off = ref_start;
        r.act_len = ref_end - ref_start;
        recs.push_back(std::move(r));
    }
    // _consolidate_repeat_calls (3003-3036): stable sort by (start, end), then a
    // fold merging overlapping calls with equal motifs into bare records
    std::stable_sort(recs.begin(), recs.end(), [](const Rec &a, const Rec &b) {
        return a.start != b.start ? a.start < b.start : a.end < b.end;
    });
    if (recs.empty()) return;
    Rec cur = recs[0];
    for (size_t k = 1; k < recs.size(); ++k) {
        const Rec &r = recs[k];
        if (r.start <= cur.end && r.motif == cur.motif) {
            Rec m;
            m.chrom = cur.chrom;
            m.start = std::min(cur.start, r.start);
            m.end = std::max(cur.end, r.end);
            m.motif = cur.motif;
            m.copies = (cur.copies + r.copies) / 2;
            m.length = m.end - m.start;
            m.tier = cur.tier;
            m.confidence = std::min(cur.confidence, r.confidence);
            m.stats_none = true;   // composition None, entropy 0.0, the other fields at their defaults
            cur = std::move(m);
        } else {
            out.push_back(std::move(cur));
            cur = r;
        }
    }
    out.push_back(std::move(cur));
}


// ------------------------------------------------- simple period scan (host)
namespace {
struct SimRes {
    int64_t as, ae, copies, fs, fe;
};

inline int64_t max_mm_for_array_host(int64_t L, int64_t c) {
    const int64_t tot = L * c;
    if (L == 1) return 0;
    const double f = L <= 6 ? 0.05 : 0.08;
    return std::max<int64_t>(1, (int64_t)std::ceil(f * (double)tot));
}

// _extend_with_mismatches (bwt.py:2392-2498), exact, any alphabet.  Each
// column keeps the symbols it has seen with their counts (a handful); the
// majority is the largest count, the smallest symbol on ties (the reference's
// first maximum over symbols in byte order).
SimRes simple_extend_host(const uint8_t *t, int64_t n, int64_t s0, int64_t p, bool allow) {
    struct Col {
        std::vector<std::pair<uint8_t, uint32_t>> v;
        void add(uint8_t b, int d) {
            for (auto &e : v)
                if (e.first == b) { e.second = (uint32_t)((int64_t)e.second + d); return; }
            v.push_back({b, (uint32_t)d});
        }
        char major(uint32_t &mx) const {
            mx = 0;
            int sym = 0;
            for (const auto &e : v)
                if (e.second > mx || (e.second == mx && e.second > 0 && e.first < sym)) { mx = e.second; sym = e.first; }
            return (char)sym;
        }
    };
    thread_local std::vector<Col> cnt;
    if ((int64_t)cnt.size() < p) cnt.resize((size_t)p);
    for (int64_t c = 0; c < p; ++c) {
        cnt[(size_t)c].v.clear();
        cnt[(size_t)c].add(t[s0 + c], 1);
    }
    std::string cons((const char *)t + s0, (size_t)p);
    int64_t start = s0, end = s0 + p, copies = 1;
    for (int dir = 0; dir < 2; ++dir) {
        for (;;) {
            if (dir == 0 ? (end + p > n) : (start - p < 0)) break;
            const int64_t at = dir == 0 ? end : start - p;
            const int64_t tc = copies + 1;
            int64_t mm = 0;
            for (int64_t c = 0; c < p; ++c) {
                cnt[(size_t)c].add(t[at + c], 1);
                uint32_t mx;
                cnt[(size_t)c].major(mx);
                mm += tc - mx;
            }
            if (mm <= (allow ? max_mm_for_array_host(p, tc) : 0)) {
                copies = tc;
                if (dir == 0) end += p;
                else start -= p;
                uint32_t mx;
                for (int64_t c = 0; c < p; ++c) cons[(size_t)c] = cnt[(size_t)c].major(mx);
            } else {
                for (int64_t c = 0; c < p; ++c) cnt[(size_t)c].add(t[at + c], -1);
                break;
            }
        }
    }
    int64_t pr = 0, pl = 0;
    while (pr < p && end + pr < n && t[end + pr] == (uint8_t)cons[(size_t)pr]) ++pr;
    while (pl < p && start - pl - 1 >= 0 && t[start - pl - 1] == (uint8_t)cons[(size_t)(p - 1 - pl)]) ++pl;
    return SimRes{start - pl, end + pr, copies, start, end};
}

struct SimWalk {
    int64_t p = 0, i = 0, iters = 0;
    bool done = false;
    std::vector<int64_t> accepts;   // positions i whose first extension was accepted, in walk order
    std::vector<int64_t> acc_iter;  // iteration number (1-based, within the walk) of each
    std::vector<SimRes> acc_res;    // and its first extension
    // first extensions of the current look-ahead, ascending positions: the walk
    // only moves forward, so a cursor replaces a map
    std::vector<int64_t> look_pos;
    std::vector<SimRes> look_res;
    size_t cur = 0;
    // the look-ahead's grid: look_start + k step <= look_last, every position
    // of it tested -- on it, "needs an extension" is membership in look_pos
    int64_t look_start = -1, look_last = -2, look_len = 0;
    bool on_grid(int64_t pos, int64_t step) const {
        return pos >= look_start && pos <= look_last && (pos - look_start) % step == 0;
    }
    const SimRes *find(int64_t pos) {
        while (cur < look_pos.size() && look_pos[cur] < pos) ++cur;
        return cur < look_pos.size() && look_pos[cur] == pos ? &look_res[cur] : nullptr;
    }
};
}  // namespace

// Tier2LCPFinder.find_long_repeats -> _find_repeats_simple (bwt.py:2097-2106,
// 2177-2390).  Walks (one per period) are independent: a step's outcome depends
// only on (position, period), and the seen-key set only decides which records
// are kept.  So every walk is simulated on the host, and the first extensions it
// needs (the costly part) are evaluated on the device in rounds of look-ahead
// batches -- the next kLook positions of the walk that pass the cheap tests
// (Tier 1 mask, '$'/'N', entropy), as if nothing were accepted before them.  The
// walks are then replayed in period order under the reference's global
// iteration cap (100,000) to build the records.  The reference also stops after
// 30 s of wall time (2238-2257); that machine-dependent stop is not reproduced.
void simple_scan_device(Ctx &c, DeviceIndex *ix, const LibParams &P, const std::vector<int64_t> &seen_pairs,
                        int32_t chrom, RecVec &out) {
    const int64_t nt = index_n(ix);
    if (nt == 0) return;
    std::vector<uint8_t> text((size_t)nt);
    index_get_text(c, ix, text.data());
    const uint8_t *t = text.data();
    int64_t n = nt;
    if (t[n - 1] == '$') --n;
    int64_t max_p = std::min<int64_t>(P.max_period, std::max<int64_t>(1, n / 2));
    if (n > 100000) max_p = std::min<int64_t>(max_p, 30);
    else if (n > 10000) max_p = std::min<int64_t>(max_p, 50);
    else if (n > 1000) max_p = std::min<int64_t>(max_p, 100);
    else max_p = std::min<int64_t>(max_p, 200);
    const int64_t min_p = std::min<int64_t>(P.min_period, max_p);
    int64_t step, pstep;
    if (n > 10000000) { step = 500; pstep = 20; }
    else if (n > 5000000) { step = 200; pstep = 10; }
    else if (n > 1000000) { step = 100; pstep = 5; }
    else if (n > 100000) { step = 50; pstep = 2; }
    else if (n > 10000) { step = 20; pstep = 1; }
    else { step = 10; pstep = 1; }
    constexpr int64_t kMaxIter = 100000;
    std::vector<uint8_t> mask((size_t)std::max<int64_t>(n, 1), 0);
    for (size_t q = 0; q + 1 < seen_pairs.size(); q += 2)
        for (int64_t x = std::max<int64_t>(0, seen_pairs[q]); x < std::min(seen_pairs[q + 1], n); ++x) mask[(size_t)x] = 1;
    std::vector<SimWalk> walks;
    for (int64_t p = min_p; p <= max_p; p += pstep) {
        SimWalk w;
        w.p = p;
        walks.push_back(w);
    }
    // cheap tests of position i for period p: true = the first extension is needed
    auto needs_ext = [&](int64_t i, int64_t p) {
        if (i < n && mask[(size_t)i]) return false;
        for (int64_t q = 0; q < p; ++q)
            if (t[i + q] == '$' || t[i + q] == 'N') return false;
        return !(entropy_of((const char *)t + i, p) < P.min_entropy);
    };
    const bool allow_all = P.allow_mismatches != 0;
    constexpr int kLook = 512;   // look-ahead positions per walk and round
    hipStream_t st = c.stream;
    using clk = std::chrono::steady_clock;
    const bool stats = stats_on();
    double t_host = 0, t_dev = 0;
    int64_t rounds = 0, nreq = 0;
    auto T0 = clk::now();
    std::vector<int64_t> req;        // (i, p | allow << 16)
    std::vector<int32_t> req_w;
    std::vector<std::vector<int64_t>> wreq(walks.size());   // each walk's look-ahead requests
    std::vector<int64_t> lower(walks.size(), 0);
    const int nthr = std::max(1, host_cpu_budget(nullptr, nullptr));
    for (;;) {
        // advance every walk until it needs an unknown extension; collect look-ahead
        // requests.  The walks run in parallel; each takes as the iterations of the
        // earlier walks (period order) their counts after the last round -- a lower
        // bound, so a walk stops at the global cap no earlier than in a serial pass
        // and the replay (which applies the cap exactly) sees the same accepts.
        for (size_t wi = 1; wi < walks.size(); ++wi) lower[wi] = lower[wi - 1] + walks[wi - 1].iters;
        run_tasks((int64_t)walks.size(), nthr, [&](int64_t wk) {
            const size_t wi = (size_t)wk;
            SimWalk &w = walks[wi];
            std::vector<int64_t> &wr = wreq[wi];
            wr.clear();
            const int64_t p = w.p;
            const bool allow = allow_all && p <= 64;
            while (!w.done) {
                if (w.i + 2 * p > n) { w.done = true; break; }
                if (lower[wi] + w.iters + 1 > kMaxIter) { w.done = true; break; }   // beyond the global cap
                const int64_t i = w.i;
                const SimRes *rp;
                if (w.on_grid(i, step)) {   // tested when the look-ahead was built
                    rp = w.find(i);
                    if (!rp) { ++w.iters; w.i += step; continue; }
                } else {
                    if (!needs_ext(i, p)) { ++w.iters; w.i += step; continue; }
                    rp = w.find(i);
                }
                SimRes wide;
                if (!rp && p > kSimMaxP) {            // wider than a wave's columns
                    wide = simple_extend_host(t, n, i, p, allow);
                    rp = &wide;
                }
                if (!rp) {   // a new look-ahead from i (positions of the old one are behind or off this grid)
                    // its length adapts: twice what the walk used of the last one
                    // (a walk that keeps jumping after accepts wastes little), 32..kLook
                    const int64_t used = (int64_t)w.cur;
                    w.look_len = w.look_len == 0 ? kLook : std::max<int64_t>(32, std::min<int64_t>(kLook, 2 * used));
                    w.look_pos.clear();
                    w.look_res.clear();
                    w.cur = 0;
                    w.look_start = i;
                    int64_t j = i, q = 0;
                    for (; q < w.look_len && j + 2 * p <= n; j += step) {
                        if (!needs_ext(j, p)) continue;
                        wr.push_back(j);
                        w.look_pos.push_back(j);
                        ++q;
                    }
                    w.look_last = j - step;
                    break;
                }
                ++w.iters;
                const SimRes &r = *rp;
                const int64_t alen = r.ae - r.as;
                bool acc = false;
                if (alen >= P.min_array_length) {
                    const int64_t part = std::max<int64_t>(0, alen - r.copies * p);
                    const double pf = (double)part / (double)p;
                    const int64_t eff = r.copies + (pf >= 0.75 ? 1 : 0);
                    acc = r.copies >= P.min_copies || eff >= P.min_copies;
                }
                if (!acc) { w.i += step; continue; }
                w.accepts.push_back(i);
                w.acc_iter.push_back(w.iters);
                w.acc_res.push_back(r);
                // the walk resumes at the (second-extension) array end, decided on the host
                const int64_t fs = r.fs;
                const int64_t prim = smallest_period((const char *)t + fs, p);
                const int64_t pe = prim < p ? prim : p;
                const SimRes r2 = simple_extend_host(t, n, fs, pe, allow_all && pe <= 64);
                int64_t ae = r2.ae;
                const int64_t alen2 = r2.ae - r2.as;
                const int64_t part2 = std::max<int64_t>(0, alen2 - r2.copies * pe);
                const double pf2 = (double)part2 / (double)pe;
                const int64_t eff2 = r2.copies + (pf2 >= 0.75 ? 1 : 0);
                if (r2.copies < P.min_copies && eff2 < P.min_copies) { w.i += step; continue; }
                std::string cons;
                double mm = 0;
                int64_t maxmm = 0;
                if (!consensus_array(t, nt, r2.fs, pe, r2.copies, cons, mm, maxmm)) { w.i += step; continue; }
                const int64_t pl = smallest_period(cons.data(), (int64_t)cons.size());
                if (pl < (int64_t)cons.size()) {
                    const int64_t cf = std::max<int64_t>(1, (r2.ae - r2.as) / pl);
                    ae = r2.as + cf * pl;
                    if (!consensus_array(t, nt, r2.as, pl, cf, cons, mm, maxmm)) { w.i += step; continue; }
                }
                w.i = ae;
            }
        });
        req.clear();
        req_w.clear();
        for (size_t wi = 0; wi < walks.size(); ++wi) {
            const int64_t pw = walks[wi].p | (allow_all && walks[wi].p <= 64 ? (1 << 16) : 0);
            for (int64_t j : wreq[wi]) {
                req.push_back(j);
                req.push_back(pw);
                req_w.push_back((int32_t)wi);
            }
        }
        auto T1 = clk::now();
        t_host += std::chrono::duration<double, std::milli>(T1 - T0).count();
        T0 = T1;
        if (req.empty()) {
            for (auto &w : walks)
                if (!w.done) fail(BWTMI_E_STATE, "simple scan: walk of period %lld stalled", (long long)w.p);
            break;
        }
        // device batch through the context's pinned staging buffer: requests
        // in, (5 words + overflow flag) per request out
        const int64_t nr = (int64_t)req_w.size();
        ++rounds;
        nreq += nr;
        c.slot[S_IDX1].ensure((size_t)nr * 16);
        c.slot[S_IDX2].ensure((size_t)nr * 48);
        HBuf &hb = c.host[0];
        hb.ensure((size_t)nr * 48);
        std::memcpy(hb.p, req.data(), (size_t)nr * 16);
        HIPCHECK(hipMemcpyAsync(c.slot[S_IDX1].p, hb.p, (size_t)nr * 16, hipMemcpyHostToDevice, st));
        int64_t *d_res = c.slot[S_IDX2].as<int64_t>();
        uint8_t *d_ovf = reinterpret_cast<uint8_t *>(d_res + 5 * nr);
        // the index's own text (the bytes downloaded above), not a fresh upload per batch
        KLAUNCH("k_simple_extend", 0.0, k_simple_extend, dim3((unsigned)((nr + 3) / 4)), dim3(256), 0, st,
                index_text_device(ix), n, c.slot[S_IDX1].as<int64_t>(), nr, d_res, d_ovf);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(hb.p, d_res, (size_t)nr * 41, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        const int64_t *res = hb.as<int64_t>();
        const uint8_t *ovf = reinterpret_cast<const uint8_t *>(res + 5 * nr);
        for (int64_t q = 0; q < nr; ++q) {
            const int64_t i = req[(size_t)(2 * q)], pw = req[(size_t)(2 * q + 1)];
            SimRes r;
            if (ovf[q])
                r = simple_extend_host(t, n, i, pw & 0xFFFF, (pw >> 16) & 1);
            else
                r = SimRes{res[5 * q], res[5 * q + 1], res[5 * q + 2], res[5 * q + 3], res[5 * q + 4]};
            walks[(size_t)req_w[(size_t)q]].look_res.push_back(r);   // requests of a walk: ascending, in order
        }
        T1 = clk::now();
        t_dev += std::chrono::duration<double, std::milli>(T1 - T0).count();
        T0 = T1;
    }
    if (stats)
        std::fprintf(stderr, "  simple scan: %lld walks, %lld rounds, %lld requests, host walk %.1f ms, device batches %.1f ms\n",
                     (long long)walks.size(), (long long)rounds, (long long)nreq, t_host, t_dev);
    // replay in period order under the global cap: records of the accepted positions
    std::set<std::tuple<int64_t, int64_t, std::string>> seen;
    const std::string seq((const char *)t, (size_t)nt);
    AlignSummary summ;
    int64_t cum = 0;
    for (size_t wi = 0; wi < walks.size(); ++wi) {
        const SimWalk &w = walks[wi];
        const int64_t p = w.p;
        for (size_t a = 0; a < w.accepts.size(); ++a) {
            if (cum + w.acc_iter[a] > kMaxIter) break;
            const SimRes &r = w.acc_res[a];
            const int64_t prim = smallest_period((const char *)t + r.fs, p);
            int64_t pe = prim < p ? prim : p;
            const SimRes r2 = simple_extend_host(t, n, r.fs, pe, allow_all && pe <= 64);
            int64_t as = r2.as, ae = r2.ae, cf = r2.copies;
            const int64_t alen2 = ae - as;
            const int64_t part2 = std::max<int64_t>(0, alen2 - cf * pe);
            const double pf2 = (double)part2 / (double)pe;
            const int64_t eff2 = cf + (pf2 >= 0.75 ? 1 : 0);
            if (cf < P.min_copies && eff2 < P.min_copies) continue;
            std::string cons;
            double mm = 0;
            int64_t maxmm = 0;
            if (!consensus_array(t, nt, r2.fs, pe, cf, cons, mm, maxmm)) continue;
            const int64_t pl = smallest_period(cons.data(), (int64_t)cons.size());
            if (pl < (int64_t)cons.size()) {
                pe = pl;
                cf = std::max<int64_t>(1, (ae - as) / pe);
                ae = as + cf * pe;
                if (!consensus_array(t, nt, as, pe, cf, cons, mm, maxmm)) continue;
            }
            std::string canon;
            char strand = '+';
            canonical_stranded(cons, canon, strand);
            if (!seen.insert(std::make_tuple(as, ae, canon)).second) continue;
            Rec rec;
            rec.chrom = chrom;
            rec.tier = 2;
            rec.start = as;
            rec.end = ae;
            rec.length = ae - as;
            rec.motif = cons;
            rec.copies = (double)cf;
            rec.confidence = std::max(0.5, 0.95 - mm);
            rec.mismatch_rate = mm;
            rec.max_mm = maxmm;
            rec.n_eval = cf;
            rec.strand = strand;
            rec.pmatch = (1.0 - mm) * 100.0;
            rec.pindel = 0.0;
            rec.score = trf_score(ae - as, mm);
            rec.act_kind = ACT_FULL;
            rec.act_off = as;
            rec.act_len = ae - as;
            if (ae > as && align_repeat_region(seq.data(), nt, as, ae, cons, 1, summ) && summ.any_variation)
                rec.variations = summ.variations;
            out.push_back(std::move(rec));
        }
        cum += w.iters;
        if (cum >= kMaxIter) break;
    }
    if (stats)
        std::fprintf(stderr, "  simple scan: replay %.1f ms (%zu records)\n",
                     std::chrono::duration<double, std::milli>(clk::now() - T0).count(), out.size());
}

}  // namespace bwtmi
