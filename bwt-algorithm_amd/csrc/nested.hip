// nested.hip -- nested-repeat suppression, position sort and dedup of one
// contig's strict hits, on the device where the scan left them.
//
// Replaces, for strict hits (mismatch_rate 0, one class), the worker-side
// _filter_nested_repeats (bwt.py:3402-3497), the (start, end) sort that
// follows it and _deduplicate_repeats (bwt.py:3189-3220):
//
//   * a hit r (start s0, end e0, primitive motif length m) is suppressed when
//     a KEPT hit of strictly longer motif M overlaps it by ov with
//     ov / (e0 - s0) >= t(M / m) (t = 0.1 / 0.3 / 0.5, or 0.8 when m == 1);
//     hits are decided in descending m, so the kept set a query sees is
//     exactly the reference's;
//   * the survivors, stable-sorted by (start, end), keep the reference's tie
//     order (m desc, then worker order), i.e. the total order
//     (start, end, m desc, hit index);
//   * dedup keys (start, end, motif) of strict hits reduce to (start, end, m)
//     (the motif is text[start, start + m)); equal keys are adjacent in that
//     order and share the nested decision, and every field dedup compares
//     (confidence 0.95, mismatch 0, tier 2) ties, so the first one stays.
//
// Kernels: two stable LSD radix sorts give the position order P (by
// (len, m desc) then start) and the level order G (by m desc); the position
// arrays S/E/M and an inclusive prefix max of E (PME) are gathered once, with
// a bucket table of S (first rank per 64 bp).  One launch per distinct m
// (descending) decides that level: each hit finds the last span starting
// before e0 (bucket + short binary search) and walks P backwards until PME
// drops to s0 -- every span that can overlap r lies in that window; small
// levels (long motifs, long walks) use a wave per hit, 64 ranks per step.  A
// final flag/scan/compact pass writes the kept, deduplicated hits in P order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kB = 256;
constexpr int kTile = 4096;

inline unsigned blocks(int64_t n) { return (unsigned)((n + kB - 1) / kB); }
inline int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b) != 0) ++b;
    return b;
}

__global__ void k_maxlen(const bwtmi_hit *__restrict__ H, int64_t n, unsigned long long *__restrict__ out) {
    __shared__ unsigned long long red[kB];
    unsigned long long v = 0;
    for (int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        v = max(v, (unsigned long long)(H[i].end - H[i].start));
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = kB / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(out, red[0]);
}

// position sort, stage 1 key: (len << mb) | (lmax - m); group key: lmax - m
// sshift >= 0: the start goes above (len, g) in the same key, so one sort
// orders by (start, len, g) -- what the two stable sorts give
__global__ void k_keys(const bwtmi_hit *__restrict__ H, int64_t n, int mb, int64_t lmax, uint64_t *__restrict__ kpos,
                       uint32_t *__restrict__ vpos, uint64_t *__restrict__ kgrp, uint32_t *__restrict__ vgrp,
                       int sshift) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const bwtmi_hit h = H[i];
    const uint64_t g = (uint64_t)(lmax - h.prim_len);
    kpos[i] = ((uint64_t)(h.end - h.start) << mb) | g | (sshift >= 0 ? (uint64_t)h.start << sshift : 0ull);
    vpos[i] = (uint32_t)i;
    kgrp[i] = g;
    vgrp[i] = (uint32_t)i;
}

// stage 2 key: start of the hit now at rank k
__global__ void k_keys_start(const bwtmi_hit *__restrict__ H, int64_t n, const uint32_t *__restrict__ vpos,
                             uint64_t *__restrict__ kpos) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    kpos[k] = (uint64_t)H[vpos[k]].start;
}

__global__ void k_gather(const bwtmi_hit *__restrict__ H, int64_t n, const uint32_t *__restrict__ vpos,
                         int64_t *__restrict__ S, int64_t *__restrict__ E, int32_t *__restrict__ M,
                         uint32_t *__restrict__ rank_of, uint8_t *__restrict__ kept) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const uint32_t idx = vpos[k];
    const bwtmi_hit h = H[idx];
    S[k] = h.start;
    E[k] = h.end;
    M[k] = h.prim_len;
    rank_of[idx] = (uint32_t)k;
    kept[k] = 0;
}

// level boundaries: first[g] = first position of group key g in the G order
__global__ void k_bounds(const uint64_t *__restrict__ kgrp, int64_t n, int64_t *__restrict__ first) {
    const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (j >= n) return;
    if (j == 0 || kgrp[j] != kgrp[j - 1]) first[kgrp[j]] = j;
}

// ---- inclusive prefix max (int64), tiles of 4096
__global__ __launch_bounds__(kB) void k_tile_max(const int64_t *__restrict__ in, int64_t *__restrict__ out, int64_t n) {
    __shared__ int64_t red[kB];
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int64_t v = INT64_MIN;
    for (int i = 0; i < kTile / kB; ++i) {
        const int64_t idx = base + (int64_t)i * kB + threadIdx.x;
        if (idx < n) v = max(v, in[idx]);
    }
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = kB / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + o]);
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// inclusive max scan of one tile, seeded with the inclusive max of all
// earlier tiles (pre[blockIdx.x - 1]).  Wave w owns 1024 consecutive items
// in the (item, lane) layout, so every load and store is one coalesced
// 512-byte row; each row is max-scanned across the lanes (shuffles) and
// carries its last lane into the next row, then the four wave totals seed
// the waves after them.  (Sixteen consecutive items per thread made each
// load instruction touch 64 lines: 121 us at C3 for 43 MB, r05fc.)
__device__ __forceinline__ int64_t wave_incl_max(int64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t u = __shfl_up(x, o, 64);
        if (lane >= o) x = max(x, u);
    }
    return x;
}
// (in == out is allowed: a wave reads all its items before it writes them)
__global__ __launch_bounds__(kB) void k_tile_scan_max(const int64_t *in, int64_t *out, const int64_t *__restrict__ pre,
                                                      int64_t n) {
    constexpr int kI = kTile / kB;   // rows of 64 items per wave
    __shared__ int64_t wtot[kB / 64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)wv * (kI * 64) + lane;
    int64_t loc[kI];
#pragma unroll
    for (int i = 0; i < kI; ++i) {
        const int64_t idx = base + (int64_t)i * 64;
        loc[i] = idx < n ? in[idx] : INT64_MIN;
    }
    int64_t carry = INT64_MIN;
#pragma unroll
    for (int i = 0; i < kI; ++i) {
        const int64_t x = max(wave_incl_max(loc[i]), carry);
        loc[i] = x;
        carry = __shfl(x, 63, 64);
    }
    if (lane == 0) wtot[wv] = carry;
    __syncthreads();
    int64_t seed = INT64_MIN;
    for (int w = 0; w < wv; ++w) seed = max(seed, wtot[w]);
    if (pre && blockIdx.x > 0) seed = max(seed, pre[blockIdx.x - 1]);
#pragma unroll
    for (int i = 0; i < kI; ++i) {
        const int64_t idx = base + (int64_t)i * 64;
        if (idx < n) out[idx] = max(loc[i], seed);
    }
}

void prefix_max(Ctx &c, const int64_t *in, int64_t *out, int64_t n, int64_t *tmp) {
    const int64_t nt = (n + kTile - 1) / kTile;
    if (nt == 1) {
        KLAUNCH("k_tile_scan_max", 0.0, k_tile_scan_max, dim3(1), dim3(kB), 0, c.stream, in, out, (const int64_t *)nullptr, n);
        return;
    }
    int64_t *tm = tmp;
    KLAUNCH("k_tile_max", 0.0, k_tile_max, dim3((unsigned)nt), dim3(kB), 0, c.stream, in, tm, n);
    prefix_max(c, tm, tm, nt, tmp + nt);   // inclusive max over tiles
    KLAUNCH("k_tile_scan_max", 0.0, k_tile_scan_max, dim3((unsigned)nt), dim3(kB), 0, c.stream, in, out, (const int64_t *)tm, n);
}

// position buckets: B[b] = first rank k with S[k] >= b << kBucketShift (n if
// none), so a search for "first rank with S >= x" starts inside one bucket
// (a few hits) instead of spanning all n ranks with ~23 dependent loads
constexpr int kBucketShift = 6;
constexpr int64_t kWaveLevelMax = 65536;   // levels up to this many hits use k_level_wave

__global__ void k_buckets(const int64_t *__restrict__ S, int64_t n, int64_t nb, uint32_t *__restrict__ B) {
    const int64_t b = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (b >= nb) return;
    const int64_t x = b << kBucketShift;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (S[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    B[b] = (uint32_t)lo;
}

// the nested test of hit (s0, e0, m) against a kept span (Sk, Ek) of longer
// motif Mk > m (bwt.py:3460-3490, overlap_threshold 0.5 as both CLI call
// sites pass it, bwt.py:3829 / 3928), in integers: for the thresholds t =
// p / q in {0.1, 0.3, 0.5, 0.8} the reference's float test ov / rl >= t holds
// exactly when q ov >= p rl (a ratio below p / q differs from it by at least
// 1 / (q rl), far above the rounding of either double), and Mk / m >= 10 / 5
// exactly when Mk >= 10 m / 5 m.  No division in the walks.
__device__ __forceinline__ bool nested_by(int64_t s0, int64_t e0, int64_t m, int64_t rl, int64_t Sk, int64_t Ek,
                                          int64_t Mk) {
    const int64_t ov = min(e0, Ek) - max(s0, Sk);
    if (ov <= 0) return false;
    if (m == 1 && Mk > 1 && 5 * ov >= 4 * rl) return true;   // frac >= 0.8
    if (Mk >= 10 * m) return 10 * ov >= rl;                    // >= 0.1
    if (Mk >= 5 * m) return 10 * ov >= 3 * rl;                 // >= 0.3
    return 2 * ov >= rl;                                       // >= 0.5
}

// All levels in one launch, segment by segment.  Hits overlap only inside a
// "segment" of the position order (k starts one iff PME[k-1] <= S[k]: no
// earlier span reaches past it), so segments are independent and the level
// order only matters inside each.  Window w = the segments that START in
// positions [w W, (w+1) W) of the order; a workgroup copies its window's spans
// to LDS and decides them level by level (descending m, a workgroup barrier
// between levels) -- instead of one launch per distinct m (119 launches, ~1.5
// ms of a 12.5 Mbp scan).  Two sizes: 256-thread workgroups holding up to
// kSegCapS hits (many per CU), and for the windows whose segments overflow
// them (long arrays: chains of overlapping spans) 1024-thread workgroups
// holding kSegCapL; past that the caller falls back to the per-level launches.
constexpr int kSegWin = 512;           // nominal positions per window
constexpr int kSegCapS = 1024;         // hits a small workgroup holds
constexpr int kSegCapL = 4096;         // hits a large workgroup holds

// LARGE = false: window blockIdx.x, overflowing windows are appended to ovf_win;
// LARGE = true: the windows listed in ovf_win (*ovf_n of them), a grid-stride
// loop; a window past kSegCapL sets *fallback
template <int T, int CAP, int WIN, bool LARGE>
__global__ __launch_bounds__(T) void k_seg_levels(const int64_t *__restrict__ S, const int64_t *__restrict__ E,
                                                  const int32_t *__restrict__ M, const int64_t *__restrict__ PME,
                                                  int64_t n, uint8_t *__restrict__ kept, uint32_t *__restrict__ ovf_win,
                                                  unsigned int *__restrict__ ovf_n, unsigned int *__restrict__ fallback) {
    __shared__ int64_t sS[CAP], sE[CAP], sP[CAP];
    __shared__ int32_t sM[CAP];
    __shared__ uint8_t sK[CAP];
    __shared__ int16_t sF[CAP];
    __shared__ unsigned long long found;
    __shared__ int64_t pm1;   // PME[w0 - 1]
    __shared__ int pend[3];
    const int tid = threadIdx.x;
    const int64_t nwin = LARGE ? (int64_t)*ovf_n : (int64_t)gridDim.x;
    for (int64_t q = blockIdx.x; q < nwin; q += LARGE ? (int64_t)gridDim.x : nwin) {
        const int64_t w = LARGE ? (int64_t)ovf_win[q] : q;
        const int64_t w0 = w * WIN;
        const int64_t w1 = w0 + WIN < n ? w0 + WIN : n;
        // The window's entries from w0 on, up to CAP of them, go to LDS in one
        // pass: its segments start at a >= w0 and end at b <= a + CAP, so that
        // copy is the window's whenever a == w0 (nearly always), and the two
        // head searches below read LDS -- one round trip to memory per window
        // instead of three (head search, end search, copy).
        // (the window and a quarter more: its segments nearly always end
        // there; loading all CAP entries read twice what a window uses)
        constexpr int64_t kLoad = WIN + WIN / 4 < CAP ? WIN + WIN / 4 : CAP;
        const int64_t L0 = w0 + kLoad < n ? kLoad : n - w0;
        for (int i = tid; i < L0; i += T) {
            sS[i] = S[w0 + i];
            sE[i] = E[w0 + i];
            sP[i] = PME[w0 + i];
            sM[i] = M[w0 + i];
        }
        if (tid == 0) {
            found = ~0ull;
            pm1 = w0 > 0 ? PME[w0 - 1] : INT64_MIN;
        }
        __syncthreads();
        // k >= w0 starts a segment: k == 0 or PME[k - 1] <= S[k] (LDS where loaded)
        auto head_at = [&](int64_t k) -> bool {
            if (k == 0) return true;
            const int64_t j = k - w0;
            const int64_t pp = j == 0 ? pm1 : (j - 1 < L0 ? sP[j - 1] : PME[k - 1]);
            return pp <= (j < L0 ? sS[j] : S[k]);
        };
        // a = the window's first segment head (none: a segment from an earlier window covers it)
        for (int64_t k = w0 + tid; k < w1; k += T)
            if (head_at(k)) atomicMin(&found, (unsigned long long)k);
        __syncthreads();
        const int64_t a = (int64_t)found;   // uniform
        __syncthreads();
        if (a == (int64_t)~0ull) continue;
        // b = the first segment head at or after w1 (n if none), looked for up to a + CAP
        if (tid == 0) found = ~0ull;
        __syncthreads();
        const int64_t lim = a + CAP < n ? a + CAP : n;
        for (int64_t k = w1 + tid; k <= lim; k += T)
            if (k == n || head_at(k)) atomicMin(&found, (unsigned long long)k);
        __syncthreads();
        const int64_t b = (int64_t)found;
        __syncthreads();
        if (b == (int64_t)~0ull || b - a > CAP) {   // the window's segments do not fit
            if (tid == 0) {
                if (LARGE) atomicOr(fallback, 1u);
                else ovf_win[atomicAdd(ovf_n, 1u)] = (uint32_t)w;
            }
            continue;
        }
        const int len = (int)(b - a);
        if (a != w0 || b - w0 > L0) {   // not the loaded range: the window's own copy
            for (int i = tid; i < len; i += T) {
                sS[i] = S[a + i];
                sE[i] = E[a + i];
                sP[i] = PME[a + i];
                sM[i] = M[a + i];
            }
            __syncthreads();
        }
        // a hit that no span of a longer motif could nest (kept or not) is kept
        // whatever the levels decide: only the others (kUndecided) take part in
        // the level loop, whose levels are then the distinct motif lengths among them
        constexpr uint8_t kUndecided = 2;
        // the first pass walks each hit's window back from its end to the first
        // span of a longer motif that would nest it (kept or not) and remembers
        // where: a hit with none is kept whatever the others decide, the rest
        // (kUndecided) resume their walk there -- no nester lies above it
        auto first_nester = [&](int i) -> int {   // local rank of the first possible nester, -1 none
            const int64_t s0 = sS[i], e0 = sE[i], rl = e0 - s0;
            const int64_t m = sM[i];
            if (rl <= 0) return -1;
            int lo = i + 1, hi = len;   // first local rank with S >= e0 (S[i] = s0 < e0)
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (sS[mid] < e0) lo = mid + 1;
                else hi = mid;
            }
            for (int k = lo - 1; k >= 0 && sP[k] > s0; --k) {
                const int64_t Mk = sM[k];
                if (Mk > m && nested_by(s0, e0, m, rl, sS[k], sE[k], Mk)) return k;
            }
            return -1;
        };
        for (int i = tid; i < len; i += T) {
            const int k = first_nester(i);
            sK[i] = k >= 0 ? kUndecided : 1;
            sF[i] = (int16_t)k;
        }
        // Rounds instead of levels: an undecided hit is decided as soon as the
        // longer-motif spans that would nest it are decided -- suppressed by the
        // first KEPT one (final, whatever else is pending), kept when none is
        // kept and none is pending.  That is the reference's level order's
        // outcome (a hit only ever reads decisions of strictly longer motifs),
        // reached in as many rounds as the longest chain of such dependencies
        // (a handful) instead of one barrier pair per distinct motif length.
        volatile uint8_t *vK = sK;   // entries of other hits change during a round
        auto decide = [&](int i) -> uint8_t {   // 0 nested, 1 kept, kUndecided: wait
            const int64_t s0 = sS[i], e0 = sE[i], rl = e0 - s0;
            const int64_t m = sM[i];
            bool wait = false;
            for (int k = sF[i]; k >= 0 && sP[k] > s0; --k) {
                const int64_t Mk = sM[k];
                if (Mk <= m) continue;
                const uint8_t dk = vK[k];
                if (dk == 0) continue;
                if (nested_by(s0, e0, m, rl, sS[k], sE[k], Mk)) {
                    if (dk == 1) return 0;
                    wait = true;
                }
            }
            return wait ? kUndecided : 1;
        };
        if (tid == 0) pend[0] = pend[1] = pend[2] = 0;
        __syncthreads();
        for (int r = 0;; ++r) {
            for (int i = tid; i < len; i += T) {
                if (vK[i] != kUndecided) continue;
                const uint8_t res = decide(i);
                if (res == kUndecided) pend[r % 3] = 1;
                else vK[i] = res;
            }
            // the flag of round r + 1: last read after round r - 2's barrier
            if (tid == 0) pend[(r + 1) % 3] = 0;
            __syncthreads();
            if (!pend[r % 3]) break;   // uniform: not reset before round r + 2
        }
        for (int i = tid; i < len; i += T) kept[a + i] = sK[i];
        __syncthreads();   // the LDS is refilled by the next window
    }
}

// one level (all hits of one primitive length m): nested test against the
// kept spans of longer motif (bwt.py:3460-3490), predicate division for division
__global__ __launch_bounds__(kB) void k_level(const uint32_t *__restrict__ lvl, int64_t cnt,
                                              const bwtmi_hit *__restrict__ H, const uint32_t *__restrict__ rank_of,
                                              const int64_t *__restrict__ S, const int64_t *__restrict__ E,
                                              const int32_t *__restrict__ M, const int64_t *__restrict__ PME,
                                              const uint32_t *__restrict__ B, uint8_t *__restrict__ kept, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (t >= cnt) return;
    const uint32_t idx = lvl[t];
    const bwtmi_hit h = H[idx];
    const int64_t s0 = h.start, e0 = h.end, m = h.prim_len, rl = e0 - s0;
    bool nested = false;
    if (rl > 0) {
        // first rank with S >= e0: inside bucket e0 >> shift (e0 <= text_len)
        const int64_t bk = e0 >> kBucketShift;
        int64_t lo = B[bk], hi = B[bk + 1];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (S[mid] < e0) lo = mid + 1;
            else hi = mid;
        }
        for (int64_t k = lo - 1; k >= 0 && PME[k] > s0; --k) {
            const int64_t Mk = M[k];
            if (Mk <= m || !kept[k]) continue;   // same-level entries are being written now: never read
            if (nested_by(s0, e0, m, rl, S[k], E[k], Mk)) { nested = true; break; }
        }
    }
    kept[rank_of[idx]] = nested ? 0 : 1;
}

// the same test with one WAVE per hit: the 64 lanes walk 64 consecutive ranks
// at a time.  Long-motif levels hold few hits but long spans, whose backward
// walks cover hundreds of ranks -- one lane walking them serially leaves the
// launch latency-bound.  The visited set {k <= lo-1 : PME[k] > s0} is a
// contiguous range (PME is non-decreasing), and the outcome is an "any".
__global__ __launch_bounds__(kB) void k_level_wave(const uint32_t *__restrict__ lvl, int64_t cnt,
                                                   const bwtmi_hit *__restrict__ H, const uint32_t *__restrict__ rank_of,
                                                   const int64_t *__restrict__ S, const int64_t *__restrict__ E,
                                                   const int32_t *__restrict__ M, const int64_t *__restrict__ PME,
                                                   const uint32_t *__restrict__ B, uint8_t *__restrict__ kept,
                                                   int64_t n) {
    const int lane = threadIdx.x & 63;
    const int64_t t = ((int64_t)blockIdx.x * kB + threadIdx.x) >> 6;
    if (t >= cnt) return;   // wave-uniform
    const uint32_t idx = lvl[t];
    const bwtmi_hit h = H[idx];
    const int64_t s0 = h.start, e0 = h.end, m = h.prim_len, rl = e0 - s0;
    bool nested = false;
    if (rl > 0) {
        const int64_t bk = e0 >> kBucketShift;
        int64_t lo = B[bk], hi = B[bk + 1];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (S[mid] < e0) lo = mid + 1;
            else hi = mid;
        }
        for (int64_t top = lo - 1; top >= 0; top -= 64) {
            const int64_t k = top - lane;
            const bool live = k >= 0 && PME[k] > s0;
            bool hit = false;
            if (live) {
                const int64_t Mk = M[k];
                if (Mk > m && kept[k])   // same-level entries are being written now: never read
                    hit = nested_by(s0, e0, m, rl, S[k], E[k], Mk);
            }
            if (__any(hit)) {
                nested = true;
                break;
            }
            if (!__all(live)) break;
        }
    }
    if (lane == 0) kept[rank_of[idx]] = nested ? 0 : 1;
}

// ---- records the post-processing would only carry to its final filter.
// A kept hit that fails the final filter on its own (bwt.py:3940-3944:
// (end - start) // prim < min_copies or end - start < 6 -- an unmerged strict
// record keeps its span and copies) and that no other record can reach leaves
// the output unchanged when it is dropped here:
//   merge (bwt.py:3222-3289): a merge needs same canonical motifs (equal
//     motif lengths M) within a gap of M + 1.  A record built from records
//     before the hit ends at most at max(e, s + M min_copies) + 2 ext(M) of
//     one of them (the recompute's walk limit, motif.cpp / post.cpp, once for
//     the merge and once for the refine; ext(M) = max(3M, 4 min(10, M/2 or 1))),
//     A one-base record is the closed form: the run of its first base through
//     its start, capped at the walk limit -- a unit-1 strict hit is a maximal
//     run, so a record built from such hits ends at its first hit's end, and
//     it has no mismatches to refine: its bound is its end.
//     So with R = max over the earlier kept hits of that bound,
//     start - R > M_hit + 1 keeps every earlier record out of reach; with
//     next.start - end > max(M_hit, M_next) + 1 the hit merges with nothing
//     after it, and neither does the record before it once it is gone (the
//     removed hit's own gap lies between them);
//   collapse (bwt.py:3499-3513) needs an overlap: the hit overlaps nothing, and
//     nothing that was separated by it overlaps after it is gone.
// R over the kept hits in screen order is an inclusive prefix max of reach()
// (non-kept entries contribute nothing; k_final_flags writes it); the next
// kept hit is found by a short probe forward (kept hits are dense: a probe
// that finds none within kDropProbe ranks keeps the hit).
constexpr int kDropProbe = 64;
__device__ __forceinline__ int64_t screen_reach(int64_t s, int64_t e, int64_t m, int32_t mc) {
    if (m == 1) return e;
    const int64_t mi = m >= 4 ? min<int64_t>(10, m / 2) : 1;
    const int64_t ext = max<int64_t>(3 * m, 4 * mi);
    return max(e, s + m * (int64_t)mc) + 2 * ext;
}
// out[k] = flag[k], cleared for a droppable kept hit (R: inclusive prefix max;
// flag is read only, so every probe sees the kept set before the drop)
__global__ void k_drop_flags(const int64_t *__restrict__ S, const int64_t *__restrict__ E,
                             const int32_t *__restrict__ M, const uint32_t *__restrict__ flag,
                             const int64_t *__restrict__ R, int64_t n, int32_t mc, uint32_t *__restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const uint32_t f = flag[k];
    out[k] = f;
    if (!f) return;
    const int64_t s = S[k], e = E[k], m = max<int64_t>(1, M[k]), len = e - s;
    if (len / m >= (int64_t)mc && len >= 6) return;   // passes the final filter: kept
    if (k > 0 && R[k - 1] != INT64_MIN && s - R[k - 1] <= m + 1) return;
    int64_t q = k + 1;
    while (q < n && !flag[q] && q - k < kDropProbe) ++q;
    if (q < n) {
        if (!flag[q]) return;   // no kept hit within the probe: keep
        const int64_t mq = max<int64_t>(1, M[q]);
        if (S[q] - e <= max(m, mq) + 1) return;
    }
    out[k] = 0u;
}

// R (drop_mc > 0): the reach of each kept hit, INT64_MIN elsewhere (k_drop_flags)
__global__ void k_final_flags(const int64_t *__restrict__ S, const int64_t *__restrict__ E,
                              const int32_t *__restrict__ M, const uint8_t *__restrict__ kept, int64_t n,
                              uint32_t *__restrict__ flag, int32_t drop_mc, int64_t *__restrict__ R) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    bool f = kept[k] != 0;
    if (f && k > 0 && S[k - 1] == S[k] && E[k - 1] == E[k] && M[k - 1] == M[k]) f = false;
    flag[k] = f ? 1u : 0u;
    if (drop_mc > 0) R[k] = f ? screen_reach(S[k], E[k], max<int64_t>(1, M[k]), drop_mc) : INT64_MIN;
}

// kept hits in screen order, one 64-bit word each (lbits >= 0: start | len << 32
// | prim << (32 + lbits)) or two ({start, len | prim << 32}); common.h ScreenedVec
__global__ void k_final_compact(const bwtmi_hit *__restrict__ H, const uint32_t *__restrict__ vpos,
                                const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos, int64_t n,
                                int lbits, uint64_t *__restrict__ out) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= n || !flag[k]) return;
    const bwtmi_hit h = H[vpos[k]];
    const uint64_t len = (uint64_t)(h.end - h.start), prim = (uint64_t)(uint32_t)h.prim_len;
    if (lbits >= 0) {
        out[pos[k]] = (uint64_t)(uint32_t)h.start | len << 32 | prim << (32 + lbits);
    } else {
        out[2 * (int64_t)pos[k]] = (uint64_t)h.start;
        out[2 * (int64_t)pos[k] + 1] = (len & 0xFFFFFFFFull) | prim << 32;
    }
}

}  // namespace

// the per-level path: the hits in level order G (descending m), one launch per
// level (also the fallback of k_seg_levels when segments exceed its LDS)
static void screen_levels(Ctx &c, const bwtmi_hit *d_hits, int64_t n, int32_t lmax, int mb, uint64_t *kgrp,
                          uint32_t *vgrp, const uint32_t *rank_of, const int64_t *S, const int64_t *E, const int32_t *M,
                          const int64_t *PME, uint8_t *kept, int64_t nb) {
    hipStream_t st = c.stream;
    const int gb = ((mb + 7) / 8) * 8;
    radix_sort_pairs32(c, kgrp, vgrp, n, 0, gb);
    uint32_t *B = c.slot[S_IDX6].as<uint32_t>();
    KLAUNCH("k_buckets", 0.0, k_buckets, dim3(blocks(nb)), dim3(kB), 0, st, S, n, nb, B);
    int64_t *first = c.slot[S_COUNTS].as<int64_t>();
    HIPCHECK(hipMemsetAsync(first, 0xff, (size_t)(lmax + 2) * 8, st));
    KLAUNCH("k_bounds", 0.0, k_bounds, dim3(blocks(n)), dim3(kB), 0, st, kgrp, n, first);
    std::vector<int64_t> fh((size_t)lmax + 2);
    HIPCHECK(hipMemcpyAsync(fh.data(), first, fh.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipGetLastError());
    scan_wait(st);
    // levels in descending m (ascending group key)
    std::vector<std::pair<int64_t, int64_t>> lv;   // (first, group key)
    for (int64_t g = 0; g <= lmax; ++g)
        if (fh[(size_t)g] >= 0) lv.push_back({fh[(size_t)g], g});
    for (size_t q = 0; q < lv.size(); ++q) {
        const int64_t a = lv[q].first, b = q + 1 < lv.size() ? lv[q + 1].first : n;
        if (b - a <= kWaveLevelMax)   // few hits (long motifs, long walks): a wave per hit
            KLAUNCH("k_level_wave", 0.0, k_level_wave, dim3(blocks((b - a) * 64)), dim3(kB), 0, st, vgrp + a, b - a, d_hits,
                    rank_of, S, E, M, PME, B, kept, n);
        else
            KLAUNCH("k_level", 0.0, k_level, dim3(blocks(b - a)), dim3(kB), 0, st, vgrp + a, b - a, d_hits, rank_of, S, E,
                    M, PME, B, kept, n);
    }
}

void screen_hits_device(Ctx &c, const bwtmi_hit *d_hits, int64_t n, int64_t text_len, int32_t lmax,
                        ScreenedVec &out, int64_t maxlen_known, int32_t drop_min_copies) {
    out.clear();
    if (n <= 0) return;
    if (n >= (int64_t)UINT32_MAX) fail(BWTMI_E_ARG, "too many strict hits for one contig (%lld)", (long long)n);
    if (text_len >= (int64_t)UINT32_MAX) fail(BWTMI_E_ARG, "contig too long for the screened-hit records (%lld)", (long long)text_len);
    hipStream_t st = c.stream;
    c.slot[S_CAND_K].ensure((size_t)n * 8);
    c.slot[S_CAND_V].ensure((size_t)n * 4);
    c.slot[S_CAND_K2].ensure((size_t)n * 8);
    c.slot[S_CAND_V2].ensure((size_t)n * 4);
    c.slot[S_MISC0].ensure((size_t)n * 8);
    c.slot[S_MISC1].ensure((size_t)n * 8);
    c.slot[S_IDX0].ensure((size_t)n * 8);
    c.slot[S_IDX1].ensure((size_t)n * 4);
    c.slot[S_IDX2].ensure((size_t)n * 4);
    c.slot[S_IDX3].ensure((size_t)n + 64);
    c.slot[S_IDX4].ensure((size_t)n * sizeof(bwtmi_hit));
    c.slot[S_IDX5].ensure((size_t)(n / kTile + 64) * 2 * 8);
    c.slot[S_FLAG].ensure((size_t)(n + 1) * 4);
    c.slot[S_SCAN].ensure((size_t)(n + 1) * 4);
    c.slot[S_COUNTS].ensure((size_t)(lmax + 2) * 8);
    const int64_t nb = (text_len >> kBucketShift) + 2;   // hit ends are <= text_len
    c.slot[S_IDX6].ensure((size_t)nb * 4);
    uint64_t *kpos = c.slot[S_CAND_K].as<uint64_t>(), *kgrp = c.slot[S_CAND_K2].as<uint64_t>();
    uint32_t *vpos = c.slot[S_CAND_V].as<uint32_t>(), *vgrp = c.slot[S_CAND_V2].as<uint32_t>();
    int64_t *S = c.slot[S_MISC0].as<int64_t>(), *E = c.slot[S_MISC1].as<int64_t>();
    int64_t *PME = c.slot[S_IDX0].as<int64_t>();
    int32_t *M = c.slot[S_IDX1].as<int32_t>();
    uint32_t *rank_of = c.slot[S_IDX2].as<uint32_t>();
    uint8_t *kept = c.slot[S_IDX3].as<uint8_t>();
    uint64_t *dout = c.slot[S_IDX4].as<uint64_t>();   // n * 32 B: room for either layout
    uint32_t *flag = c.slot[S_FLAG].as<uint32_t>(), *pos = c.slot[S_SCAN].as<uint32_t>();
    unsigned long long *d_max = c.slot[S_COUNTS].as<unsigned long long>();

    // longest span -> key widths
    unsigned long long *mb = c.mailbox<unsigned long long>(4);
    unsigned long long maxlen = 0;
    if (maxlen_known >= 0) {
        maxlen = (unsigned long long)maxlen_known;
    } else {
        HIPCHECK(hipMemsetAsync(d_max, 0, 8, st));
        KLAUNCH("k_maxlen", 0.0, k_maxlen, dim3((unsigned)std::min<int64_t>(1024, blocks(n))), dim3(kB), 0, st, d_hits,
                n, d_max);
        HIPCHECK(hipMemcpyAsync(mb, d_max, 8, hipMemcpyDeviceToHost, st));
        scan_wait(st);
        maxlen = mb[0];
    }
    const int mb_bits = std::max(1, bits_for((uint64_t)lmax));
    const int lb = std::max(1, bits_for(maxlen));
    if (lb + mb_bits > 64) fail(BWTMI_E_ARG, "span too long for the screen keys");
    auto round8 = [](int b) { return ((b + 7) / 8) * 8; };

    // (start, len, g) in one key when it fits 64 bits (C3: 27 + 10 + 10 bits, 6
    // passes instead of 3 + 4), else two stable sorts
    const int sb = std::max(1, bits_for((uint64_t)text_len));   // start < text_len
    const bool one_key = sb + lb + mb_bits <= 64;
    KLAUNCH("k_keys", 0.0, k_keys, dim3(blocks(n)), dim3(kB), 0, st, d_hits, n, mb_bits, (int64_t)lmax, kpos, vpos, kgrp,
            vgrp, one_key ? lb + mb_bits : -1);
    if (one_key) {
        radix_sort_pairs32(c, kpos, vpos, n, 0, round8(sb + lb + mb_bits));
    } else {
        radix_sort_pairs32(c, kpos, vpos, n, 0, round8(lb + mb_bits));
        KLAUNCH("k_keys_start", 0.0, k_keys_start, dim3(blocks(n)), dim3(kB), 0, st, d_hits, n, vpos, kpos);
        radix_sort_pairs32(c, kpos, vpos, n, 0, round8(sb));
    }
    KLAUNCH("k_gather", 0.0, k_gather, dim3(blocks(n)), dim3(kB), 0, st, d_hits, n, vpos, S, E, M, rank_of, kept);
    prefix_max(c, E, PME, n, c.slot[S_IDX5].as<int64_t>());
    // every level, segment by segment, in one launch (BWTMI_SEG_LEVELS=0: per-level launches)
    const bool seg_levels = knob(KN_SEG_LEVELS) != 0;
    unsigned int *d_ovf = reinterpret_cast<unsigned int *>(d_max);   // [0] fallback flag, [1] overflow windows
    // one word per kept hit when the start fits the low half and the longest span
    // and the longest primitive motif fit the high half (BWTMI_SCREEN_WIDE=1:
    // always two)
    const bool wide = knob(KN_SCREEN_WIDE) != 0;
    const int lbits = lb;   // bits of the longest span (hit lengths are <= maxlen)
    const int pbits = std::max(1, bits_for((uint64_t)lmax));
    out.lbits = !wide && lbits + pbits <= 32 && bits_for((uint64_t)text_len) <= 32 ? lbits : -1;
    // the kept flags -> their order -> the packed records, and the kept count
    // with the screen's overflow flag (mb[1]) in the same stream wait
    // records only the final filter would see are dropped here (k_drop_flags;
    // BWTMI_SCREEN_DROP=0 keeps them): at C3 most kept hits are short runs
    const bool drop = drop_min_copies > 0 && knob(KN_SCREEN_DROP) != 0;
    if (drop) c.slot[S_IDX7].ensure((size_t)(n + 1) * 4);
    auto final_pass = [&] {
        int64_t *R = drop ? c.slot[S_CAND_K].as<int64_t>() : nullptr;   // (the sorted keys are spent)
        KLAUNCH("k_final_flags", 0.0, k_final_flags, dim3(blocks(n)), dim3(kB), 0, st, S, E, M, kept, n, flag,
                drop ? drop_min_copies : 0, R);
        uint32_t *fl = flag;   // the flags the compaction takes
        if (drop) {
            fl = c.slot[S_IDX7].as<uint32_t>();
            prefix_max(c, R, R, n, c.slot[S_IDX5].as<int64_t>());
            KLAUNCH("k_drop_flags", 0.0, k_drop_flags, dim3(blocks(n)), dim3(kB), 0, st, S, E, M, flag, R, n,
                    drop_min_copies, fl);
        }
        HIPCHECK(hipMemsetAsync(fl + n, 0, 4, st));
        exclusive_scan<uint32_t>(c, fl, pos, n + 1);
        KLAUNCH("k_final_compact", 0.0, k_final_compact, dim3(blocks(n)), dim3(kB), 0, st, d_hits, vpos, fl, pos, n,
                out.lbits, dout);
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(reinterpret_cast<uint32_t *>(mb), pos + n, 4, hipMemcpyDeviceToHost, st));
    };
    unsigned int ovf = 1;
    if (seg_levels) {
        uint32_t *ovf_win = pos;   // the final-pass scan buffer is free until then (n + 1 words >= nwin)
        HIPCHECK(hipMemsetAsync(d_ovf, 0, 8, st));
        // windows of 512 positions, up to 1024 hits per 256-thread workgroup
        // (r05i, C3: 0.44 ms for both launches; 256 / 512: 0.48; 128 / 256: 0.46)
        const int64_t nwin = (n + kSegWin - 1) / kSegWin;
        KLAUNCH("k_seg_levels", 0.0, (k_seg_levels<256, kSegCapS, kSegWin, false>), dim3((unsigned)nwin), dim3(256), 0,
                st, S, E, M, PME, n, kept, ovf_win, d_ovf + 1, d_ovf);
        KLAUNCH("k_seg_levels_l", 0.0, (k_seg_levels<1024, kSegCapL, kSegWin, true>), dim3(256), dim3(1024), 0, st, S,
                E, M, PME, n, kept, ovf_win, d_ovf + 1, d_ovf);
        // the window list (ovf_win) is spent: the final pass runs before the
        // host sees the fallback flag, and runs again after a fallback (rare)
        final_pass();
        HIPCHECK(hipMemcpyAsync(mb + 1, d_ovf, 8, hipMemcpyDeviceToHost, st));
        scan_wait(st);
        const unsigned int *o2 = reinterpret_cast<const unsigned int *>(mb + 1);
        ovf = o2[0];
        if (stats_on())
            std::fprintf(stderr, "  screen: %lld hits, %u overflow windows, fallback %u\n", (long long)n, o2[1], o2[0]);
    }
    if (ovf) {
        screen_levels(c, d_hits, n, lmax, mb_bits, kgrp, vgrp, rank_of, S, E, M, PME, kept, nb);
        final_pass();
        scan_wait(st);
    }
    const uint32_t nk = *reinterpret_cast<const uint32_t *>(mb);
    const int wph = out.lbits >= 0 ? 1 : 2;   // words per hit
    const size_t words = (size_t)nk * (size_t)wph;
    out.w.resize(words);
    if (c.timing) HIPCHECK(hipEventRecord(c.ev1, st));   // the end of the scan's kernels
    if (!nk) return;
    // into a registered block: a pinned DMA instead of a staged pageable copy.
    // The download goes in pieces, an event behind each, and the call returns:
    // the merge fold's first tasks read their hits while the rest lands
    // (ScreenedVec::wait), instead of the whole copy (~0.6 ms at 100 Mbp)
    // standing between the scan and the post-processing
    (void)ensure_pinned(out.w.data(), out.w.data(), words * 8);
    struct Pieces final : Landing {
        std::vector<hipEvent_t> ev;
        std::vector<int64_t> end;   // hits landed once ev[p] has completed: [0, end[p])
        // runs on whichever thread drops the hits (job reset, rescan, job_free, a
        // post-processing worker): event waits need no current device, so the
        // thread's device is left alone
        ~Pieces() override {
            for (hipEvent_t e : ev) {
                (void)hipEventSynchronize(e);
                (void)hipEventDestroy(e);
            }
        }
        void wait(int64_t k) override {
            if (k <= 0) return;
            size_t p = 0;
            while (p + 1 < end.size() && end[p] < k) ++p;
            for (;;) {   // a short wait: poll (a blocking one sleeps the thread)
                const hipError_t e = hipEventQuery(ev[p]);
                if (e == hipSuccess) return;
                if (e != hipErrorNotReady) HIPCHECK(e);
                __builtin_ia32_pause();
            }
        }
    };
    auto pc = std::make_shared<Pieces>();
    const int P = (int)std::max<int64_t>(1, std::min<int64_t>(8, (int64_t)words / (1 << 16)));   // >= 512 KB pieces
    for (int q = 0; q < P; ++q) {
        const int64_t h0 = (int64_t)nk * q / P, h1 = (int64_t)nk * (q + 1) / P;
        if (h1 > h0)
            HIPCHECK(hipMemcpyAsync(out.w.data() + h0 * wph, dout + h0 * wph, (size_t)(h1 - h0) * wph * 8,
                                    hipMemcpyDeviceToHost, st));
        hipEvent_t e;
        HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        pc->ev.push_back(e);
        pc->end.push_back(h1);
        HIPCHECK(hipEventRecord(e, st));
    }
    out.landing = std::move(pc);
}

}  // namespace bwtmi
