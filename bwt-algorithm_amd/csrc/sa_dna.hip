// sa_dna.hip -- suffix array + BWT of an ACGT text with its single final '$'
// (BWTCore._build_suffix_array / _build_bwt_array, bwt.py:212-274), the text
// every CLI contig produces (seq + '$', bwt.py:3053 / 3782) -- and of a text
// over up to 7 other symbols that all sort above '$' (ACGT with assembly gaps:
// N runs, IUPAC codes), whose first sort key is 16 symbols of 3 bits (48-bit
// keys, 6 passes) instead of 16 bases of 2 bits; everything after the first
// sort is the same.  Any other text (an inner '$', more symbols, a byte below
// '$') takes index.hip's general prefix doubling.
//
// The reference orders suffixes by byte value with the unique '$' smallest;
// 2-bit codes A0 C1 G2 T3 keep that order among bases.  Instead of doubling
// over a rank array, suffixes are sorted as strings:
//   1. the text is packed to 2 bits (32 bases per 64-bit word);
//   2. one LSD radix sort of (first 16 bases: 32-bit key, value) -- 4 passes
//      of 8 B keys+values instead of 8+ passes of 12 B; the value carries the
//      suffix start and the code of the base before it (BWT symbol);
//   3. runs of equal keys (groups): one tiled pass finds them (gs / ge in SA
//      order) and every suffix's run head; the first ranks go out through two
//      partition passes by the top 16 position bits, after which each tile of
//      pairs is one window of positions, written from LDS;
//   4. groups are finished by prefix doubling over a rank array
//      (Larsson-Sadakane): rank[i] = SA index of the head of i's group; a
//      round with h sorts every group by rank[i + h] -- the groups are then
//      2h-sorted -- and writes the new heads.  Only group members take part,
//      and each group is sorted where it fits:
//        <= 64 members     one wave (4, 16, 32 or 64 lanes per group), bitonic
//                          over lane shuffles
//        <= kMedium        one workgroup, bitonic in LDS
//        larger            one segmented radix pass over all such groups
//      The sorts read rank[a + h] as the round found it and push their rank
//      changes to a list that is stored after all of them: a mix of old and
//      new heads would order suffixes wrongly.  The next round's groups and
//      the changes are appended through 8 counters (sharded chunks).
//   5. one streaming pass writes SA and BWT.
// The end of the text: keys pad past the end with A, so the (at most 16)
// suffixes with fewer than 16 bases before '$' tie with suffixes that really
// continue with A.  One small fix-up moves each of them to the front of its
// group (a suffix ending sooner is smaller) before the rounds start, so the
// first round's ranks are an exact 16-sort.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kB = 256;
constexpr int kMedium = 1024;                   // largest group sorted by one workgroup
constexpr uint32_t kPosMask = (1u << 29) - 1;   // value: start (29 bits) | BWT code << 29

inline unsigned nblocks(int64_t n, int b = kB) { return (unsigned)((n + b - 1) / b); }

__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

__device__ __forceinline__ uint32_t code2(uint8_t c) { return (uint32_t)(((c >> 2) ^ (c >> 1)) & 3u); }   // A0 C1 G2 T3

// P[w] = bases 32w .. 32w+31, first base in the top bits; '$' and past the end read as A (0)
__global__ __launch_bounds__(kB) void k_dna_pack(const uint8_t *__restrict__ t, int64_t n, uint64_t *__restrict__ P,
                                                 int64_t nw) {
    const int64_t w = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (w >= nw) return;
    const int64_t base = w * 32;
    uint64_t v = 0;
    if (base + 32 <= n - 1) {
        const uint4 a = *reinterpret_cast<const uint4 *>(t + base);
        const uint4 b = *reinterpret_cast<const uint4 *>(t + base + 16);
        const uint32_t ws[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) v = (v << 2) | code2((uint8_t)(ws[q] >> (8 * k)));
    } else {
        for (int k = 0; k < 32; ++k) {
            const int64_t i = base + k;
            v = (v << 2) | (i < n - 1 ? code2(t[i]) : 0u);
        }
    }
    P[w] = v;
}

// bases pos .. pos+31 (P is padded with two zero words)
__device__ __forceinline__ uint64_t window(const uint64_t *__restrict__ P, int64_t pos) {
    const int64_t w = pos >> 5;
    const int sh = (int)(pos & 31) * 2;
    const uint64_t hi = P[w];
    return sh ? (hi << sh) | (P[w + 1] >> (64 - sh)) : hi;
}

__device__ __forceinline__ uint32_t base_code(const uint64_t *__restrict__ P, int64_t i) {
    return (uint32_t)((P[i >> 5] >> (62 - 2 * (i & 31))) & 3u);
}

// key = first 16 bases of suffix i; value = i | BWT code << 29 (code of the base
// before i, '$' = 4 for i == 0)
__global__ __launch_bounds__(kB) void k_dna_keys(const uint64_t *__restrict__ P, int64_t n, uint32_t *__restrict__ keys,
                                                 uint32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    keys[i] = (uint32_t)(window(P, i) >> 32);
    const uint32_t prev = i == 0 ? 4u : base_code(P, i - 1);
    vals[i] = (uint32_t)i | (prev << 29);
}

// ---- small alphabets (<= 7 symbols above '$'): symbol codes 0..6 by byte
// order, 4-bit nibbles in the packed words (16 per word, first in the top
// nibble), '$' and past the end read as code 0 (the end fix-up below serves
// both paths); the 48-bit key holds 16 codes of 3 bits
__global__ __launch_bounds__(kB) void k_sym_pack(const uint8_t *__restrict__ t, int64_t n,
                                                 const uint8_t *__restrict__ lut, uint64_t *__restrict__ P, int64_t nw) {
    __shared__ uint8_t cm[256];
    cm[threadIdx.x] = lut[threadIdx.x];
    __syncthreads();
    const int64_t w = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (w >= nw) return;
    const int64_t base = w * 16;
    uint64_t v = 0;
    if (base + 16 <= n - 1) {
        const uint4 a = *reinterpret_cast<const uint4 *>(t + base);
        const uint32_t ws[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int k = 0; k < 4; ++k) v = (v << 4) | cm[(ws[q] >> (8 * k)) & 255u];
    } else {
        for (int k = 0; k < 16; ++k) {
            const int64_t i = base + k;
            v = (v << 4) | (i < n - 1 ? cm[t[i]] : 0u);
        }
    }
    P[w] = v;
}

// key = the 16 symbols from i (3 bits each, first in the top bits of 48);
// value = i | code of the symbol before i << 29 ('$' = 7 for i == 0)
__global__ __launch_bounds__(kB) void k_sym_keys(const uint64_t *__restrict__ P, int64_t n, uint64_t *__restrict__ keys,
                                                 uint32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (i >= n) return;
    const int64_t w = i >> 4;
    const int sh = (int)(i & 15) * 4;
    const uint64_t x = sh ? (P[w] << sh) | (P[w + 1] >> (64 - sh)) : P[w];
    uint64_t k = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) k = (k << 3) | ((x >> (60 - 4 * j)) & 7u);
    keys[i] = k;
    const uint32_t prev = i == 0 ? 7u : (uint32_t)((P[(i - 1) >> 4] >> (60 - 4 * ((i - 1) & 15))) & 15u);
    vals[i] = (uint32_t)i | (prev << 29);
}

// flags of the multi-member groups (runs of equal keys): S = first member, E = last member
__global__ __launch_bounds__(kB) void k_dna_compact2(const uint32_t *__restrict__ fs, const uint32_t *__restrict__ ps,
                                                     const uint32_t *__restrict__ fe, const uint32_t *__restrict__ pe,
                                                     int64_t n, uint32_t *__restrict__ gs, uint32_t *__restrict__ ge) {
    const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (r >= n) return;
    if (fs[r]) gs[ps[r]] = (uint32_t)r;
    if (fe[r]) ge[pe[r]] = (uint32_t)r + 1;   // exclusive end
}

// Groups of equal 16-base keys, three launches over the sorted keys instead of
// flags + two scans + compaction + heads (five passes over n):
//   count : per 4096-key tile, the group starts and ends (runs of >= 2 equal
//           keys) and the last run start
//   scan  : one workgroup, exclusive sums / max over the tiles
//   apply : the tile again: gs / ge in SA order (ballot prefix counts), and
//           hd[r] = the SA index where r's run starts (r itself when alone)
constexpr int kGRows = 16;                 // 256-key rows per tile
constexpr int kGTile = kGRows * kB;        // 4096
struct RunFlags {
    bool run, gstart, gend;   // r starts a run; starts / ends a group of >= 2
};
// one coalesced load per key: the neighbours come from the adjacent lanes
// (lanes 0 and 63 load theirs); every lane of the wave must call it
template <class K>
__device__ __forceinline__ RunFlags run_flags(const K *__restrict__ keys, int64_t r, int64_t n) {
    const int lane = threadIdx.x & 63;
    const K k = r < n ? keys[r] : K(0);
    K kp = __shfl_up(k, 1, 64), kn = __shfl_down(k, 1, 64);
    if (lane == 0 && r > 0 && r < n) kp = keys[r - 1];
    if (lane == 63 && r + 1 < n) kn = keys[r + 1];
    RunFlags f{false, false, false};
    if (r >= n) return f;
    const bool head = r == 0 || kp != k;
    const bool tail = r + 1 == n || kn != k;
    f.run = head;
    f.gstart = head && !tail;
    f.gend = tail && !head;
    return f;
}

template <class K>
__global__ __launch_bounds__(kB) void k_grp_count(const K *__restrict__ keys, int64_t n,
                                                  uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t ws[kB / 64], we[kB / 64], wl[kB / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kGTile;
    uint32_t cs = 0, ce = 0, last = 0;
    for (int i = 0; i < kGRows; ++i) {
        const int64_t r = base + (int64_t)i * kB + threadIdx.x;
        const RunFlags f = run_flags(keys, r, n);
        const uint64_t mr = __ballot(f.run);
        cs += (uint32_t)__popcll(__ballot(f.gstart));
        ce += (uint32_t)__popcll(__ballot(f.gend));
        if (mr) last = (uint32_t)(r - lane) + 63u - (uint32_t)__clzll((long long)mr);
    }
    if (lane == 0) {
        ws[wv] = cs;
        we[wv] = ce;
        wl[wv] = last;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0, b = 0, l = 0;
        for (int w = 0; w < kB / 64; ++w) {
            a += ws[w];
            b += we[w];
            l = max(l, wl[w]);
        }
        const int64_t nt = (n + kGTile - 1) / kGTile;
        tcnt[blockIdx.x] = a;
        tcnt[nt + blockIdx.x] = b;
        tcnt[2 * nt + blockIdx.x] = l;
    }
}

// in place: exclusive sums of the start / end counts, exclusive max of the
// last run starts; the total start count (G) at tcnt[3 * nt].  One workgroup,
// 1024 tiles per step (coalesced), a block scan per step.
__global__ __launch_bounds__(1024) void k_grp_scan(uint32_t *__restrict__ tcnt, int64_t nt) {
    __shared__ uint32_t wa[16], wb[16], wl[16];
    __shared__ uint32_t carry[3];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t < 3) carry[t] = 0;
    __syncthreads();
    for (int64_t x0 = 0; x0 < nt; x0 += 1024) {
        const int64_t x = x0 + t;
        const uint32_t a = x < nt ? tcnt[x] : 0u, b = x < nt ? tcnt[nt + x] : 0u, l = x < nt ? tcnt[2 * nt + x] : 0u;
        uint32_t ia = a, ib = b, il = l;   // inclusive wave scans
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t pa = __shfl_up(ia, o, 64), pb = __shfl_up(ib, o, 64), pl = __shfl_up(il, o, 64);
            if (lane >= o) {
                ia += pa;
                ib += pb;
                il = max(il, pl);
            }
        }
        if (lane == 63) {
            wa[wv] = ia;
            wb[wv] = ib;
            wl[wv] = il;
        }
        __syncthreads();
        uint32_t ea = carry[0], eb = carry[1], el = carry[2];
        for (int w = 0; w < wv; ++w) {
            ea += wa[w];
            eb += wb[w];
            el = max(el, wl[w]);
        }
        const uint32_t pl = __shfl_up(il, 1, 64);   // exclusive max: the previous lane's inclusive one
        if (x < nt) {
            tcnt[x] = ea + ia - a;
            tcnt[nt + x] = eb + ib - b;
            tcnt[2 * nt + x] = lane ? max(el, pl) : el;
        }
        __syncthreads();
        if (t == 1023) {
            carry[0] = ea + ia;
            carry[1] = eb + ib;
            carry[2] = max(el, il);
        }
        __syncthreads();
    }
    if (t == 0) tcnt[3 * nt] = carry[0];
}

template <class K>
__global__ __launch_bounds__(kB) void k_grp_apply(const K *__restrict__ keys, int64_t n,
                                                  const uint32_t *__restrict__ tcnt, uint32_t *__restrict__ gs,
                                                  uint32_t *__restrict__ ge, uint32_t *__restrict__ hd) {
    __shared__ uint32_t ws[kB / 64], we[kB / 64], wl[kB / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nt = (n + kGTile - 1) / kGTile;
    const int64_t base = (int64_t)blockIdx.x * kGTile;
    uint32_t cs = tcnt[blockIdx.x], ce = tcnt[nt + blockIdx.x], cl = tcnt[2 * nt + blockIdx.x];   // carries
    const uint64_t below = lanes_below(lane);
    for (int i = 0; i < kGRows; ++i) {
        const int64_t r = base + (int64_t)i * kB + threadIdx.x;
        const RunFlags f = run_flags(keys, r, n);
        const uint64_t ms = __ballot(f.gstart), me = __ballot(f.gend), mr = __ballot(f.run);
        const uint32_t wbase = (uint32_t)(r - lane);
        if (lane == 0) {
            ws[wv] = (uint32_t)__popcll(ms);
            we[wv] = (uint32_t)__popcll(me);
            wl[wv] = mr ? wbase + 63u - (uint32_t)__clzll((long long)mr) : 0u;
        }
        __syncthreads();
        uint32_t ps = cs, pe = ce, pl = cl;
        for (int w = 0; w < wv; ++w) {
            ps += ws[w];
            pe += we[w];
            pl = max(pl, wl[w]);
        }
        if (r < n) {
            if (f.gstart) gs[ps + (uint32_t)__popcll(ms & below)] = (uint32_t)r;
            if (f.gend) ge[pe + (uint32_t)__popcll(me & below)] = (uint32_t)r + 1;   // exclusive end
            const uint64_t mine = mr & (below | (1ull << lane));
            hd[r] = mine ? wbase + 63u - (uint32_t)__clzll((long long)mine) : pl;
        }
        for (int w = wv; w < kB / 64; ++w) {   // carries into the next row (every thread, same values)
            ps += ws[w];
            pe += we[w];
            pl = max(pl, wl[w]);
        }
        cs = ps;
        ce = pe;
        cl = pl;
        __syncthreads();   // ws / we / wl are rewritten by the next row
    }
}

// rank[pos] = head, from (position | code, head) pairs: after a pass that
// orders the pairs by the position's top 8 bits, each workgroup's writes stay
// in one 2^shift-position window that its XCD's L2 holds, so the scattered
// 4-byte stores reach HBM as whole lines
// NT: the (position, head) stream is read with nontemporal loads, so it does
// not displace the window's partly written rank lines from the L2
constexpr int kPutItems = 16;
template <bool NT>
__global__ __launch_bounds__(kB) void k_dna_rank_put(const uint32_t *__restrict__ pv, const uint32_t *__restrict__ hd,
                                                     int64_t n, int64_t ntiles, uint32_t *__restrict__ rank,
                                                     uint32_t *chk) {
    const int64_t base = xcd_tile(blockIdx.x, ntiles) * (kB * kPutItems) + threadIdx.x;
    uint32_t p[kPutItems], h[kPutItems];
#pragma unroll
    for (int i = 0; i < kPutItems; ++i) {
        const int64_t r = base + (int64_t)i * kB;
        if (NT) {
            p[i] = r < n ? __builtin_nontemporal_load(pv + r) : 0u;
            h[i] = r < n ? __builtin_nontemporal_load(hd + r) : 0u;
        } else {
            p[i] = r < n ? pv[r] : 0u;
            h[i] = r < n ? hd[r] : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < kPutItems; ++i)
        if (base + (int64_t)i * kB < n) {
            if (chk && (int64_t)(p[i] & kPosMask) >= n) atomicOr(chk, kChkRankPut);
            else rank[p[i] & kPosMask] = h[i];
        }
}

// The same writes after the pairs are ordered by the top 16 position bits: every
// position occurs once, so with 2^(bits-16) dividing the 4096-pair tile, tile t
// holds exactly the positions [4096 t, 4096 t + 4096).  The ranks are placed in
// an LDS copy of that window and leave as one coalesced 16 KB store (scattered
// 4-byte stores, even L2-local ones, issue one cache line per lane).  A pair
// outside the window (not expected) is stored directly.
template <bool NT>
__global__ __launch_bounds__(kB) void k_dna_rank_put_tile(const uint32_t *__restrict__ pv, const uint32_t *__restrict__ hd,
                                                          int64_t n, uint32_t *__restrict__ rank, uint32_t *chk) {
    constexpr int kT = kB * kPutItems;
    __shared__ uint32_t win[kT];
    const int64_t t0 = (int64_t)blockIdx.x * kT;
    uint32_t p[kPutItems], h[kPutItems];
#pragma unroll
    for (int i = 0; i < kPutItems; ++i) {
        const int64_t r = t0 + (int64_t)i * kB + threadIdx.x;
        if (NT) {
            p[i] = r < n ? __builtin_nontemporal_load(pv + r) : 0u;
            h[i] = r < n ? __builtin_nontemporal_load(hd + r) : 0u;
        } else {
            p[i] = r < n ? pv[r] : 0u;
            h[i] = r < n ? hd[r] : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < kPutItems; ++i) {
        if (t0 + (int64_t)i * kB + threadIdx.x >= n) continue;
        const int64_t q = (int64_t)(p[i] & kPosMask) - t0;
        if (q >= 0 && q < kT) win[q] = h[i];
        else if (chk && (int64_t)(p[i] & kPosMask) >= n) atomicOr(chk, kChkRankPut);
        else rank[p[i] & kPosMask] = h[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPutItems; ++i) {
        const int j = i * kB + threadIdx.x;
        if (t0 + j < n) rank[t0 + j] = win[j];
    }
}

// the <= 16 suffixes with fewer than 16 bases before '$' (their keys are
// A-padded): each goes to the front of its group, shorter first, and leaves
// the group; the rest of the group gets the head behind them.  One workgroup.
__global__ __launch_bounds__(1024) void k_dna_short_fix(uint32_t *__restrict__ vals, uint32_t *__restrict__ rank,
                                                        uint32_t *__restrict__ gs, const uint32_t *__restrict__ ge,
                                                        int64_t G, int64_t n, uint32_t *chk) {
    __shared__ int64_t grp[16];      // group index of the short suffix with r bases left, or -1
    __shared__ uint32_t where[16];   // its index in vals
    const int ns = (int)min<int64_t>(16, n);
    if (threadIdx.x < 16) {
        grp[threadIdx.x] = -1;
        where[threadIdx.x] = ~0u;
        if ((int)threadIdx.x < ns) {
            const uint32_t hd = rank[n - 1 - threadIdx.x];
            int64_t lo = 0, hi = G;   // gs ascends: find gs[x] == hd
            while (lo < hi) {
                const int64_t mid = (lo + hi) / 2;
                if (gs[mid] < hd) lo = mid + 1;
                else hi = mid;
            }
            if (lo < G && gs[lo] == hd && ge[lo] - gs[lo] >= 2) grp[threadIdx.x] = lo;
        }
    }
    __syncthreads();
    for (int r0 = 0; r0 < ns; ++r0) {
        const int64_t g = grp[r0];
        bool first = g >= 0;
        for (int r = 0; r < r0 && first; ++r) first = grp[r] != g;
        if (!first) continue;   // each group once, at its shortest member
        const uint32_t s = gs[g], e = ge[g];
        for (uint32_t x = s + threadIdx.x; x < e; x += blockDim.x) {
            const int64_t pos = vals[x] & kPosMask;
            if (pos >= n - 16) where[n - 1 - pos] = x;
        }
        __syncthreads();
        __shared__ uint32_t k_sh;
        if (threadIdx.x == 0) {   // swap the shorts to s, s+1, ... in order of r
            uint32_t k = 0;
            for (int r = 0; r < ns; ++r) {
                if (grp[r] != g) continue;
                const uint32_t t = s + k, from = where[r];
                if (chk && (from < s || from >= e || t >= e)) {   // the short suffix was not found in its group
                    atomicOr(chk, kChkShortFix);
                    continue;
                }
                const uint32_t moved = vals[t];
                vals[t] = vals[from];
                vals[from] = moved;
                const int64_t mp = moved & kPosMask;
                if (mp >= n - 16) where[n - 1 - mp] = from;
                rank[n - 1 - r] = t;
                ++k;
            }
            k_sh = k;
            gs[g] = s + k;
        }
        __syncthreads();
        const uint32_t k = k_sh;
        for (uint32_t x = s + k + threadIdx.x; x < e; x += blockDim.x) rank[vals[x] & kPosMask] = s + k;
        __syncthreads();
    }
}

// groups by size class; the order inside a class does not matter (groups are disjoint)
// <= 4, <= 16, <= 32, <= 64 members (W-lane segments of one wave), <= kMedium
// (one workgroup), larger (segmented radix)
constexpr int kClasses = 6;
__device__ __forceinline__ int size_class(uint32_t sz) {
    return sz <= 4 ? 0 : sz <= 16 ? 1 : sz <= 32 ? 2 : sz <= 64 ? 3 : sz <= (uint32_t)kMedium ? 4 : 5;
}


// append (start, end) to a list, one atomic per workgroup of NT threads (a
// single counter hit once per wave by ~10^6 waves serialises in L2); every
// thread of the workgroup must call it
template <int NT>
__device__ __forceinline__ void block_append(bool on, uint32_t st, uint32_t en, uint32_t *__restrict__ ls,
                                             uint32_t *__restrict__ le, uint32_t *__restrict__ cnt) {
    __shared__ uint32_t wc[NT / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = __ballot(on);
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NT / 64; ++w) {
            const uint32_t x = wc[w];
            wc[w] = tot;
            tot += x;
        }
        wc[NT / 64] = tot ? atomicAdd(cnt, tot) : 0u;
    }
    __syncthreads();
    if (on) {
        const uint32_t at = wc[NT / 64] + wc[wv] + (uint32_t)__popcll(m & lanes_below(lane));
        ls[at] = st;
        le[at] = en;
    }
    __syncthreads();   // wc is reused by the next call
}

// The next round's group list is appended by ~10^4 workgroups per pass; one
// counter would serialise them in L2 (~10 ns each).  Eight counters instead,
// one per blockIdx % 8: shard q owns list chunks q, q + 8, q + 16, ... of kCH
// slots, so an entry's slot follows from its shard and its index there.  The
// unused tail of each shard's last chunk is a hole the reader skips
// (ShardedList::live).  A slot past cap raises *ovf (the caller then takes
// the general path).
constexpr uint32_t kCH = 1024;
__device__ __forceinline__ uint32_t shard_slot(uint32_t v, uint32_t q) { return ((v / kCH) * 8 + q) * kCH + v % kCH; }

struct ShardedList {
    uint32_t cnt[8];   // entries of each shard
    uint32_t S;        // slots [0, S) are sharded; [S, G) are plain
    __device__ __forceinline__ bool live(uint32_t j) const {
        if (j >= S) return true;
        const uint32_t ch = j / kCH;
        return (ch / 8) * kCH + j % kCH < cnt[ch % 8];
    }
};

template <int NT>
__device__ __forceinline__ void block_append_sharded(bool on, uint32_t st, uint32_t en, uint32_t *__restrict__ ls,
                                                     uint32_t *__restrict__ le, uint32_t *__restrict__ cnt8,
                                                     uint32_t cap, uint32_t *__restrict__ ovf) {
    __shared__ uint32_t wc[NT / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t q = blockIdx.x & 7u;
    const uint64_t m = __ballot(on);
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NT / 64; ++w) {
            const uint32_t x = wc[w];
            wc[w] = tot;
            tot += x;
        }
        wc[NT / 64] = tot ? atomicAdd(&cnt8[q], tot) : 0u;
    }
    __syncthreads();
    if (on) {
        const uint32_t at = shard_slot(wc[NT / 64] + wc[wv] + (uint32_t)__popcll(m & lanes_below(lane)), q);
        if (at < cap) {
            ls[at] = st;
            le[at] = en;
        } else {
            atomicOr(ovf, 1u);
        }
    }
    __syncthreads();   // wc is reused by the next call
}

// a round's rank changes, (position << 32 | new head), pushed like the group
// lists (sharded chunks, holes skipped by the reader) and stored after every
// sort of the round has read its keys: the sorts gather rank[a + h] from the
// state at the start of the round
template <int NT>
__device__ __forceinline__ void block_push_sharded(bool on, uint64_t item, uint64_t *__restrict__ ls,
                                                   uint32_t *__restrict__ cnt8, uint32_t cap,
                                                   uint32_t *__restrict__ ovf) {
    __shared__ uint32_t wc[NT / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t q = blockIdx.x & 7u;
    const uint64_t m = __ballot(on);
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NT / 64; ++w) {
            const uint32_t x = wc[w];
            wc[w] = tot;
            tot += x;
        }
        wc[NT / 64] = tot ? atomicAdd(&cnt8[q], tot) : 0u;
    }
    __syncthreads();
    if (on) {
        const uint32_t at = shard_slot(wc[NT / 64] + wc[wv] + (uint32_t)__popcll(m & lanes_below(lane)), q);
        if (at < cap) ls[at] = item;
        else atomicOr(ovf, 1u);
    }
    __syncthreads();
}

// where a round's sorts write: the next round's groups and the rank changes
struct LsOut {
    uint32_t *ngs, *nge, *ncnt;   // ncnt[0..7] shard counts, ncnt[8] overflow
    uint32_t cap;
    uint64_t *chg;
    uint32_t *ccnt;               // ccnt[0..7], ccnt[8] overflow
    uint32_t ccap;
};

__global__ __launch_bounds__(kB) void k_ls_apply(const uint64_t *__restrict__ chg, int64_t S, ShardedList sl,
                                                 uint32_t *__restrict__ rank) {
    const int64_t j = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (j >= S || !sl.live((uint32_t)j)) return;
    const uint64_t e = chg[j];
    rank[e >> 32] = (uint32_t)e;
}

// the round's groups into the size-class lists: kCI groups per thread, slots
// inside the workgroup from wave ballots + LDS counters, then one atomic per
// class and workgroup
constexpr int kCI = 16;
__global__ __launch_bounds__(kB) void k_dna_classify(const uint32_t *__restrict__ gs, const uint32_t *__restrict__ ge,
                                                     int64_t G, ShardedList sl, uint32_t *__restrict__ cls_start,
                                                     uint32_t *__restrict__ cls_size, uint32_t *__restrict__ counts,
                                                     int64_t cap) {
    __shared__ uint32_t lc[kClasses], base[kClasses];
    const int lane = threadIdx.x & 63;
    if (threadIdx.x < kClasses) lc[threadIdx.x] = 0;
    __syncthreads();
    uint32_t st[kCI], sz[kCI], slot[kCI];
    int cl[kCI];
#pragma unroll
    for (int i = 0; i < kCI; ++i) {
        const int64_t g = (int64_t)blockIdx.x * (kB * kCI) + (int64_t)i * kB + threadIdx.x;
        cl[i] = -1;
        st[i] = sz[i] = slot[i] = 0;
        if (g < G && sl.live((uint32_t)g)) {
            st[i] = gs[g];
            sz[i] = ge[g] - st[i];
            cl[i] = size_class(sz[i]);
        }
#pragma unroll
        for (int k = 0; k < kClasses; ++k) {
            const uint64_t m = __ballot(cl[i] == k);
            if (!m) continue;
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t b = 0;
            if (lane == leader) b = atomicAdd(&lc[k], (uint32_t)__popcll(m));
            b = __shfl(b, leader, 64);
            if (cl[i] == k) slot[i] = b + (uint32_t)__popcll(m & lanes_below(lane));
        }
    }
    __syncthreads();
    if (threadIdx.x < kClasses) base[threadIdx.x] = lc[threadIdx.x] ? atomicAdd(&counts[threadIdx.x], lc[threadIdx.x]) : 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kCI; ++i)
        if (cl[i] >= 0) {
            const int64_t at = (int64_t)cl[i] * cap + base[cl[i]] + slot[i];
            cls_start[at] = st[i];
            cls_size[at] = sz[i];
        }
}

// Long runs of one symbol ("deep" suffixes: the first 16 symbols all equal c).
// A run of R copies of c puts R - 15 suffixes into one 16-symbol group that
// plain doubling resolves only h symbols per round (16 rounds for the 958 kbp
// N runs of an assembly).  Their order is known in closed form instead: a
// deep suffix is c^r X with X[0] != c (r = symbols to the run's end); every
// one whose X[0] < c sorts before every one whose X[0] > c (b = 0 / 1), then
// b = 0 by r ascending, b = 1 by r descending, then by X.
// The doubling invariant must hold for every group, deep or not: after the
// round with h, the members of a group share their first 2h symbols, because
// other suffixes read a group's rank through rank[a + h] as standing for h
// symbols in the next round.  A (b, r) group shares exactly r symbols, so:
//   round h = 16 (the c^16 group [gs, gs + gsz)): members with r >= 32 get
//     gs + (r - 32) (b = 0) or gs + gsz - 1 - (r - 32) (b = 1) -- inside the
//     group's own SA range, b = 0 below b = 1 (the group holds R - 15 members
//     per run of length R, so the two ranges never meet); members with
//     r < 32 keep rank[a + 16], which already falls below gs (b = 0) or at or
//     after gs + gsz (b = 1);
//   rounds h >= 32 (groups are uniform in r from here on): rank[a + r] -- the
//     rank of X, h symbols of it -- while r >= h (r + h >= 2h symbols), and
//     rank[a + h] once r < h.
// (Round 5 keyed every run member by (b, r) and then rank[a + r] whatever r
// was: a (b, r) group with r < 2h then claimed 2h symbols, and Z c^r x W
// against Z c^r y V with |Z| = h tied and skipped x)
// Deep groups hold only deep suffixes (their 16-prefix is c^16), so every
// group is keyed one way.  re[a >> 4] = the end of the run holding position
// 16 (a >> 4) + 15, which lies inside a's run whenever a is deep.
struct Deep {
    const uint64_t *P;    // packed text (2-bit bases, or 4-bit symbol codes when small)
    const uint32_t *re;   // run end per 16-position block (valid for deep suffixes' blocks)
    int small;            // symbol codes of the small-alphabet path
    int on;               // any run of >= 16 equal symbols
    uint32_t *chk;        // Ctx::checks (nullptr: off)
};

// the 16 symbols from a (the packed words are padded): c when all equal, else -1
__device__ __forceinline__ int homopolymer16(const Deep &d, int64_t a) {
    if (d.small) {
        const int64_t w = a >> 4;
        const int sh = (int)(a & 15) * 4;
        const uint64_t x = sh ? (d.P[w] << sh) | (d.P[w + 1] >> (64 - sh)) : d.P[w];
        const uint64_t c = x >> 60;
        return x == c * 0x1111111111111111ull ? (int)c : -1;
    }
    const uint64_t w = window(d.P, a) >> 32;   // 16 bases, 2 bits each
    const uint64_t c = w >> 30;
    return w == c * 0x55555555ull ? (int)c : -1;
}
__device__ __forceinline__ int sym_at(const Deep &d, int64_t i) {
    return d.small ? (int)((d.P[i >> 4] >> (60 - 4 * (i & 15))) & 15u) : (int)base_code(d.P, i);
}

// the doubling key of member v of the group [gs, gs + gsz): rank of the suffix
// h bases on (a group member always has more than h bases before '$': its
// h-prefix is shared); deep suffixes as above
__device__ __forceinline__ uint32_t ls_key(const uint32_t *__restrict__ rank, uint32_t v, int64_t n, int64_t h,
                                          const Deep &d, uint32_t gs, uint32_t gsz) {
    const int64_t a = v & kPosMask;
    if (d.on && a + 16 < n) {
        const int c = homopolymer16(d, a);
        if (c >= 0) {
            const int64_t e = d.re[a >> 4];   // first position past the run (<= n - 1: '$' ends every run)
            const int64_t r = e - a;
            if (d.chk && (e < a + 16 || e >= n)) {   // a run-end block the run-end pass did not write
                atomicOr(d.chk, kChkDeepEnd);
                return 0u;
            }
            if (h == 16) {
                if (r >= 32) {
                    const bool b = e < n - 1 && sym_at(d, e) > c;
                    return b ? gs + gsz - 1u - (uint32_t)(r - 32) : gs + (uint32_t)(r - 32);
                }
            } else if (r >= h) {
                return rank[e];
            }
        }
    }
    return a + h < n ? rank[a + h] : 0u;
}

// runs of >= 16 equal symbols in t[0, n - 1): their first positions, appended
// (unordered) to rs through one atomic per workgroup
// (16 consecutive positions per thread: a run starts at most once among them
// -- two starts need a run of >= 16 between them)
__global__ __launch_bounds__(kB) void k_run_starts(Deep d, int64_t n, uint32_t *__restrict__ rs,
                                                   uint32_t *__restrict__ kcount, uint32_t cap) {
    const int64_t p0 = ((int64_t)blockIdx.x * kB + threadIdx.x) * 16;
    bool st = false;
    int64_t p = 0;
    for (int j = 0; j < 16 && !st; ++j) {
        p = p0 + j;
        if (p + 16 >= n) break;   // 16 real symbols from p
        const int c = homopolymer16(d, p);
        st = c >= 0 && (p == 0 || sym_at(d, p - 1) != c);
    }
    __shared__ uint32_t wc[kB / 64 + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = __ballot(st);
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < kB / 64; ++w) {
            const uint32_t x = wc[w];
            wc[w] = tot;
            tot += x;
        }
        wc[kB / 64] = tot ? atomicAdd(kcount, tot) : 0u;
    }
    __syncthreads();
    if (st) {
        const uint32_t at = wc[kB / 64] + wc[wv] + (uint32_t)__popcll(m & lanes_below(lane));
        if (at < cap) rs[at] = (uint32_t)p;
        else if (d.chk) atomicOr(d.chk, kChkRunList);
    }
}

// one workgroup per run (grid-stride over the K runs): its end e (the first
// position >= start + 16 whose symbol differs, or n - 1: '$'), found 16
// positions per thread and 8 windows in flight, then re[b] = e for every block
// b whose last position 16 b + 15 lies in [start, e)
__global__ __launch_bounds__(kB) void k_run_ends(Deep d, int64_t n, const uint32_t *__restrict__ rs,
                                                 const uint32_t *__restrict__ kcount, uint32_t *__restrict__ re) {
    __shared__ unsigned long long first;
    const uint32_t K = *kcount;
    for (uint32_t k = blockIdx.x; k < K; k += gridDim.x) {
        const int64_t s0 = rs[k];
        const int c = sym_at(d, s0);
        if (threadIdx.x == 0) first = (unsigned long long)(n - 1);
        __syncthreads();
        for (int64_t base = s0 + 16;; base += (int64_t)kB * 16 * 8) {   // uniform (first is read after a barrier)
            int64_t mine = n - 1;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int64_t pos = base + ((int64_t)q * kB + threadIdx.x) * 16;
                if (pos >= n - 1 || mine < n - 1) continue;
                if (pos + 16 <= n - 1 && homopolymer16(d, pos) == c) continue;
                for (int j = 0; j < 16; ++j)
                    if (pos + j >= n - 1 || sym_at(d, pos + j) != c) {
                        mine = pos + j;
                        break;
                    }
            }
            if (mine < n - 1) atomicMin(&first, (unsigned long long)mine);
            __syncthreads();
            const int64_t e = (int64_t)first;
            if (e < n - 1 || base + (int64_t)kB * 16 * 8 >= n - 1) break;
            __syncthreads();
        }
        const int64_t e0 = (int64_t)first;
        const int64_t b0 = s0 >> 4, b1 = (e0 - 16) >> 4;   // 16 b + 15 in [s0, e0)
        if (d.chk && (e0 < s0 + 16 || e0 > n - 1 || b1 > (n - 1) / 16)) {
            if (threadIdx.x == 0) atomicOr(d.chk, kChkRunEnd);
        } else {
            for (int64_t b = b0 + threadIdx.x; b <= b1; b += kB) re[b] = (uint32_t)e0;
        }
        __syncthreads();   // `first` is reset for the next run
    }
}

// one doubling pass over groups of <= W members, 64/W groups per wave: bitonic
// sort of (rank[a+h], value) in W-lane segments, new heads from ballots, the
// still-tied runs appended to the next round's list
// (KEYS: the gather pass -- kb[i] = key of the member at vals[i])
constexpr int kLB = 1024;   // threads per workgroup of the wave-sort passes
template <int W>
__global__ __launch_bounds__(kLB) void k_ls_wave(const uint32_t *__restrict__ starts, const uint32_t *__restrict__ sizes,
                                                int64_t cnt, uint32_t *__restrict__ vals,
                                                const uint32_t *__restrict__ rank, int64_t n, int64_t h, LsOut o,
                                                Deep dp) {
    const int lane = threadIdx.x & 63, kk = lane & (W - 1);
    const int64_t g = (((int64_t)blockIdx.x * kLB + threadIdx.x) >> 6) * (64 / W) + lane / W;
    uint32_t s = 0, sz = 0;
    if (g < cnt) {
        s = starts[g];
        sz = sizes[g];
    }
    const bool live = kk < (int)sz;
    const uint32_t orig = live ? vals[s + kk] : 0u;
    uint64_t x = live ? ((uint64_t)ls_key(rank, orig, n, h, dp, s, sz) << 32) | orig : ~0ull;
#pragma unroll
    for (int k2 = 2; k2 <= W; k2 <<= 1)
#pragma unroll
        for (int j = k2 >> 1; j > 0; j >>= 1) {
            const uint64_t y = __shfl_xor(x, j, 64);
            const bool keep_min = ((kk & j) == 0) == ((kk & k2) == 0);
            x = keep_min ? (y < x ? y : x) : (y > x ? y : x);
        }
    const uint32_t key = (uint32_t)(x >> 32), v = (uint32_t)x;
    const uint32_t kp = __shfl(key, (lane + 63) & 63, 64), kn = __shfl(key, (lane + 1) & 63, 64);
    const bool start = live && (kk == 0 || kp != key);
    const bool tail = live && (kk == (int)sz - 1 || kn != key);
    const uint64_t S = __ballot(start), T = __ballot(tail);
    const int seg = lane - kk;
    // every member's rank is s when the round starts: only the members of the
    // later subgroups change rank, and only moved values are stored
    if (live) {
        if (v != orig) vals[s + kk] = v;
    }
    const int hl = live ? 63 - __clzll((long long)(S & (lanes_below(lane) | (1ull << lane)))) : seg;
    block_push_sharded<kLB>(hl != seg, ((uint64_t)(v & kPosMask) << 32) | (s + (uint32_t)(hl - seg)), o.chg, o.ccnt,
                            o.ccap, o.ccnt + 8);
    const bool multi = start && !tail;
    const int el = multi ? __ffsll((unsigned long long)(T & (~0ull << lane))) - 1 : 0;
    block_append_sharded<kLB>(multi, s + kk, s + (uint32_t)(el - seg) + 1, o.ngs, o.nge, o.ncnt, o.cap, o.ncnt + 8);
}

// one doubling pass over a group of <= kMedium members in one workgroup
constexpr int kWB = 1024;
__global__ __launch_bounds__(kWB) void k_ls_block(const uint32_t *__restrict__ starts, const uint32_t *__restrict__ sizes,
                                                  uint32_t *__restrict__ vals, const uint32_t *__restrict__ rank,
                                                  int64_t n, int64_t h, LsOut o, Deep dp) {
    __shared__ uint64_t x[kMedium];
    __shared__ int wl[kWB / 64], wf[kWB / 64];
    const uint32_t s = starts[blockIdx.x], sz = sizes[blockIdx.x];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t p2 = 1;
    while (p2 < sz) p2 <<= 1;
    const uint32_t orig = t < (int)sz ? vals[s + t] : 0u;
    if (t < (int)p2) x[t] = t < (int)sz ? ((uint64_t)ls_key(rank, orig, n, h, dp, s, sz) << 32) | orig : ~0ull;
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= p2; k2 <<= 1)
        for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
            const uint32_t q = (uint32_t)t ^ j;
            if (t < (int)p2 && q > (uint32_t)t) {
                const uint64_t a = x[t], b = x[q];
                if ((a > b) == (((uint32_t)t & k2) == 0)) {
                    x[t] = b;
                    x[q] = a;
                }
            }
            __syncthreads();
        }
    const bool live = t < (int)sz;
    const uint64_t me = live ? x[t] : ~0ull;
    const uint32_t key = (uint32_t)(me >> 32);
    const bool start = live && (t == 0 || (uint32_t)(x[t - 1] >> 32) != key);
    const bool tail = live && (t == (int)sz - 1 || (uint32_t)(x[t + 1] >> 32) != key);
    const uint64_t S = __ballot(start), T = __ballot(tail);
    if (lane == 0) {
        wl[wv] = S ? wv * 64 + 63 - __clzll((long long)S) : -1;
        wf[wv] = T ? wv * 64 + __ffsll((unsigned long long)T) - 1 : 1 << 30;
    }
    __syncthreads();
    int head = -1;
    const uint64_t Sb = S & (lanes_below(lane) | (1ull << lane));
    if (Sb) head = wv * 64 + 63 - __clzll((long long)Sb);
    else
        for (int w = 0; w < wv; ++w) head = max(head, wl[w]);
    const uint32_t v = (uint32_t)me;   // as in k_ls_wave: moved values, changed ranks
    if (live && v != orig) vals[s + t] = v;
    block_push_sharded<kWB>(live && head != 0, ((uint64_t)(v & kPosMask) << 32) | (s + (uint32_t)head), o.chg,
                            o.ccnt, o.ccap, o.ccnt + 8);
    const bool multi = start && !tail;
    int end = 1 << 30;
    if (multi) {
        const uint64_t Ta = T & (~0ull << lane);
        if (Ta) end = wv * 64 + __ffsll((unsigned long long)Ta) - 1;
        else
            for (int w = wv + 1; w < kWB / 64; ++w) end = min(end, wf[w]);
    }
    block_append_sharded<kWB>(multi, s + (uint32_t)t, s + (uint32_t)end + 1, o.ngs, o.nge, o.ncnt, o.cap, o.ncnt + 8);
}

// one wave-class pass over the cnt groups of a class list
template <int W>
void ls_wave_pass(Ctx &c, const char *name, const uint32_t *cs, const uint32_t *cz, uint32_t cnt, uint32_t *vals,
                  const uint32_t *rank, int64_t n, int64_t h, const LsOut &o, const Deep &dp) {
    if (!cnt) return;
    const unsigned grid = (unsigned)((cnt + (kLB / 64) * (64 / W) - 1) / ((kLB / 64) * (64 / W)));
    KLAUNCH(name, 0.0, (k_ls_wave<W>), dim3(grid), dim3(kLB), 0, c.stream, cs, cz, (int64_t)cnt, vals, rank, n, h, o,
            dp);
}

// groups larger than kMedium: (group index << 30 | rank[a+h]) keys gathered
// into one segmented radix sort; starts/sizes/offs = the large-group table
__global__ __launch_bounds__(kB) void k_dna_refine_keys(const uint32_t *__restrict__ starts, const uint32_t *__restrict__ sizes,
                                                        const uint32_t *__restrict__ offs, const uint32_t *__restrict__ vals,
                                                        const uint32_t *__restrict__ rank, int64_t n, int64_t h,
                                                        uint64_t *__restrict__ rk, uint32_t *__restrict__ rv, Deep dp) {
    const uint32_t q = blockIdx.y;
    const uint32_t s = starts[q], sz = sizes[q], at = offs[q];
    for (uint32_t k = blockIdx.x * kB + threadIdx.x; k < sz; k += gridDim.x * kB) {
        const uint32_t v = vals[s + k];
        rk[at + k] = ((uint64_t)q << 30) | ls_key(rank, v, n, h, dp, s, sz);
        rv[at + k] = v;
    }
}

__global__ __launch_bounds__(kB) void k_dna_refine_back(const uint32_t *__restrict__ starts, const uint32_t *__restrict__ sizes,
                                                        const uint32_t *__restrict__ offs, const uint32_t *__restrict__ rv,
                                                        uint32_t *__restrict__ vals) {
    const uint32_t q = blockIdx.y;
    const uint32_t s = starts[q], sz = sizes[q], at = offs[q];
    for (uint32_t k = blockIdx.x * kB + threadIdx.x; k < sz; k += gridDim.x * kB) vals[s + k] = rv[at + k];
}

// subgroups after the pass: runs of equal keys (same q)
__global__ __launch_bounds__(kB) void k_dna_refine_flags(const uint64_t *__restrict__ rk, int64_t m,
                                                         uint32_t *__restrict__ fs, uint32_t *__restrict__ fe) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= m) return;
    const uint64_t x = rk[k];
    const bool head = k == 0 || rk[k - 1] != x;
    const bool tail = k + 1 == m || rk[k + 1] != x;
    fs[k] = head && !tail;
    fe[k] = tail && !head;
}

// new heads of the large groups' members: the subgroup start (gs, gathered
// index) when inside a tied run, else the member itself, mapped to vals
__global__ __launch_bounds__(kB) void k_dna_refine_rank(const uint64_t *__restrict__ rk, const uint32_t *__restrict__ rv,
                                                        const uint32_t *__restrict__ ps, const uint32_t *__restrict__ pe,
                                                        const uint32_t *__restrict__ gs, const uint32_t *__restrict__ starts,
                                                        const uint32_t *__restrict__ offs, int64_t m,
                                                        uint32_t *__restrict__ rank) {
    const int64_t k = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (k >= m) return;
    const uint32_t started = ps[k + 1];
    const uint32_t hk = started > pe[k] ? gs[started - 1] : (uint32_t)k;
    const uint32_t q = (uint32_t)(rk[k] >> 30);
    rank[rv[k] & kPosMask] = starts[q] + (hk - offs[q]);
}

// subgroup bounds from gathered indices to positions in vals: index k of large
// group q = rk[k] >> 30 sits at starts[q] + (k - offs[q]); ends are exclusive
__global__ __launch_bounds__(kB) void k_dna_refine_pos(const uint64_t *__restrict__ rk, const uint32_t *__restrict__ starts,
                                                       const uint32_t *__restrict__ offs, uint32_t *__restrict__ gs,
                                                       uint32_t *__restrict__ ge, int64_t G) {
    const int64_t x = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (x >= G) return;
    const uint32_t k = gs[x], kl = ge[x] - 1;
    const uint32_t q = (uint32_t)(rk[k] >> 30);
    gs[x] = starts[q] + (k - offs[q]);
    ge[x] = starts[q] + (kl - offs[q]) + 1;
}

struct Sym8 {
    uint8_t s[8];   // byte of each BWT code
};
__global__ __launch_bounds__(kB) void k_dna_final(const uint32_t *__restrict__ vals, int64_t n, uint32_t *__restrict__ sa,
                                                  uint8_t *__restrict__ bwt, int32_t *__restrict__ sampled,
                                                  int32_t sample, Sym8 sym) {
    const int64_t r = (int64_t)blockIdx.x * kB + threadIdx.x;
    if (r >= n) return;
    const uint32_t v = vals[r];
    sa[r] = v & kPosMask;
    if (r % sample == 0) sampled[r / sample] = (int32_t)(v & kPosMask);   // the SA row is already in hand
    bwt[r] = sym.s[v >> 29];
}

}  // namespace

bool sa_dna_eligible(const uint8_t last, int64_t n, const int64_t *totals) {
    if (n < 2 || n > (int64_t)kPosMask || last != '$' || totals['$'] != 1) return false;
    return totals['A'] + totals['C'] + totals['G'] + totals['T'] + 1 == n;
}

int sa_small_alphabet(const uint8_t last, int64_t n, const int64_t *totals, uint8_t *lut, uint8_t *sym) {
    if (n < 2 || n > (int64_t)kPosMask || last != '$' || totals['$'] != 1) return 0;
    int k = 0;
    std::memset(lut, 0, 256);
    for (int b = 0; b < 256; ++b) {
        if (!totals[b] || b == '$') continue;
        if (b < '$' || k == 7) return 0;   // '$' must sort first; codes 0..6 (7 is '$' in the values)
        lut[b] = (uint8_t)k;
        sym[k++] = (uint8_t)b;
    }
    sym[7] = '$';
    return k;
}

namespace {
// SA (uint32[n]) and BWT (uint8[n]) of t[0, n) = the text with its single
// final '$': ACGT (lut == nullptr: 2-bit bases, 32-bit keys) or a small
// alphabet (lut: symbol codes, 48-bit keys); false when a round outgrows its
// lists (the caller then runs the general prefix doubling)
bool sa_sort(Ctx &c, const uint8_t *t, int64_t n, uint32_t *SA, uint8_t *BWT, int32_t *sampled, int32_t sample,
             const uint8_t *lut, const uint8_t *symtab) {
    hipStream_t st = c.stream;
    const bool small = lut != nullptr;
    const int64_t nw = small ? (n + 15) / 16 + 2 : (n + 31) / 32 + 2;
    c.slot[S_IDX0].ensure((size_t)n * (small ? 8 : 4) + 64);      // keys, then class lists
    c.slot[S_IDX1].ensure((size_t)n * 4 + 64);      // values
    c.slot[S_IDX2].ensure((size_t)nw * 8 + 64);     // packed text
    c.slot[S_IDX3].ensure((size_t)(n + 1) * 4);     // group-start flags
    c.slot[S_IDX4].ensure((size_t)(n + 1) * 4 + 256);   // their positions (first: the group tiles' counts)
    c.slot[S_IDX5].ensure((size_t)(n + 1) * 4);     // group-end flags
    c.slot[S_IDX6].ensure((size_t)(n + 1) * 4);     // their positions
    c.slot[S_MISC3].ensure(512);   // 6 class counts | 8 + 1 group-list counters | 8 + 1 change counters; symbol lut
    uint32_t *keys = c.slot[S_IDX0].as<uint32_t>();
    uint32_t *vals = c.slot[S_IDX1].as<uint32_t>();
    uint64_t *P = c.slot[S_IDX2].as<uint64_t>();
    uint32_t *fs = c.slot[S_IDX3].as<uint32_t>(), *ps = c.slot[S_IDX4].as<uint32_t>();
    uint32_t *fe = c.slot[S_IDX5].as<uint32_t>(), *pe = c.slot[S_IDX6].as<uint32_t>();
    uint32_t *counts = c.slot[S_MISC3].as<uint32_t>();

    uint64_t *keys64 = c.slot[S_IDX0].as<uint64_t>();
    Sym8 sym{{'A', 'C', 'G', 'T', '$', 0, 0, 0}};
    if (small) {
        std::memcpy(sym.s, symtab, 8);
        uint8_t *d_lut = reinterpret_cast<uint8_t *>(c.slot[S_MISC3].as<char>() + 256);
        HIPCHECK(hipMemcpyAsync(d_lut, lut, 256, hipMemcpyHostToDevice, st));
        KLAUNCH("sym_pack", (double)n + (double)n / 2.0, k_sym_pack, dim3(nblocks(nw)), dim3(kB), 0, st, t, n, d_lut, P,
                nw);
        KLAUNCH("sym_keys", (double)n / 2.0 + 12.0 * (double)n, k_sym_keys, dim3(nblocks(n)), dim3(kB), 0, st, P, n,
                keys64, vals);
        radix_sort_pairs32(c, keys64, vals, n, 0, 48);
    } else {
        KLAUNCH("dna_pack", (double)n + (double)n / 4.0, k_dna_pack, dim3(nblocks(nw)), dim3(kB), 0, st, t, n, P, nw);
        KLAUNCH("dna_keys", (double)n / 4.0 + 8.0 * (double)n, k_dna_keys, dim3(nblocks(n)), dim3(kB), 0, st, P, n,
                keys, vals);
        radix_sort_pairs_k32(c, keys, vals, n, 0, 32);
    }

    // groups of equal 16-base prefixes -> (start, end) lists
    auto groups = [&](const uint32_t *f_s, uint32_t *p_s, const uint32_t *f_e, uint32_t *p_e, int64_t m,
                      uint32_t *gs, uint32_t *ge) -> int64_t {
        HIPCHECK(hipMemsetAsync(const_cast<uint32_t *>(f_s) + m, 0, 4, st));
        exclusive_scan<uint32_t>(c, f_s, p_s, m + 1);
        exclusive_scan<uint32_t>(c, f_e, p_e, m);
        uint32_t G = 0;
        HIPCHECK(hipMemcpyAsync(&G, p_s + m, 4, hipMemcpyDeviceToHost, st));
        KLAUNCH("dna_compact", 0.0, k_dna_compact2, dim3(nblocks(m)), dim3(kB), 0, st, f_s, p_s, f_e, p_e, m, gs, ge);
        HIPCHECK(hipStreamSynchronize(st));
        return (int64_t)G;
    };
    // group lists: current round and next round, (start, exclusive end) in vals
    // (<= n/2 groups; the sharded appends leave holes: slack for them and for
    // uneven shards -- a list that would outgrow it takes the general path)
    const int64_t lalloc = n / 2 + n / 8 + 16 * (int64_t)kCH + 64;
    for (int q : {S_MISC0, S_MISC1, S_IDX9, S_IDX10}) c.slot[q].ensure((size_t)lalloc * 4);
    int64_t lcap = lalloc;
    if (knob(KN_LS_CAP) >= 0) lcap = std::min<int64_t>(lcap, knob(KN_LS_CAP));   // test hook
    c.slot[S_IDX8].ensure((size_t)n * 4 + 64);
    // a round's rank changes (<= its members; holes and uneven shards as above)
    const int64_t calloc_ = n + n / 4 + 16 * (int64_t)kCH + 64;
    c.slot[S_IDX11].ensure((size_t)calloc_ * 8);
    int64_t ccap = calloc_;
    if (knob(KN_LS_CAP) >= 0) ccap = std::min<int64_t>(ccap, 2 * knob(KN_LS_CAP));
    uint64_t *chg = c.slot[S_IDX11].as<uint64_t>();
    uint32_t *gs = c.slot[S_MISC0].as<uint32_t>(), *ge = c.slot[S_MISC1].as<uint32_t>();
    uint32_t *xs = c.slot[S_IDX9].as<uint32_t>(), *xe = c.slot[S_IDX10].as<uint32_t>();
    uint32_t *rank = c.slot[S_IDX8].as<uint32_t>();
    // the 16-base groups: gs / ge in SA order and every suffix's run head (in
    // the flag buffer, dead until the large-group rounds)
    uint32_t *hd = fs;
    int64_t G = 0;
    {
        const int64_t nt = (n + kGTile - 1) / kGTile;
        uint32_t *tcnt = ps;   // 3 nt + 1 words
        if (small) {
            KLAUNCH("dna_grp_count", 8.0 * (double)n, k_grp_count<uint64_t>, dim3((unsigned)nt), dim3(kB), 0, st,
                    keys64, n, tcnt);
            KLAUNCH("dna_grp_scan", 0.0, k_grp_scan, dim3(1), dim3(1024), 0, st, tcnt, nt);
            KLAUNCH("dna_grp_apply", 12.0 * (double)n, k_grp_apply<uint64_t>, dim3((unsigned)nt), dim3(kB), 0, st,
                    keys64, n, tcnt, gs, ge, hd);
        } else {
            KLAUNCH("dna_grp_count", 4.0 * (double)n, k_grp_count<uint32_t>, dim3((unsigned)nt), dim3(kB), 0, st, keys,
                    n, tcnt);
            KLAUNCH("dna_grp_scan", 0.0, k_grp_scan, dim3(1), dim3(1024), 0, st, tcnt, nt);
            KLAUNCH("dna_grp_apply", 8.0 * (double)n, k_grp_apply<uint32_t>, dim3((unsigned)nt), dim3(kB), 0, st, keys,
                    n, tcnt, gs, ge, hd);
        }
        uint32_t g32 = 0;
        HIPCHECK(hipMemcpyAsync(&g32, tcnt + 3 * nt, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        c.checks_verify("the suffix sort's 16-symbol groups");
        G = g32;
    }
    // rank[pos] = head
    const int64_t nput = (n + kB * kPutItems - 1) / (kB * kPutItems);
    if (n <= (1 << 16)) {
        KLAUNCH("dna_rank_put", 12.0 * (double)n, k_dna_rank_put<false>, dim3((unsigned)nput), dim3(kB), 0, st, vals,
                hd, n, nput, rank, c.checks());
    } else {
        // through a position partition (the pass output in the sort's buffers):
        // two stable passes order the pairs by the top 16 position bits, so one
        // workgroup's 4096 pairs cover about 4096 consecutive ranks (16 KB written
        // whole inside the workgroup) instead of 4096 scattered ranks of a
        // 2^(bits-8) window merged across workgroups in the XCD's L2 (one pass:
        // 3.3x write amplification, PMC r03i; the direct scatter 2.35 ms at C3)
        int bits = 0;
        while ((int64_t{1} << bits) < n) ++bits;
        c.slot[S_SORT_TMP0].ensure((size_t)n * 4);
        c.slot[S_SORT_TMP1].ensure((size_t)n * 4);
        uint32_t *pv = c.slot[S_SORT_TMP0].as<uint32_t>(), *ph = c.slot[S_SORT_TMP1].as<uint32_t>();
        radix_pass_k32(c, vals, hd, pv, ph, n, bits - 16);
        radix_pass_k32(c, pv, ph, fe, pe, n, bits - 8);   // fe / pe are free until the refine rounds
        if (bits - 16 <= 12)   // 2^(bits-16) positions per 16-bit window divide the 4096-pair tile
            KLAUNCH("dna_rank_put", 12.0 * (double)n, k_dna_rank_put_tile<true>, dim3((unsigned)nput), dim3(kB), 0, st,
                    fe, pe, n, rank, c.checks());
        else   // texts past 2^28 bases: streaming stores into the 2^(bits-16) windows
            KLAUNCH("dna_rank_put", 12.0 * (double)n, k_dna_rank_put<true>, dim3((unsigned)nput), dim3(kB), 0, st, fe,
                    pe, n, nput, rank, c.checks());
    }
    if (G) KLAUNCH("dna_short_fix", 0.0, k_dna_short_fix, dim3(1), dim3(1024), 0, st, vals, rank, gs, ge, G, n,
                   c.checks());

    // runs of >= 16 equal symbols: their blocks' run ends (Deep); the flag
    // buffers are free until the large-group rounds
    Deep dp{P, nullptr, small ? 1 : 0, 0, c.checks()};
    if (G > 0) {
        const int64_t cap = n / 16 + 64;   // runs of >= 16 are disjoint
        c.slot[S_IDX12].ensure((size_t)(n / 16 + 2) * 4 + (size_t)cap * 4 + 64);
        uint32_t *re = c.slot[S_IDX12].as<uint32_t>(), *rs = re + n / 16 + 2;
        uint32_t *kcount = counts + 40;   // past the class / list / change counters
        HIPCHECK(hipMemsetAsync(kcount, 0, 4, st));
        KLAUNCH("dna_run_starts", 0.0, k_run_starts, dim3(nblocks((n + 15) / 16)), dim3(kB), 0, st, dp, n, rs, kcount,
                (uint32_t)cap);
        uint32_t K = 0;
        HIPCHECK(hipMemcpyAsync(&K, kcount, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        c.checks_verify("the suffix sort's first ranks and run starts");
        if (K) {
            KLAUNCH("dna_run_ends", 0.0, k_run_ends, dim3((unsigned)std::min<uint32_t>(K, 2048)), dim3(kB), 0, st, dp, n,
                    rs, kcount, re);
            dp.re = re;
            dp.on = 1;
        }
    }

    std::vector<uint32_t> lstart, lsize, loff;
    ShardedList sl{};   // the first list is plain
    for (int64_t h = 16; G > 0; h *= 2) {
        if (h >= 2 * n) return false;   // cannot happen ('$' is unique); the general path if it does
        // the keys are dead: class lists (5 x (start, size), capacity G each) and
        // the large-group table (3 x <= G) live in their buffer
        c.slot[S_IDX0].ensure((size_t)((2 * kClasses + 3) * G + 16) * 4);
        keys = c.slot[S_IDX0].as<uint32_t>();
        uint32_t *cs = keys, *cz = keys + kClasses * G;
        HIPCHECK(hipMemsetAsync(counts, 0, 256, st));
        KLAUNCH("dna_classify", 0.0, k_dna_classify, dim3(nblocks(G, kB * kCI)), dim3(kB), 0, st, gs, ge, G, sl, cs, cz,
                counts, G);
        uint32_t cnt[kClasses];
        HIPCHECK(hipMemcpyAsync(cnt, counts, sizeof cnt, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        c.checks_verify("a doubling round");
        if (FILE *tf = Ctx::ktrace_file())
            std::fprintf(tf, "# round h=%lld G=%lld classes %u %u %u %u %u %u\n", (long long)h, (long long)G, cnt[0],
                         cnt[1], cnt[2], cnt[3], cnt[4], cnt[5]);
        uint32_t *ncnt = counts + 8;   // [0, 8) shards, [8] overflow; the changes' at +16
        const LsOut o{xs, xe, ncnt, (uint32_t)lcap, chg, counts + 24, (uint32_t)ccap};
        const int64_t L = cnt[5];
        int64_t M = 0;
        uint32_t *tab = keys + 2 * kClasses * G;
        uint64_t *rk = nullptr;
        uint32_t *rv = nullptr;
        dim3 grid2;
        if (L) {
            if (L > 65535) return false;   // grid.y bound: such texts take the general path
            lstart.resize((size_t)L);
            lsize.resize((size_t)L);
            loff.resize((size_t)L);
            HIPCHECK(hipMemcpyAsync(lstart.data(), cs + 5 * G, (size_t)L * 4, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipMemcpyAsync(lsize.data(), cz + 5 * G, (size_t)L * 4, hipMemcpyDeviceToHost, st));
            HIPCHECK(hipStreamSynchronize(st));
            uint32_t mx = 0;
            for (int64_t q = 0; q < L; ++q) {
                loff[(size_t)q] = (uint32_t)M;
                M += lsize[(size_t)q];
                mx = std::max(mx, lsize[(size_t)q]);
            }
            c.slot[S_IDX7].ensure((size_t)M * 8 + 64);
            c.slot[S_MISC2].ensure((size_t)M * 4 + 64);
            rk = c.slot[S_IDX7].as<uint64_t>();
            rv = c.slot[S_MISC2].as<uint32_t>();
            HIPCHECK(hipMemcpyAsync(tab, lstart.data(), (size_t)L * 4, hipMemcpyHostToDevice, st));
            HIPCHECK(hipMemcpyAsync(tab + L, lsize.data(), (size_t)L * 4, hipMemcpyHostToDevice, st));
            HIPCHECK(hipMemcpyAsync(tab + 2 * L, loff.data(), (size_t)L * 4, hipMemcpyHostToDevice, st));
            grid2 = dim3((unsigned)std::min<int64_t>(64, (mx + kB - 1) / kB), (unsigned)L);
            KLAUNCH("dna_refine_keys", 0.0, k_dna_refine_keys, grid2, dim3(kB), 0, st, tab, tab + L, tab + 2 * L, vals,
                    rank, n, h, rk, rv, dp);
        }
        // the sorts read rank[a + h] as the round found it (the large groups'
        // keys are gathered above); their rank changes are stored after them
        ls_wave_pass<4>(c, "dna_ls_w4", cs, cz, cnt[0], vals, rank, n, h, o, dp);
        ls_wave_pass<16>(c, "dna_ls_w16", cs + G, cz + G, cnt[1], vals, rank, n, h, o, dp);
        ls_wave_pass<32>(c, "dna_ls_w32", cs + 2 * G, cz + 2 * G, cnt[2], vals, rank, n, h, o, dp);
        ls_wave_pass<64>(c, "dna_ls_w64", cs + 3 * G, cz + 3 * G, cnt[3], vals, rank, n, h, o, dp);
        if (cnt[4])
            KLAUNCH("dna_ls_block", 0.0, k_ls_block, dim3(cnt[4]), dim3(kWB), 0, st, cs + 4 * G, cz + 4 * G, vals,
                    rank, n, h, o, dp);
        uint32_t sc[25];   // group shards, overflow | 7 unused | change shards, overflow
        HIPCHECK(hipMemcpyAsync(sc, ncnt, sizeof sc, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        if (sc[8] || sc[24]) return false;
        ShardedList csl{};
        for (int q = 0; q < 8; ++q) {
            csl.cnt[q] = sc[16 + q];
            if (sc[16 + q]) csl.S = std::max<uint32_t>(csl.S, (((sc[16 + q] - 1) / kCH) * 8 + (uint32_t)q + 1) * kCH);
        }
        if (csl.S)
            KLAUNCH("dna_ls_apply", 0.0, k_ls_apply, dim3(nblocks(csl.S)), dim3(kB), 0, st, chg, (int64_t)csl.S, csl,
                    rank);
        if (sc[8]) return false;
        ShardedList nsl{};
        for (int q = 0; q < 8; ++q) {
            nsl.cnt[q] = sc[q];
            if (sc[q]) nsl.S = std::max<uint32_t>(nsl.S, (((sc[q] - 1) / kCH) * 8 + (uint32_t)q + 1) * kCH);
        }
        const int64_t nc = nsl.S;
        int64_t next = nc;
        if (L) {   // large groups: one segmented radix pass
            if (nc + M / 2 + 1 > lcap) return false;
            int qb = 1;
            while ((1ll << qb) < L) ++qb;
            radix_sort_pairs32(c, rk, rv, M, 0, ((30 + qb + 7) / 8) * 8);
            KLAUNCH("dna_refine_back", 0.0, k_dna_refine_back, grid2, dim3(kB), 0, st, tab, tab + L, tab + 2 * L, rv,
                    vals);
            KLAUNCH("dna_refine_flags", 0.0, k_dna_refine_flags, dim3(nblocks(M)), dim3(kB), 0, st, rk, M, fs, fe);
            const int64_t Gl = groups(fs, ps, fe, pe, M, xs + nc, xe + nc);
            KLAUNCH("dna_refine_rank", 0.0, k_dna_refine_rank, dim3(nblocks(M)), dim3(kB), 0, st, rk, rv, ps, pe,
                    xs + nc, tab, tab + 2 * L, M, rank);
            if (Gl)
                KLAUNCH("dna_refine_pos", 0.0, k_dna_refine_pos, dim3(nblocks(Gl)), dim3(kB), 0, st, rk, tab,
                        tab + 2 * L, xs + nc, xe + nc, Gl);
            next += Gl;
        }
        std::swap(gs, xs);
        std::swap(ge, xe);
        G = next;
        sl = nsl;
    }
    KLAUNCH("dna_final", 9.0 * (double)n + 4.0 * (double)((n + sample - 1) / sample), k_dna_final, dim3(nblocks(n)),
            dim3(kB), 0, st, vals, n, SA, BWT, sampled, sample, sym);
    HIPCHECK(hipGetLastError());
    return true;
}
}  // namespace

bool sa_dna_device(Ctx &c, const uint8_t *t, int64_t n, uint32_t *SA, uint8_t *BWT, int32_t *sampled, int32_t sample) {
    return sa_sort(c, t, n, SA, BWT, sampled, sample, nullptr, nullptr);
}

bool sa_small_device(Ctx &c, const uint8_t *t, int64_t n, uint32_t *SA, uint8_t *BWT, int32_t *sampled, int32_t sample,
                     const uint8_t *lut, const uint8_t *sym) {
    return sa_sort(c, t, n, SA, BWT, sampled, sample, lut, sym);
}

}  // namespace bwtmi
