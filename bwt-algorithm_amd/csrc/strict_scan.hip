// strict_scan.hip -- exact adjacent-copy tandem scan on gfx950.
//
// Replaces Tier2LCPFinder.find_long_unit_repeats_strict (bwt.py:1891-2001)
// with max_mismatch = 0.  For one unit length L the reference's while-loop is
// equivalent to a run formulation:
//   M_L[j] = (t[j] == t[j+L]), j < n-L; for each maximal 1-run [s,e) in
//   position order, i = max(s, carry); if e - i >= (min_copies-1)*L emit
//   count = 1 + (e-i)/L and set carry = i + count*L.
// Kernel pipeline (one launch each, all on the ctx stream):
//   k_pack       bytes -> B-bit codes (B = 2/4/8 from the contig's alphabet),
//                64-bit words, coalesced
//   k_runs       grid (word tiles x L chunks): every lane owns 32 positions
//                for every L of its chunk; equality masks by XOR of packed windows, neighbour
//                masks by wave shuffles; emits the maximal runs long enough
//                to hold min_copies copies (candidates)
//   radix sort   candidates by (L desc, s asc) -- the reference order
//   k_resolve    chains of candidates closer than L (where carry can act) are
//                walked by their head lane; all others resolve independently
//   scan+compact hits in candidate order, each with the smallest divisor
//                period of its first unit (k_period on the min_copies = 1 path)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr uint32_t FULL = 0xFFFFFFFFu;

// ------------------------------------------------------------------ pack
// Bit-plane layout: word w (positions 32w .. 32w+31) is B uint32 planes,
// plane p holding bit p of each position's code (bit k <-> position 32w+k).
// The equality mask of two windows is then ~OR_p(a_p ^ b_p): no bit
// compaction, and an unaligned window is one v_alignbit per plane.
template <int B>
__global__ __launch_bounds__(256) void k_pack(const uint8_t *__restrict__ text, int64_t n,
                                              const uint8_t *__restrict__ code, uint32_t *__restrict__ P,
                                              int64_t nwords) {
    __shared__ uint8_t cmap[256];
    cmap[threadIdx.x] = code[threadIdx.x];
    __syncthreads();
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwords) return;
    const int64_t j0 = w * 32;
    uint32_t pl[B];
#pragma unroll
    for (int p = 0; p < B; ++p) pl[p] = 0;
    if (j0 + 32 <= n) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint64_t v = *reinterpret_cast<const uint64_t *>(text + j0 + 8 * q);
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t cd = cmap[(v >> (8 * b)) & 255u];
#pragma unroll
                for (int p = 0; p < B; ++p) pl[p] |= ((cd >> p) & 1u) << (8 * q + b);
            }
        }
    } else {
        for (int k = 0; k < 32; ++k)
            if (j0 + k < n) {
                const uint32_t cd = cmap[text[j0 + k]];
#pragma unroll
                for (int p = 0; p < B; ++p) pl[p] |= ((cd >> p) & 1u) << k;
            }
    }
#pragma unroll
    for (int p = 0; p < B; ++p) P[w * B + p] = pl[p];
}

// M_L for positions 32w .. 32w+31 (bit k <-> position 32w+k), from global planes
template <int B>
__device__ __forceinline__ uint32_t eq32(const uint32_t *__restrict__ P, int64_t w, int64_t L, int64_t n) {
    const int64_t j0 = w * 32;
    const int64_t lim = n - L - j0;  // positions j0+k valid iff k < lim
    if (w < 0 || lim <= 0) return 0u;
    const int64_t q = w + (L >> 5);
    const uint32_t r = (uint32_t)(L & 31);
    uint32_t x = 0;
#pragma unroll
    for (int p = 0; p < B; ++p)
        x |= P[w * B + p] ^ __builtin_amdgcn_alignbit(P[(q + 1) * B + p], P[q * B + p], r);
    uint32_t m = ~x;
    if (lim < 32) m &= (1u << lim) - 1u;
    return m;
}

// Candidates go to kCandSegs segments of seg_cap slots, each with its own
// counter (segment = workgroup index mod kCandSegs): one counter for the whole
// grid serialises ~1.5M same-address atomics at the memory side.  The host
// compacts the segments afterwards (their order is irrelevant: a radix sort
// follows).
constexpr int kCandSegs = 256;

struct CandOut {
    uint64_t *keys;   // [kCandSegs][seg_cap]
    uint64_t *vals;
    unsigned long long *count;   // [kCandSegs]
    int64_t seg_cap;
    int32_t umax;
    int32_t sb;   // key = (umax - L) << sb | s, sb = bits of the text length
    // streaks whose end lies more than one 64-word step away: (L, start, first
    // word still to scan) triples, ended by k_streak_end one wave each
    int64_t *pend;                 // [pend_cap][3]
    unsigned long long *npend;     // entries pushed (may exceed pend_cap: the host retries)
    int64_t pend_cap;
};

// defer the end search of a streak (one lane)
__device__ __forceinline__ void push_pending(const CandOut &o, int64_t L, int64_t s, int64_t q0) {
    const unsigned long long at = atomicAdd(o.npend, 1ull);
    if ((int64_t)at < o.pend_cap) {
        o.pend[3 * at] = L;
        o.pend[3 * at + 1] = s;
        o.pend[3 * at + 2] = q0;
    }
}

// candidate at slot idx of segment seg, reserved by the wave (slots past
// seg_cap are counted, not written: the host retries with larger segments)
__device__ __forceinline__ void put(const CandOut &o, int seg, unsigned long long idx, int64_t L, int64_t s,
                                    int64_t e) {
    if ((int64_t)idx < o.seg_cap) {
        const int64_t at = (int64_t)seg * o.seg_cap + (int64_t)idx;
        o.keys[at] = ((uint64_t)(o.umax - L) << o.sb) | (uint64_t)s;
        o.vals[at] = (uint64_t)e;
    }
}

// segments -> one contiguous array (segment order)
__global__ void k_cand_gather(const uint64_t *__restrict__ ksegs, const uint64_t *__restrict__ vsegs,
                              const unsigned long long *__restrict__ count, const int64_t *__restrict__ off,
                              int64_t seg_cap, uint64_t *__restrict__ kout, uint64_t *__restrict__ vout) {
    const int seg = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)count[seg]) return;
    kout[off[seg] + i] = ksegs[(int64_t)seg * seg_cap + i];
    vout[off[seg] + i] = vsegs[(int64_t)seg * seg_cap + i];
}

constexpr int kOwn = 62;   // words owned per wave: lanes 1..62; lanes 0 and 63 only feed neighbours

// grid.x: tiles of 4 waves x 62 words; grid.y: runs of gper groups of unit
// lengths, group g = L in [32g, 32g+31].  All L of a group read the same two
// words q = w+g, q+1, so a lane holds its planes in registers and derives
// every M_L of the group from them; a workgroup walks its groups in turn.
template <int B>
__global__ __launch_bounds__(256) void k_runs(const uint32_t *__restrict__ P, int64_t n, int64_t nwords32,
                                              int32_t lmin, int32_t lmax, int64_t mc, int32_t gper, CandOut out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_base = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kOwn;
    const int64_t w = wave_base - 1 + lane;
    const bool owned = lane >= 1 && lane <= kOwn && w < nwords32;
    const int64_t j0 = w * 32;
    const int64_t tile_j0 = (int64_t)blockIdx.x * 4 * kOwn * 32;
    const bool inb = w >= 0 && w < nwords32;
    // this block's unit-length groups: g in [g0, g1), group g = L in [32g, 32g+31]
    const int64_t g0 = (int64_t)blockIdx.y * gper + (lmin >> 5);
    const int64_t g1 = min(g0 + (int64_t)gper, (int64_t)(lmax >> 5) + 1);
    // words past the text (the planes are zero-padded by 8 words) only feed
    // positions that the `lim` mask below discards
    auto word = [&](int64_t q, int p) { return inb && q < nwords32 + 8 ? P[q * B + p] : 0u; };
    // group g compares word w with words w+g, w+g+1: consecutive groups share
    // one of them, so each group loads one new word per plane (prefetched a
    // group ahead)
    uint32_t a[B], lo[B], hi[B], nx[B];
#pragma unroll
    for (int p = 0; p < B; ++p) {
        a[p] = inb ? P[w * B + p] : 0u;
        lo[p] = word(w + g0, p);
        hi[p] = word(w + g0 + 1, p);
    }
    for (int64_t g = g0; g < g1; ++g) {
#pragma unroll
    for (int p = 0; p < B; ++p) nx[p] = g + 1 < g1 ? word(w + g + 2, p) : 0u;
    // this group's unit lengths, bounds hoisted out of the loop (the kernel is
    // scalar-issue bound: every uniform test per L costs SALU slots): L >= lmin,
    // L <= lmax, and the tile must hold positions below n - L
    const int64_t Lg = g * 32;
    const int r_lo = (int)max((int64_t)0, (int64_t)lmin - Lg);
    const int r_hi = (int)min(min((int64_t)31, (int64_t)lmax - Lg), n - tile_j0 - 1 - Lg);
    const bool done = r_hi < 31;   // later groups have no work
    // positions j0 + k are valid for k < n - L - j0: only the text's last words need the mask
    const bool tail = !inb || j0 + 32 + Lg + 31 >= n;
    int64_t K = (mc - 1) * (Lg + r_lo);
    for (int r = r_lo; r <= r_hi; ++r, K += mc - 1) {
        const int64_t L = Lg + r;
        uint32_t x = 0;
#pragma unroll
        for (int p = 0; p < B; ++p) x |= a[p] ^ __builtin_amdgcn_alignbit(hi[p], lo[p], (uint32_t)r);
        uint32_t M = ~x;
        if (tail) {
            const int64_t lim = n - L - j0;
            if (!inb || lim <= 0) M = 0u;
            else if (lim < 32) M &= (1u << lim) - 1u;
        }
        if (K > 62) {
            // a qualifying run is >= 64 long, so it contains a full aligned
            // word: only the first full word of a streak can own it
            if (!__any(M == FULL)) continue;
        } else if (!__any(M != 0u)) {
            continue;
        }
        const uint32_t Mp = (uint32_t)__shfl_up((int)M, 1, 64);
        const uint32_t Mn = (uint32_t)__shfl_down((int)M, 1, 64);
        // This lane's candidates are counted first -- at most one streak
        // (first full word) or the short runs starting in its word -- so the
        // wave reserves all its output slots with ONE atomic: per-candidate
        // atomics on the single counter serialise millions of same-address
        // operations across the chip.
        int cnt = 0;
        int64_t s1 = 0, e1 = 0;   // streak candidate
        uint32_t qual = 0;        // qualifying short-run starts (bit k <-> position j0 + k)
        // end of the run that starts at bit k of this word (exclusive), or -1
        // when it joins a streak owned by word w+1
        auto run_end = [&](int k) -> int64_t {
            const uint32_t rr = M >> k;
            const int len_in = __ffs(~rr) - 1;   // ~rr has its top k bits set
            if (k + len_in < 32) return j0 + k + len_in;
            if (Mn == FULL) return -1;
            return j0 + 32 + (int64_t)__ffs(~Mn) - 1;
        };
        // Streaks (runs of full words): the first full word of each owns the
        // run.  Its end lies in the first non-full word after it -- found by a
        // ballot when that word is in this wave, else by the whole wave
        // scanning 64 words per step (long exact arrays repeat for many L, and
        // one lane walking them word by word stalls its wave on dependent loads).
        const bool sstart = owned && M == FULL && Mp != FULL;
        int64_t e_streak = -1;
        if (__any(sstart)) {   // (short unit lengths: rarely) the streak ends
            const uint64_t nf = __ballot(M != FULL);
            const uint64_t above = lane == 63 ? 0ull : (nf & (~0ull << (lane + 1)));
            const int src = above ? __ffsll((unsigned long long)above) - 1 : lane;
            const uint32_t Mend = (uint32_t)__shfl((int)M, src, 64);
            if (sstart && above) e_streak = (w + (src - lane)) * 32 + (int64_t)__ffs(~Mend) - 1;
            const bool beyond = sstart && !above;
            if (__any(beyond)) {   // at most one lane: the streak runs past lane 63's word
                // one 64-word step here; a streak longer than that (an assembly gap's
                // N run is one for every unit length) is ended by k_streak_end, so
                // the unit lengths' walks do not chain through this wave
                const int64_t q0 = wave_base + 63;
                const uint32_t Mq = eq32<B>(P, q0 + lane, L, n);   // 0 past the text: ends the scan
                const uint64_t nb = __ballot(Mq != FULL);
                if (nb) {
                    const int f = __ffsll((unsigned long long)nb) - 1;
                    const uint32_t Mf = (uint32_t)__shfl((int)Mq, f, 64);
                    if (beyond) e_streak = (q0 + f) * 32 + (int64_t)__ffs(~Mf) - 1;
                } else if (beyond) {
                    push_pending(out, L, j0 - (int64_t)__clz(~Mp), q0 + 64);
                }
            }
        }
        if (owned) {
            if (M == FULL) {
                if (sstart) {   // first full word of a streak
                    const int64_t s = j0 - (int64_t)__clz(~Mp);
                    if (e_streak - s >= K) {
                        cnt = 1;
                        s1 = s;
                        e1 = e_streak;
                    }
                }
            } else if (K <= 62 && M != 0u) {
                // runs that start in this word and contain no full aligned word;
                // only starts with K ones ahead (within M:Mn) can qualify
                uint32_t starts = M & ~((M << 1) | (Mp >> 31));
                const uint64_t V = (uint64_t)M | ((uint64_t)Mn << 32);
                uint64_t A = V;
                for (int64_t have = 1; have < K;) {
                    const int64_t s = have < K - have ? have : K - have;
                    A &= A >> s;
                    have += s;
                }
                starts &= (uint32_t)A;
                while (starts) {
                    const int k = __ffs(starts) - 1;
                    starts &= starts - 1;
                    const int64_t e = run_end(k);
                    if (e >= 0 && e - (j0 + k) >= K) {
                        qual |= 1u << k;
                        ++cnt;
                    }
                }
            }
        }
        if (!__any(cnt != 0)) continue;   // most (unit length, word) steps: no candidate, no prefix scan
        int incl = cnt;   // wave inclusive prefix of the counts
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const int tot = __builtin_amdgcn_readlane(incl, 63);   // scalar: the `continue` below is uniform
        if (tot == 0) continue;   // wave-uniform
        const int seg = (int)(blockIdx.x & (kCandSegs - 1));
        unsigned long long base = 0;
        if (lane == 63) base = atomicAdd(out.count + seg, (unsigned long long)tot);
        base = __shfl(base, 63, 64);
        unsigned long long at = base + (unsigned long long)(incl - cnt);
        if (cnt == 0) continue;
        if (M == FULL) {
            put(out, seg, at, L, s1, e1);
        } else {
            while (qual) {
                const int k = __ffs(qual) - 1;
                qual &= qual - 1;
                put(out, seg, at++, L, j0 + k, run_end(k));
            }
        }
    }
    if (done) break;
#pragma unroll
    for (int p = 0; p < B; ++p) {
        lo[p] = hi[p];
        hi[p] = nx[p];
    }
    }
}

// min_copies == 1: every position starts a hit; one lane walks one L.  Row
// `row` (L = lmax - row) owns hits[off[row] ..), at most n/L + 1 of them.
__global__ void k_mc1(const uint8_t *__restrict__ t, int64_t n, int32_t lmin, int32_t lmax,
                      const int64_t *__restrict__ off, bwtmi_hit *__restrict__ hits, int64_t *__restrict__ nper) {
    const int64_t L = lmax - (int64_t)(blockIdx.x * blockDim.x + threadIdx.x);
    if (L < lmin) return;
    const int64_t row = lmax - L;
    int64_t i = 0, k = 0;
    while (i + L <= n) {
        int64_t c = 1;
        while (i + (c + 1) * L <= n) {
            bool eq = true;
            for (int64_t x = 0; x < L && eq; ++x) eq = t[i + (c - 1) * L + x] == t[i + c * L + x];
            if (!eq) break;
            ++c;
        }
        bwtmi_hit h;
        h.start = i;
        h.end = i + c * L;
        h.unit_len = (int32_t)L;
        h.prim_len = 0;
        h.copies = c;
        hits[off[row] + k] = h;
        ++k;
        i += c * L;
    }
    nper[row] = k;
}

// ------------------------------------------------ max_mismatch > 0
// find_long_unit_repeats_strict with a Hamming tolerance (bwt.py:1929-1944):
// blocks j and j + L "match" iff D_L(j) = #{x in [j, j + L): t[x] != t[x + L]}
// <= m.  Row l (L = L0 - l) gets the bit P(j) = (j + 2L <= n and D_L(j) <= m)
// for every j, each thread sliding the window over kMmSeg positions
// (D_L(j + 1) = D_L(j) - [t[j] != t[j+L]] + [t[j+L] != t[j+2L]]).
constexpr int kMmSeg = 1024;
__global__ __launch_bounds__(256) void k_mm_pbits(const uint8_t *__restrict__ t, int64_t n, int32_t L0, int32_t m,
                                                  int64_t nw, uint32_t *__restrict__ P) {
    const int64_t L = L0 - (int64_t)blockIdx.y;
    const int64_t j0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kMmSeg;
    if (j0 >= n) return;
    uint32_t *row = P + (int64_t)blockIdx.y * (nw + 1);
    const int64_t jend = j0 + kMmSeg < n ? j0 + kMmSeg : n;
    int64_t D = 0;
    if (j0 + 2 * L <= n)
        for (int64_t x = j0; x < j0 + L; ++x) D += t[x] != t[x + L];
    uint32_t word = 0;
    for (int64_t j = j0; j < jend; ++j) {
        const bool p = j + 2 * L <= n && D <= m;
        word |= (uint32_t)p << (j & 31);
        if ((j & 31) == 31 || j == jend - 1) {
            row[j >> 5] = word;
            word = 0;
        }
        if (j + 2 * L < n) D += (int64_t)(t[j + L] != t[j + 2 * L]) - (int64_t)(t[j] != t[j + L]);
    }
}

// The scan itself, one wave per unit length: i = the first position >= carry
// with count >= mc, i.e. Q(i) = (i + L*mc <= n) and P(i), P(i+L), ...,
// P(i+(mc-2)L) (64 Q words per step, ballot); count = 1 + the run of P along
// i, i+L, ... (64 copies per step); hit [i, i + count*L); carry = its end.
// Carry and count are wave-uniform scalars (readfirstlane / ballot), so the
// loop exits together.  Row l writes (start, count) pairs at out + off[l].
__device__ __forceinline__ uint32_t pword_at(const uint32_t *row, int64_t bit) {
    const int64_t w = bit >> 5;
    const int s = (int)(bit & 31);
    const uint32_t lo = row[w];
    return s ? (lo >> s) | (row[w + 1] << (32 - s)) : lo;
}

__global__ __launch_bounds__(64) void k_mm_walk(const uint32_t *__restrict__ P, int64_t n, int64_t nw, int32_t L0,
                                                int32_t mc, const int64_t *__restrict__ off,
                                                int64_t *__restrict__ out, int64_t *__restrict__ nper) {
    const int64_t L = L0 - (int64_t)blockIdx.x;
    const int lane = threadIdx.x;
    const uint32_t *row = P + (int64_t)blockIdx.x * (nw + 1);
    int64_t *dst = out + 2 * off[blockIdx.x];
    const int64_t last = n - L * (int64_t)mc;   // the greatest i the loop visits (bwt.py:1923)
    int64_t carry = 0, k = 0;
    while (carry <= last) {
        const int64_t w0 = carry >> 5;
        const int64_t w = w0 + lane;
        uint32_t q = 0;
        if (w <= (last >> 5)) {
            q = ~0u;
            if (w == w0) q &= ~0u << (carry & 31);
            if (w == (last >> 5)) q &= (uint32_t)(~0ull >> (63 - (last & 31))) ;
            for (int c = 0; c + 1 < mc && q; ++c) q &= pword_at(row, (w << 5) + (int64_t)c * L);
        }
        const uint64_t bal = __ballot(q != 0);
        if (!bal) {
            carry = (w0 + 64) << 5;
            continue;
        }
        const int f = __ffsll((unsigned long long)bal) - 1;
        const uint32_t qf = (uint32_t)__builtin_amdgcn_readlane((int)q, f);
        const int64_t i = ((w0 + f) << 5) + (__ffs(qf) - 1);
        int64_t cnt = 1;
        for (;;) {   // the run of P(i + cL) for c = cnt - 1, cnt, ...
            const int64_t j = i + (cnt - 1 + lane) * L;
            const bool p = j < n && ((row[j >> 5] >> (j & 31)) & 1u);
            const uint64_t stop = __ballot(!p);
            if (stop) {
                cnt += __ffsll((unsigned long long)stop) - 1;
                break;
            }
            cnt += 64;
        }
        if (lane == 0) {
            dst[2 * k] = i;
            dst[2 * k + 1] = cnt;
        }
        ++k;
        carry = i + cnt * L;
    }
    if (lane == 0) nper[blockIdx.x] = k;
}

// ---------------------------------------------------------- resolution
__global__ __launch_bounds__(256) void k_resolve(const uint64_t *__restrict__ keys, const uint64_t *__restrict__ vals,
                                                 int64_t nc, int32_t umax, int sb, int64_t mc,
                                                 int64_t *__restrict__ hit_i, int64_t *__restrict__ hit_c,
                                                 uint32_t *__restrict__ flag) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    const uint64_t smask = (1ull << sb) - 1;
    auto Lof = [&](int64_t j) { return (int64_t)umax - (int64_t)(keys[j] >> sb); };
    const int64_t L = Lof(k);
    const int64_t s = (int64_t)(keys[k] & smask);
    const bool head = (k == 0) || Lof(k - 1) != L || s >= (int64_t)vals[k - 1] + L;
    if (!head) return;
    const int64_t K = (mc - 1) * L;
    int64_t carry = 0;
    for (int64_t j = k; j < nc; ++j) {
        const int64_t sj = (int64_t)(keys[j] & smask);
        if (j > k && (Lof(j) != L || sj >= (int64_t)vals[j - 1] + L)) break;
        const int64_t e = (int64_t)vals[j];
        const int64_t i = sj > carry ? sj : carry;
        if (e - i >= K) {
            const int64_t cnt = 1 + (e - i) / L;
            hit_i[j] = i;
            hit_c[j] = cnt;
            flag[j] = 1;
            carry = i + cnt * L;
        } else {
            flag[j] = 0;
        }
    }
}

// smallest_period_str of s[0 : L) (bwt.py:1125-1133): the first divisor d of L
// with s[x] == s[x - d] for all x in [d, L)
__device__ __forceinline__ int32_t smallest_period(const uint8_t *__restrict__ s, int32_t L) {
    for (int32_t d = 1; d < L; ++d) {   // 32-bit: the divisor tests are 32-bit remainders
        if (L % d) continue;
        int32_t x = d;
        while (x < L && s[x] == s[x - d]) ++x;
        if (x == L) return d;
    }
    return L;
}

// smallest_period of s[0, L) for L <= 32 in registers: the 32 bytes from
// three aligned 16-byte loads (every device text carries 128 zero bytes of
// padding: upload_text, the device loader),
// and each divisor d <= 16 of L tested as one comparison of the byte string
// with itself shifted by d (compile-time shifts): no chain of dependent byte
// loads per divisor
template <int D>
__device__ __forceinline__ bool shift_equal(const uint64_t (&w)[6], int32_t L) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int32_t lo = 8 * q;   // bytes [lo, lo + 8) of s[D..] against the same of s[0..]
        if (lo >= L - D) break;
        constexpr int W = D / 8, B = 8 * (D % 8);
        const uint64_t sh = B == 0 ? w[q + W] : (w[q + W] >> B) | (w[q + W + 1] << (64 - B));
        const int32_t nb = min(8, L - D - lo);
        const uint64_t m = nb >= 8 ? ~0ull : ((1ull << (8 * nb)) - 1ull);
        if ((sh ^ w[q]) & m) return false;
    }
    return true;
}
__device__ __forceinline__ int32_t period_le32(const uint8_t *__restrict__ t, int64_t start, int32_t L) {
    const uintptr_t addr = (uintptr_t)(t + start);
    const uint4 *a = reinterpret_cast<const uint4 *>(addr & ~(uintptr_t)15);
    const int off = (int)(addr & 15);
    const uint4 x0 = a[0], x1 = a[1], x2 = a[2];
    const uint64_t v[6] = {(uint64_t)x0.x | (uint64_t)x0.y << 32, (uint64_t)x0.z | (uint64_t)x0.w << 32,
                           (uint64_t)x1.x | (uint64_t)x1.y << 32, (uint64_t)x1.z | (uint64_t)x1.w << 32,
                           (uint64_t)x2.x | (uint64_t)x2.y << 32, (uint64_t)x2.z | (uint64_t)x2.w << 32};
    const int ws = off >> 3, bs = 8 * (off & 7);
    uint64_t w[6];
#pragma unroll
    for (int q = 0; q < 4; ++q) {   // bytes [8q, 8q + 8) of s
        const uint64_t lo = ws ? v[q + 1] : v[q], hi = ws ? v[q + 2] : v[q + 1];
        w[q] = bs ? (lo >> bs) | (hi << (64 - bs)) : lo;
    }
    w[4] = w[5] = 0;
    // bytes at or past L are not compared (masks), so what follows the unit is irrelevant
#define BWTMI_PERIOD_TRY(D) \
    if (D < L && L % D == 0 && shift_equal<D>(w, L)) return D;
    BWTMI_PERIOD_TRY(1) BWTMI_PERIOD_TRY(2) BWTMI_PERIOD_TRY(3) BWTMI_PERIOD_TRY(4)
    BWTMI_PERIOD_TRY(5) BWTMI_PERIOD_TRY(6) BWTMI_PERIOD_TRY(7) BWTMI_PERIOD_TRY(8)
    BWTMI_PERIOD_TRY(9) BWTMI_PERIOD_TRY(10) BWTMI_PERIOD_TRY(11) BWTMI_PERIOD_TRY(12)
    BWTMI_PERIOD_TRY(13) BWTMI_PERIOD_TRY(14) BWTMI_PERIOD_TRY(15) BWTMI_PERIOD_TRY(16)
#undef BWTMI_PERIOD_TRY
    return L;
}

// hits of unit length up to kThreadPeriodL get their period from one thread
// (at most kThreadPeriodL - 1 divisor candidates over a few cached bytes);
// longer units from one wave (k_period_wave): a thread walking a 1000-byte unit
// byte by byte is a serial chain of loads that held every launch for ~2.6 ms
constexpr int32_t kThreadPeriodL = 32;
static_assert(kThreadPeriodL <= 32, "period_le32 holds 32 bytes of the unit");

// compaction of the resolved hits, with the smallest period of each hit's
// first unit and the count after primitive reduction (bwt.py:1956-1961)
// Also the hits' longest span (the screen's key width): a workgroup maximum,
// and an atomic only when it beats the value already stored (one address for
// the whole grid: unconditional atomics serialise; maxlen zero before the launch)
__global__ __launch_bounds__(256) void k_compact(const uint64_t *__restrict__ keys, int64_t nc, int32_t umax, int sb,
                                                 const int64_t *__restrict__ hit_i, const int64_t *__restrict__ hit_c,
                                                 const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                 const uint8_t *__restrict__ t, bwtmi_hit *__restrict__ hits,
                                                 unsigned long long *__restrict__ maxlen) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = k < nc && flag[k];
    const int64_t L = live ? (int64_t)umax - (int64_t)(keys[k] >> sb) : 0;
    unsigned long long span = live ? (unsigned long long)(hit_c[k] * L) : 0ull;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) span = max(span, (unsigned long long)__shfl_xor(span, o, 64));
    __shared__ unsigned long long wmax[4];
    if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = span;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m > __hip_atomic_load(maxlen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxlen, m);
    }
    if (!live) return;
    bwtmi_hit h;
    h.start = hit_i[k];
    h.end = hit_i[k] + hit_c[k] * L;
    h.unit_len = (int32_t)L;
    if (L > kThreadPeriodL) {   // k_period_wave fills prim_len / copies
        h.prim_len = (int32_t)L;
        h.copies = hit_c[k];
        hits[pos[k]] = h;
        return;
    }
    const int32_t p = period_le32(t, h.start, (int32_t)L);
    h.prim_len = p;
    h.copies = p < L ? (h.end - h.start) / p : hit_c[k];
    hits[pos[k]] = h;
}

// number of candidates with unit length > lthr: a prefix of the (L desc) order
__global__ void k_count_long(const uint64_t *__restrict__ keys, int64_t nc, int32_t umax, int sb, int32_t lthr,
                             int64_t *__restrict__ out) {
    if (blockIdx.x || threadIdx.x) return;
    int64_t lo = 0, hi = nc;   // first k with L(k) <= lthr
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)umax - (int64_t)(keys[mid] >> sb) > lthr) lo = mid + 1;
        else hi = mid;
    }
    *out = lo;
}

// smallest_period_str (bwt.py:1125-1133) of one long first unit per wave: the
// lanes mark which of 64 consecutive d divide L (ballot), each divisor in
// ascending order is tested over the unit 64 bytes at a time (coalesced), the
// first one without a mismatch is the period
__device__ __forceinline__ void period_wave_one(const uint64_t *__restrict__ keys, int64_t k, int32_t umax, int sb,
                                                const int64_t *__restrict__ hit_i, const int64_t *__restrict__ hit_c,
                                                const uint32_t *__restrict__ pos, const uint8_t *__restrict__ t,
                                                bwtmi_hit *__restrict__ hits) {
    const int lane = threadIdx.x & 63;
    const int32_t L = (int32_t)((int64_t)umax - (int64_t)(keys[k] >> sb));
    const uint8_t *s = t + hit_i[k];
    int32_t p = L;
    for (int32_t base = 1; base < L && p == L; base += 64) {
        const int32_t dl = base + lane;
        uint64_t m = __ballot(dl < L && L % dl == 0);
        while (m) {
            const int32_t d = base + (__ffsll((unsigned long long)m) - 1);
            m &= m - 1;
            bool ok = true;
            for (int32_t x0 = d; x0 < L; x0 += 64) {
                const int32_t x = x0 + lane;
                if (__any(x < L && s[x] != s[x - d])) { ok = false; break; }
            }
            if (ok) { p = d; break; }
        }
    }
    if (lane == 0) {
        bwtmi_hit &h = hits[pos[k]];
        h.prim_len = p;
        h.copies = p < L ? (h.end - h.start) / p : hit_c[k];
    }
}

// The count of long units comes from the device (k_count_long): the launch
// is sized from the candidate count, and each wave takes units nwaves apart.
__global__ __launch_bounds__(256) void k_period_wave(const uint64_t *__restrict__ keys, const int64_t *__restrict__ d_nlong,
                                                     int32_t umax, int sb,
                                                     const int64_t *__restrict__ hit_i, const int64_t *__restrict__ hit_c,
                                                     const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                     const uint8_t *__restrict__ t, bwtmi_hit *__restrict__ hits) {
    const int64_t nlong = *d_nlong;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; k < nlong; k += nwaves)
        if (flag[k]) period_wave_one(keys, k, umax, sb, hit_i, hit_c, pos, t, hits);   // wave-uniform
}

// smallest_period_str of text[i : i+L] (bwt.py:1125-1133), then
// count = length // p when p < L (bwt.py:1957-1961)
__global__ __launch_bounds__(256) void k_period(const uint8_t *__restrict__ t, bwtmi_hit *__restrict__ hits, int64_t nh) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nh) return;
    bwtmi_hit h = hits[k];
    const int32_t L = h.unit_len;
    const int32_t p = smallest_period(t + h.start, L);
    h.prim_len = (int32_t)p;
    if (p < L) h.copies = (h.end - h.start) / p;
    hits[k] = h;
}

// which byte values occur in the text (the alphabet: only presence matters):
// 16 bytes per load, a 256-bit mask per lane in registers, OR-reduced per
// wave.  (A 256-bin LDS histogram spent 0.17 ms on a 100 Mbp text serialising
// on the 4 ACGT bins.)
__device__ __forceinline__ void mark(uint64_t (&m)[4], uint32_t b) {
    const uint64_t bit = 1ull << (b & 63u);
    const uint32_t q = b >> 6;
    m[0] |= q == 0 ? bit : 0ull;
    m[1] |= q == 1 ? bit : 0ull;
    m[2] |= q == 2 ? bit : 0ull;
    m[3] |= q == 3 ? bit : 0ull;
}
__device__ __forceinline__ void mark4(uint64_t (&m)[4], uint32_t w) {
    if ((w & 0xC0C0C0C0u) == 0x40404040u) {   // four bytes in 64..127 (letters): word 1 only
        m[1] |= (1ull << (w & 63u)) | (1ull << ((w >> 8) & 63u)) | (1ull << ((w >> 16) & 63u)) |
                (1ull << ((w >> 24) & 63u));
        return;
    }
    mark(m, w & 255u);
    mark(m, (w >> 8) & 255u);
    mark(m, (w >> 16) & 255u);
    mark(m, w >> 24);
}
__global__ __launch_bounds__(256) void k_present(const uint8_t *__restrict__ t, int64_t n,
                                                 unsigned long long *__restrict__ mask) {
    uint64_t m[4] = {0, 0, 0, 0};
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t head = std::min<int64_t>(n, (int64_t)((16 - ((uintptr_t)t & 15)) & 15));
    const int64_t nv = (n - head) / 16;
    const uint4 *v = reinterpret_cast<const uint4 *>(t + head);
    // four 16-byte loads in flight per thread and step (one at a time was
    // latency-bound: 69 us for 100 MB, r05zg)
    int64_t i = gid;
    for (; i + 3 * stride < nv; i += 4 * stride) {
        uint4 w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = v[i + q * stride];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mark4(m, w[q].x);
            mark4(m, w[q].y);
            mark4(m, w[q].z);
            mark4(m, w[q].w);
        }
    }
    for (; i < nv; i += stride) {
        const uint4 w = v[i];
        mark4(m, w.x);
        mark4(m, w.y);
        mark4(m, w.z);
        mark4(m, w.w);
    }
    if (gid == 0) {   // unaligned head and tail bytes
        for (int64_t i = 0; i < head; ++i) mark(m, t[i]);
        for (int64_t i = head + nv * 16; i < n; ++i) mark(m, t[i]);
    }
    // OR-reduced per wave, then per workgroup in LDS: one global atomic per
    // workgroup and word (per-wave atomics on the same few addresses serialised
    // at L2: 53 us on a 12.5 Mbp text, r05r)
    __shared__ unsigned long long bm[4];
    if (threadIdx.x < 4) bm[threadIdx.x] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint64_t x = m[j];
        for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o, 64);
        if ((threadIdx.x & 63) == 0 && x) atomicOr(&bm[j], (unsigned long long)x);
    }
    __syncthreads();
    if (threadIdx.x < 4 && bm[threadIdx.x]) atomicOr(mask + threadIdx.x, bm[threadIdx.x]);
}

// Long unit lengths, sampled.  When K = (mc-1)L >= 95, every qualifying run
// (length >= K) holds at least s = floor((K - 31) / 32) >= 2 consecutive full
// aligned words (a run of length R holds floor((R - 31) / 32) of them at
// least), so looking at every s-th word finds each such run: the work per
// group of 32 unit lengths drops from every word to every s-th one (s ~ 2g for
// group g at min_copies 3).  A sampled lane whose word is full (all 32
// positions match at distance L) owns the run when one of the s words before
// it is not full -- the first sample inside the run; the wave then finds the
// run's start among those s words and its end by scanning forward 64 words a
// step, for one owner at a time.  Runs and candidates are exactly the dense
// kernel's (K > 62: only streaks of full words qualify there too).
constexpr int kSparseMax = 48;   // groups per launch
struct SparseGroups {
    int32_t ng;
    int32_t g[kSparseMax];           // group: L in [32g, 32g+31] (clipped to [lmin, lmax])
    int32_t s[kSparseMax];           // sample stride in words
    int64_t woff[kSparseMax + 1];    // first wave of each group in the launch
};

template <int B>
__global__ __launch_bounds__(256) void k_runs_sparse(const uint32_t *__restrict__ P, int64_t n, int64_t nwords32,
                                                     int32_t lmin, int32_t lmax, int64_t mc, SparseGroups sg,
                                                     CandOut out) {
    const int lane = threadIdx.x & 63;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // wave of the launch
    int gi = 0;
    while (gi + 1 < sg.ng && q >= sg.woff[gi + 1]) ++gi;   // uniform
    if (q >= sg.woff[sg.ng]) return;
    const int64_t g = sg.g[gi], s = sg.s[gi];
    const int64_t w = ((q - sg.woff[gi]) * 64 + lane) * s;   // this lane's sampled word
    const bool inb = w < nwords32;
    auto word = [&](int64_t x, int p) { return inb && x < nwords32 + 8 ? P[x * B + p] : 0u; };
    uint32_t a[B], lo[B], hi[B];
#pragma unroll
    for (int p = 0; p < B; ++p) {
        a[p] = inb ? P[w * B + p] : 0u;
        lo[p] = word(w + g, p);
        hi[p] = word(w + g + 1, p);
    }
    const int64_t Lg = g * 32;
    const int r_lo = (int)max((int64_t)0, (int64_t)lmin - Lg);
    const int r_hi = (int)min((int64_t)31, (int64_t)lmax - Lg);
    const int64_t j0 = w * 32;
    const bool tail = !inb || j0 + 32 + Lg + 31 >= n;
    const int seg = (int)(blockIdx.x & (kCandSegs - 1));
    for (int r = r_lo; r <= r_hi; ++r) {
        const int64_t L = Lg + r, K = (mc - 1) * L;
        uint32_t x = 0;
#pragma unroll
        for (int p = 0; p < B; ++p) x |= a[p] ^ __builtin_amdgcn_alignbit(hi[p], lo[p], (uint32_t)r);
        uint32_t M = ~x;
        if (tail) {
            const int64_t lim = n - L - j0;
            if (!inb || lim <= 0) M = 0u;
            else if (lim < 32) M &= (1u << lim) - 1u;
        }
        // owner test, every full lane at once: the first non-full word among
        // w-1 .. w-s gives the run's start (word w-s is the previous sample: all
        // s full means that sample's run, not ours).  Inside a long streak every
        // sample is full, so the s words are checked 8 loads at a time per lane
        // rather than one lane after another for the whole wave.
        int64_t start = -1;
        if (__any(M == FULL) && M == FULL) {
            for (int64_t k0 = 1; k0 <= s && start < 0; k0 += 8) {
                uint32_t Mq[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) Mq[i] = k0 + i <= s ? eq32<B>(P, w - (k0 + i), L, n) : FULL;   // 0 before the text
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (start < 0 && Mq[i] != FULL) start = (w - (k0 + i) + 1) * 32 - (int64_t)__clz(~Mq[i]);
            }
        }
        uint64_t own = __ballot(start >= 0);   // uniform
        while (own) {
            const int src = __ffsll((unsigned long long)own) - 1;
            own &= own - 1;
            const int64_t ws = (int64_t)__builtin_amdgcn_readlane((int)(w / s), src) * s;   // the owner's word
            const int64_t st = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)start, src)) |
                               ((int64_t)__builtin_amdgcn_readlane((int)(start >> 32), src) << 32);
            // end: the first non-full word after ws -- one 64-word step here, a
            // longer streak is ended by k_streak_end
            const int64_t q0 = ws + 1;
            const uint32_t Mq = eq32<B>(P, q0 + lane, L, n);   // 0 past the text: ends the scan
            const uint64_t nb = __ballot(Mq != FULL);
            if (!nb) {
                if (lane == 0) push_pending(out, L, st, q0 + 64);
                continue;
            }
            const int f = __ffsll((unsigned long long)nb) - 1;
            const uint32_t Mf = (uint32_t)__builtin_amdgcn_readlane((int)Mq, f);
            const int64_t end = (q0 + f) * 32 + (int64_t)__ffs(~Mf) - 1;
            if (end - st >= K && lane == 0) {
                const unsigned long long at = atomicAdd(out.count + seg, 1ull);
                put(out, seg, at, L, st, end);
            }
        }
    }
}

// The sampled groups of unit lengths over LDS tiles: a workgroup copies its
// tile of kRunTile words (and the halo the sampled windows and owner tests
// reach: the largest stride before, one group plus two words after) into LDS
// once, coalesced, and then examines every sample of every group of the
// launch inside the tile from there -- the planes are read once per launch
// instead of three scattered lines per sample and group.  Samples of all
// groups are flattened over the lanes (the large-stride groups have few).
// Candidates and their order-free output are exactly k_runs_sparse's.
template <int B>
constexpr int run_tile() { return 2048 / B; }   // words per workgroup: <= 64 KB of LDS with a 256-word halo
constexpr int kRunGroupSplit = 2;   // gridDim.y: workgroups share a tile's groups (gi mod 2): 2x the
                                    // workgroups of a short contig, each tile read twice
template <int B>
__global__ __launch_bounds__(256) void k_runs_tiled(const uint32_t *__restrict__ P, int64_t n, int64_t nwords32,
                                                    int32_t lmin, int32_t lmax, int64_t mc, SparseGroups sg,
                                                    int32_t halo, int32_t after, CandOut out) {
    extern __shared__ uint32_t tl[];   // words base .. base + span - 1, B planes each
    __shared__ int64_t pre[kSparseMax + 1], first[kSparseMax];
    constexpr int kRunTile = run_tile<B>();
    const int64_t w0 = (int64_t)blockIdx.x * kRunTile;
    const int64_t base = w0 - halo;
    const int64_t span = halo + kRunTile + after;   // a sample w < w0 + kRunTile reads up to word w + g + 1
    for (int64_t k = threadIdx.x; k < span * B; k += 256) {
        const int64_t w = base + k / B;
        tl[k] = w >= 0 && w < nwords32 + 8 ? P[base * B + k] : 0u;
    }
    const int64_t wend = min(w0 + (int64_t)kRunTile, nwords32);
    if (threadIdx.x == 0) {   // samples j * s of this workgroup's groups in [w0, wend): [first, first + count)
        pre[0] = 0;
        for (int gi = 0; gi < sg.ng; ++gi) {
            const int64_t s = sg.s[gi];
            first[gi] = (w0 + s - 1) / s;
            const bool mine = gi % (int)gridDim.y == (int)blockIdx.y;
            pre[gi + 1] = pre[gi] + (mine ? max((int64_t)0, (wend + s - 1) / s - first[gi]) : 0);
        }
    }
    __syncthreads();
    // M_L of word w (bit k <-> position 32w + k), from the tile
    auto eqL = [&](int64_t w, int64_t L) -> uint32_t {
        const int64_t lim = n - L - w * 32;   // positions 32w + k valid iff k < lim
        if (w < 0 || lim <= 0) return 0u;
        const int64_t q = w + (L >> 5) - base;
        const uint32_t r = (uint32_t)(L & 31);
        const int64_t a = (w - base) * B;
        uint32_t x = 0;
#pragma unroll
        for (int p = 0; p < B; ++p) x |= tl[a + p] ^ __builtin_amdgcn_alignbit(tl[(q + 1) * B + p], tl[q * B + p], r);
        uint32_t m = ~x;
        if (lim < 32) m &= (1u << lim) - 1u;
        return m;
    };
    const int lane = threadIdx.x & 63;
    const int seg = (int)((blockIdx.x * gridDim.y + blockIdx.y) & (kCandSegs - 1));
    const int64_t total = pre[sg.ng];
    for (int64_t f0 = 0; f0 < total; f0 += 256) {   // uniform
        const int64_t f = f0 + threadIdx.x;
        const bool live = f < total;
        int gi = 0;
        while (gi + 1 < sg.ng && f >= pre[gi + 1]) ++gi;
        const int64_t s = sg.s[gi];
        const int64_t w = live ? (first[gi] + (f - pre[gi])) * s : w0;
        const int64_t g = sg.g[gi], Lg = g * 32;
        // every L of the group compares word w with words w+g, w+g+1: three words
        // per plane from the tile, once per sample
        uint32_t a[B], lo[B], hi[B];
#pragma unroll
        for (int p = 0; p < B; ++p) {
            a[p] = tl[(w - base) * B + p];
            lo[p] = tl[(w + g - base) * B + p];
            hi[p] = tl[(w + g + 1 - base) * B + p];
        }
        for (int r = 0; r < 32; ++r) {   // uniform
            const int64_t L = Lg + r;
            const bool ok = live && L >= lmin && L <= lmax;
            uint32_t M = 0u;
            if (ok) {
                uint32_t x = 0;
#pragma unroll
                for (int p = 0; p < B; ++p) x |= a[p] ^ __builtin_amdgcn_alignbit(hi[p], lo[p], (uint32_t)r);
                M = ~x;
                const int64_t lim = n - L - w * 32;
                if (lim <= 0) M = 0u;
                else if (lim < 32) M &= (1u << lim) - 1u;
            }
            // owner test: the first non-full word among w-1 .. w-s gives the
            // run's start (all full: the previous sample owns the run)
            int64_t start = -1;
            if (__any(M == FULL) && M == FULL) {
                for (int64_t k0 = 1; k0 <= s && start < 0; k0 += 8) {
                    uint32_t Mq[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) Mq[i] = k0 + i <= s ? eqL(w - (k0 + i), L) : FULL;
#pragma unroll
                    for (int i = 0; i < 8; ++i)
                        if (start < 0 && Mq[i] != FULL) start = (w - (k0 + i) + 1) * 32 - (int64_t)__clz(~Mq[i]);
                }
            }
            uint64_t own = __ballot(start >= 0);   // uniform
            while (own) {
                const int src = __ffsll((unsigned long long)own) - 1;
                own &= own - 1;
                const int64_t ws = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)w, src)) |
                                   ((int64_t)__builtin_amdgcn_readlane((int)(w >> 32), src) << 32);
                const int64_t st = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)start, src)) |
                                   ((int64_t)__builtin_amdgcn_readlane((int)(start >> 32), src) << 32);
                const int64_t Lo = ((int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)L, src));
                const int64_t Ko = (mc - 1) * Lo;
                // end: the first non-full word after ws -- one 64-word step here
                // (global: it may leave the tile), a longer streak is ended by k_streak_end
                const int64_t q0 = ws + 1;
                const uint32_t Mq = eq32<B>(P, q0 + lane, Lo, n);   // 0 past the text: ends the scan
                const uint64_t nb = __ballot(Mq != FULL);
                if (!nb) {
                    if (lane == 0) push_pending(out, Lo, st, q0 + 64);
                    continue;
                }
                const int fb = __ffsll((unsigned long long)nb) - 1;
                const uint32_t Mf = (uint32_t)__builtin_amdgcn_readlane((int)Mq, fb);
                const int64_t end = (q0 + fb) * 32 + (int64_t)__ffs(~Mf) - 1;
                if (end - st >= Ko && lane == 0) {
                    const unsigned long long at = atomicAdd(out.count + seg, 1ull);
                    put(out, seg, at, Lo, st, end);
                }
            }
        }
    }
}

// End search of the deferred streaks, one wave per streak (grid-stride over
// the list; every wave leaves when the list is exhausted): 8 x 64 words per
// step, their loads issued before any ballot.  A candidate is put when the
// run is long enough (e - s >= K), exactly as the kernel that found it would.
constexpr int kWide = 8;
template <int B>
__global__ __launch_bounds__(256) void k_streak_end(const uint32_t *__restrict__ P, int64_t n, int64_t mc,
                                                    CandOut out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t np = min((int64_t)*out.npend, out.pend_cap);
    for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < np; e += nw) {   // uniform
        const int64_t L = out.pend[3 * e], st = out.pend[3 * e + 1];
        int64_t end = -1;
        for (int64_t q0 = out.pend[3 * e + 2]; end < 0; q0 += 64 * kWide) {
            uint32_t Mq[kWide];
#pragma unroll
            for (int i = 0; i < kWide; ++i) Mq[i] = eq32<B>(P, q0 + 64 * i + lane, L, n);   // 0 past the text
#pragma unroll
            for (int i = 0; i < kWide; ++i) {
                const uint64_t nb = __ballot(Mq[i] != FULL);
                if (end < 0 && nb) {
                    const int f = __ffsll((unsigned long long)nb) - 1;
                    const uint32_t Mf = (uint32_t)__builtin_amdgcn_readlane((int)Mq[i], f);
                    end = (q0 + 64 * i + f) * 32 + (int64_t)__ffs(~Mf) - 1;
                }
            }
        }
        if (end - st >= (mc - 1) * L && lane == 0) {
            const int seg = (int)(e & (kCandSegs - 1));
            const unsigned long long at = atomicAdd(out.count + seg, 1ull);
            put(out, seg, at, L, st, end);
        }
    }
}

// first group (of 32 unit lengths) whose runs are found by sampling: K >= 95 for its shortest L
inline int64_t sparse_stride(int64_t g, int32_t lmin, int64_t mc) {
    const int64_t L = std::max<int64_t>(g * 32, lmin), K = (mc - 1) * L;
    return K >= 95 ? (K - 31) / 32 : 0;
}

template <int B>
void launch_runs(Ctx &c, const uint32_t *P, int64_t n, int32_t lmin, int32_t lmax, int64_t mc, CandOut out) {
    const int64_t nwords32 = (n + 31) / 32;
    const bool dense_only = knob(KN_RUNS_DENSE) != 0;   // A/B and parity cross-check: every group dense
    int64_t gs = std::max<int64_t>(1, lmin >> 5);   // group 0 (L < 32) stays dense: its short runs
    while (!dense_only && gs <= (lmax >> 5) && sparse_stride(gs, lmin, mc) < 2) ++gs;
    if (dense_only) gs = (lmax >> 5) + 1;
    const int32_t lmax_dense = (int32_t)std::min<int64_t>(lmax, gs * 32 - 1);
    if (lmin <= lmax_dense) {
        const int64_t tiles = (nwords32 + 4 * kOwn - 1) / (4 * kOwn);
        const int64_t groups = (int64_t)(lmax_dense >> 5) - (int64_t)(lmin >> 5) + 1;
        const int32_t gper = 8;   // unit-length groups per workgroup (32 L each)
        const int64_t gblocks = (groups + gper - 1) / gper;
        KLAUNCH("k_runs", 0.0, (k_runs<B>), dim3((unsigned)tiles, (unsigned)gblocks), dim3(256), 0, c.stream, P, n,
                nwords32, lmin, lmax_dense, mc, gper, out);
    }
    for (int64_t g0 = gs; g0 <= (lmax >> 5); g0 += kSparseMax) {
        SparseGroups sg{};
        sg.ng = 0;
        for (int64_t g = g0; g <= (lmax >> 5) && sg.ng < kSparseMax; ++g) {
            const int64_t s = sparse_stride(g, lmin, mc);
            sg.g[sg.ng] = (int32_t)g;
            sg.s[sg.ng] = (int32_t)s;
            const int64_t samples = (nwords32 + s - 1) / s;
            sg.woff[sg.ng + 1] = sg.woff[sg.ng] + (samples + 63) / 64;
            ++sg.ng;
        }
        const int64_t waves = sg.woff[sg.ng];
        if (waves == 0) continue;
        // the tile's halo: the largest stride before it (owner tests), the
        // largest group + 2 words after it (words w + g and w + g + 1 of its last sample)
        int32_t halo = 0, after = 0;
        for (int gi = 0; gi < sg.ng; ++gi) {
            halo = std::max(halo, sg.s[gi]);
            after = std::max(after, sg.g[gi] + 2);
        }
        const bool untiled = knob(KN_RUNS_UNTILED) != 0;
        constexpr int T = run_tile<B>();
        const size_t lds = (size_t)(halo + T + after) * B * 4;
        if (!untiled && halo <= 256 && lds <= 64 * 1024) {   // LDS tiles (BWTMI_RUNS_UNTILED=1: the scattered-sample kernel)
            KLAUNCH("k_runs_sparse", 0.0, (k_runs_tiled<B>),
                    dim3((unsigned)((nwords32 + T - 1) / T), (unsigned)std::min(kRunGroupSplit, sg.ng)), dim3(256), lds,
                    c.stream, P, n, nwords32, lmin, lmax, mc, sg, halo, after, out);
        } else {
            KLAUNCH("k_runs_sparse", 0.0, (k_runs_sparse<B>), dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, c.stream,
                    P, n, nwords32, lmin, lmax, mc, sg, out);
        }
    }
    KLAUNCH("k_streak_end", 0.0, (k_streak_end<B>), dim3(512), dim3(256), 0, c.stream, P, n, mc, out);
}

}  // namespace

// max_mismatch > 0 (library calls; the CLI passes 0, bwt.py:3105): hits in the
// reference's emission order, prim_len / copies as bwt.py:1956-1961
void strict_scan_mm_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t min_unit, int32_t max_unit,
                           int32_t max_mismatch, int32_t min_copies, HitVec &hits) {
    hits.clear();
    if (min_copies <= 0) fail(BWTMI_E_ARG, "min_copies must be positive");
    const int64_t maxL = std::min<int64_t>(max_unit, n / min_copies);   // bwt.py:1920
    if (n <= 0 || maxL < min_unit || maxL < 1) return;
    const int64_t lmin = std::max<int32_t>(1, min_unit), lmax = maxL;
    hipStream_t st = c.stream;
    const int64_t nw = (n + 31) / 32;
    // rows per batch: P bits (nw + 1 words per row) and the (start, count) slots
    // of the row (at most n / (mc L) + 1 hits: a row's hits are disjoint)
    const int64_t budget = int64_t{1} << 30;
    std::vector<int64_t> np;
    for (int64_t L0 = lmax; L0 >= lmin;) {
        int64_t rows = 0, slots = 0;
        std::vector<int64_t> off;
        while (L0 - rows >= lmin && rows < 65535) {   // rows are gridDim.y of k_mm_pbits
            const int64_t cap = n / (min_copies * (L0 - rows)) + 1;
            if (rows && (rows + 1) * (nw + 1) * 4 + (slots + cap) * 16 > budget) break;
            off.push_back(slots);
            slots += cap;
            ++rows;
        }
        c.slot[S_PACK].ensure((size_t)rows * (nw + 1) * 4);
        c.slot[S_MISC0].ensure((size_t)slots * 16);
        c.slot[S_MISC1].ensure((size_t)rows * 8);
        c.slot[S_MISC2].ensure((size_t)rows * 8);
        uint32_t *P = c.slot[S_PACK].as<uint32_t>();
        HIPCHECK(hipMemsetAsync(P, 0, (size_t)rows * (nw + 1) * 4, st));
        HIPCHECK(hipMemcpyAsync(c.slot[S_MISC1].p, off.data(), (size_t)rows * 8, hipMemcpyHostToDevice, st));
        const int64_t segs = (n + kMmSeg - 1) / kMmSeg;
        KLAUNCH("k_mm_pbits", 0.0, k_mm_pbits, dim3((unsigned)((segs + 255) / 256), (unsigned)rows), dim3(256), 0, st,
                d_text, n, (int32_t)L0, max_mismatch, nw, P);
        KLAUNCH("k_mm_walk", 0.0, k_mm_walk, dim3((unsigned)rows), dim3(64), 0, st, P, n, nw, (int32_t)L0, min_copies,
                c.slot[S_MISC1].as<int64_t>(), c.slot[S_MISC0].as<int64_t>(), c.slot[S_MISC2].as<int64_t>());
        HIPCHECK(hipGetLastError());
        std::vector<int64_t> cnt((size_t)rows), sc((size_t)slots * 2);
        HIPCHECK(hipMemcpyAsync(cnt.data(), c.slot[S_MISC2].p, (size_t)rows * 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(sc.data(), c.slot[S_MISC0].p, (size_t)slots * 16, hipMemcpyDeviceToHost, st));
        scan_wait(st);
        for (int64_t r = 0; r < rows; ++r) {
            const int64_t L = L0 - r;
            for (int64_t k = 0; k < cnt[(size_t)r]; ++k) {
                const int64_t i = sc[(size_t)(2 * (off[(size_t)r] + k))], cc = sc[(size_t)(2 * (off[(size_t)r] + k) + 1)];
                hits.push_back(bwtmi_hit{i, i + cc * L, (int32_t)L, 0, cc});
            }
        }
        L0 -= rows;
    }
    const int64_t nh = (int64_t)hits.size();
    if (!nh) return;
    c.slot[S_HITS].ensure((size_t)nh * sizeof(bwtmi_hit));
    HIPCHECK(hipMemcpyAsync(c.slot[S_HITS].p, hits.data(), (size_t)nh * sizeof(bwtmi_hit), hipMemcpyHostToDevice, st));
    KLAUNCH("k_period", 0.0, k_period, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, d_text,
            c.slot[S_HITS].as<bwtmi_hit>(), nh);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(hits.data(), c.slot[S_HITS].p, (size_t)nh * sizeof(bwtmi_hit), hipMemcpyDeviceToHost, st));
    scan_wait(st);
}

void strict_scan_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t min_unit, int32_t max_unit,
                        int32_t min_copies, ScanResult &res, bool screen, int32_t drop_min_copies) {
    res.hits.clear();
    res.shits.clear();
    res.candidates = 0;
    res.kernel_ms = 0;
    res.raw = 0;
    res.screened = screen;
    if (min_copies <= 0) fail(BWTMI_E_ARG, "min_copies must be positive");
    // bwt.py:1920-1921
    const int64_t maxL = std::min<int64_t>(max_unit, n / min_copies);
    if (n <= 0 || maxL < min_unit || maxL < 1) return;
    const int32_t lmin = std::max<int32_t>(1, min_unit), lmax = (int32_t)maxL;
    hipStream_t st = c.stream;
    if (c.timing) HIPCHECK(hipEventRecord(c.ev0, st));

    if (min_copies == 1) {   // degenerate but reachable from --min-copies 1
        const int64_t nL = lmax - lmin + 1;
        std::vector<int64_t> off((size_t)nL + 1, 0);
        for (int64_t row = 0; row < nL; ++row) off[(size_t)row + 1] = off[(size_t)row] + n / (lmax - row) + 1;
        const int64_t tot = off[(size_t)nL];
        c.slot[S_MISC0].ensure((size_t)(nL + 1) * sizeof(int64_t));
        c.slot[S_MISC1].ensure((size_t)tot * sizeof(bwtmi_hit));
        c.slot[S_MISC2].ensure((size_t)nL * sizeof(int64_t));
        HIPCHECK(hipMemcpyAsync(c.slot[S_MISC0].p, off.data(), off.size() * 8, hipMemcpyHostToDevice, st));
        KLAUNCH("k_mc1", 0.0, k_mc1, dim3((unsigned)((nL + 63) / 64)), dim3(64), 0, st, d_text, n, lmin, lmax,
                           c.slot[S_MISC0].as<int64_t>(), c.slot[S_MISC1].as<bwtmi_hit>(),
                           c.slot[S_MISC2].as<int64_t>());
        HIPCHECK(hipGetLastError());
        std::vector<int64_t> np((size_t)nL);
        HIPCHECK(hipMemcpyAsync(np.data(), c.slot[S_MISC2].p, np.size() * 8, hipMemcpyDeviceToHost, st));
        scan_wait(st);
        int64_t nh = 0;
        for (auto v : np) nh += v;
        c.slot[S_HITS].ensure((size_t)std::max<int64_t>(nh, 1) * sizeof(bwtmi_hit));
        int64_t w = 0;
        for (int64_t row = 0; row < nL; ++row) {   // rows are already in (L desc, start asc) order
            if (np[(size_t)row])
                HIPCHECK(hipMemcpyAsync(c.slot[S_HITS].as<bwtmi_hit>() + w,
                                        c.slot[S_MISC1].as<bwtmi_hit>() + off[(size_t)row],
                                        (size_t)np[(size_t)row] * sizeof(bwtmi_hit), hipMemcpyDeviceToDevice, st));
            w += np[(size_t)row];
        }
        if (nh > 0)
            KLAUNCH("k_period", 0.0, k_period, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, d_text,
                               c.slot[S_HITS].as<bwtmi_hit>(), nh);
        HIPCHECK(hipGetLastError());
        res.raw = nh;
        if (screen) {
            screen_hits_device(c, c.slot[S_HITS].as<bwtmi_hit>(), nh, n, lmax, res.shits, -1, drop_min_copies);
            c.kresolve();
            return;
        }
        res.hits.resize((size_t)nh);
        if (nh > 0)
            HIPCHECK(hipMemcpyAsync(res.hits.data(), c.slot[S_HITS].p, (size_t)nh * sizeof(bwtmi_hit),
                                    hipMemcpyDeviceToHost, st));
        scan_wait(st);
        return;
    }

    // 1. alphabet -> code width
    c.slot[S_COUNTS].ensure(256 * sizeof(unsigned long long));
    HIPCHECK(hipMemsetAsync(c.slot[S_COUNTS].p, 0, 256 * sizeof(unsigned long long), st));
    KLAUNCH("k_present", (double)n, k_present, dim3(1024), dim3(256), 0, st, d_text, n,
            c.slot[S_COUNTS].as<unsigned long long>());
    // the small host reads below go through the pinned mailbox, one wait per step
    unsigned long long *mb = c.mailbox<unsigned long long>(kCandSegs + 8);
    unsigned long long present[4];
    HIPCHECK(hipMemcpyAsync(mb, c.slot[S_COUNTS].p, sizeof present, hipMemcpyDeviceToHost, st));
    scan_wait(st);
    std::memcpy(present, mb, sizeof present);
    uint8_t code[256] = {0};
    int sigma = 0;
    for (int b = 0; b < 256; ++b)
        if ((present[b >> 6] >> (b & 63)) & 1ull) code[b] = (uint8_t)sigma++;
    const int B = sigma <= 2 ? 1 : (sigma <= 4 ? 2 : (sigma <= 16 ? 4 : 8));
    const int64_t nwords = (n + 31) / 32 + 8;   // + padding read by the window of the last words
    int sb = 1;   // candidate keys hold starts < n in their low sb bits
    while (sb < 63 && (1ll << sb) < n) ++sb;
    c.slot[S_PACK].ensure((size_t)nwords * B * sizeof(uint32_t) + 256);
    uint8_t *d_code = c.slot[S_PACK].as<uint8_t>() + nwords * B * sizeof(uint32_t);
    HIPCHECK(hipMemcpyAsync(d_code, code, 256, hipMemcpyHostToDevice, st));
    uint32_t *P = c.slot[S_PACK].as<uint32_t>();
    HIPCHECK(hipMemsetAsync(P, 0, (size_t)nwords * B * sizeof(uint32_t), st));
    const unsigned pgrid = (unsigned)((nwords + 255) / 256);
    if (B == 1) KLAUNCH("k_pack", 0.0, k_pack<1>, dim3(pgrid), dim3(256), 0, st, d_text, n, d_code, P, nwords - 8);
    else if (B == 2) KLAUNCH("k_pack", 0.0, k_pack<2>, dim3(pgrid), dim3(256), 0, st, d_text, n, d_code, P, nwords - 8);
    else if (B == 4) KLAUNCH("k_pack", 0.0, k_pack<4>, dim3(pgrid), dim3(256), 0, st, d_text, n, d_code, P, nwords - 8);
    else KLAUNCH("k_pack", 0.0, k_pack<8>, dim3(pgrid), dim3(256), 0, st, d_text, n, d_code, P, nwords - 8);
    HIPCHECK(hipGetLastError());

    // 2. candidate runs (segmented output, compacted below)
    int64_t seg_cap = std::max<int64_t>(1 << 12, n / 8 / kCandSegs + 1024);
    unsigned long long segn[kCandSegs] = {0};
    unsigned long long ncand = 0;
    c.slot[S_MISC3].ensure(kCandSegs * (sizeof(unsigned long long) + sizeof(int64_t)) + 64);
    unsigned long long *d_count = c.slot[S_MISC3].as<unsigned long long>();
    int64_t *d_off = reinterpret_cast<int64_t *>(d_count + kCandSegs);
    // deferred streak ends: the counter sits after the segment counts (both reset per attempt)
    unsigned long long *d_npend = reinterpret_cast<unsigned long long *>(d_count + kCandSegs + kCandSegs + 2);
    int64_t pend_cap = 1 << 16;
    for (int attempt = 0;; ++attempt) {
        c.slot[S_CAND_K2].ensure((size_t)(seg_cap * kCandSegs) * sizeof(uint64_t));
        c.slot[S_CAND_V2].ensure((size_t)(seg_cap * kCandSegs) * sizeof(uint64_t));
        c.slot[S_MISC2].ensure((size_t)pend_cap * 3 * sizeof(int64_t));
        HIPCHECK(hipMemsetAsync(d_count, 0, kCandSegs * sizeof(unsigned long long), st));
        HIPCHECK(hipMemsetAsync(d_npend, 0, sizeof(unsigned long long), st));
        CandOut co{c.slot[S_CAND_K2].as<uint64_t>(), c.slot[S_CAND_V2].as<uint64_t>(), d_count, seg_cap, lmax, sb,
                   c.slot[S_MISC2].as<int64_t>(), d_npend, pend_cap};
        hipEvent_t ka = nullptr, kb = nullptr;
        if (c.timing) {
            HIPCHECK(hipEventCreate(&ka));
            HIPCHECK(hipEventCreate(&kb));
            HIPCHECK(hipEventRecord(ka, st));
        }
        if (B == 1) launch_runs<1>(c, P, n, lmin, lmax, min_copies, co);
        else if (B == 2) launch_runs<2>(c, P, n, lmin, lmax, min_copies, co);
        else if (B == 4) launch_runs<4>(c, P, n, lmin, lmax, min_copies, co);
        else launch_runs<8>(c, P, n, lmin, lmax, min_copies, co);
        HIPCHECK(hipGetLastError());
        if (c.timing) HIPCHECK(hipEventRecord(kb, st));
        HIPCHECK(hipMemcpyAsync(mb, d_count, sizeof segn, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(mb + kCandSegs, d_npend, 8, hipMemcpyDeviceToHost, st));
        scan_wait(st);
        std::memcpy(segn, mb, sizeof segn);
        const unsigned long long npend = mb[kCandSegs];
        if (c.timing) {
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, ka, kb));
            c.last_dom_ms = ms;
            c.last_dom_launches = 1;
            c.dom_name = "k_runs";
            res.kernel_ms = ms;
            (void)hipEventDestroy(ka);
            (void)hipEventDestroy(kb);
        }
        unsigned long long mx = 0;
        ncand = 0;
        for (int q = 0; q < kCandSegs; ++q) {
            ncand += segn[q];
            mx = std::max(mx, segn[q]);
        }
        if ((int64_t)mx <= seg_cap && (int64_t)npend <= pend_cap) break;
        if (attempt >= 2) fail(BWTMI_E_STATE, "strict scan: candidate segments overflow after %d attempts", attempt + 1);
        if ((int64_t)mx > seg_cap) seg_cap = (int64_t)mx + (int64_t)mx / 4 + 1024;   // exact counts: the next attempt fits
        // (lost streaks were not counted as candidates: the next attempt may find more)
        if ((int64_t)npend > pend_cap) pend_cap = (int64_t)npend + (int64_t)npend / 4 + 1024;
        else if ((int64_t)npend > pend_cap / 2) pend_cap *= 2;
    }
    if (ncand > 0) {
        int64_t off[kCandSegs];
        unsigned long long mx = 0;
        for (int q = 0; q < kCandSegs; ++q) {
            off[q] = q ? off[q - 1] + (int64_t)segn[q - 1] : 0;
            mx = std::max(mx, segn[q]);
        }
        c.slot[S_CAND_K].ensure((size_t)ncand * sizeof(uint64_t));
        c.slot[S_CAND_V].ensure((size_t)ncand * sizeof(uint64_t));
        HIPCHECK(hipMemcpyAsync(d_off, off, sizeof off, hipMemcpyHostToDevice, st));
        KLAUNCH("k_cand_gather", 0.0, k_cand_gather, dim3((unsigned)((mx + 255) / 256), kCandSegs), dim3(256), 0, st,
                           c.slot[S_CAND_K2].as<uint64_t>(), c.slot[S_CAND_V2].as<uint64_t>(), d_count, d_off,
                           seg_cap, c.slot[S_CAND_K].as<uint64_t>(), c.slot[S_CAND_V].as<uint64_t>());
        HIPCHECK(hipGetLastError());
    }
    const int64_t nc = (int64_t)ncand;
    res.candidates = nc;
    if (nc == 0) return;

    // 3. order candidates as the reference emits them: L desc, start asc
    int hb = 0;
    while ((1ll << hb) <= (int64_t)lmax) ++hb;
    radix_sort_pairs(c, c.slot[S_CAND_K].as<uint64_t>(), c.slot[S_CAND_V].as<uint64_t>(), nc, 0,
                     ((sb + hb + 7) / 8) * 8);

    // 4. carry resolution + compaction
    c.slot[S_MISC0].ensure((size_t)nc * sizeof(int64_t));
    c.slot[S_MISC1].ensure((size_t)nc * sizeof(int64_t));
    c.slot[S_FLAG].ensure((size_t)nc * sizeof(uint32_t));
    c.slot[S_SCAN].ensure((size_t)(nc + 1) * sizeof(uint32_t));
    const unsigned g = (unsigned)((nc + 255) / 256);
    KLAUNCH("k_resolve", 0.0, k_resolve, dim3(g), dim3(256), 0, st, c.slot[S_CAND_K].as<uint64_t>(),
                       c.slot[S_CAND_V].as<uint64_t>(), nc, lmax, sb, (int64_t)min_copies, c.slot[S_MISC0].as<int64_t>(),
                       c.slot[S_MISC1].as<int64_t>(), c.slot[S_FLAG].as<uint32_t>());
    HIPCHECK(hipMemsetAsync(c.slot[S_SCAN].as<uint32_t>() + nc, 0, sizeof(uint32_t), st));
    exclusive_scan<uint32_t>(c, c.slot[S_FLAG].as<uint32_t>(), c.slot[S_SCAN].as<uint32_t>(), nc);
    int64_t *d_nlong = d_off + kCandSegs;   // after the segment offsets
    KLAUNCH("k_count_long", 0.0, k_count_long, dim3(1), dim3(64), 0, st, c.slot[S_CAND_K].as<uint64_t>(), nc, lmax,
            sb, kThreadPeriodL, d_nlong);
    // hits are a subset of the candidates: the compaction and the long units'
    // periods run before the host learns the hit count, which it reads with the
    // longest span in one wait
    c.slot[S_HITS].ensure((size_t)nc * sizeof(bwtmi_hit));
    unsigned long long *d_maxlen = d_npend + 1;   // the hits' longest span, reduced by k_compact
    HIPCHECK(hipMemsetAsync(d_maxlen, 0, 8, st));
    KLAUNCH("k_compact", 0.0, k_compact, dim3(g), dim3(256), 0, st, c.slot[S_CAND_K].as<uint64_t>(), nc, lmax, sb,
                       c.slot[S_MISC0].as<int64_t>(), c.slot[S_MISC1].as<int64_t>(), c.slot[S_FLAG].as<uint32_t>(),
                       c.slot[S_SCAN].as<uint32_t>(), d_text, c.slot[S_HITS].as<bwtmi_hit>(), d_maxlen);
    KLAUNCH("k_period_wave", 0.0, k_period_wave, dim3((unsigned)std::min<int64_t>(2048, (nc * 64 + 255) / 256)),
            dim3(256), 0, st, c.slot[S_CAND_K].as<uint64_t>(), d_nlong, lmax, sb, c.slot[S_MISC0].as<int64_t>(),
            c.slot[S_MISC1].as<int64_t>(), c.slot[S_FLAG].as<uint32_t>(), c.slot[S_SCAN].as<uint32_t>(), d_text,
            c.slot[S_HITS].as<bwtmi_hit>());
    HIPCHECK(hipGetLastError());
    uint32_t *mb32 = reinterpret_cast<uint32_t *>(mb);
    HIPCHECK(hipMemcpyAsync(mb32, c.slot[S_SCAN].as<uint32_t>() + nc - 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(mb32 + 1, c.slot[S_FLAG].as<uint32_t>() + nc - 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(mb + 1, d_maxlen, 8, hipMemcpyDeviceToHost, st));
    scan_wait(st);
    c.checks_verify("the strict scan's hit count");
    const int64_t nh = (int64_t)mb32[0] + mb32[1];
    const int64_t maxlen = (int64_t)mb[1];
    res.raw = nh;
    if (screen) {
        // records c.ev1 behind its kernels; its hits download may still be landing
        // (res.shits.wait), every kernel has finished
        screen_hits_device(c, c.slot[S_HITS].as<bwtmi_hit>(), nh, n, lmax, res.shits, maxlen, drop_min_copies);
        if (c.timing && !res.shits.landing) HIPCHECK(hipEventRecord(c.ev1, st));
        if (!res.shits.landing) scan_wait(st);
        else if (c.timing) while (hipEventQuery(c.ev1) == hipErrorNotReady) __builtin_ia32_pause();
    } else {
        if (c.timing) HIPCHECK(hipEventRecord(c.ev1, st));
        res.hits.resize((size_t)nh);
        if (nh > 0)
            HIPCHECK(hipMemcpyAsync(res.hits.data(), c.slot[S_HITS].p, (size_t)nh * sizeof(bwtmi_hit),
                                    hipMemcpyDeviceToHost, st));
        scan_wait(st);
    }
    c.kresolve();
    if (c.timing) {
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        c.last_total_ms = ms;
    }
}

}  // namespace bwtmi
