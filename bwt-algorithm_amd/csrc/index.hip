// index.hip -- FM-index construction on gfx950 (replaces BWTCore.__init__,
// bwt.py:106-136) plus the library queries built on it.
//
// Suffix array (bwt.py:212-264).  The reference sorts suffixes of seq+'$' by
// byte value with "end of text" smallest; '$' unique makes the order total.
// Here: prefix doubling over radix sorts.
//   round 0  key = k symbols of b bits (b = bits for sigma+1 codes, code 0 =
//            past the end, k = 64/b; ACGT$ -> 21 symbols), one 64-bit radix sort
//   round r  only suffixes in groups of size >= 2 survive; each gets the key
//            (group start, rank[i+h] + 1) -- sorted with one radix sort whose
//            digit range covers exactly those bits -- and its group is split;
//            singletons are dropped (h doubles each round)
// BWT/C/Occ/sampled SA are single streaming kernels; the 8-mer hash is a
// stable 16-bit radix sort of (window code, position) pairs; LCP is chunked
// Kasai; backward search runs one pattern per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "device.h"

namespace bwtmi {

struct DeviceIndex {
    int64_t n = 0;
    int32_t sa_sample = 32, occ_sample = 128;
    int sigma = 0;
    uint8_t code_of[256];        // byte -> occ row (valid when totals > 0)
    int64_t totals[256], C[256];
    DBuf text;                   // copy of the text (n + pad)
    DBuf sa;                     // int32[n]
    DBuf bwt;                    // uint8[n + pad]
    DBuf occ;                    // int32[sigma][occ_len]
    DBuf sampled;                // int32[ceil(n/s)]
    DBuf kmer_off;               // int64[65537]
    DBuf kmer_pos;               // int32[count]
    int64_t kmer_count = 0;
    bool has_kmer = false;
    int64_t occ_len = 0, sampled_len = 0;
    // ACGT* '$' texts: packed rank structure, one 32-byte block per 64 BWT rows:
    // uint32 count[4] of A C G T before the block, then the rows' 2-bit codes
    // as two bit planes (row 64b + k at bit k; '$' stored as A, dollar_row)
    DBuf fm2;
    bool has_fm2 = false;
    int64_t dollar_row = -1;
};

namespace {

__global__ void k_hist_bytes(const uint8_t *__restrict__ t, int64_t n, unsigned long long *__restrict__ h) {
    __shared__ unsigned int lh[256];
    lh[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&lh[t[i]], 1u);
    __syncthreads();
    if (lh[threadIdx.x]) atomicAdd(&h[threadIdx.x], (unsigned long long)lh[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_init_keys(const uint8_t *__restrict__ t, int64_t n,
                                                   const uint8_t *__restrict__ code, int b, int k,
                                                   uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    __shared__ uint8_t cm[256];
    cm[threadIdx.x] = code[threadIdx.x];
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t key = 0;
    for (int q = 0; q < k; ++q) {
        const uint64_t c = (i + q < n) ? cm[t[i + q]] : 0u;
        key = (key << b) | c;
    }
    keys[i] = key;
    vals[i] = (uint32_t)i;
}

// head flag of sorted position r (key differs from r-1)
__global__ __launch_bounds__(256) void k_heads(const uint64_t *__restrict__ keys, int64_t m, uint32_t *__restrict__ head) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    head[r] = (r == 0 || keys[r] != keys[r - 1]) ? 1u : 0u;
}

// after round 0: SA = vals; rank[SA[r]] = start of r's group; flag[r] = group size >= 2
__global__ __launch_bounds__(256) void k_rank0(const uint32_t *__restrict__ head, const uint32_t *__restrict__ gid,
                                               const uint32_t *__restrict__ sa, int64_t m,
                                               uint32_t *__restrict__ gstart, uint32_t *__restrict__ rank,
                                               uint32_t *__restrict__ flag, int pass) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    if (pass == 0) {
        if (head[r]) gstart[gid[r]] = (uint32_t)r;
        return;
    }
    const uint32_t g = gid[r];
    rank[sa[r]] = gstart[g];
    const bool single = head[r] && (r + 1 == m || head[r + 1]);
    flag[r] = single ? 0u : 1u;
}

// compaction of flagged indices (ascending)
__global__ __launch_bounds__(256) void k_compact_idx(const uint32_t *__restrict__ flag, const uint32_t *__restrict__ pos,
                                                     int64_t m, uint32_t *__restrict__ out, const uint32_t *__restrict__ src) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m || !flag[r]) return;
    out[pos[r]] = src ? src[r] : (uint32_t)r;
}

// keys for the surviving suffixes: (group start << nb) | (rank[i+h] + 1 or 0)
__global__ __launch_bounds__(256) void k_round_keys(const uint32_t *__restrict__ U, int64_t m, const uint32_t *__restrict__ sa,
                                                    const uint32_t *__restrict__ rank, int64_t n, int64_t h, int nb,
                                                    uint64_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= m) return;
    const uint32_t i = sa[U[u]];
    const uint64_t g = rank[i];
    const uint64_t r2 = ((int64_t)i + h < n) ? (uint64_t)rank[i + h] + 1u : 0u;
    keys[u] = (g << nb) | r2;
    vals[u] = i;
}

// write back: SA[U[u]] = vals[u]; group starts at heads
__global__ __launch_bounds__(256) void k_round_apply(const uint32_t *__restrict__ U, int64_t m, const uint32_t *__restrict__ vals,
                                                     const uint32_t *__restrict__ head, const uint32_t *__restrict__ gid,
                                                     uint32_t *__restrict__ sa, uint32_t *__restrict__ gstart, int pass,
                                                     uint32_t *__restrict__ rank, uint32_t *__restrict__ flag) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= m) return;
    if (pass == 0) {
        sa[U[u]] = vals[u];
        if (head[u]) gstart[gid[u]] = U[u];
        return;
    }
    rank[vals[u]] = gstart[gid[u]];
    const bool single = head[u] && (u + 1 == m || head[u + 1]);
    flag[u] = single ? 0u : 1u;
}

__global__ void k_gid(const uint32_t *__restrict__ head_scan_excl, const uint32_t *__restrict__ head, int64_t m,
                      uint32_t *__restrict__ gid) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= m) return;
    gid[r] = head_scan_excl[r] + head[r] - 1u;
}

__global__ __launch_bounds__(256) void k_bwt(const uint8_t *__restrict__ t, const uint32_t *__restrict__ sa, int64_t n,
                                             uint8_t *__restrict__ bwt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int64_t p = (int64_t)sa[r] - 1;
    bwt[r] = t[p < 0 ? p + n : p];
}

// zero bytes of y, exactly (no carries between bytes)
__device__ __forceinline__ uint32_t zero_bytes(uint64_t y) {
    constexpr uint64_t lo7 = 0x7f7f7f7f7f7f7f7full;
    const uint64_t t = ~(((y & lo7) + lo7) | y | lo7);
    return (uint32_t)__popcll(t);
}

// per occ_sample-byte block counts of each present code: one thread per block,
// 16-byte loads, SWAR byte compares + popcount (the BWT buffer is padded)
__global__ __launch_bounds__(256) void k_occ_blocks(const uint8_t *__restrict__ bwt, int64_t n, int64_t nblk, int blk,
                                                    const uint8_t *__restrict__ present, int sigma,
                                                    uint32_t *__restrict__ cnt /* [sigma][nblk+1] */) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    constexpr int kMaxSig = 16;
    uint32_t s[kMaxSig] = {0};
    uint64_t pat[kMaxSig];
    // 16-byte loads need 16-aligned blocks; other sample rates take the byte loop
    const int sg = (blk & 15) ? 0 : (sigma < kMaxSig ? sigma : kMaxSig);
    for (int c = 0; c < sg; ++c) pat[c] = 0x0101010101010101ull * present[c];
    const int64_t base = b * blk;
    for (int o = 0; o < blk && sg; o += 16) {
        const int64_t i = base + o;
        if (i >= n) break;
        const uint4 v = *reinterpret_cast<const uint4 *>(bwt + i);
        uint64_t w0 = ((uint64_t)v.y << 32) | v.x, w1 = ((uint64_t)v.w << 32) | v.z;
        const int64_t left = n - i;   // bytes past n must not count: force them to differ
        uint64_t m0 = ~0ull, m1 = ~0ull;
        if (left < 16) {
            m0 = left >= 8 ? ~0ull : (left <= 0 ? 0ull : (~0ull >> (64 - 8 * left)));
            m1 = left <= 8 ? 0ull : (~0ull >> (64 - 8 * (left - 8)));
        }
        for (int c = 0; c < sg; ++c) {
            // a byte outside the text is made to differ from the pattern
            const uint64_t y0 = (w0 ^ pat[c]) | (~m0 & 0x0101010101010101ull);
            const uint64_t y1 = (w1 ^ pat[c]) | (~m1 & 0x0101010101010101ull);
            s[c] += zero_bytes(y0) + zero_bytes(y1);
        }
    }
    for (int c = 0; c < sg; ++c) cnt[(int64_t)c * (nblk + 1) + b] = s[c];
    for (int c = sg; c < sigma; ++c) {   // alphabets past 16 symbols: byte loop
        uint32_t x = 0;
        for (int o = 0; o < blk && base + o < n; ++o) x += bwt[base + o] == present[c];
        cnt[(int64_t)c * (nblk + 1) + b] = x;
    }
}

// The same counts with G = blk / 16 lanes per block (blk a power of two in
// [16, 1024]): lane j of a group loads bytes [16j, 16j + 16) of its block, so a
// wave's loads are 64 consecutive 16-byte pieces (1 KB, coalesced) instead of
// 64 pieces 128 B apart; the group's counts meet by G-lane shuffles and the
// group's first lane writes them.  SWAR compares as above.
template <int G>
__global__ __launch_bounds__(256) void k_occ_groups(const uint8_t *__restrict__ bwt, int64_t n, int64_t nblk,
                                                    const uint8_t *__restrict__ present, int sigma,
                                                    uint32_t *__restrict__ cnt /* [sigma][nblk+1] */) {
    constexpr int kMaxSig = 16;
    const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t b = gt / G;            // every lane of a group has the same b
    const int64_t i = gt * 16;           // = b * blk + 16 * (lane in group)
    uint64_t w0 = 0, w1 = 0, m0 = 0, m1 = 0;
    if (b < nblk && i < n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(bwt + i);
        w0 = ((uint64_t)v.y << 32) | v.x;
        w1 = ((uint64_t)v.w << 32) | v.z;
        const int64_t left = n - i;   // bytes past n must not count
        m0 = left >= 8 ? ~0ull : (~0ull >> (64 - 8 * left));
        m1 = left >= 16 ? ~0ull : (left <= 8 ? 0ull : (~0ull >> (64 - 8 * (left - 8))));
    }
    const int sg = sigma < kMaxSig ? sigma : kMaxSig;
    for (int c = 0; c < sg; ++c) {
        const uint64_t pat = 0x0101010101010101ull * present[c];
        const uint64_t y0 = (w0 ^ pat) | (~m0 & 0x0101010101010101ull);
        const uint64_t y1 = (w1 ^ pat) | (~m1 & 0x0101010101010101ull);
        uint32_t s = zero_bytes(y0) + zero_bytes(y1);
#pragma unroll
        for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (b < nblk && (gt & (G - 1)) == 0) cnt[(int64_t)c * (nblk + 1) + b] = s;
    }
}

__global__ void k_sample(const uint32_t *__restrict__ sa, int64_t n, int32_t s, int32_t *__restrict__ out, int64_t m) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    out[j] = (int32_t)sa[j * s];
}

// ---- 8-mer hash (bwt.py:138-171)
__device__ __forceinline__ int kbits(uint8_t ch) {
    if (ch >= 'a' && ch <= 'z') ch = (uint8_t)(ch - 32);
    switch (ch) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        case 'N': return 0;
        default: return -1;
    }
}

__global__ void k_kvalid(const uint8_t *__restrict__ t, int64_t n, uint32_t *__restrict__ v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = kbits(t[i]) >= 0 ? 1u : 0u;
}

__global__ void k_kcompact(const uint8_t *__restrict__ t, int64_t n, const uint32_t *__restrict__ vpos,
                           uint8_t *__restrict__ V) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int b = kbits(t[i]);
    if (b >= 0) V[vpos[i]] = (uint8_t)b;
}

// entries in position order: [first window at 0 if all k leading chars valid]
// then every valid i >= k -> (window of the last k valid codes, i-k+1)
// 16-bit codes (k <= 8): 6 bytes per entry written and per radix pass moved
// (64-bit codes: 12), the layout of the ACGT path's k_kmer_dna
__global__ void k_kentries(const uint8_t *__restrict__ t, int64_t n, int k, const uint32_t *__restrict__ vpos,
                           const uint8_t *__restrict__ V, int first, uint16_t *__restrict__ keys,
                           uint32_t *__restrict__ vals, uint32_t vbase_k) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == k - 1 && first) {
        uint32_t w = 0;
        for (int q = 0; q < k; ++q) w = (w << 2) | V[q];
        keys[0] = (uint16_t)w;
        vals[0] = 0;
    }
    if (i < k || kbits(t[i]) < 0) return;
    const int64_t v = vpos[i];
    uint32_t w = 0;
    for (int q = k - 1; q >= 0; --q) {
        const int64_t x = v - q;
        w = (w << 2) | (x >= 0 ? V[x] : 0u);
    }
    const int64_t e = (int64_t)first + (v - vbase_k);
    keys[e] = (uint16_t)w;
    vals[e] = (uint32_t)(i - k + 1);
}

// ACGT* '$' texts: every 8-mer that ends before the '$' is an entry, in
// position order (p = 0 .. n-9), so the entries need no compaction; codes
// A0 C1 G2 T3 as kbits.  Four positions per thread from one 12-byte window.
__global__ __launch_bounds__(256) void k_kmer_dna(const uint8_t *__restrict__ t, int64_t n,
                                                  uint16_t *__restrict__ keys, uint32_t *__restrict__ pos) {
    const int64_t p0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int64_t m = n - 8;
    if (p0 >= m) return;
    uint32_t w = 0;   // codes of t[p0 .. p0+10], first in the high bits
#pragma unroll
    for (int q = 0; q < 11; ++q) {
        const int64_t i = p0 + q;
        const uint8_t ch = i < n ? t[i] : (uint8_t)'A';
        w = (w << 2) | (uint32_t)(((ch >> 2) ^ (ch >> 1)) & 3u);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (p0 + q < m) {
            keys[p0 + q] = (uint16_t)(w >> (2 * (3 - q)));
            pos[p0 + q] = (uint32_t)(p0 + q);
        }
}

// CSR offsets from the sorted k-mer codes: off[code] = the first entry whose
// code is >= code (off[65536] = m), one binary search per code -- 65,537
// searches of ~27 steps whose top levels every thread shares in the cache,
// instead of a pass over all m sorted codes
template <typename KT>
__global__ void k_kbounds(const KT *__restrict__ keys, int64_t m, int64_t *__restrict__ off) {
    const int64_t code = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (code > 65536) return;
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)keys[mid] < code) lo = mid + 1;
        else hi = mid;
    }
    off[code] = lo;
}

// ---- LCP: chunked Kasai (exact while the only rank-0 suffix is the last one)
__global__ void k_isa(const uint32_t *__restrict__ sa, int64_t n, uint32_t *__restrict__ isa) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) isa[sa[r]] = (uint32_t)r;
}

// bytes p .. p+7 of t (little-endian: byte p lowest), from two aligned words;
// t is 8-byte aligned and zero-padded by >= 16 bytes past the text
__device__ __forceinline__ uint64_t load8(const uint8_t *__restrict__ t, int64_t p) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(t + (p & ~int64_t{7}));
    const int sh = (int)(p & 7) * 8;
    const uint64_t lo = w[0], hi = w[1];
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// Chunked Kasai: each thread owns kKasaiChunk consecutive text positions and
// carries h through them (h restarts at 0 per chunk: exact, only less
// amortised).  The workgroup's ISA slice is staged in LDS by coalesced loads
// (a thread's own positions lie kKasaiChunk apart from its neighbours'), and
// suffixes are compared 8 bytes per step.  The text's unique final '$' ends
// every comparison before the padding (the caller checks SA[0] == n - 1).
constexpr int kKasaiChunk = 64;
__global__ __launch_bounds__(256) void k_kasai(const uint8_t *__restrict__ t, const uint32_t *__restrict__ sa,
                                               const uint32_t *__restrict__ isa, int64_t n,
                                               int32_t *__restrict__ lcp) {
    __shared__ uint32_t ri[256 * (kKasaiChunk + 1)];   // + 1: a thread's slice starts in its own bank
    const int64_t base = (int64_t)blockIdx.x * 256 * kKasaiChunk;
    for (int k = threadIdx.x; k < 256 * kKasaiChunk; k += 256) {
        const int64_t i = base + k;
        ri[(k / kKasaiChunk) * (kKasaiChunk + 1) + k % kKasaiChunk] = i < n ? isa[i] : 0u;
    }
    __syncthreads();
    const int64_t i0 = base + (int64_t)threadIdx.x * kKasaiChunk;
    int64_t h = 0;
    for (int q = 0; q < kKasaiChunk; ++q) {
        const int64_t i = i0 + q;
        if (i >= n) break;
        const int64_t r = ri[threadIdx.x * (kKasaiChunk + 1) + q];
        if (r > 0) {
            const int64_t j = sa[r - 1];
            for (;;) {
                const uint64_t x = load8(t, i + h) ^ load8(t, j + h);
                if (x) {
                    h += __builtin_ctzll(x) >> 3;
                    break;
                }
                h += 8;
            }
            lcp[r] = (int32_t)h;
            if (h > 0) --h;
        }
    }
}

__global__ void k_kasai_serial(const uint8_t *__restrict__ t, const uint32_t *__restrict__ sa,
                               const uint32_t *__restrict__ isa, int64_t n, int32_t *__restrict__ lcp) {
    if (blockIdx.x || threadIdx.x) return;
    int64_t h = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t r = isa[i];
        if (r > 0) {
            const int64_t j = sa[r - 1];
            while (i + h < n && j + h < n && t[i + h] == t[j + h]) ++h;
            lcp[r] = (int32_t)h;
            if (h > 0) --h;
        }
    }
}

// ---- packed FM rank for ACGT* '$' texts (bwt.py:335-357 semantics)
// per block: planes and counts of A C G T (the '$' row is not counted)
__global__ __launch_bounds__(256) void k_fm2_local(const uint8_t *__restrict__ bwt, int64_t n, int64_t nb,
                                                   uint64_t *__restrict__ fm2, uint32_t *__restrict__ cnt4,
                                                   unsigned long long *__restrict__ dollar) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    uint64_t lo = 0, hi = 0;
    uint32_t c[4] = {0, 0, 0, 0};
    const int64_t base = b * 64;
    for (int q = 0; q < 4; ++q) {   // 16 rows per load (the BWT buffer is padded)
        const uint4 v = *reinterpret_cast<const uint4 *>(bwt + base + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        for (int k = 0; k < 16; ++k) {
            const int64_t i = base + 16 * q + k;
            if (i >= n) break;
            const uint8_t ch = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
            if (ch == '$') {
                *dollar = (unsigned long long)i;
                continue;
            }
            const uint32_t code = ((ch >> 2) ^ (ch >> 1)) & 3u;   // A0 C1 G2 T3
            ++c[code];
            lo |= (uint64_t)(code & 1u) << (16 * q + k);
            hi |= (uint64_t)(code >> 1) << (16 * q + k);
        }
    }
    fm2[4 * b + 2] = lo;
    fm2[4 * b + 3] = hi;
    for (int q = 0; q < 4; ++q) cnt4[(int64_t)q * (nb + 1) + b] = c[q];
    if (b == nb - 1)
        for (int q = 0; q < 4; ++q) cnt4[(int64_t)q * (nb + 1) + nb] = 0;   // the rows' last word (scanned to the total)
}

__global__ __launch_bounds__(256) void k_fm2_counts(const uint32_t *__restrict__ cnt4, int64_t nb,
                                                    uint32_t *__restrict__ fm2u32) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    for (int q = 0; q < 4; ++q) fm2u32[8 * b + q] = cnt4[(int64_t)q * (nb + 1) + b];
}

struct FM2View {
    const uint4 *blk;      // 2 x uint4 per block
    int64_t C[5], tot[5];  // codes A C G T $
    int64_t n, dollar;
};

// occurrences of code c (0-3; 4 = '$') in bwt[0, i), 0 <= i <= n
__device__ __forceinline__ int64_t rank2(const FM2View &f, int c, int64_t i) {
    if (c == 4) return f.dollar < i ? 1 : 0;
    const int64_t b = i >> 6;
    const int r = (int)(i & 63);
    const uint4 h = f.blk[2 * b], p = f.blk[2 * b + 1];
    const uint32_t cnt = c == 0 ? h.x : c == 1 ? h.y : c == 2 ? h.z : h.w;
    const uint64_t lo = ((uint64_t)p.y << 32) | p.x, hi = ((uint64_t)p.w << 32) | p.z;
    const uint64_t m = ((c & 1) ? lo : ~lo) & ((c & 2) ? hi : ~hi);
    const uint64_t below = r ? (~0ull >> (64 - r)) : 0ull;
    int64_t x = (int64_t)cnt + __popcll(m & below);
    if (c == 0 && f.dollar >= 64 * b && f.dollar < i) --x;   // the '$' row reads as A in the planes
    return x;
}

__device__ __forceinline__ int code5(uint8_t ch) {
    switch (ch) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        case '$': return 4;
        default: return -1;
    }
}

// backward search over the packed rank, one pattern per lane: each step is
// two 32-byte block loads and two popcounts
__global__ __launch_bounds__(256) void k_bsearch2(FM2View f, const uint8_t *__restrict__ pats,
                                                  const int64_t *__restrict__ off, int64_t np,
                                                  int64_t *__restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const int64_t a = off[p], b = off[p + 1];
    int64_t sp = -1, ep = -1;
    if (b == a) {
        sp = 0;
        ep = f.n - 1;
    } else {
        int c = code5(pats[b - 1]);
        if (c >= 0 && f.tot[c] > 0) {
            sp = f.C[c];
            ep = sp + f.tot[c] - 1;
            for (int64_t i = b - 2; i >= a; --i) {
                c = code5(pats[i]);
                if (c < 0 || f.tot[c] == 0) { sp = ep = -1; break; }
                sp = f.C[c] + rank2(f, c, sp);
                ep = f.C[c] + rank2(f, c, ep + 1) - 1;
                if (sp > ep) { sp = ep = -1; break; }
            }
        }
    }
    out[2 * p] = sp;
    out[2 * p + 1] = ep;
}

// ---- backward search (bwt.py:335-389), one pattern per lane
struct FMView {
    const uint8_t *bwt;
    const int32_t *occ;
    const int64_t *C;
    const int64_t *tot;
    const uint8_t *row;
    int64_t n, olen;
    int32_t k;
};

__device__ int64_t d_rank(const FMView &f, uint8_t c, int64_t pos) {
    if (pos <= 0) return 0;
    if (pos > f.n) pos = f.n;
    const int64_t ci = pos / f.k, cpos = ci * f.k;
    int64_t base = f.occ[(int64_t)f.row[c] * f.olen + ci];
    for (int64_t i = cpos; i < pos; ++i) base += f.bwt[i] == c;
    return base;
}

__global__ void k_bsearch(FMView f, const uint8_t *__restrict__ pats, const int64_t *__restrict__ off, int64_t np,
                          int64_t *__restrict__ out) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    const int64_t a = off[p], b = off[p + 1];
    int64_t sp = -1, ep = -1;
    if (b == a) {
        sp = 0;
        ep = f.n - 1;
    } else {
        uint8_t c = pats[b - 1];
        if (f.tot[c] > 0) {
            sp = f.C[c];
            ep = sp + f.tot[c] - 1;
            for (int64_t i = b - 2; i >= a; --i) {
                c = pats[i];
                if (f.tot[c] == 0) { sp = ep = -1; break; }
                sp = f.C[c] + d_rank(f, c, sp);
                ep = f.C[c] + d_rank(f, c, ep + 1) - 1;
                if (sp > ep) { sp = ep = -1; break; }
            }
        }
    }
    out[2 * p] = sp;
    out[2 * p + 1] = ep;
}

inline unsigned blocks(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

// Suffix array of any text by prefix doubling over radix sorts (see the file
// header), then the BWT gather.
void sa_doubling(Ctx &c, DeviceIndex *ix, const uint8_t *T, int64_t n, int sigma, const uint8_t *code) {
    hipStream_t st = c.stream;
    int b = 1;
    while ((1 << b) < sigma + 1) ++b;
    const int k = 64 / b;
    c.slot[S_IDX0].ensure((size_t)n * 8);    // keys
    c.slot[S_IDX1].ensure((size_t)n * 4);    // vals
    c.slot[S_IDX2].ensure((size_t)n * 4);    // rank
    c.slot[S_IDX3].ensure((size_t)(n + 1) * 4);  // head
    c.slot[S_IDX4].ensure((size_t)(n + 1) * 4);  // scan / gid
    c.slot[S_IDX5].ensure((size_t)(n + 1) * 4);  // gstart
    c.slot[S_IDX6].ensure((size_t)(n + 1) * 4);  // flag
    c.slot[S_IDX7].ensure((size_t)(n + 1) * 4);  // U (surviving SA slots)
    c.slot[S_MISC2].ensure((size_t)(n + 1) * 4); // next U
    c.slot[S_MISC3].ensure(256);
    uint64_t *keys = c.slot[S_IDX0].as<uint64_t>();
    uint32_t *vals = c.slot[S_IDX1].as<uint32_t>();
    uint32_t *rank = c.slot[S_IDX2].as<uint32_t>();
    uint32_t *head = c.slot[S_IDX3].as<uint32_t>();
    uint32_t *gid = c.slot[S_IDX4].as<uint32_t>();
    uint32_t *gstart = c.slot[S_IDX5].as<uint32_t>();
    uint32_t *flag = c.slot[S_IDX6].as<uint32_t>();
    uint32_t *U = c.slot[S_IDX7].as<uint32_t>();
    uint32_t *U2 = c.slot[S_MISC2].as<uint32_t>();
    uint32_t *SA = ix->sa.as<uint32_t>();
    HIPCHECK(hipMemcpyAsync(c.slot[S_MISC3].p, code, 256, hipMemcpyHostToDevice, st));
    KLAUNCH("sa_init_keys", (double)n * (1.0 + 12.0), k_init_keys, dim3(blocks(n)), dim3(256), 0, st, T, n, c.slot[S_MISC3].as<uint8_t>(), b, k, keys,
                       vals);
    radix_sort_pairs32(c, keys, vals, n, 0, ((b * k + 7) / 8) * 8);
    HIPCHECK(hipMemcpyAsync(SA, vals, (size_t)n * 4, hipMemcpyDeviceToDevice, st));
    auto group_ids = [&](int64_t m) {   // head -> gid (group index), uses flag as scratch
        exclusive_scan<uint32_t>(c, head, flag, m);
        KLAUNCH("k_gid", 0.0, k_gid, dim3(blocks(m)), dim3(256), 0, st, flag, head, m, gid);
    };
    KLAUNCH("k_heads", 0.0, k_heads, dim3(blocks(n)), dim3(256), 0, st, keys, n, head);
    group_ids(n);
    KLAUNCH("k_rank0", 0.0, k_rank0, dim3(blocks(n)), dim3(256), 0, st, head, gid, SA, n, gstart, rank, flag, 0);
    KLAUNCH("k_rank0", 0.0, k_rank0, dim3(blocks(n)), dim3(256), 0, st, head, gid, SA, n, gstart, rank, flag, 1);
    // U = SA slots in groups of size >= 2
    auto compact = [&](int64_t m, const uint32_t *src, uint32_t *dst) -> int64_t {
        exclusive_scan<uint32_t>(c, flag, head, m);   // head reused as positions
        uint32_t lastp = 0, lastf = 0;
        HIPCHECK(hipMemcpyAsync(&lastp, head + m - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(&lastf, flag + m - 1, 4, hipMemcpyDeviceToHost, st));
        KLAUNCH("k_compact_idx", 0.0, k_compact_idx, dim3(blocks(m)), dim3(256), 0, st, flag, head, m, dst, src);
        HIPCHECK(hipStreamSynchronize(st));
        return (int64_t)lastp + lastf;
    };
    int64_t m = compact(n, nullptr, U);
    int nb = 1;
    while ((1ll << nb) <= n) ++nb;   // rank + 1 <= n fits in nb bits
    int64_t hlen = k;
    while (m > 0) {
        KLAUNCH("k_round_keys", 0.0, k_round_keys, dim3(blocks(m)), dim3(256), 0, st, U, m, SA, rank, n, hlen, nb, keys, vals);
        radix_sort_pairs32(c, keys, vals, m, 0, ((2 * nb + 7) / 8) * 8);
        KLAUNCH("k_heads", 0.0, k_heads, dim3(blocks(m)), dim3(256), 0, st, keys, m, head);
        group_ids(m);
        KLAUNCH("k_round_apply", 0.0, k_round_apply, dim3(blocks(m)), dim3(256), 0, st, U, m, vals, head, gid, SA, gstart, 0,
                           rank, flag);
        KLAUNCH("k_round_apply", 0.0, k_round_apply, dim3(blocks(m)), dim3(256), 0, st, U, m, vals, head, gid, SA, gstart, 1,
                           rank, flag);
        m = compact(m, U, U2);
        std::swap(U, U2);
        hlen *= 2;
        if (hlen > 4 * n + 64) fail(BWTMI_E_STATE, "suffix array doubling did not converge");
    }
    HIPCHECK(hipGetLastError());

    // BWT (bwt.py:266-274)
    KLAUNCH("bwt_gather", (double)n * (4.0 + 1.0 + 1.0), k_bwt, dim3(blocks(n)), dim3(256), 0, st, T, SA, n, ix->bwt.as<uint8_t>());
}

DeviceIndex *index_build_device(Ctx &c, const uint8_t *d_text, int64_t n, int32_t sa_sample, int32_t occ_sample,
                                uint32_t flags, DeviceIndex *reuse) {
    auto *ix = reuse ? reuse : new DeviceIndex();   // reuse: keep the buffers of an earlier build
    ix->has_kmer = false;
    ix->kmer_count = 0;
    hipStream_t st = c.stream;
    ix->n = n;
    ix->sa_sample = sa_sample;
    ix->occ_sample = occ_sample;
    ix->text.ensure((size_t)n + 128);
    HIPCHECK(hipMemsetAsync(ix->text.p, 0, (size_t)n + 128, st));
    if (n) HIPCHECK(hipMemcpyAsync(ix->text.p, d_text, (size_t)n, hipMemcpyDeviceToDevice, st));
    const uint8_t *T = ix->text.as<uint8_t>();
    // histogram -> alphabet, totals, C (bwt.py:129-134, 276-286)
    c.slot[S_COUNTS].ensure(256 * 8);
    HIPCHECK(hipMemsetAsync(c.slot[S_COUNTS].p, 0, 256 * 8, st));
    if (n) KLAUNCH("k_hist_bytes", 0.0, k_hist_bytes, dim3(1024), dim3(256), 0, st, T, n, c.slot[S_COUNTS].as<unsigned long long>());
    unsigned long long h[256];
    HIPCHECK(hipMemcpyAsync(h, c.slot[S_COUNTS].p, sizeof h, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    int64_t cum = 0;
    uint8_t code[256] = {0}, present[256] = {0};
    int sigma = 0;
    std::memset(ix->code_of, 0, sizeof ix->code_of);
    for (int b = 0; b < 256; ++b) {
        ix->totals[b] = (int64_t)h[b];
        ix->C[b] = cum;
        cum += (int64_t)h[b];
        if (h[b]) {
            present[sigma] = (uint8_t)b;
            ix->code_of[b] = (uint8_t)sigma;
            code[b] = (uint8_t)(++sigma);   // 0 = past the end
        }
    }
    ix->sigma = sigma;
    ix->sa.ensure((size_t)std::max<int64_t>(n, 1) * 4);
    ix->occ_len = ix->sampled_len = 0;
    if (n == 0) return ix;
    ix->bwt.ensure((size_t)n + 128);
    HIPCHECK(hipMemsetAsync(ix->bwt.p, 0, (size_t)n + 128, st));
    uint8_t last = 0;
    HIPCHECK(hipMemcpyAsync(&last, T + n - 1, 1, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    // ACGT* '$' (every CLI contig): string sort over 2-bit words (sa_dna.hip)
    ix->sampled_len = (n + sa_sample - 1) / sa_sample;
    ix->sampled.ensure((size_t)ix->sampled_len * 4 + 4);
    const bool dna = sa_dna_eligible(last, n, ix->totals) &&
                     sa_dna_device(c, T, n, ix->sa.as<uint32_t>(), ix->bwt.as<uint8_t>(), ix->sampled.as<int32_t>(),
                                   sa_sample);
    // ACGT with assembly gaps (N runs, a few IUPAC codes): the same string sort
    // over 3-bit symbol codes (BWTMI_SA_SMALL=0: the general doubling instead)
    const bool small_ok = knob(KN_SA_SMALL) != 0;
    uint8_t slut[256], ssym[8];
    const bool small = !dna && small_ok && sa_small_alphabet(last, n, ix->totals, slut, ssym) > 0 &&
                       sa_small_device(c, T, n, ix->sa.as<uint32_t>(), ix->bwt.as<uint8_t>(),
                                       ix->sampled.as<int32_t>(), sa_sample, slut, ssym);
    if (!dna && !small) sa_doubling(c, ix, T, n, sigma, code);
    // scratch of the Occ / k-mer / packed-rank stages
    c.slot[S_IDX0].ensure((size_t)n * 8);
    c.slot[S_IDX3].ensure((size_t)std::max<int64_t>(n + 1, 4 * (n / 64 + 2)) * 4);
    c.slot[S_IDX4].ensure((size_t)(n + 1) * 4);
    c.slot[S_IDX6].ensure((size_t)(n + 1) * 4);
    uint64_t *keys = c.slot[S_IDX0].as<uint64_t>();
    uint32_t *head = c.slot[S_IDX3].as<uint32_t>();
    uint32_t *gid = c.slot[S_IDX4].as<uint32_t>();
    uint32_t *flag = c.slot[S_IDX6].as<uint32_t>();
    const uint32_t *SA = ix->sa.as<uint32_t>();

    const int64_t nblk = (n + occ_sample - 1) / occ_sample;
    ix->occ_len = 1 + n / occ_sample + (n % occ_sample != 0);   // == nblk + 1
    ix->occ.ensure((size_t)sigma * (nblk + 1) * 4);
    HIPCHECK(hipMemsetAsync(ix->occ.p, 0, (size_t)sigma * (nblk + 1) * 4, st));
    HIPCHECK(hipMemcpyAsync(c.slot[S_MISC3].p, present, 256, hipMemcpyHostToDevice, st));
    {
        const double ob = (double)n + (double)sigma * (double)(nblk + 1) * 4.0;   // BWT read + counts written
        const uint8_t *pres = c.slot[S_MISC3].as<uint8_t>();
        uint32_t *occ = ix->occ.as<uint32_t>();
        const uint8_t *B = ix->bwt.as<uint8_t>();
        const bool pow2 = occ_sample >= 16 && occ_sample <= 1024 && (occ_sample & (occ_sample - 1)) == 0;
        const unsigned gl = blocks(nblk * (occ_sample / 16));   // one lane per 16 bytes
        if (pow2 && sigma <= 16) {
            switch (occ_sample) {
                case 16: KLAUNCH("occ_blocks", ob, k_occ_groups<1>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                case 32: KLAUNCH("occ_blocks", ob, k_occ_groups<2>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                case 64: KLAUNCH("occ_blocks", ob, k_occ_groups<4>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                case 128: KLAUNCH("occ_blocks", ob, k_occ_groups<8>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                case 256: KLAUNCH("occ_blocks", ob, k_occ_groups<16>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                case 512: KLAUNCH("occ_blocks", ob, k_occ_groups<32>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
                default: KLAUNCH("occ_blocks", ob, k_occ_groups<64>, dim3(gl), dim3(256), 0, st, B, n, nblk, pres, sigma, occ); break;
            }
        } else {   // other sample rates / alphabets: a thread per block
            KLAUNCH("occ_blocks", ob, k_occ_blocks, dim3(blocks(nblk)), dim3(256), 0, st, B, n, nblk, occ_sample, pres,
                    sigma, occ);
        }
    }
    // the sigma rows of nblk + 1 counts, one launch
    exclusive_scan_rows(c, ix->occ.as<uint32_t>(), ix->occ.as<uint32_t>(), nblk + 1, sigma, nblk + 1);
    if (!dna && !small)   // the string sort wrote the samples in its final pass
        KLAUNCH("k_sample", 0.0, k_sample, dim3(blocks(ix->sampled_len)), dim3(256), 0, st, SA, n, sa_sample,
                ix->sampled.as<int32_t>(), ix->sampled_len);

    // ------------------------------------------------ packed rank (ACGT* '$')
    ix->has_fm2 = false;
    if (dna) {
        const int64_t nb = n / 64 + 1;   // rank(c, n) reads block n >> 6
        ix->fm2.ensure((size_t)nb * 32);
        uint32_t *cnt4 = head;   // 4 x (nb + 1) words, sized above
        unsigned long long *d_dollar = reinterpret_cast<unsigned long long *>(c.slot[S_COUNTS].p);
        HIPCHECK(hipMemsetAsync(d_dollar, 0, 8, st));
        KLAUNCH("fm2_local", (double)n + 16.0 * (double)nb + 16.0 * (double)nb, k_fm2_local, dim3(blocks(nb)),
                dim3(256), 0, st, ix->bwt.as<uint8_t>(), n, nb, ix->fm2.as<uint64_t>(), cnt4, d_dollar);
        // k_fm2_local zeroed each row's last word: 4 rows of nb + 1, one launch
        exclusive_scan_rows(c, cnt4, cnt4, nb + 1, 4, nb + 1);
        KLAUNCH("fm2_counts", 32.0 * (double)nb, k_fm2_counts, dim3(blocks(nb)), dim3(256), 0, st, cnt4, nb,
                ix->fm2.as<uint32_t>());
        unsigned long long dr = 0;
        HIPCHECK(hipMemcpyAsync(&dr, d_dollar, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        ix->dollar_row = (int64_t)dr;
        ix->has_fm2 = true;
    }

    // ------------------------------------------------------------ 8-mer hash
    const int K = 8;
    if (!(flags & BWTMI_INDEX_NO_KMER) && n >= K + 1 && dna) {
        // every char but the final '$' is valid: n-8 entries, one stable
        // 16-bit radix sort of (code, position)
        ix->has_kmer = true;
        const int64_t nent = n - K;
        uint16_t *k16 = c.slot[S_IDX0].as<uint16_t>();   // 16-bit codes: 6 B per entry and pass
        ix->kmer_pos.ensure((size_t)nent * 4);
        KLAUNCH("kmer_dna", (double)n + 6.0 * (double)nent, k_kmer_dna, dim3(blocks((nent + 3) / 4)), dim3(256),
                0, st, T, n, k16, ix->kmer_pos.as<uint32_t>());
        radix_sort_pairs_k16(c, k16, ix->kmer_pos.as<uint32_t>(), nent, 0, 16);
        ix->kmer_off.ensure((size_t)(65537) * 8);
        KLAUNCH("k_kbounds", 0.0, k_kbounds<uint16_t>, dim3(blocks(65537)), dim3(256), 0, st, k16, nent,
                ix->kmer_off.as<int64_t>());
        ix->kmer_count = nent;
    } else if (!(flags & BWTMI_INDEX_NO_KMER) && n >= K) {
        ix->has_kmer = true;
        KLAUNCH("k_kvalid", 0.0, k_kvalid, dim3(blocks(n)), dim3(256), 0, st, T, n, flag);
        exclusive_scan<uint32_t>(c, flag, head, n);   // head = vpos
        uint32_t *mb = c.mailbox<uint32_t>(4);          // four reads, one wait
        HIPCHECK(hipMemcpyAsync(mb + 0, head + K - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(mb + 1, flag + K - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(mb + 2, head + n - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipMemcpyAsync(mb + 3, flag + n - 1, 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        const uint32_t vk = mb[0], vkf = mb[1], vlast = mb[2], vlastf = mb[3];
        const int64_t nvalid = (int64_t)vlast + vlastf;
        const int64_t valid_first = (int64_t)vk + vkf;   // valid among the first K chars
        const int first = valid_first == K ? 1 : 0;
        const int64_t nent = first + (nvalid - valid_first);
        uint8_t *V = (uint8_t *)gid;   // reuse: nvalid bytes <= 4n
        KLAUNCH("k_kcompact", 0.0, k_kcompact, dim3(blocks(n)), dim3(256), 0, st, T, n, head, V);
        ix->kmer_pos.ensure((size_t)std::max<int64_t>(nent, 1) * 4);
        uint16_t *k16 = reinterpret_cast<uint16_t *>(keys);
        if (nent > 0) {
            KLAUNCH("k_kentries", 0.0, k_kentries, dim3(blocks(n)), dim3(256), 0, st, T, n, K, head, V, first, k16,
                               ix->kmer_pos.as<uint32_t>(), (uint32_t)valid_first);
            radix_sort_pairs_k16(c, k16, ix->kmer_pos.as<uint32_t>(), nent, 0, 16);
        }
        ix->kmer_off.ensure((size_t)(65537) * 8);
        KLAUNCH("k_kbounds", 0.0, k_kbounds<uint16_t>, dim3(blocks(65537)), dim3(256), 0, st, k16, nent,
                           ix->kmer_off.as<int64_t>());
        ix->kmer_count = nent;
    }
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(st));
    c.checks_verify("the end of the index build");
    c.kresolve();
    return ix;
}

void index_free(DeviceIndex *ix) {
    if (!ix) return;
    (void)hipDeviceSynchronize();
    ix->text.release();
    ix->sa.release();
    ix->bwt.release();
    ix->occ.release();
    ix->sampled.release();
    ix->kmer_off.release();
    ix->kmer_pos.release();
    ix->fm2.release();
    delete ix;
}

int64_t index_n(const DeviceIndex *ix) { return ix->n; }
int64_t index_occ_len(const DeviceIndex *ix) { return ix->n ? ix->occ_len : 0; }
int64_t index_sampled_len(const DeviceIndex *ix) { return ix->sampled_len; }
int64_t index_kmer_count(const DeviceIndex *ix) { return ix->kmer_count; }

void index_get_sa(Ctx &c, const DeviceIndex *ix, int32_t *out) {
    if (ix->n) HIPCHECK(hipMemcpy(out, ix->sa.p, (size_t)ix->n * 4, hipMemcpyDeviceToHost));
}
void index_get_bwt(Ctx &c, const DeviceIndex *ix, uint8_t *out) {
    if (ix->n) HIPCHECK(hipMemcpy(out, ix->bwt.p, (size_t)ix->n, hipMemcpyDeviceToHost));
}
void index_get_counts(const DeviceIndex *ix, int64_t *totals, int64_t *C) {
    std::memcpy(totals, ix->totals, sizeof ix->totals);
    std::memcpy(C, ix->C, sizeof ix->C);
}
void index_get_occ(Ctx &c, const DeviceIndex *ix, uint8_t code, int32_t *out) {
    const int64_t len = index_occ_len(ix);
    if (!len) return;
    if (!ix->totals[code]) {   // absent alphabet codes read as zeros (bwt.py:318-325)
        std::memset(out, 0, (size_t)len * 4);
        return;
    }
    HIPCHECK(hipMemcpy(out, ix->occ.as<int32_t>() + (int64_t)ix->code_of[code] * len, (size_t)len * 4,
                       hipMemcpyDeviceToHost));
}
void index_get_sampled(Ctx &c, const DeviceIndex *ix, int32_t *out) {
    if (ix->sampled_len) HIPCHECK(hipMemcpy(out, ix->sampled.p, (size_t)ix->sampled_len * 4, hipMemcpyDeviceToHost));
}
void index_get_kmer(Ctx &c, const DeviceIndex *ix, int64_t *offsets, int32_t *pos) {
    if (!ix->has_kmer) {
        std::memset(offsets, 0, 65537 * 8);
        return;
    }
    HIPCHECK(hipMemcpy(offsets, ix->kmer_off.p, 65537 * 8, hipMemcpyDeviceToHost));
    if (ix->kmer_count) HIPCHECK(hipMemcpy(pos, ix->kmer_pos.p, (size_t)ix->kmer_count * 4, hipMemcpyDeviceToHost));
}

const uint8_t *index_text_device(const DeviceIndex *ix) { return ix->text.as<uint8_t>(); }
const uint32_t *index_sa_device(const DeviceIndex *ix) { return ix->sa.as<uint32_t>(); }

void index_get_text(Ctx &c, const DeviceIndex *ix, uint8_t *out) {
    if (!ix->n) return;
    HIPCHECK(hipMemcpyAsync(out, ix->text.p, (size_t)ix->n, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
}

void index_lcp(Ctx &c, DeviceIndex *ix, int32_t *out) {
    const int64_t n = ix->n;
    if (!n) return;
    const int32_t *lcp = index_lcp_device(c, ix);
    HIPCHECK(hipMemcpyAsync(out, lcp, (size_t)n * 4, hipMemcpyDeviceToHost, c.stream));
    HIPCHECK(hipStreamSynchronize(c.stream));
}

// Kasai LCP left in the S_MISC1 slot (valid until that slot is reused)
const int32_t *index_lcp_device(Ctx &c, DeviceIndex *ix) {
    const int64_t n = ix->n;
    if (!n) return nullptr;
    hipStream_t st = c.stream;
    c.slot[S_MISC0].ensure((size_t)n * 4);
    c.slot[S_MISC1].ensure((size_t)n * 4);
    uint32_t *isa = c.slot[S_MISC0].as<uint32_t>();
    int32_t *lcp = c.slot[S_MISC1].as<int32_t>();
    HIPCHECK(hipMemsetAsync(lcp, 0, (size_t)n * 4, st));
    KLAUNCH("k_isa", 8.0 * (double)n, k_isa, dim3(blocks(n)), dim3(256), 0, st, ix->sa.as<uint32_t>(), n, isa);
    uint32_t sa0 = 0;
    HIPCHECK(hipMemcpyAsync(&sa0, ix->sa.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    uint8_t last = 0;
    if (n > 0) HIPCHECK(hipMemcpy(&last, ix->text.as<uint8_t>() + n - 1, 1, hipMemcpyDeviceToHost));
    if ((int64_t)sa0 == n - 1 && ix->totals[last] == 1) {   // a unique smallest last symbol ends every compare
        const int64_t per = 256 * (int64_t)kKasaiChunk;
        KLAUNCH("k_kasai", 13.0 * (double)n, k_kasai, dim3((unsigned)((n + per - 1) / per)), dim3(256), 0, st,
                ix->text.as<uint8_t>(), ix->sa.as<uint32_t>(), isa, n, lcp);
    } else {
        // the smallest suffix is not the last one (no unique final sentinel):
        // Kasai's h then carries over the skipped rank-0 step, so replay it serially
        KLAUNCH("k_kasai_serial", 0.0, k_kasai_serial, dim3(1), dim3(64), 0, st, ix->text.as<uint8_t>(), ix->sa.as<uint32_t>(),
                           isa, n, lcp);
    }
    HIPCHECK(hipGetLastError());
    return lcp;
}

namespace {
__global__ void k_sa_rows(const uint32_t *__restrict__ sa, const int64_t *__restrict__ rows, int64_t k,
                          int64_t *__restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < k) out[j] = (int64_t)sa[rows[j]];
}
}  // namespace

// SA[rows[j]] for k rows (host arrays; every row < n)
void index_sa_rows(Ctx &c, const DeviceIndex *ix, const int64_t *rows, int64_t k, int64_t *out) {
    if (k <= 0) return;
    for (int64_t j = 0; j < k; ++j)
        if (rows[j] < 0 || rows[j] >= ix->n) fail(BWTMI_E_ARG, "SA row %lld out of range", (long long)rows[j]);
    hipStream_t st = c.stream;
    c.slot[S_MISC0].ensure((size_t)k * 8);
    c.slot[S_MISC1].ensure((size_t)k * 8);
    HIPCHECK(hipMemcpyAsync(c.slot[S_MISC0].p, rows, (size_t)k * 8, hipMemcpyHostToDevice, st));
    KLAUNCH("k_sa_rows", 0.0, k_sa_rows, dim3(blocks(k)), dim3(256), 0, st, ix->sa.as<uint32_t>(),
                       c.slot[S_MISC0].as<int64_t>(), k, c.slot[S_MISC1].as<int64_t>());
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(out, c.slot[S_MISC1].p, (size_t)k * 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
}

void index_backward_search(Ctx &c, DeviceIndex *ix, const uint8_t *pats, const int64_t *off, int64_t npat,
                           int64_t *sp_ep) {
    if (npat <= 0) return;
    hipStream_t st = c.stream;
    const int64_t plen = off[npat];
    c.slot[S_MISC0].ensure((size_t)plen + 8);
    c.slot[S_MISC1].ensure((size_t)(npat + 1) * 8);
    c.slot[S_MISC2].ensure((size_t)npat * 16);
    c.slot[S_MISC3].ensure(256 * 8 * 2 + 256);
    if (plen) HIPCHECK(hipMemcpyAsync(c.slot[S_MISC0].p, pats, (size_t)plen, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(c.slot[S_MISC1].p, off, (size_t)(npat + 1) * 8, hipMemcpyHostToDevice, st));
    int64_t *tabs = c.slot[S_MISC3].as<int64_t>();
    HIPCHECK(hipMemcpyAsync(tabs, ix->C, 256 * 8, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(tabs + 256, ix->totals, 256 * 8, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(tabs + 512, ix->code_of, 256, hipMemcpyHostToDevice, st));
    if (ix->has_fm2 && !knob(KN_FM_BYTES)) {
        FM2View g;
        g.blk = ix->fm2.as<uint4>();
        const char sym[5] = {'A', 'C', 'G', 'T', '$'};
        for (int q = 0; q < 5; ++q) {
            g.C[q] = ix->C[(uint8_t)sym[q]];
            g.tot[q] = ix->totals[(uint8_t)sym[q]];
        }
        g.n = ix->n;
        g.dollar = ix->dollar_row;
        KLAUNCH("k_bsearch2", 0.0, k_bsearch2, dim3(blocks(npat)), dim3(256), 0, st, g, c.slot[S_MISC0].as<uint8_t>(),
                c.slot[S_MISC1].as<int64_t>(), npat, c.slot[S_MISC2].as<int64_t>());
        HIPCHECK(hipGetLastError());
        HIPCHECK(hipMemcpyAsync(sp_ep, c.slot[S_MISC2].p, (size_t)npat * 16, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
        return;
    }
    FMView f;
    f.bwt = ix->bwt.as<uint8_t>();
    f.occ = ix->occ.as<int32_t>();
    f.C = tabs;
    f.tot = tabs + 256;
    f.row = (const uint8_t *)(tabs + 512);
    f.n = ix->n;
    f.olen = index_occ_len(ix);
    f.k = ix->occ_sample;
    KLAUNCH("k_bsearch", 0.0, k_bsearch, dim3(blocks(npat)), dim3(256), 0, st, f, c.slot[S_MISC0].as<uint8_t>(),
                       c.slot[S_MISC1].as<int64_t>(), npat, c.slot[S_MISC2].as<int64_t>());
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(sp_ep, c.slot[S_MISC2].p, (size_t)npat * 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
}

}  // namespace bwtmi
