// radix.hip -- hand-written device primitives for gfx950: a single-pass
// exclusive scan and a stable LSD radix sort (8-bit digits) over 16-, 32- or
// 64-bit keys with 32/64-bit values.
//
// Radix pass = two launches:
//   hist    : k_hist_lb -- per-wave LDS histograms of 1-16 scatter tiles per
//             workgroup (a run of equal digits in a 16-byte load is one add),
//             then a two-level look-back per digit (this block of 16 tickets,
//             then the earlier blocks' aggregates) gives every tile's
//             exclusive prefix of each digit (tile-major rows) and the last
//             workgroup the digit bases; no count table scan
//   scatter : each of the 8 waves owns 1024 consecutive keys of the tile; it
//             ranks keys of equal digit with 8 ballots (wave64 match-any) in
//             index order, so the pass is stable; the tile is reordered by
//             digit in LDS and streamed out in that order, so each digit's
//             run of the tile is one contiguous, coalesced write.  Keys and
//             then values take turns in one 64 KB LDS buffer (2 workgroups
//             of 8 waves per CU; 32 KB with 32-bit keys).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096
constexpr int kWaves = kBlock / 64;

template <class T>
__device__ inline T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        T u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
    }
    return v;
}

__device__ inline uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------ look-back
// Single-pass prefix sums (decoupled look-back): the workgroups of a launch
// take their tile in ticket order (an agent-scope atomic counter, so a
// workgroup only ever waits on tiles whose owners are already running),
// publish their tile's aggregate, then walk back over the predecessors'
// published values until one carries an inclusive prefix.  Each published
// value is ONE 8-byte granule written and read with agent-scope (sc1)
// atomics -- {value:32, flag:2, epoch:30} -- so it needs no fence: a reader
// accepts a granule only when its epoch is this launch's (every launch on a
// context draws a fresh one, so the buffer never needs clearing between
// launches) and its flag is set.  The last ticket holder resets the counter
// for the next launch.
constexpr uint64_t kLbA = 1, kLbP = 2;   // aggregate / inclusive prefix
constexpr int kMaxScanRows = 64;         // rows of one exclusive_scan_rows launch (a ticket each)
__device__ __forceinline__ uint64_t lb_pack(uint32_t epoch, uint64_t flag, uint32_t v) {
    return ((uint64_t)epoch << 34) | (flag << 32) | v;
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lb_load(uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool lb_ready(uint64_t s, uint32_t epoch) {
    return (uint32_t)(s >> 34) == epoch && ((s >> 32) & 3u) != 0;
}
// the tile of this workgroup (thread 0 draws it; every thread returns it)
__device__ __forceinline__ int64_t lb_ticket(unsigned *ticket, int64_t ntickets) {
    __shared__ unsigned tk;
    if (threadIdx.x == 0) {
        tk = atomicAdd(ticket, 1u);
        if ((int64_t)tk == ntickets - 1) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return (int64_t)tk;
}

// exclusive scan of uint32 in one launch: 4096 elements per workgroup (16
// consecutive ones per thread, 16-byte loads when aligned), wave 0 walks the
// predecessors 64 tiles per step (lane l reads tile t - 1 - l; the ballot of
// inclusive flags says where to stop, the ballot of unready lanes whether to
// wait).  In place (in == out) is allowed: a tile reads its elements before
// it writes them and no other tile touches them.
// gridDim.y rows of n elements, `stride` apart, scanned independently (one
// ticket and one granule range per row)
__global__ __launch_bounds__(kBlock) void k_scan_lb(const uint32_t *__restrict__ in, uint32_t *out, int64_t n,
                                                    int64_t ntiles, uint64_t *status, unsigned *ticket,
                                                    uint32_t epoch, int vec, int64_t stride) {
    in += (int64_t)blockIdx.y * stride;
    out += (int64_t)blockIdx.y * stride;
    status += (int64_t)blockIdx.y * ntiles;
    const int64_t tile = lb_ticket(ticket + blockIdx.y, ntiles);
    const int64_t base = tile * kTile + (int64_t)threadIdx.x * kItems;
    uint32_t x[kItems];
    const bool full = vec && base + kItems <= n;
    if (full) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
        uint4 v[kItems / 4];
#pragma unroll
        for (int q = 0; q < kItems / 4; ++q) v[q] = p[q];
        __builtin_memcpy(x, v, sizeof v);
    } else {
#pragma unroll
        for (int i = 0; i < kItems; ++i) x[i] = base + i < n ? in[base + i] : 0u;
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const uint32_t t = x[i];
        x[i] = s;
        s += t;
    }
    const uint32_t inc = wave_incl_scan<uint32_t>(s);
    __shared__ uint32_t ws[kWaves];
    __shared__ uint32_t tile_excl;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    if (wv == 0) {
        uint32_t agg = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) agg += ws[w];
        uint32_t excl = 0;
        if (tile == 0) {
            if (lane == 0) lb_store(status, lb_pack(epoch, kLbP, agg));
        } else {
            if (lane == 0) lb_store(status + tile, lb_pack(epoch, kLbA, agg));
            for (int64_t top = tile - 1;;) {   // every exit and wait is decided by a ballot (uniform)
                const int64_t idx = top - lane;
                const uint64_t v = idx >= 0 ? lb_load(status + idx) : lb_pack(epoch, kLbP, 0);
                const bool ready = lb_ready(v, epoch);
                const uint64_t nr = __ballot(!ready);
                const uint64_t pm = __ballot(ready && ((v >> 32) & 3u) == kLbP);
                const int fp = pm ? __ffsll((unsigned long long)pm) - 1 : 64;
                if (nr && __ffsll((unsigned long long)nr) - 1 <= fp) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += wave_sum_u32(lane <= fp ? (uint32_t)v : 0u);
                if (fp < 64) break;
                top -= 64;
            }
            if (lane == 0) lb_store(status + tile, lb_pack(epoch, kLbP, excl + agg));
        }
        if (lane == 0) tile_excl = excl;
    }
    __syncthreads();
    uint32_t e = inc - s + tile_excl;
    for (int w = 0; w < wv; ++w) e += ws[w];
#pragma unroll
    for (int i = 0; i < kItems; ++i) x[i] += e;
    if (full) {
        uint4 v[kItems / 4];
        __builtin_memcpy(v, x, sizeof v);
        uint4 *p = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int q = 0; q < kItems / 4; ++q) p[q] = v[q];
    } else {
#pragma unroll
        for (int i = 0; i < kItems; ++i)
            if (base + i < n) out[base + i] = x[i];
    }
}

// ------------------------------------------------------------------ radix
// Histogram + offsets of one pass in one launch.  Scatter tiles hold kSub
// keys; a histogram workgroup counts S consecutive scatter tiles (S = 1..16:
// fewer workgroups on large inputs), one LDS histogram per wave,
// and thread d owns digit d: it publishes the workgroup's count of d, sums
// the count of d in all earlier workgroups, and writes every scatter
// tile's exclusive prefix of d -- tile-major rows prefix[tile][256], one
// coalesced 1 KB row per tile.  The workgroup holding the last ticket also
// knows every digit's total and writes the digit bases (exclusive scan over
// the 256 totals).  The scatter's global slot of a key of digit d in tile t is
// then base[d] + prefix[t][d] + its rank in the tile.
constexpr int kSub = 8192;   // keys per scatter tile (512 threads x 16)
constexpr int kMaxSub = 16;
constexpr int kLbBlk = 16;   // tickets per look-back block (and granules a digit's look-back reads per step)
template <class KT>
__device__ __forceinline__ void hist_load(const KT *__restrict__ keys, int64_t tile, int64_t n, int vec,
                                          uint4 (&v)[kSub / kBlock / (16 / sizeof(KT))]) {
    constexpr int NV = kSub / kBlock / (16 / sizeof(KT));
    const int64_t b0 = tile * kSub;
    if (vec && b0 + kSub <= n) {
        const uint4 *src = reinterpret_cast<const uint4 *>(keys + b0);
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = src[i * kBlock + threadIdx.x];
    }
}
template <class KT>
__global__ __launch_bounds__(kBlock) void k_hist_lb(const KT *__restrict__ keys, int64_t n, int shift, int64_t ntiles,
                                                    int S, int64_t nhist, uint64_t *status,
                                                    uint32_t *__restrict__ prefix, uint32_t *__restrict__ base,
                                                    unsigned *ticket, uint32_t epoch, int vec, uint32_t *chk) {
    constexpr int VEC = 16 / sizeof(KT);
    constexpr int NV = kSub / kBlock / VEC;   // 16-byte loads per thread and scatter tile
    __shared__ uint32_t h[kWaves][256];
    const int64_t ht = lb_ticket(ticket, nhist);
    if (chk && ht >= nhist) {   // (uniform: the ticket is shared) a counter left non-zero by an earlier launch
        if (threadIdx.x == 0) atomicOr(chk, kChkHistTicket);
        return;
    }
    const int wv = threadIdx.x >> 6, d = threadIdx.x, lane = threadIdx.x & 63;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) h[w][d] = 0;
    // each sub-tile is loaded right before it is counted: a ring of
    // prefetched sub-tiles ran slower (tools/hist_bench: 100M bytes 31 -> 50 us)
    __syncthreads();
    uint32_t cnt[kMaxSub];
    uint32_t total = 0;
#pragma unroll
    for (int s = 0; s < kMaxSub; ++s) {
        cnt[s] = 0;
        const int64_t tile = ht * S + s;
        if (s >= S || tile >= ntiles) continue;   // uniform
        uint4 cur[NV];
        hist_load<KT>(keys, tile, n, vec, cur);
        const int64_t b0 = tile * kSub;
        if (vec && b0 + kSub <= n) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                // a run of equal digits among the load's VEC consecutive keys is
                // one add: same-digit lanes serialise an LDS atomic, and partly
                // ordered keys (the later passes, the refine rounds' digit bytes)
                // have long runs (tools/hist_bench: 100M bytes in runs of 8-263,
                // 145 -> 32 us; random 32-bit keys 99 -> 79 us, the read floor)
                const KT *k = reinterpret_cast<const KT *>(&cur[i]);
                uint32_t run = (uint32_t)(k[0] >> shift) & 255u, rc = 1;
#pragma unroll
                for (int e = 1; e < VEC; ++e) {
                    const uint32_t dg = (uint32_t)(k[e] >> shift) & 255u;
                    if (dg != run) {
                        atomicAdd(&h[wv][run], rc);
                        run = dg;
                        rc = 1;
                    } else {
                        ++rc;
                    }
                }
                atomicAdd(&h[wv][run], rc);
            }
        } else {
            const int64_t e1 = min(n, b0 + (int64_t)kSub);
            for (int64_t i = b0 + threadIdx.x; i < e1; i += kBlock) atomicAdd(&h[wv][(uint32_t)(keys[i] >> shift) & 255u], 1u);
        }
        __syncthreads();
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) {
            c += h[w][d];
            h[w][d] = 0;   // thread d alone touches column d until the next barrier
        }
        cnt[s] = c;
        total += c;
        __syncthreads();
    }
    // two-level look-back: the workgroups of a launch count at the same time,
    // so a one-level chain of inclusive prefixes would advance a window of
    // predecessors per round trip (~48 round trips for 763 workgroups).
    // Instead: the sum of the earlier workgroups of this block of kLbBlk
    // tickets, then of the earlier blocks' aggregates, which the last
    // workgroup of each block publishes -- about 4 round trips.  Every wait is
    // on lower tickets (running or done).
    const int64_t blk = ht / kLbBlk, b0 = blk * kLbBlk;
    lb_store(status + ht * 256 + d, lb_pack(epoch, kLbA, total));
    auto sum_ready = [&](int64_t first, int cntw) -> uint32_t {   // granules [first, first + cntw) of digit d, waited for
        uint32_t acc = 0;
        uint32_t have = 0;   // bit i: granule i already summed
        const uint32_t want = cntw >= 32 ? 0xffffffffu : ((1u << cntw) - 1u);
        while (have != want) {
            uint64_t v[kLbBlk];
#pragma unroll
            for (int i = 0; i < kLbBlk; ++i)
                v[i] = i < cntw && !((have >> i) & 1u) ? lb_load(status + (first + i) * 256 + d) : 0ull;
#pragma unroll
            for (int i = 0; i < kLbBlk; ++i)
                if (i < cntw && !((have >> i) & 1u) && lb_ready(v[i], epoch)) {
                    acc += (uint32_t)v[i];
                    have |= 1u << i;
                }
            if (have != want) __builtin_amdgcn_s_sleep(1);
        }
        return acc;
    };
    const uint32_t local = sum_ready(b0, (int)(ht - b0));
    if (ht - b0 == kLbBlk - 1) lb_store(status + (nhist + blk) * 256 + d, lb_pack(epoch, kLbA, local + total));
    uint32_t excl = local;
    for (int64_t q = 0; q < blk; q += kLbBlk) excl += sum_ready(nhist + q, (int)min<int64_t>(kLbBlk, blk - q));
    uint32_t run = excl;
#pragma unroll
    for (int s = 0; s < kMaxSub; ++s) {
        const int64_t tile = ht * S + s;
        if (s < S && tile < ntiles) prefix[tile * 256 + d] = run;
        run += cnt[s];
    }
    if (ht == nhist - 1) {   // run = the total of digit d
        __shared__ uint32_t dsum[kWaves];
        const uint32_t inc = wave_incl_scan<uint32_t>(run);
        if (lane == 63) dsum[wv] = inc;
        __syncthreads();
        uint32_t b = inc - run;
        for (int w = 0; w < wv; ++w) b += dsum[w];
        base[d] = b;
    }
}

template <bool NT, class T>
__device__ __forceinline__ void st(T *p, T v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Scatter of one tile, staged through LDS so that the global writes are
// coalesced: every key is ranked inside the tile (stable: wave order, then
// item order, then lane order), written to LDS at its tile-sorted slot, and the
// tile is then streamed out in slot order -- consecutive lanes write
// consecutive addresses inside each digit's run.
//   NT    : nontemporal (streaming) global stores -- the pass output is not
//           re-read before it has left the caches anyway
//   SPLIT : keys and values take turns in one LDS staging buffer (the slot ->
//           global position map stays in registers), so a tile needs 8 B of
//           LDS per key instead of 8 + sizeof(V) and more workgroups fit a CU
template <class KT, class V, int BLOCK, int ITEMS, bool NT, bool SPLIT>
__global__ __launch_bounds__(BLOCK) void k_scatter(const KT *__restrict__ kin, const V *__restrict__ vin,
                                                   KT *__restrict__ kout, V *__restrict__ vout,
                                                   const uint32_t *__restrict__ prefix,
                                                   const uint32_t *__restrict__ dbase, int64_t n, int shift,
                                                   int64_t ntiles, uint32_t *chk, uint8_t *__restrict__ dnext = nullptr,
                                                   int nshift = 0) {
    constexpr int kT = BLOCK * ITEMS;
    constexpr int NW = BLOCK / 64;
    static_assert(BLOCK >= 256 && BLOCK % 64 == 0, "threads 0..255 own one digit each");
    static_assert(!SPLIT || sizeof(V) <= sizeof(KT), "values are staged in the key buffer");
    // static LDS: the 256 per-wave digit counters of every wave, the digit bases,
    // the 256/64 wave sums of the digit scan and the key (and value) staging
    static_assert(sizeof(uint32_t) * (NW * 256 + 256 + 256 / 64) + sizeof(KT) * kT + (SPLIT ? (sizeof(KT) == 4 ? kT : 0) : sizeof(V) * kT) <=
                      160 * 1024, "exceeds gfx950's 160 KB of LDS per workgroup");
    __shared__ uint32_t wcnt[NW][256];   // per-wave digit counts, then per-wave digit bases
    __shared__ uint32_t gdelta[256];     // global position of tile slot j = gdelta[digit] + j
    __shared__ uint32_t dsum[256 / 64];  // waves 0-3 own the 256 digits of the scan
    __shared__ KT ks[kT];
    __shared__ V vs_own[SPLIT ? 1 : kT];
    // 32-bit keys: the digit of tile slot j, from which the value pass re-derives
    // its global position (no per-item positions held in registers: 80 VGPRs,
    // 3 workgroups of 8 waves per CU); 64-bit keys keep the positions in registers
    constexpr bool DG = SPLIT && sizeof(KT) == 4;
    __shared__ uint8_t dg_s[DG ? kT : 1];
    V *vs = SPLIT ? reinterpret_cast<V *>(ks) : vs_own;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < NW * 256; i += BLOCK) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const int64_t tile = xcd_tile(blockIdx.x, ntiles);
    const int64_t tbase = tile * kT;
    const int64_t wbase = tbase + (int64_t)wv * (ITEMS * 64);
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // items of this wave that exist: item i of this lane iff i * 64 + lane < lim
    const int lim = (int)max<int64_t>(0, min<int64_t>(n - wbase, ITEMS * 64));
    const KT *const kw = kin + wbase + lane;
    const V *const vw = vin ? vin + wbase + lane : nullptr;
    KT k[ITEMS];
    V v[ITEMS];
    uint32_t slot[ITEMS];   // rank among the wave's earlier keys of the same digit, then the tile slot
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const bool valid = i * 64 + lane < lim;
        k[i] = valid ? kw[i * 64] : (KT)0;
        if (!DG && vin) v[i] = valid ? vw[i * 64] : (V)0;   // DG: loaded once the keys are staged
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const bool valid = i * 64 + lane < lim;
        const uint32_t d = (uint32_t)((k[i] >> shift) & 255u);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bt = 0; bt < 8; ++bt) {
            const bool bit = (d >> bt) & 1u;
            const uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t before = (uint32_t)__popcll(peers & lt);
        slot[i] = valid ? wcnt[wv][d] + before : 0u;
        __builtin_amdgcn_wave_barrier();
        if (valid && before == 0) wcnt[wv][d] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // threads 0..255 own one digit each: tile count, exclusive scan over
    // digits (waves 0-3), per-wave bases
    const int dg = threadIdx.x;
    uint32_t cnt[NW], tot = 0, inc = 0;
    if (dg < 256) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            cnt[w] = wcnt[w][dg];
            tot += cnt[w];
        }
        inc = wave_incl_scan<uint32_t>(tot);
        if (lane == 63) dsum[wv] = inc;
    }
    __syncthreads();
    if (dg < 256) {
        uint32_t toff = inc - tot;
        for (int w = 0; w < wv; ++w) toff += dsum[w];
        gdelta[dg] = dbase[dg] + prefix[tile * 256 + dg] - toff;
        uint32_t b = toff;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            wcnt[w][dg] = b;
            b += cnt[w];
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        if (i * 64 + lane < lim) {
            const uint32_t d = (uint32_t)((k[i] >> shift) & 255u);
            slot[i] += wcnt[wv][d];
            ks[slot[i]] = k[i];
            if (!SPLIT && vin) vs[slot[i]] = v[i];
        }
    }
    if constexpr (DG) {   // the value loads fly while the keys go out (the keys' registers are free now)
        if (vin) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) v[i] = i * 64 + lane < lim ? vw[i * 64] : (V)0;
        }
    }
    __syncthreads();
    const int64_t rem = n - tbase;
    const int cntt = rem < kT ? (int)rem : kT;
    uint32_t pos[DG ? 1 : ITEMS];   // 64-bit keys: global position of tile slot i * BLOCK + t
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int j = i * BLOCK + threadIdx.x;
        if (j < cntt) {
            const KT key = ks[j];
            const uint32_t d = (uint32_t)((key >> shift) & 255u);
            const uint32_t p = gdelta[d] + (uint32_t)j;
            if constexpr (DG) dg_s[j] = (uint8_t)d;
            else pos[i] = p;
            if (chk && (int64_t)p >= n) {   // a count table that does not match the keys
                atomicOr(chk, kChkScatter);
                continue;
            }
            st<NT>(kout + p, key);
            if (dnext) dnext[p] = (uint8_t)((key >> nshift) & 255u);   // the next pass's histogram input
            if (!SPLIT && vout) st<NT>(vout + p, vs[j]);
        }
    }
    if (SPLIT && vin) {
        __syncthreads();   // every key has left the staging buffer
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if (i * 64 + lane < lim) vs[slot[i]] = v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const int j = i * BLOCK + threadIdx.x;
            if (j < cntt) {
                if constexpr (DG) {
                    const uint32_t p = gdelta[dg_s[j]] + (uint32_t)j;
                    if (!chk || (int64_t)p < n) st<NT>(vout + p, vs[j]);
                } else if (!chk || (int64_t)pos[i] < n) {
                    st<NT>(vout + pos[i], vs[j]);
                }
            }
        }
    }
}

// The look-back state of a context: the granule buffer (shared by the
// histogram and scan launches, which never overlap on one stream), the ticket
// counter and a fresh epoch per launch.  A (re)allocated granule buffer is
// cleared once, so no stale granule can carry a future epoch.
struct LbState {
    uint64_t *status;
    unsigned *ticket;
    uint32_t epoch;
};
LbState lb_prepare(Ctx &c, int64_t granules) {
    DBuf &g = c.slot[S_LB];
    const void *p0 = g.p;
    const size_t b0 = g.bytes;
    g.ensure((size_t)granules * 8 + 64);
    const bool fresh = g.p != p0 || g.bytes != b0;
    if (++c.lb_epoch >= (1u << 30)) c.lb_epoch = 1;   // epochs wrap: clear again
    if (fresh || c.lb_epoch == 1) HIPCHECK(hipMemsetAsync(g.p, 0, g.bytes, c.stream));
    if (!c.lb_ticket.p) {
        c.lb_ticket.ensure(kMaxScanRows * sizeof(unsigned));
        HIPCHECK(hipMemsetAsync(c.lb_ticket.p, 0, c.lb_ticket.bytes, c.stream));
    }
    return {g.as<uint64_t>(), c.lb_ticket.as<unsigned>(), c.lb_epoch};
}

// one pass's histogram and offsets: prefix rows in S_SORT_HIST, digit bases after them
template <class KT>
void launch_hist(Ctx &c, const KT *keys, int64_t n, int shift, int64_t ntiles, uint32_t **prefix, uint32_t **base) {
    const int64_t fs = knob(KN_HIST_S);
    // scatter tiles per histogram workgroup: ~512-1024 workgroups -- the
    // look-back chains, not the reads, set the time of larger grids (r05j, C3
    // 32-bit pass: 12207 / 6104 / 3052 / 763 workgroups 292 / 198 / 164 / 140 us)
    const int S = fs > 0 ? (int)std::min<int64_t>(fs, kMaxSub) : (int)std::max<int64_t>(1, std::min<int64_t>(kMaxSub, ntiles / 512));
    const int64_t nhist = (ntiles + S - 1) / S;
    c.slot[S_SORT_HIST].ensure((size_t)(ntiles + 1) * 256 * sizeof(uint32_t));
    *prefix = c.slot[S_SORT_HIST].as<uint32_t>();
    *base = *prefix + ntiles * 256;
    const LbState lb = lb_prepare(c, (nhist + (nhist + kLbBlk - 1) / kLbBlk) * 256);
    KLAUNCH(sizeof(KT) == 1 ? "radix_hist_k1" : sizeof(KT) == 2 ? "radix_hist_k2" : sizeof(KT) == 4 ? "radix_hist_k4"
                                                                                        : "radix_hist_k8",
            (double)n * (double)sizeof(KT), k_hist_lb<KT>, dim3((unsigned)nhist), dim3(kBlock), 0,
            c.stream, keys, n, shift, ntiles, S, nhist, lb.status, *prefix, *base, lb.ticket, lb.epoch,
            ((uintptr_t)keys & 15) == 0 ? 1 : 0, c.checks());
}

template <class KT, class V, int BLOCK, int ITEMS, bool NT, bool SPLIT>
void radix_sort_cfg(Ctx &c, KT *keys, V *vals, int64_t n, int bit0, int bit1) {
    constexpr int kT = BLOCK * ITEMS;
    static_assert(kT == kSub, "the histogram counts the scatter's tiles");
    const int64_t ntiles = (n + kT - 1) / kT;
    c.slot[S_SORT_TMP0].ensure((size_t)n * sizeof(KT));
    if (vals) c.slot[S_SORT_TMP1].ensure((size_t)n * sizeof(V));
    KT *ka = keys, *kb = c.slot[S_SORT_TMP0].as<KT>();
    V *va = vals, *vb = vals ? c.slot[S_SORT_TMP1].as<V>() : nullptr;
    // 64-bit keys: each pass but the last also writes the next pass's digit of
    // every key it places (one byte, at the key's new position), and the next
    // histogram reads n bytes instead of 8n (C3N: histograms 3.34 -> 2.56 ms,
    // the kv12 scatters +0.3 ms for their byte stores, r04zo).  For 32- and
    // 16-bit keys the byte stores cost the scatter more than the histogram
    // saves (C3: kv8 1.54 -> 1.86 ms for 1.21 -> 0.97), so they read the keys.
    const bool dig = sizeof(KT) == 8 && bit0 + 8 < bit1;
    uint8_t *dg = nullptr;
    if (dig) {
        c.slot[S_SORT_DIG].ensure((size_t)n + 64);
        dg = c.slot[S_SORT_DIG].as<uint8_t>();
    }
    int passes = 0;
    for (int sh = bit0; sh < bit1; sh += 8) {
        uint32_t *prefix, *base;
        // read the keys (the first pass) or their digit bytes once
        if (dig && sh > bit0) launch_hist<uint8_t>(c, dg, n, 0, ntiles, &prefix, &base);
        else launch_hist<KT>(c, ka, n, sh, ntiles, &prefix, &base);
        // read (key, value) once, write it once
        const bool more = dig && sh + 8 < bit1;
        const char *name = sizeof(KT) == 2 ? "radix_scatter_kv6" : sizeof(KT) == 4 ? "radix_scatter_kv8"
                           : sizeof(V) == 4 ? "radix_scatter_kv12" : "radix_scatter_kv16";
        const double bytes = (double)n * 2.0 * ((double)sizeof(KT) + (vals ? (double)sizeof(V) : 0.0));
        KLAUNCH(name, bytes, (k_scatter<KT, V, BLOCK, ITEMS, NT, SPLIT>), dim3((unsigned)ntiles), dim3(BLOCK), 0,
                c.stream, ka, va, kb, vb, prefix, base, n, sh, ntiles, c.checks(), more ? dg : nullptr, sh + 8);
        std::swap(ka, kb);
        std::swap(va, vb);
        ++passes;
    }
    HIPCHECK(hipGetLastError());
    if (passes & 1) {
        HIPCHECK(hipMemcpyAsync(keys, ka, (size_t)n * sizeof(KT), hipMemcpyDeviceToDevice, c.stream));
        if (vals) HIPCHECK(hipMemcpyAsync(vals, va, (size_t)n * sizeof(V), hipMemcpyDeviceToDevice, c.stream));
    }
}

// Pass geometry measured on the bench workload (radix_scatter_kv12 = fraction
// of the 8 TB/s peak).  r01r/r01s, 256-thread workgroups: 16 items + shared
// staging 0.50-0.51 (20 items 0.52, 12 items 0.50, 8 items 0.47); separate key
// and value staging 0.44-0.45; nontemporal stores 0.34-0.41 in every geometry.
// r01ak, same box session for every variant: 512x16 0.50, 256x16 0.47, 512x8
// 0.47, 1024x4 0.47, 256x20 0.48, 1024x8 0.44, 256x32 0.43; r02w (32-bit keys):
// 512x32, 256x32, 1024x16, 512x24 within 5 % of 512x16.  r06l/r06m (C3, same
// box): 16 K / 32 K-key tiles staged in LDS rounds, which lengthen each digit's
// written run 2-4x, are slower -- 1024x16 2.05-2.17 ms per step, 1024x32 2.33,
// 512x32 in two rounds (2 workgroups per CU) 1.80, against 1.54-1.56 for 512x16:
// with one or two workgroups per CU the ranking and the streaming phases of a
// CU's workgroups no longer overlap (profiles/r06/radix_tiles).
template <class KT, class V>
void radix_sort_impl(Ctx &c, KT *keys, V *vals, int64_t n, int bit0, int bit1) {
    if (n <= 1) return;
    if (n >= (int64_t{1} << 32)) fail(BWTMI_E_ARG, "radix sort: %lld keys exceed the 32-bit offsets", (long long)n);
    // 512 threads x 16 keys: 8192-key tiles, 8 waves per workgroup, ~75 KB of
    // LDS with 64-bit keys (64 KB staging + 8 KB wave counters + digit tables),
    // ~43 KB with 32-bit keys; 2 (3) workgroups per CU within gfx950's 160 KB
    radix_sort_cfg<KT, V, 512, 16, false, true>(c, keys, vals, n, bit0, bit1);
}

}  // namespace

void Ctx::checks_verify(const char *where) {
    if (!chk.p || !knob(KN_DEVICE_CHECKS)) return;
    uint32_t v = 0;
    HIPCHECK(hipMemcpyAsync(&v, chk.p, 4, hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    if (!v) return;
    HIPCHECK(hipMemsetAsync(chk.p, 0, 4, stream));
    static const char *const names[] = {"histogram ticket", "scatter slot", "first-rank position", "end fix-up",
                                        "run list", "run end", "deep run end"};
    std::string what;
    for (int b = 0; b < 7; ++b)
        if (v >> b & 1u) what += std::string(what.empty() ? "" : ", ") + names[b];
    fail(BWTMI_E_STATE, "device check failed before %s: %s (BWTMI_DEVICE_CHECKS)", where, what.c_str());
}

void exclusive_scan_rows(Ctx &c, const uint32_t *in, uint32_t *out, int64_t n, int rows, int64_t stride) {
    if (n <= 0 || rows <= 0) return;
    if (rows > kMaxScanRows) fail(BWTMI_E_ARG, "exclusive_scan_rows: %d rows (at most %d)", rows, kMaxScanRows);
    const int64_t ntiles = (n + kTile - 1) / kTile;
    const LbState lb = lb_prepare(c, ntiles * rows);
    // 16-byte vectors need aligned bases in every row
    const int vec = (((uintptr_t)in | (uintptr_t)out) & 15) == 0 && (rows == 1 || (stride & 3) == 0) ? 1 : 0;
    KLAUNCH("k_scan", 2.0 * (double)n * rows * 4.0, k_scan_lb, dim3((unsigned)ntiles, (unsigned)rows), dim3(kBlock), 0,
            c.stream, in, out, n, ntiles, lb.status, lb.ticket, lb.epoch, vec, stride);
    HIPCHECK(hipGetLastError());
}

template <class T>
void exclusive_scan(Ctx &c, const T *in, T *out, int64_t n) {
    static_assert(sizeof(T) == 4, "32-bit scans");
    exclusive_scan_rows(c, (const uint32_t *)in, (uint32_t *)out, n, 1, 0);
}

template void exclusive_scan<uint32_t>(Ctx &, const uint32_t *, uint32_t *, int64_t);

void radix_sort_pairs(Ctx &c, uint64_t *keys, uint64_t *vals, int64_t n, int bit0, int bit1) {
    radix_sort_impl<uint64_t, uint64_t>(c, keys, vals, n, bit0, bit1);
}
void radix_sort_pairs32(Ctx &c, uint64_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1) {
    radix_sort_impl<uint64_t, uint32_t>(c, keys, vals, n, bit0, bit1);
}
// one pass: (kin, vin) -> (kout, vout) ordered by the 8-bit digit at `shift`
void radix_pass_k32(Ctx &c, const uint32_t *kin, const uint32_t *vin, uint32_t *kout, uint32_t *vout, int64_t n,
                    int shift) {
    if (n <= 0) return;
    constexpr int BLOCK = 512, ITEMS = 16, kT = BLOCK * ITEMS;
    const int64_t ntiles = (n + kT - 1) / kT;
    uint32_t *prefix, *base;
    launch_hist<uint32_t>(c, kin, n, shift, ntiles, &prefix, &base);
    KLAUNCH("radix_partition_kv8", (double)n * 16.0, (k_scatter<uint32_t, uint32_t, BLOCK, ITEMS, false, true>),
            dim3((unsigned)ntiles), dim3(BLOCK), 0, c.stream, kin, vin, kout, vout, prefix, base, n, shift, ntiles,
            c.checks());
    HIPCHECK(hipGetLastError());
}

// 16-bit keys (the 8-mer codes), 32-bit values: keys and values staged apart
// (a value does not fit a key's LDS slot), positions kept in registers
void radix_sort_pairs_k16(Ctx &c, uint16_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1) {
    if (n <= 1) return;
    if (n >= (int64_t{1} << 32)) fail(BWTMI_E_ARG, "radix sort: %lld keys exceed the 32-bit offsets", (long long)n);
    radix_sort_cfg<uint16_t, uint32_t, 512, 16, false, false>(c, keys, vals, n, bit0, bit1);
}

void radix_sort_pairs_k32(Ctx &c, uint32_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1) {
    radix_sort_impl<uint32_t, uint32_t>(c, keys, vals, n, bit0, bit1);
}

}  // namespace bwtmi
