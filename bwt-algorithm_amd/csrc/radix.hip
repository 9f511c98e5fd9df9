// radix.hip -- hand-written device primitives for gfx950: exclusive scan and a
// stable LSD radix sort (8-bit digits) over 64- or 32-bit keys with 32/64-bit
// values.
//
// Radix pass = three launches:
//   hist    : one workgroup per 8192-key tile, LDS histogram -> counts[d][tile]
//   scan    : exclusive scan of counts (digit-major) -> global offsets
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

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kBlock = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlock * kItems;  // 4096
constexpr int kWaves = kBlock / 64;

// ------------------------------------------------------------------ scan
template <class T>
__global__ __launch_bounds__(kBlock) void k_chunk_sums(const T *__restrict__ in, T *__restrict__ sums, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * kTile;
    T s = 0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
        if (idx < n) s += in[idx];
    }
    __shared__ T red[kBlock];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = red[0];
}

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

// Blocked variants of the two chunk kernels: thread t owns the 16 consecutive
// elements [16t, 16t + 16) of the chunk, read and written as 16-byte vectors
// (a wave moves 4 KB per 4-8 instructions), scanned in registers; only the
// 4 wave totals pass through LDS.  The kernels above staged every element in
// LDS and read it back at a 16-element stride (bank conflicts) -- each of the
// ~20 scans of a C3 index build over 3.1M tile counts ran at < 1 TB/s.
template <class T>
__device__ __forceinline__ bool load_blocked(const T *__restrict__ in, int64_t base, int64_t n, T (&x)[kItems]) {
    constexpr int NV = kItems * (int)sizeof(T) / 16;
    if (base + kItems <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
        uint4 v[NV];
#pragma unroll
        for (int q = 0; q < NV; ++q) v[q] = p[q];
        __builtin_memcpy(x, v, sizeof v);
        return true;
    }
#pragma unroll
    for (int i = 0; i < kItems; ++i) x[i] = base + i < n ? in[base + i] : (T)0;
    return false;
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_chunk_sums_v(const T *__restrict__ in, T *__restrict__ sums, int64_t n) {
    T x[kItems];
    load_blocked<T>(in, (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems, n, x);
    T s = 0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) s += x[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ T ws[kWaves];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += ws[w];
        sums[blockIdx.x] = t;
    }
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_chunk_scan_v(const T *__restrict__ in, T *__restrict__ out,
                                                         const T *__restrict__ offs, int64_t n) {
    constexpr int NV = kItems * (int)sizeof(T) / 16;
    const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
    T x[kItems];
    const bool full = load_blocked<T>(in, base, n, x);
    T s = 0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const T t = x[i];
        x[i] = s;
        s += t;
    }
    const T inc = wave_incl_scan<T>(s);
    __shared__ T ws[kWaves];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) ws[wv] = inc;
    __syncthreads();
    T excl = inc - s + (offs ? offs[blockIdx.x] : (T)0);
    for (int w = 0; w < wv; ++w) excl += ws[w];
#pragma unroll
    for (int i = 0; i < kItems; ++i) x[i] += excl;
    if (full) {
        uint4 v[NV];
        __builtin_memcpy(v, x, sizeof v);
        uint4 *p = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int q = 0; q < NV; ++q) p[q] = v[q];
    } else {
#pragma unroll
        for (int i = 0; i < kItems; ++i)
            if (base + i < n) out[base + i] = x[i];
    }
}

// exclusive scan of one chunk, adding offs[blockIdx.x] (exclusive chunk prefix)
template <class T>
__global__ __launch_bounds__(kBlock) void k_chunk_scan(const T *__restrict__ in, T *__restrict__ out,
                                                       const T *__restrict__ offs, int64_t n) {
    __shared__ T buf[kTile];
    __shared__ T wsum[kWaves];
    const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
        buf[i * kBlock + threadIdx.x] = idx < n ? in[idx] : (T)0;
    }
    __syncthreads();
    T loc[kItems];
    T s = 0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        loc[i] = s;
        s += buf[threadIdx.x * kItems + i];
    }
    const T inc = wave_incl_scan<T>(s);
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    T wpre = 0;
    for (int w = 0; w < wv; ++w) wpre += wsum[w];
    const T excl = inc - s + wpre + (offs ? offs[blockIdx.x] : (T)0);
#pragma unroll
    for (int i = 0; i < kItems; ++i) buf[threadIdx.x * kItems + i] = loc[i] + excl;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
        if (idx < n) out[idx] = buf[i * kBlock + threadIdx.x];
    }
}

// ------------------------------------------------------------------ radix
// Pass geometry: 256-thread workgroups (thread t owns digit t in the tile
// scan), ITEMS keys per thread, tile = 256 * ITEMS.
template <int ITEMS, class KT>
__global__ __launch_bounds__(kBlock) void k_hist(const KT *__restrict__ keys, uint32_t *__restrict__ counts,
                                                 int64_t n, int shift, int64_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * (kBlock * ITEMS);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const int64_t idx = base + (int64_t)i * kBlock + threadIdx.x;
        if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 255u], 1u);
    }
    __syncthreads();
    counts[(int64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// The same counts, read as 16-byte vectors (every key of a full tile is loaded
// before the first LDS atomic, so the loads are all in flight together) and
// counted into one histogram per wave (no atomics between waves on one bin);
// the tile's last partial piece takes the scalar path.
template <int ITEMS, class KT>
__global__ __launch_bounds__(kBlock) void k_hist_vec(const KT *__restrict__ keys, uint32_t *__restrict__ counts,
                                                     int64_t n, int shift, int64_t ntiles) {
    constexpr int VEC = 16 / sizeof(KT);
    constexpr int NV = ITEMS / VEC;   // 16-byte loads per thread
    static_assert(ITEMS % VEC == 0, "whole vectors per thread");
    __shared__ uint32_t h[kWaves][256];
    for (int i = threadIdx.x; i < kWaves * 256; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    const int wv = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * (kBlock * ITEMS);
    if (base + kBlock * ITEMS <= n) {
        uint4 v[NV];
        const uint4 *src = reinterpret_cast<const uint4 *>(keys + base);
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = src[i * kBlock + threadIdx.x];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const KT *k = reinterpret_cast<const KT *>(&v[i]);
#pragma unroll
            for (int e = 0; e < VEC; ++e) atomicAdd(&h[wv][(k[e] >> shift) & 255u], 1u);
        }
    } else {
        for (int64_t idx = base + threadIdx.x; idx < n; idx += kBlock) atomicAdd(&h[wv][(keys[idx] >> shift) & 255u], 1u);
    }
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += h[w][threadIdx.x];
    counts[(int64_t)threadIdx.x * ntiles + blockIdx.x] = t;
}

template <int ITEMS, class KT>
void launch_hist(Ctx &c, const KT *keys, uint32_t *cnt, int64_t n, int sh, int64_t ntiles) {
    static const int vec = [] { const char *e = std::getenv("BWTMI_HIST_VEC"); return e ? std::atoi(e) : 1; }();
    if (vec && ((uintptr_t)keys & 15) == 0)
        KLAUNCH("radix_hist", (double)n * (double)sizeof(KT), (k_hist_vec<ITEMS, KT>), dim3((unsigned)ntiles),
                dim3(kBlock), 0, c.stream, keys, cnt, n, sh, ntiles);
    else
        KLAUNCH("radix_hist", (double)n * (double)sizeof(KT), (k_hist<ITEMS, KT>), dim3((unsigned)ntiles),
                dim3(kBlock), 0, c.stream, keys, cnt, n, sh, ntiles);
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
                                                   const uint32_t *__restrict__ offs, int64_t n, int shift,
                                                   int64_t ntiles, int swz, uint8_t *__restrict__ dnext = nullptr,
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
    const int64_t tile = swz ? xcd_tile(blockIdx.x, ntiles) : (int64_t)blockIdx.x;
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
        gdelta[dg] = offs[(int64_t)dg * ntiles + tile] - toff;
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
            st<NT>(kout + p, key);
            if (dnext) dnext[p] = (uint8_t)((key >> nshift) & 255u);   // the next pass's histogram input
            if constexpr (DG) dg_s[j] = (uint8_t)d;
            else pos[i] = p;
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
                if constexpr (DG) st<NT>(vout + gdelta[dg_s[j]] + (uint32_t)j, vs[j]);
                else st<NT>(vout + pos[i], vs[j]);
            }
        }
    }
}

template <class KT, class V, int BLOCK, int ITEMS, bool NT, bool SPLIT>
void radix_sort_cfg(Ctx &c, KT *keys, V *vals, int64_t n, int bit0, int bit1) {
    constexpr int kT = BLOCK * ITEMS;
    static_assert(kT % kBlock == 0, "histogram tiles are 256-thread tiles");
    const int64_t ntiles = (n + kT - 1) / kT;
    c.slot[S_SORT_TMP0].ensure((size_t)n * sizeof(KT));
    if (vals) c.slot[S_SORT_TMP1].ensure((size_t)n * sizeof(V));
    c.slot[S_SORT_HIST].ensure((size_t)ntiles * 256 * sizeof(uint32_t));
    KT *ka = keys, *kb = c.slot[S_SORT_TMP0].as<KT>();
    V *va = vals, *vb = vals ? c.slot[S_SORT_TMP1].as<V>() : nullptr;
    uint32_t *cnt = c.slot[S_SORT_HIST].as<uint32_t>();
    static const int swz = [] { const char *e = std::getenv("BWTMI_RADIX_SWZ"); return e ? std::atoi(e) : 1; }();
    // 64-bit keys: each pass but the last also writes the next pass's digit of
    // every key it places (one byte, at the key's new position), and the next
    // histogram reads n bytes instead of 8n (C3N: histograms 3.34 -> 2.56 ms,
    // the kv12 scatters +0.3 ms for their byte stores, r04zo).  For 32- and
    // 16-bit keys the byte stores cost the scatter more than the histogram
    // saves (C3: kv8 1.54 -> 1.86 ms for 1.21 -> 0.97), so they read the keys.
    // BWTMI_RADIX_DIGITS=0: never, =2: every key width.
    static const int digits = [] { const char *e = std::getenv("BWTMI_RADIX_DIGITS"); return e && *e ? std::atoi(e) : 1; }();
    const bool dig = (digits == 2 || (digits == 1 && sizeof(KT) == 8)) && bit0 + 8 < bit1;
    uint8_t *dg = nullptr;
    if (dig) {
        c.slot[S_SORT_DIG].ensure((size_t)n + 64);
        dg = c.slot[S_SORT_DIG].as<uint8_t>();
    }
    int passes = 0;
    for (int sh = bit0; sh < bit1; sh += 8) {
        // read the keys (the first pass) or their digit bytes once
        if (dig && sh > bit0) launch_hist<kT / kBlock, uint8_t>(c, dg, cnt, n, 0, ntiles);
        else launch_hist<kT / kBlock, KT>(c, ka, cnt, n, sh, ntiles);
        exclusive_scan<uint32_t>(c, cnt, cnt, ntiles * 256);
        // read (key, value) once, write it once
        const bool more = dig && sh + 8 < bit1;
        KLAUNCH(sizeof(KT) == 2 ? "radix_scatter_kv6" : sizeof(KT) == 4 ? "radix_scatter_kv8"
                : sizeof(V) == 4 ? "radix_scatter_kv12" : "radix_scatter_kv16",
                (double)n * 2.0 * ((double)sizeof(KT) + (vals ? (double)sizeof(V) : 0.0)),
                (k_scatter<KT, V, BLOCK, ITEMS, NT, SPLIT>), dim3((unsigned)ntiles), dim3(BLOCK), 0, c.stream, ka, va,
                kb, vb, cnt, n, sh, ntiles, swz, more ? dg : nullptr, sh + 8);
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
// 0.47, 1024x4 0.47, 256x20 0.48, 1024x8 0.44, 256x32 0.43.
template <class KT, class V>
void radix_sort_impl(Ctx &c, KT *keys, V *vals, int64_t n, int bit0, int bit1) {
    if (n <= 1) return;
    // 512 threads x 16 keys: 8192-key tiles, 8 waves per workgroup, ~75 KB of
    // LDS with 64-bit keys (64 KB staging + 8 KB wave counters + digit tables),
    // ~43 KB with 32-bit keys; 2 (3) workgroups per CU within gfx950's 160 KB
    radix_sort_cfg<KT, V, 512, 16, false, true>(c, keys, vals, n, bit0, bit1);
}

}  // namespace

// Mid-size arrays (the radix count tables of short inputs, flag arrays of
// a few tens of thousands): one workgroup walks the array 4096 elements a step
// with a running carry -- one launch instead of the sums / scan / scan chain
// (three launches and their gaps on a launch-bound 12.5 Mbp scan)
constexpr int64_t kOneBlockScan = 32768;
template <class T>
__global__ __launch_bounds__(kBlock) void k_scan_one(const T *__restrict__ in, T *__restrict__ out, int64_t n) {
    __shared__ T ws[kWaves];
    __shared__ T carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t c0 = 0; c0 < n; c0 += kTile) {
        const int64_t base = c0 + (int64_t)threadIdx.x * kItems;
        T x[kItems];
#pragma unroll
        for (int i = 0; i < kItems; ++i) x[i] = base + i < n ? in[base + i] : (T)0;
        T s = 0;
#pragma unroll
        for (int i = 0; i < kItems; ++i) {
            const T t = x[i];
            x[i] = s;
            s += t;
        }
        const T inc = wave_incl_scan<T>(s);
        const int wv = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 63) ws[wv] = inc;
        __syncthreads();
        T excl = inc - s + carry;
        for (int w = 0; w < wv; ++w) excl += ws[w];
#pragma unroll
        for (int i = 0; i < kItems; ++i)
            if (base + i < n) out[base + i] = x[i] + excl;
        __syncthreads();   // every thread has read carry and ws
        if (threadIdx.x == kBlock - 1) carry = excl + s;
        __syncthreads();
    }
}

// in place (in == out) is allowed: a chunk's elements are read before any is written
template <class T>
static void scan_rec(Ctx &c, const T *in, T *out, int64_t n, T *tmp) {
    static const int vec = [] { const char *e = std::getenv("BWTMI_SCAN_VEC"); return e ? std::atoi(e) : 1; }();
    const bool v = vec && (((uintptr_t)in | (uintptr_t)out) & 15) == 0;   // 16-byte vectors need aligned bases
    const int64_t nch = (n + kTile - 1) / kTile;
    const double bytes = 2.0 * (double)n * (double)sizeof(T);
    static const bool one = [] { const char *e = std::getenv("BWTMI_SCAN_ONE"); return !(e && *e == '0'); }();
    if (nch > 1 && n <= kOneBlockScan && one) {
        KLAUNCH("k_chunk_scan", bytes, k_scan_one<T>, dim3(1), dim3(kBlock), 0, c.stream, in, out, n);
        return;
    }
    if (nch == 1) {
        if (v) KLAUNCH("k_chunk_scan", bytes, k_chunk_scan_v<T>, dim3(1), dim3(kBlock), 0, c.stream, in, out, (const T *)nullptr, n);
        else KLAUNCH("k_chunk_scan", bytes, k_chunk_scan<T>, dim3(1), dim3(kBlock), 0, c.stream, in, out, (const T *)nullptr, n);
        return;
    }
    T *sums = tmp;
    if (v) KLAUNCH("k_chunk_sums", bytes / 2, k_chunk_sums_v<T>, dim3((unsigned)nch), dim3(kBlock), 0, c.stream, in, sums, n);
    else KLAUNCH("k_chunk_sums", bytes / 2, k_chunk_sums<T>, dim3((unsigned)nch), dim3(kBlock), 0, c.stream, in, sums, n);
    scan_rec<T>(c, sums, sums, nch, tmp + nch);
    if (v) KLAUNCH("k_chunk_scan", bytes, k_chunk_scan_v<T>, dim3((unsigned)nch), dim3(kBlock), 0, c.stream, in, out, (const T *)sums, n);
    else KLAUNCH("k_chunk_scan", bytes, k_chunk_scan<T>, dim3((unsigned)nch), dim3(kBlock), 0, c.stream, in, out, (const T *)sums, n);
}

template <class T>
void exclusive_scan(Ctx &c, const T *in, T *out, int64_t n) {
    if (n <= 0) return;
    int64_t need = 0;
    for (int64_t m = n; m > kTile;) {
        m = (m + kTile - 1) / kTile;
        need += m;
    }
    c.slot[S_SCAN_TMP].ensure((size_t)(need + 1) * sizeof(T));
    scan_rec<T>(c, in, out, n, c.slot[S_SCAN_TMP].as<T>());
    HIPCHECK(hipGetLastError());
}

template void exclusive_scan<uint32_t>(Ctx &, const uint32_t *, uint32_t *, int64_t);
template void exclusive_scan<uint64_t>(Ctx &, const uint64_t *, uint64_t *, int64_t);
template void exclusive_scan<int64_t>(Ctx &, const int64_t *, int64_t *, int64_t);

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
    c.slot[S_SORT_HIST].ensure((size_t)ntiles * 256 * sizeof(uint32_t));
    uint32_t *cnt = c.slot[S_SORT_HIST].as<uint32_t>();
    launch_hist<kT / kBlock, uint32_t>(c, kin, cnt, n, shift, ntiles);
    exclusive_scan<uint32_t>(c, cnt, cnt, ntiles * 256);
    KLAUNCH("radix_partition_kv8", (double)n * 16.0, (k_scatter<uint32_t, uint32_t, BLOCK, ITEMS, false, true>),
            dim3((unsigned)ntiles), dim3(BLOCK), 0, c.stream, kin, vin, kout, vout, cnt, n, shift, ntiles, 1);
    HIPCHECK(hipGetLastError());
}

// 16-bit keys (the 8-mer codes), 32-bit values: keys and values staged apart
// (a value does not fit a key's LDS slot), positions kept in registers
void radix_sort_pairs_k16(Ctx &c, uint16_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1) {
    if (n <= 1) return;
    radix_sort_cfg<uint16_t, uint32_t, 512, 16, false, false>(c, keys, vals, n, bit0, bit1);
}

void radix_sort_pairs_k32(Ctx &c, uint32_t *keys, uint32_t *vals, int64_t n, int bit0, int bit1) {
    static const int v = [] { const char *e = std::getenv("BWTMI_RADIX32"); return e ? std::atoi(e) : 0; }();
    switch (v) {   // geometry A/B (tools/gpu_radix_ab.sh)
        case 1: radix_sort_cfg<uint32_t, uint32_t, 512, 32, false, true>(c, keys, vals, n, bit0, bit1); return;
        case 2: radix_sort_cfg<uint32_t, uint32_t, 256, 32, false, true>(c, keys, vals, n, bit0, bit1); return;
        case 3: radix_sort_cfg<uint32_t, uint32_t, 1024, 16, false, true>(c, keys, vals, n, bit0, bit1); return;
        case 4: radix_sort_cfg<uint32_t, uint32_t, 512, 24, false, true>(c, keys, vals, n, bit0, bit1); return;
        default: radix_sort_impl<uint32_t, uint32_t>(c, keys, vals, n, bit0, bit1);
    }
}

}  // namespace bwtmi
