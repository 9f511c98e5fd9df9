// Counting phase of the radix histogram, in isolation (measurement tool, not
// product code): 256-thread workgroups each count S = 16 tiles of 8192 keys
// into LDS and write every tile's 256 counts (tile-major), as k_hist_lb does
// before its look-back.  Variants:
//   atom   : one LDS histogram per wave, ds_add per key (the product's way)
//   match  : wave match-any over the 8 digit bits (ballots); one ds_add per
//            distinct digit of the 64 lanes, by the lowest lane holding it
//   peel1/2: the first lane's digit group (then the next one's) added once,
//            the other lanes one by one
//   run16 / runslice: runs of equal digits among a thread's consecutive keys
//            (per 16-byte load / over the thread's contiguous slice) added once
//   ring_run16: run16 with k_hist_lb's prefetch ring (one tile ahead)
//   none   : the same loads, keys summed in a register (no counting): the
//            read floor of this loop
// Inputs: random bytes, and "runs" (bytes constant over runs of 4096 keys --
// the digit stream of partly ordered keys).  u8 and u32 keys (digit = low byte).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/hist_bench tools/hist_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int kB = 256, kSub = 8192, kS = 16;

template <int MODE, class KT>
__global__ __launch_bounds__(kB) void k_count(const KT *__restrict__ keys, int64_t ntiles, uint32_t *__restrict__ out,
                                              uint32_t *__restrict__ sink) {
    constexpr int VEC = 16 / sizeof(KT), NV = kSub / kB / VEC;
    __shared__ uint32_t h[4][256];
    const int wv = threadIdx.x >> 6, d = threadIdx.x, lane = threadIdx.x & 63;
    const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
    for (int w = 0; w < 4; ++w) h[w][d] = 0;
    __syncthreads();
    uint32_t acc = 0;
    if constexpr (MODE == 7) {   // k_hist_lb's loop: one tile prefetched while one is counted
        constexpr int D = NV >= 8 ? 1 : 8 / NV;
        uint4 buf[D + 1][NV];
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const uint4 *src = reinterpret_cast<const uint4 *>(keys + ((int64_t)blockIdx.x * kS + q) * kSub);
#pragma unroll
            for (int i = 0; i < NV; ++i) buf[q][i] = src[i * kB + threadIdx.x];
        }
#pragma unroll
        for (int s = 0; s < kS; ++s) {
            const int64_t tile = (int64_t)blockIdx.x * kS + s;
            if (tile >= ntiles) continue;
            if (s + D < kS && tile + D < ntiles) {
                const uint4 *src = reinterpret_cast<const uint4 *>(keys + (tile + D) * kSub);
#pragma unroll
                for (int i = 0; i < NV; ++i) buf[(s + D) % (D + 1)][i] = src[i * kB + threadIdx.x];
            }
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const KT *k = reinterpret_cast<const KT *>(&buf[s % (D + 1)][i]);
                uint32_t run = (uint32_t)k[0] & 255u, rc = 1;
#pragma unroll
                for (int e = 1; e < VEC; ++e) {
                    const uint32_t dg = (uint32_t)k[e] & 255u;
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
            __syncthreads();
            uint32_t c = 0;
            for (int w = 0; w < 4; ++w) {
                c += h[w][d];
                h[w][d] = 0;
            }
            out[tile * 256 + d] = c;
            __syncthreads();
        }
        return;
    }
    for (int s = 0; s < kS; ++s) {
        const int64_t tile = (int64_t)blockIdx.x * kS + s;
        if (tile >= ntiles) break;
        const uint4 *src = reinterpret_cast<const uint4 *>(keys + tile * kSub);
        uint4 v[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = MODE == 6 ? src[threadIdx.x * NV + i] : src[i * kB + threadIdx.x];
        if constexpr (MODE == 5 || MODE == 6) {
            // runs of equal digits inside the thread's consecutive keys (MODE 5:
            // each 16-byte load; MODE 6: the thread's whole contiguous slice)
            // are added once per run
            uint32_t cur = 0xffffffffu, cnt = 0;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const KT *k = reinterpret_cast<const KT *>(&v[i]);
#pragma unroll
                for (int e = 0; e < VEC; ++e) {
                    const uint32_t dg = (uint32_t)k[e] & 255u;
                    if (dg != cur) {
                        if (cnt) atomicAdd(&h[wv][cur], cnt);
                        cur = dg;
                        cnt = 1;
                    } else {
                        ++cnt;
                    }
                }
                if (MODE == 5) {
                    atomicAdd(&h[wv][cur], cnt);
                    cur = 0xffffffffu;
                    cnt = 0;
                }
            }
            if (cnt) atomicAdd(&h[wv][cur], cnt);
        } else
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const KT *k = reinterpret_cast<const KT *>(&v[i]);
#pragma unroll
            for (int e = 0; e < VEC; ++e) {
                const uint32_t dg = (uint32_t)k[e] & 255u;
                if constexpr (MODE == 0) {
                    atomicAdd(&h[wv][dg], 1u);
                } else if constexpr (MODE == 1) {
                    uint64_t peers = ~0ull;
#pragma unroll
                    for (int bt = 0; bt < 8; ++bt) {
                        const bool bit = (dg >> bt) & 1u;
                        const uint64_t bal = __ballot(bit);
                        peers &= bit ? bal : ~bal;
                    }
                    if ((peers & lt) == 0) atomicAdd(&h[wv][dg], (uint32_t)__popcll(peers));
                } else if constexpr (MODE == 3 || MODE == 4) {
                    // peel the first lane's digit group (MODE 4: then the next
                    // remaining lane's), one add each; the rest add one by one
                    uint64_t left = __ballot(true);
                    bool done = false;
#pragma unroll
                    for (int pass = 0; pass < MODE - 2; ++pass) {
                        if (!left) break;
                        const int fl = __ffsll((unsigned long long)left) - 1;
                        const uint32_t ld = __shfl(dg, fl, 64);
                        const uint64_t eq = __ballot(!done && dg == ld);
                        if (lane == fl) atomicAdd(&h[wv][ld], (uint32_t)__popcll(eq));
                        done = done || dg == ld;
                        left &= ~eq;
                    }
                    if (!done) atomicAdd(&h[wv][dg], 1u);
                } else {
                    acc += dg;
                }
            }
        }
        __syncthreads();
        uint32_t c = 0;
        for (int w = 0; w < 4; ++w) {
            c += h[w][d];
            h[w][d] = 0;
        }
        out[tile * 256 + d] = c;
        __syncthreads();
    }
    if (MODE == 2 && acc == 0xdeadbeef) sink[0] = acc;
}

template <class KT>
void run(const char *tag, int64_t n, int runs, uint32_t *out, uint32_t *sink) {
    // runs: 0 random; 1 constant over 4096 keys; 2 constant over random lengths 8..263
    std::vector<KT> hkeys((size_t)n);
    uint32_t x = 12345, y = 777;
    int64_t next = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (runs == 0 || (runs == 1 && i % 4096 == 0) || (runs == 2 && i >= next)) {
            x = x * 1664525u + 1013904223u;
            y = y * 22695477u + 1u;
            next = i + 8 + (int64_t)((y >> 16) & 255u);
        }
        hkeys[(size_t)i] = (KT)((x >> 8) ^ (runs ? 0u : (uint32_t)(i * 2654435761u)));
    }
    KT *d;
    CK(hipMalloc(&d, n * sizeof(KT)));
    CK(hipMemcpy(d, hkeys.data(), n * sizeof(KT), hipMemcpyHostToDevice));
    const int64_t ntiles = n / kSub, grid = (ntiles + kS - 1) / kS;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto k) {
        for (int w = 0; w < 3; ++w) k<<<grid, kB>>>(d, ntiles, out, sink);
        CK(hipEventRecord(a));
        for (int r = 0; r < 20; ++r) k<<<grid, kB>>>(d, ntiles, out, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1000.0 / 20.0;
    };
    const double ta = time(k_count<0, KT>), tm = time(k_count<1, KT>), tn = time(k_count<2, KT>),
                 tp1 = time(k_count<3, KT>), tp2 = time(k_count<4, KT>), tr5 = time(k_count<5, KT>),
                 tr6 = time(k_count<6, KT>), tr7 = time(k_count<7, KT>);
    std::printf("{\"keys\": \"%s\", \"n\": %lld, \"atom_us\": %.1f, \"match_us\": %.1f, \"none_us\": %.1f, "
                "\"peel1_us\": %.1f, \"peel2_us\": %.1f, \"run16_us\": %.1f, \"runslice_us\": %.1f, \"ring_run16_us\": %.1f}\n",
                tag, (long long)n, ta, tm, tn, tp1, tp2, tr5, tr6, tr7);
    CK(hipFree(d));
}

int main() {
    const int64_t n = 12207LL * kSub;
    uint32_t *out, *sink;
    CK(hipMalloc(&out, (n / kSub + 16) * 256 * 4));
    CK(hipMalloc(&sink, 64));
    run<uint8_t>("u8 random", n, 0, out, sink);
    run<uint8_t>("u8 runs4096", n, 1, out, sink);
    run<uint8_t>("u8 runs8-263", n, 2, out, sink);
    run<uint32_t>("u32 random", n, 0, out, sink);
    run<uint32_t>("u32 runs4096", n, 1, out, sink);
    run<uint32_t>("u32 runs8-263", n, 2, out, sink);
    return 0;
}
