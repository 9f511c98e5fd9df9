// Ceiling of the radix scatter's write pattern on this GPU (measurement tool,
// not product code): 100M (key, value) u32 pairs, read once and written once
// (1.6 GB), as
//   copy     : streaming 16-byte copy (the HBM ceiling of the same bytes)
//   runs     : what one LSD pass writes with uniform digits: every 8192-pair
//              tile sends 256 runs of 32 pairs to 256 buckets, run t of bucket
//              d at d * ntiles * 32 + t * 32 (+ `skew` elements per bucket, so
//              runs straddle 128-B lines as in a real pass); _xcd: tiles mapped
//              to blocks as the product's scatter does (xcd_tile)
// Each timed 20 times after 3 warm-ups; prints one JSON line.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/scatter_ceiling tools/scatter_ceiling.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr int kTile = 8192, kBlock = 512, kItems = kTile / kBlock;

__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}

__device__ __forceinline__ int64_t xcd_tile(int64_t b, int64_t ntiles) {   // as csrc/device.h
    const int64_t q = ntiles / 8, r = ntiles % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// thread t of the tile holds elements j = i * 512 + t (coalesced), element j
// belongs to run j / 32 (digit d) at offset j % 32
template <int RL>
__global__ __launch_bounds__(kBlock) void k_runs(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                 uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                 int64_t ntiles, int64_t bucket, int xcd) {
    const int64_t t = xcd ? xcd_tile(blockIdx.x, ntiles) : blockIdx.x;
    uint32_t k[kItems], v[kItems];
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        k[i] = kin[t * kTile + i * kBlock + threadIdx.x];
        v[i] = vin[t * kTile + i * kBlock + threadIdx.x];
    }
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int j = i * kBlock + threadIdx.x;
        const int64_t p = (int64_t)(j / RL) * bucket + t * RL + (j % RL);
        kout[p] = k[i];
        vout[p] = v[i];
    }
}

int main(int argc, char **argv) {
    const int64_t ntiles = 12207, n = ntiles * kTile;
    uint32_t *kin, *vin, *kout, *vout;
    const int64_t skew = 7;
    const int64_t bucket = ntiles * 32 + skew;
    const size_t outn = (size_t)(256 * bucket + 64);
    CK(hipMalloc(&kin, n * 4));
    CK(hipMalloc(&vin, n * 4));
    CK(hipMalloc(&kout, outn * 4));
    CK(hipMalloc(&vout, outn * 4));
    CK(hipMemset(kin, 1, n * 4));
    CK(hipMemset(vin, 2, n * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipEventRecord(a));
        for (int r = 0; r < 20; ++r) launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / 20.0;
    };
    const double bytes = (double)n * 16.0;
    const double t_copy = time([&] {
        k_copy<<<4096, 256>>>((const uint4 *)kin, (uint4 *)kout, n / 4);
        k_copy<<<4096, 256>>>((const uint4 *)vin, (uint4 *)vout, n / 4);
    });
    const double t_runs_aligned = time([&] {
        k_runs<32><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, ntiles * 32, 0);
    });
    const double t_runs_skew = time([&] {
        k_runs<32><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, bucket, 0);
    });
    const double t_runs_skew_xcd = time([&] {
        k_runs<32><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, bucket, 1);
    });
    const double t_runs_aligned_xcd = time([&] {
        k_runs<32><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, ntiles * 32, 1);
    });
    // runs of 64 (128 buckets per tile: what 16384-pair tiles give with 256 buckets)
    const int64_t bucket64 = ntiles * 64 + skew;
    const double t_runs64_skew_xcd = time([&] {
        k_runs<64><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, bucket64, 1);
    });
    const int64_t bucket128 = ntiles * 128 + skew;
    const double t_runs128_skew_xcd = time([&] {
        k_runs<128><<<ntiles, kBlock>>>(kin, vin, kout, vout, ntiles, bucket128, 1);
    });
    std::fprintf(stderr, "runs64_skew_xcd %.3f TB/s, runs128_skew_xcd %.3f TB/s\n", bytes / t_runs64_skew_xcd / 1e9,
                 bytes / t_runs128_skew_xcd / 1e9);
    CK(hipGetLastError());
    std::printf("{\"pairs\": %lld, \"bytes\": %.0f, \"copy_ms\": %.4f, \"copy_tbs\": %.3f, \"runs_aligned_ms\": %.4f, "
                "\"runs_aligned_tbs\": %.3f, \"runs_skew_ms\": %.4f, \"runs_skew_tbs\": %.3f, \"runs_skew_xcd_tbs\": %.3f, "
                "\"runs_aligned_xcd_tbs\": %.3f}\n",
                (long long)n, bytes, t_copy, bytes / t_copy / 1e9, t_runs_aligned, bytes / t_runs_aligned / 1e9,
                t_runs_skew, bytes / t_runs_skew / 1e9, bytes / t_runs_skew_xcd / 1e9, bytes / t_runs_aligned_xcd / 1e9);
    return 0;
}
