// Replays the merge fold's DP recomputes (BWTMI_DUMP_RECOMPUTE=path dumps
// "start end m min_copies" per call, trimmed coordinates) against the contig
// sequence through bwtmi::align_repeat_region, as post.cpp's recompute calls
// it, and reports ns per call by motif length.  Host-only (no GPU).
//   g++ -O2 -std=c++17 tools/recompute_bench.cpp -Ibwt-algorithm_amd/csrc \
//       -Lbwt-algorithm_amd -lbwtmi -Wl,-rpath,$PWD/bwt-algorithm_amd -o /tmp/rcb
//   /tmp/rcb SEQ.bin ARGS.txt [reps]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "common.h"

extern "C" int sampler_start(int hz) __attribute__((weak));
extern "C" int sampler_stop(const char *path) __attribute__((weak));

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    FILE *f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::string seq;
    char buf[1 << 16];
    size_t r;
    while ((r = std::fread(buf, 1, sizeof buf, f)) > 0) seq.append(buf, r);
    std::fclose(f);
    struct A { long long s, e, m, mc; };
    std::vector<A> args;
    FILE *g = std::fopen(argv[2], "r");
    A a;
    while (g && std::fscanf(g, "%lld %lld %lld %lld", &a.s, &a.e, &a.m, &a.mc) == 4) args.push_back(a);
    if (g) std::fclose(g);
    const int reps = argc > 3 ? std::atoi(argv[3]) : 5;
    const int64_t L = (int64_t)seq.size();
    std::map<int, std::pair<double, long>> by;   // log2 bucket of m -> (ns, calls)
    double tot = 0;
    long sink = 0, retries = 0;
    bwtmi::AlignScratch *ws = bwtmi::align_scratch_new();   // as post.cpp's workers hold it
    bwtmi::AlignSummary s;
    const char *prof = std::getenv("RCB_PROFILE");   // with tools/libsampler.so linked
    if (prof && sampler_start) sampler_start(4000);
    for (int rep = 0; rep < reps; ++rep) {
        for (const A &x : args) {
            s.want_copies = false;
            const auto t0 = std::chrono::steady_clock::now();
            std::string tmpl = seq.substr((size_t)x.s, (size_t)x.m);
            bool ok = bwtmi::align_repeat_region(seq.data(), L, x.s, x.e, tmpl, x.mc, s, 0.1, -1, ws);
            if (!ok) {
                ++retries;
                ok = bwtmi::align_repeat_region(seq.data(), L, x.s, x.e, tmpl, 1, s, 0.1, -1, ws);
            }
            const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
            sink += ok ? s.consumed : 0;
            if (rep == 0) continue;   // warm-up pass
            int b = 0;
            while ((1ll << (b + 1)) <= x.m) ++b;
            by[b].first += ns;
            by[b].second += 1;
            tot += ns;
        }
    }
    if (prof && sampler_stop) sampler_stop(prof);
    const long n = (long)args.size() * (reps - 1);
    std::printf("%zu recomputes x %d reps: %.0f ns/call (sink %ld), %.1f%% retried with min_copies 1\n", args.size(),
                reps - 1, tot / n, sink, 100.0 * retries / ((double)args.size() * reps));
    for (auto &kv : by)
        std::printf("  m %4d-%4d: %7ld calls %8.0f ns/call %5.1f%% of time\n", 1 << kv.first, (2 << kv.first) - 1,
                    kv.second.second / (reps - 1), kv.second.first / kv.second.second, 100.0 * kv.second.first / tot);
    return 0;
}
