// fixed_dec (csrc/fmtnum.h) against snprintf("%.<p>f") on values the writers
// meet (ratios of small integers, halves, binary-midpoint cases) and random doubles.
// build: g++ -O2 -std=c++17 tools/fmtnum_check.cpp -o /tmp/fmtnum_check && /tmp/fmtnum_check
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#include "../bwt-algorithm_amd/csrc/fmtnum.h"

int main() {
    std::mt19937_64 g(7);
    long checked = 0, bad = 0;
    auto check = [&](double x) {
        for (int p = 0; p <= 3; ++p) {
            char a[64], b[64];
            const int n = snprintf(a, sizeof a, "%.*f", p, x);
            char *e = bwtmi::fixed_dec(x, p, b);
            if (!e) continue;
            ++checked;
            if ((int)(e - b) != n || std::memcmp(a, b, (size_t)n) != 0) {
                if (++bad < 20) std::printf("MISMATCH p=%d x=%.17g printf=%s mine=%.*s\n", p, x, a, (int)(e - b), b);
            }
        }
    };
    for (int num = 0; num <= 20000; ++num)
        for (int den = 1; den <= 300; ++den) check((double)num / (double)den);
    for (int k = 0; k < 2000000; ++k) {
        check(std::uniform_real_distribution<double>(0, 1000)(g));
        check((double)(g() % 100000) / 1000.0 + 0.0005);
        check((double)(g() % 2000000) / 8.0);
        check(std::ldexp((double)(g() >> 11), -(int)(g() % 80)));
    }
    auto icheck = [&](int64_t v) {
        char a[32], b[32];
        char *ea = std::to_chars(a, a + 32, v).ptr, *eb = bwtmi::int_dec(v, b);
        ++checked;
        if (ea - a != eb - b || std::memcmp(a, b, (size_t)(ea - a)) != 0) {
            if (++bad < 20) std::printf("INT MISMATCH %lld\n", (long long)v);
        }
    };
    for (int64_t v = -100000; v <= 2000000; ++v) icheck(v);
    for (int s = 0; s < 63; ++s)
        for (int64_t d = -3; d <= 3; ++d) {
            icheck((int64_t(1) << s) + d);
            icheck(-(int64_t(1) << s) + d);
        }
    int64_t p = 1;
    for (int s = 0; s < 19; ++s, p *= 10)
        for (int64_t d = -2; d <= 2; ++d) icheck(p + d);
    icheck(INT64_MAX);
    icheck(INT64_MIN);
    for (int k = 0; k < 4000000; ++k) icheck((int64_t)g() >> (g() % 64));
    check(0.0); check(0.125); check(0.375); check(2.675); check(1.005); check(1e-300); check(999999999999.995);
    std::printf("%ld checked, %ld mismatches\n", checked, bad);
    return bad != 0;
}
