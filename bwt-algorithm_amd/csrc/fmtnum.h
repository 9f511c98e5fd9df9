// fmtnum.h -- printf's fixed-point formatting of non-negative doubles without
// printf, for the row formatters (render.cpp).  Python formats f"{x:.2f}" and
// "%.2f" % x like glibc: the exact binary value of x, rounded half to even at
// the last digit.  Here x = M * 2^E exactly (M < 2^53), so x * 10^p = M * 10^p
// * 2^E is split into an integer part and a remainder with 128-bit integers
// and rounded the same way.  tools/fmtnum_check.cpp compares it with snprintf.
#pragma once

#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace bwtmi {

constexpr char kDigits2[201] =
    "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
    "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
    "8081828384858687888990919293949596979899";

// decimal digits of x at out (>= 21 bytes); returns the end (std::to_chars' output)
inline char *int_dec(int64_t x, char *out) {
    static constexpr uint64_t kPow10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull,
                                            10000000ull, 100000000ull, 1000000000ull, 10000000000ull,
                                            100000000000ull, 1000000000000ull, 10000000000000ull,
                                            100000000000000ull, 1000000000000000ull, 10000000000000000ull,
                                            100000000000000000ull, 1000000000000000000ull,
                                            10000000000000000000ull};
    uint64_t v = (uint64_t)x;
    if (x < 0) {
        *out++ = '-';
        v = 0 - v;
    }
    const int lg = (64 - __builtin_clzll(v | 1)) * 1233 >> 12;   // floor(log10) of the bit length's power
    int n = lg + (v >= kPow10[lg] ? 1 : 0);
    if (n == 0) n = 1;
    char *p = out + n;
    while (v >= 100) {   // two digits a step from the end
        const uint64_t q = v / 100;
        p -= 2;
        std::memcpy(p, kDigits2 + 2 * (v - 100 * q), 2);
        v = q;
    }
    if (v >= 10) {
        p -= 2;
        std::memcpy(p, kDigits2 + 2 * v, 2);
    } else {
        *--p = (char)('0' + v);
    }
    return out + n;
}

// "%.<p>f" of x into out (>= 40 bytes), p in 0..3; returns the end, or nullptr
// when x is outside [0, 1e12) or not finite (the caller uses snprintf)
inline char *fixed_dec(double x, int p, char *out) {
    static const uint64_t S[4] = {1, 10, 100, 1000};
    if (!(x >= 0.0) || !(x < 1e12) || p < 0 || p > 3) return nullptr;
    uint64_t q = 0;
    if (x > 0.0) {
        int e;
        const double m = std::frexp(x, &e);                 // x = m * 2^e, 0.5 <= m < 1
        const uint64_t M = (uint64_t)std::ldexp(m, 53);     // exact: 2^52 <= M < 2^53
        const int k = 53 - e;                               // x = M / 2^k, k > 0 for x < 2^52
        const unsigned __int128 N = (unsigned __int128)M * S[p];   // < 2^63
        if (k < 127) {
            q = (uint64_t)(N >> k);
            const unsigned __int128 r = N - ((unsigned __int128)q << k), half = (unsigned __int128)1 << (k - 1);
            if (r > half || (r == half && (q & 1u))) ++q;
        }
    }
    char *w = std::to_chars(out, out + 24, q / S[p]).ptr;
    if (p > 0) {
        *w++ = '.';
        uint64_t f = q % S[p];
        for (int d = p - 1; d >= 0; --d) {
            w[d] = (char)('0' + f % 10);
            f /= 10;
        }
        w += p;
    }
    return w;
}

}  // namespace bwtmi
