// motif.cpp -- exact host restatement of the MotifUtils pieces on the CLI path.
// Float arithmetic follows the Python expressions operation by operation; the
// library is built with -ffp-contract=off so no FMA changes a rounding.
#include <immintrin.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace bwtmi {

// Least rotation (Booth).  MotifUtils.get_canonical_motif takes the min over
// all rotations (bwt.py:679-685); the least rotation string is unique, so any
// exact algorithm yields the same string.
// ss = s + s (2n bytes)
static int64_t least_rotation(const unsigned char *ss, int64_t n, std::vector<int32_t> &f) {
    if (n <= 1) return 0;
    if (n <= 16) {   // short motifs: direct comparison of the n rotations
        int64_t k = 0;
        for (int64_t j = 1; j < n; ++j)
            if (std::memcmp(ss + j, ss + k, (size_t)n) < 0) k = j;
        return k;
    }
    f.assign((size_t)(2 * n), -1);
    int64_t k = 0;
    for (int64_t j = 1; j < 2 * n; ++j) {
        const unsigned char sj = ss[j];
        int64_t i = f[(size_t)(j - k - 1)];
        while (i != -1 && sj != ss[k + i + 1]) {
            if (sj < ss[k + i + 1]) k = j - i - 1;
            i = f[(size_t)i];
        }
        if (sj != ss[k + i + 1]) {  // i == -1
            if (sj < ss[k]) k = j;
            f[(size_t)(j - k)] = -1;
        } else {
            f[(size_t)(j - k)] = (int32_t)(i + 1);
        }
    }
    return k % n;
}

std::string min_rotation(const std::string &s) {
    thread_local std::vector<int32_t> f;
    thread_local std::string ss;
    ss.assign(s).append(s);
    const int64_t k = least_rotation((const unsigned char *)ss.data(), (int64_t)s.size(), f);
    return ss.substr((size_t)k, s.size());
}

static inline char comp_base(char c) {       // bwt.py:688-691
    switch (c) {
        case 'A': return 'T';
        case 'T': return 'A';
        case 'C': return 'G';
        case 'G': return 'C';
        default: return c;  // 'N' -> 'N', anything else unchanged
    }
}

// 2-bit code of a byte (A0 C1 G2 T3), 4 for every other byte
static const struct Code2 {
    uint8_t v[256];
    Code2() {
        for (int b = 0; b < 256; ++b) v[b] = 4;
        v['A'] = 0;
        v['C'] = 1;
        v['G'] = 2;
        v['T'] = 3;
    }
} kCode2;

bool pack2_acgt(const char *s, int64_t n, uint64_t &x) {
    if (n > 32) return false;
    uint64_t y = 0;
    unsigned bad = 0;
    for (int64_t i = 0; i < n; ++i) {   // branch-free: the invalid bit is checked once
        const unsigned c = kCode2.v[(uint8_t)s[i]];
        bad |= c;
        y = (y << 2) | (c & 3u);
    }
    x = y;
    return (bad & 4u) == 0;
}

// canonical word of an ACGT motif of 33..64 bases (least rotation of the
// motif and of its reverse complement, as 128-bit 2-bit words)
bool canon_key128(const char *s, int64_t n, unsigned __int128 &key);

uint64_t rc2(uint64_t x, int64_t n) {
    x = ~x;   // complement: 3 - code
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0f0f0f0f0f0f0f0full) | ((x & 0x0f0f0f0f0f0f0f0full) << 4);
    x = __builtin_bswap64(x);   // 2-bit groups reversed over the whole word
    return n ? x >> (64 - 2 * n) : 0;
}

uint64_t min_rot2(uint64_t x, int64_t n) {
    if (n <= 1) return x;
    const int bits = (int)(2 * n);
    const uint64_t mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
    uint64_t best = x;
    for (int sh = 2; sh < bits; sh += 2) {
        const uint64_t r = ((x << sh) | (x >> (bits - sh))) & mask;
        best = r < best ? r : best;
    }
    return best;
}

// [n][x], n = 1..8: the canonical word (low 16 bits) and whether the forward
// strand holds it (bit 16: min_rot2(x) <= min_rot2(rc2(x)))
static const std::vector<uint32_t> *canon_table() {
    static const std::vector<uint32_t> *tab = [] {
        auto *t = new std::vector<uint32_t>[9];
        for (int k = 1; k <= 8; ++k) {
            t[k].resize((size_t)1 << (2 * k));
            for (uint64_t v = 0; v < t[k].size(); ++v) {
                const uint64_t f = min_rot2(v, k), r = min_rot2(rc2(v, k), k);
                t[k][v] = (uint32_t)(f < r ? f : r) | (f <= r ? 1u << 16 : 0u);
            }
        }
        return t;
    }();
    return tab;
}

uint64_t canon2(uint64_t x, int64_t n) {
    if (n >= 1 && n <= 8) return canon_table()[n][(size_t)x] & 0xffffu;
    const uint64_t f = min_rot2(x, n), r = min_rot2(rc2(x, n), n);
    return f < r ? f : r;
}

// 33..64 bases: the same over 128-bit words
typedef unsigned __int128 u128;
static bool pack2_acgt128(const char *s, int64_t n, u128 &x) {
    uint64_t hi, lo;
    if (n <= 32 || n > 64 || !pack2_acgt(s, n - 32, hi) || !pack2_acgt(s + (n - 32), 32, lo)) return false;
    x = ((u128)hi << 64) | lo;
    return true;
}
static u128 rc2_128(u128 x, int64_t n) {
    const uint64_t hi = (uint64_t)(x >> 64), lo = (uint64_t)x;   // hi: first n-32 bases, lo: last 32
    // reverse complement: rc(lo) (32 bases) first, then rc(hi) (n-32 bases)
    return ((u128)rc2(lo, 32) << (2 * (n - 32))) | rc2(hi, n - 32);
}
static u128 min_rot2_128(u128 x, int64_t n) {
    const int bits = (int)(2 * n);
    const u128 mask = bits == 128 ? ~(u128)0 : (((u128)1 << bits) - 1);
    u128 best = x;
    for (int sh = 2; sh < bits; sh += 2) {
        const u128 r = ((x << sh) | (x >> (bits - sh))) & mask;
        best = r < best ? r : best;
    }
    return best;
}

bool canon_key128(const char *s, int64_t n, unsigned __int128 &key) {
    u128 y;
    if (!pack2_acgt128(s, n, y)) return false;
    const u128 f = min_rot2_128(y, n), r = min_rot2_128(rc2_128(y, n), n);
    key = f < r ? f : r;
    return true;
}

void canonical_stranded(const std::string &s, std::string &canon, char &strand) {  // 694-716
    const int64_t n = (int64_t)s.size();
    if (n == 0) {
        canon.clear();
        strand = '+';
        return;
    }
    uint64_t x;
    if (pack2_acgt(s.data(), n, x)) {   // least rotations of s and rc(s) over packed words
        const uint64_t bf = min_rot2(x, n), br = min_rot2(rc2(x, n), n);
        const bool fwd = bf <= br;
        const uint64_t v = fwd ? bf : br;
        canon.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) canon[(size_t)i] = "ACGT"[(v >> (2 * (n - 1 - i))) & 3u];
        strand = fwd ? '+' : '-';
        return;
    }
    u128 y;
    if (pack2_acgt128(s.data(), n, y)) {
        const u128 bf = min_rot2_128(y, n), br = min_rot2_128(rc2_128(y, n), n);
        const bool fwd = bf <= br;
        const u128 v = fwd ? bf : br;
        canon.resize((size_t)n);
        for (int64_t i = 0; i < n; ++i) canon[(size_t)i] = "ACGT"[(unsigned)(v >> (2 * (n - 1 - i))) & 3u];
        strand = fwd ? '+' : '-';
        return;
    }
    thread_local std::vector<int32_t> f;
    thread_local std::string ss, rr;   // s+s and rc+rc: every rotation is a plain slice
    ss.resize((size_t)(2 * n));
    rr.resize((size_t)(2 * n));
    for (int64_t i = 0; i < n; ++i) {
        ss[(size_t)i] = ss[(size_t)(i + n)] = s[(size_t)i];
        rr[(size_t)i] = rr[(size_t)(i + n)] = comp_base(s[(size_t)(n - 1 - i)]);
    }
    const int64_t kf = least_rotation((const unsigned char *)ss.data(), n, f);
    const int64_t kr = least_rotation((const unsigned char *)rr.data(), n, f);
    const bool fwd = std::memcmp(ss.data() + kf, rr.data() + kr, (size_t)n) <= 0;
    canon.assign((fwd ? ss.data() + kf : rr.data() + kr), (size_t)n);
    strand = fwd ? '+' : '-';
}

char canonical_strand(const char *s, int64_t n) {
    uint64_t x;
    if (n > 0 && pack2_acgt(s, n, x)) {
        if (n <= 8) return (canon_table()[n][(size_t)x] >> 16) ? '+' : '-';
        return min_rot2(x, n) <= min_rot2(rc2(x, n), n) ? '+' : '-';
    }
    u128 y;
    if (pack2_acgt128(s, n, y)) return min_rot2_128(y, n) <= min_rot2_128(rc2_128(y, n), n) ? '+' : '-';
    thread_local std::string t, c;
    t.assign(s, (size_t)n);
    char st;
    canonical_stranded(t, c, st);
    return st;
}

int64_t smallest_period(const char *s, int64_t n) {   // bwt.py:1125-1133
    if (n <= 0) return 0;
    for (int64_t p = 1; p <= n; ++p) {
        if (n % p) continue;
        int64_t k = p;
        while (k < n && s[k] == s[k - p]) ++k;
        if (k == n) return p;
    }
    return n;
}

double entropy_of(const char *s, int64_t n) {         // bwt.py:730-745
    if (n <= 0) return 0.0;
    if (n <= 64) {   // short motifs: a first-seen list instead of clearing 256 counters per call
        unsigned char sym[64];
        int64_t c[64];
        int m = 0;
        for (int64_t i = 0; i < n; ++i) {
            const unsigned char ch = (unsigned char)s[i];
            int j = 0;
            while (j < m && sym[j] != ch) ++j;
            if (j == m) {
                sym[m] = ch;
                c[m++] = 0;
            }
            ++c[j];
        }
        double e = 0.0;
        for (int k = 0; k < m; ++k) {
            double p = (double)c[k] / (double)n;
            e -= p * std::log2(p);
        }
        return e;
    }
    int64_t cnt[256] = {0};
    unsigned char order[256];
    int nord = 0;
    for (int64_t i = 0; i < n; ++i) {
        unsigned char c = (unsigned char)s[i];
        if (cnt[c]++ == 0) order[nord++] = c;   // Counter keeps first-seen order
    }
    double e = 0.0;
    for (int k = 0; k < nord; ++k) {
        double p = (double)cnt[order[k]] / (double)n;
        e -= p * std::log2(p);
    }
    return e;
}

void composition_of(const char *s, int64_t n, double out[4]) {   // bwt.py:1290-1310
    if (n <= 0) {
        out[0] = out[1] = out[2] = out[3] = 0.0;
        return;
    }
    int64_t a = 0, c = 0, g = 0, t = 0;
    for (int64_t i = 0; i < n; ++i) {
        char x = s[i];
        if (x >= 'a' && x <= 'z') x = (char)(x - 32);
        a += x == 'A';
        c += x == 'C';
        g += x == 'G';
        t += x == 'T';
    }
    const double tot = (double)n;
    out[0] = ((double)a / tot) * 100.0;
    out[1] = ((double)c / tot) * 100.0;
    out[2] = ((double)g / tot) * 100.0;
    out[3] = ((double)t / tot) * 100.0;
}

int64_t trf_score(int64_t length, double mm) {      // bwt.py:1313-1333
    double matches = (double)length * (1.0 - mm);
    double mism = (double)length * mm;
    double v = (matches * 2.0) - (mism * 7.0);
    int64_t s = (int64_t)v;  // int() truncates toward zero
    return s < 0 ? 0 : s;
}

// ------------------------------------------------------------------------
// MotifUtils._align_unit_to_window (bwt.py:829-983) and align_repeat_region
// (998-1102).  Banded storage: row i keeps columns i-band..i+band; cells
// outside the computed band read as the reference's `inf`, row 0 / column 0
// hold its initialisation.  Ties keep sub > del > ins.  All scratch is
// thread-local and reused: no allocation per copy.
// ------------------------------------------------------------------------
namespace {

struct Scratch {
    std::vector<int32_t> cost;
    std::vector<unsigned char> wpad;           // the window with 64 bytes of 0xff on each side
    std::vector<char> ptr;
    std::vector<char> cref, cqry;              // aligned columns (reversed)
    std::vector<int64_t> obs_idx;              // observed bases of the current copy
    std::vector<char> obs_base;
    std::string ops;                           // formatted ops of the current copy ("" parts)
    std::vector<uint32_t> op_end;              // piece boundaries in ops
    // per-position Counter in insertion order: up to 8 inline entries, overflow vector
    std::vector<char> pc_c;
    std::vector<int64_t> pc_n;
    std::vector<uint8_t> pc_k;
    std::vector<std::vector<std::pair<char, int64_t>>> pc_over;
};

constexpr int KIN = 8;

struct UnitOut {
    int64_t consumed = 0, n_sub = 0, n_ins = 0, n_del = 0;
};

inline void put_num(std::string &s, int64_t v) {
    char b[24];
    const auto r = std::to_chars(b, b + sizeof b, v);
    s.append(b, (size_t)(r.ptr - b));
}

template <typename CostF>
bool finish_unit(const char *motif, int64_t m, const char *win, int64_t n, int64_t lower, int64_t upper,
                 int64_t band, int64_t W, int32_t INF, int64_t tol, int64_t max_indel, CostF cost, Scratch &S,
                 UnitOut &res);

// The banded DP of align_unit in diagonal coordinates, one AVX-512 register
// per row: cell (i, j) sits in lane d = j - i + band (W = 2 band + 1 <= 25 of
// 32 lanes), so the diagonal neighbour is lane d of the previous row, the one
// above is lane d + 1 and the left one lane d - 1.  Substitution/deletion are
// lane-parallel; the insertion chain cur[j] = min(base[j], cur[j-1] + 1) is a
// prefix minimum of base[d] - d (5 shift/min steps).  Choices and tie order are
// the scalar loop's: match/sub, then deletion if strictly cheaper, then
// insertion if strictly cheaper.  ptr rows get the same codes at the same
// offsets (row i at i*W, 32 bytes written per row: rows are written in order
// and the buffer has 32 bytes of slack).  Returns 0 = reject (the row-min
// test), 1 = done; last[d] = row m.
__attribute__((target("avx512f,avx512bw,avx512vl"))) static int dp_rows_avx512(
    const char *motif, int64_t m, const unsigned char *wp, int64_t n, int64_t band, int32_t INF, int32_t reject,
    char *ptr, int64_t W, int16_t *last) {
    const __m512i iota = _mm512_set_epi16(31, 30, 29, 28, 27, 26, 25, 24, 23, 22, 21, 20, 19, 18, 17, 16, 15, 14, 13,
                                          12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    const __m512i inf = _mm512_set1_epi16((int16_t)INF), one = _mm512_set1_epi16(1);
    const __m512i up_idx = _mm512_add_epi16(iota, one);   // lane d <- lane d + 1 (lane 31 masked)
    __m512i sh_idx[5];
    __mmask32 sh_mask[5];
    for (int q = 0; q < 5; ++q) {   // lane d <- lane d - 2^q
        sh_idx[q] = _mm512_sub_epi16(iota, _mm512_set1_epi16((int16_t)(1 << q)));
        sh_mask[q] = (__mmask32)(0xffffffffu << (1 << q));
    }
    int nsteps = 0;
    while (nsteps < 5 && (1 << nsteps) < W) ++nsteps;
    const __m512i cS = _mm512_set1_epi16('S'), cM = _mm512_set1_epi16('M'), cD = _mm512_set1_epi16('D'),
                  cI = _mm512_set1_epi16('I');
    // row 0: cost j for j in [0, n] (every column), lane d -> j = d - band
    const __m512i j0 = _mm512_sub_epi16(iota, _mm512_set1_epi16((int16_t)band));
    const __mmask32 r0 = _mm512_cmpge_epi16_mask(j0, _mm512_setzero_si512()) &
                         _mm512_cmple_epi16_mask(j0, _mm512_set1_epi16((int16_t)n));
    __m512i prev = _mm512_mask_mov_epi16(inf, r0, j0);
    for (int64_t i = 1; i <= m; ++i) {
        const int64_t jmin = std::max<int64_t>(1, i - band), jmax = std::min<int64_t>(n, i + band);
        const int64_t dlo = jmin - i + band, dhi = jmax - i + band;
        __mmask32 valid = dhi >= dlo ? (__mmask32)(((1ull << (dhi + 1)) - 1) & ~((1ull << dlo) - 1)) : 0;
        // text: lane d compares win[j - 1] = wp[i - band - 1 + d]
        const __m512i tv = _mm512_cvtepu8_epi16(_mm256_loadu_si256((const __m256i *)(wp + (i - band - 1))));
        const __mmask32 eq = _mm512_cmpeq_epi16_mask(tv, _mm512_set1_epi16((int16_t)(unsigned char)motif[i - 1]));
        const __m512i p1 = _mm512_add_epi16(prev, one);
        const __m512i sub = _mm512_mask_mov_epi16(p1, eq, prev);
        const __m512i up = _mm512_mask_permutexvar_epi16(inf, (__mmask32)0x7fffffffu, up_idx, prev);
        const __m512i dc = _mm512_add_epi16(up, one);
        const __mmask32 isD = _mm512_cmplt_epi16_mask(dc, sub);
        __m512i base = _mm512_mask_mov_epi16(inf, valid, _mm512_min_epi16(sub, dc));
        __mmask32 keep = valid;
        if (i <= band) {   // column 0 (j = 0): cost i, the left end of the chain
            const __mmask32 c0 = (__mmask32)(1u << (band - i));
            base = _mm512_mask_mov_epi16(base, c0, _mm512_set1_epi16((int16_t)i));
            keep |= c0;
        }
        __m512i t = _mm512_sub_epi16(base, iota);
        // row band + 1: column 0 (cost i) is the left neighbour of lane 0 --
        // the scalar loop's cur[jmin - 1] -- one lane below the register
        if (i == band + 1) t = _mm512_min_epi16(t, _mm512_set1_epi16((int16_t)(i + 1)));
        for (int q = 0; q < nsteps; ++q)   // ceil(log2 W) doubling steps cover the band
            t = _mm512_min_epi16(t, _mm512_mask_permutexvar_epi16(inf, sh_mask[q], sh_idx[q], t));
        const __m512i fin = _mm512_mask_mov_epi16(inf, keep, _mm512_add_epi16(t, iota));
        const __mmask32 isI = _mm512_cmplt_epi16_mask(fin, base) & valid;
        __m512i code = _mm512_mask_mov_epi16(cS, eq, cM);
        code = _mm512_mask_mov_epi16(code, isD, cD);
        code = _mm512_mask_mov_epi16(code, isI, cI);
        _mm256_storeu_si256((__m256i *)(ptr + i * W), _mm512_cvtepi16_epi8(code));
        // row minimum over the band (INF elsewhere)
        const __m512i fv = _mm512_mask_mov_epi16(inf, valid, fin);
        __m256i h = _mm256_min_epu16(_mm512_castsi512_si256(fv), _mm512_extracti64x4_epi64(fv, 1));
        __m128i h2 = _mm_min_epu16(_mm256_castsi256_si128(h), _mm256_extracti128_si256(h, 1));
        const int32_t rowmin = (int32_t)(uint16_t)_mm_cvtsi128_si32(_mm_minpos_epu16(h2));
        if (rowmin > reject && (jmin > 1 || i > reject)) return 0;
        prev = fin;
    }
    _mm512_storeu_si512((void *)last, prev);
    return 1;
}

// the CPU feature test is cached; the switch is read at every call (a
// namespace-scope initialiser could run before knobs.cpp has read the
// environment, and bwtmi_knob_set must take effect in-process)
static const bool g_cpu_avx512 = [] {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("avx512vl");
}();
static inline bool use_avx512() { return g_cpu_avx512 && !knob(KN_NO_AVX512); }

// ops of one copy are formatted with a placeholder-free prefix; the copy index
// is prepended when the copy is accepted (ops hold "pos:..." pieces)
bool align_unit(const char *motif, int64_t m, const char *win, int64_t n, int64_t max_indel, int64_t tol,
                Scratch &S, UnitOut &res) {
    if (m == 0 || n == 0) return false;
    max_indel = std::max<int64_t>(0, max_indel);
    tol = std::max<int64_t>(0, tol);
    const int64_t lower = std::max<int64_t>(0, m - max_indel);
    const int64_t upper = std::min<int64_t>(n, m + max_indel);
    if (lower > upper) return false;
    // Every in-band cell is finite (<= i + j), so the reference's `inf` only
    // has to lose every comparison: two rolling rows indexed by column, with
    // the out-of-band neighbours (left of jmin, right of the previous row's
    // jmax) set to INF, make the recurrence branch-free.
    const int32_t INF = (int32_t)(m + n + 10);
    const int64_t band = max_indel + 2;
    const int64_t W = 2 * band + 1;
    const size_t cells = (size_t)((m + 1) * W) + 32;
    if (S.ptr.size() < cells) S.ptr.resize(cells);
    const int32_t reject = (int32_t)(tol + 2 * max_indel);
    if (use_avx512() && W <= 31 && INF < 30000) {
        // 64 bytes of never-matching padding on both sides of the window
        if (S.wpad.size() < (size_t)(n + 128)) S.wpad.resize((size_t)(n + 128));
        std::memset(S.wpad.data(), 0xff, 64);
        std::memcpy(S.wpad.data() + 64, win, (size_t)n);
        std::memset(S.wpad.data() + 64 + n, 0xff, 64);
        alignas(64) int16_t last[32];
        if (!dp_rows_avx512(motif, m, S.wpad.data() + 64, n, band, INF, reject, S.ptr.data(), W, last)) return false;
        return finish_unit(motif, m, win, n, lower, upper, band, W, INF, tol, max_indel,
                           [&](int64_t j) -> int64_t { return last[j - m + band]; }, S, res);
    }
    if (S.cost.size() < (size_t)(2 * (n + 2))) S.cost.resize((size_t)(2 * (n + 2)));
    char *ptr = S.ptr.data();
    int32_t *prev = S.cost.data(), *cur = prev + (n + 2);
    for (int64_t j = 0; j <= n; ++j) prev[j] = (int32_t)j;   // row 0
    prev[n + 1] = INF;
    int64_t pjmax = n;                                        // row 0 spans every column
    // costs never decrease along a path, so once a whole row exceeds
    // tol + 2*max_indel every alignment has n_sub > tol or an indel count
    // > max_indel, and the copy is rejected below anyway
    for (int64_t i = 1; i <= m; ++i) {
        const int64_t jmin = std::max<int64_t>(1, i - band), jmax = std::min<int64_t>(n, i + band);
        const char mi = motif[i - 1];
        char *prow = ptr + i * W + band - i;
        if (pjmax + 1 <= n) prev[pjmax + 1] = INF;            // (i-1, i-1+band+1) is out of band
        cur[jmin - 1] = jmin - 1 == 0 ? (int32_t)i : INF;
        // two passes over the band: the diagonal/deletion choice has no
        // dependence along the row (vectorisable); the insertion choice
        // (cur[j-1] + 1 strictly better) is the only serial chain.  Same tie
        // order as one pass: sub/match, then deletion, then insertion.
        const int32_t *pv = prev, *pw = prev;   // prev[j - 1], prev[j]
        int32_t *cw = cur;
        const char *wj = win - 1;               // win[j - 1]
        for (int64_t j = jmin; j <= jmax; ++j) {
            const int32_t sub = pv[j - 1] + (mi == wj[j] ? 0 : 1);
            const int32_t dc = pw[j] + 1;
            cw[j] = dc < sub ? dc : sub;
            prow[j] = dc < sub ? 'D' : (mi == wj[j] ? 'M' : 'S');
        }
        int32_t rowmin = INF, left = cur[jmin - 1];
        for (int64_t j = jmin; j <= jmax; ++j) {
            int32_t best = cur[j];
            if (left + 1 < best) {
                best = left + 1;
                prow[j] = 'I';
                cur[j] = best;
            }
            left = best;
            rowmin = std::min(rowmin, best);
        }
        if (rowmin > reject && (jmin > 1 || i > reject)) return false;
        pjmax = jmax;
        std::swap(prev, cur);
    }
    // prev = row m over [max(1, m-band), min(n, m+band)]; column 0 reads m
    return finish_unit(motif, m, win, n, lower, upper, band, W, INF, tol, max_indel,
                       [&](int64_t j) -> int64_t { return j == 0 ? m : prev[j]; }, S, res);
}

// best end column on row m (first minimum in [lower, upper]), traceback and
// the copy's ops / observed bases / acceptance (cost(j) = row m, column j)
template <typename CostF>
bool finish_unit(const char *motif, int64_t m, const char *win, int64_t n, int64_t lower, int64_t upper,
                 int64_t band, int64_t W, int32_t INF, int64_t tol, int64_t max_indel, CostF cost, Scratch &S,
                 UnitOut &res) {
    const char *ptr = S.ptr.data();
    int64_t bj = -1, bc = INF;
    for (int64_t j = lower; j <= upper; ++j) {
        const int64_t c = cost(j);
        if (c < bc) { bc = c; bj = j; }
    }
    if (bj <= 0 || bc >= INF) return false;
    // an accepted copy has n_sub <= tol and both indel counts <= max_indel, so
    // its cost (= bc) is at most tol + 2 max_indel: skip the traceback otherwise
    if (bc > tol + 2 * max_indel) return false;
    // traceback (columns collected in reverse, into buffers sized once: a path
    // has at most m + bj columns)
    if (S.cref.size() < (size_t)(m + bj + 1)) {
        S.cref.resize((size_t)(m + bj + 1));
        S.cqry.resize((size_t)(m + bj + 1));
    }
    char *cr = S.cref.data(), *cq = S.cqry.data();
    size_t nc = 0;
    int64_t i = m, j = bj;
    int64_t ns = 0, ni = 0, nd = 0;
    while (i > 0 || j > 0) {
        char op;
        if (i == 0) op = 'I';
        else if (j == 0) op = 'D';
        else if (j < i - band || j > i + band) op = 0;
        else op = ptr[i * W + (j - i + band)];
        if (op == 'M' || op == 'S') { cr[nc] = motif[i - 1]; cq[nc++] = win[j - 1]; ns += op == 'S'; --i; --j; }
        else if (op == 'D') { cr[nc] = motif[i - 1]; cq[nc++] = '-'; ++nd; --i; }
        else if (op == 'I') { cr[nc] = '-'; cq[nc++] = win[j - 1]; ++ni; --j; }
        else break;
    }
    // the copy tests below, decided before any op is formatted ('S' = a
    // mismatching diagonal step, 'D' / 'I' = one deleted / inserted base)
    if (ns > tol || ni > max_indel || nd > max_indel) return false;
    S.obs_idx.clear();
    S.obs_base.clear();
    S.ops.clear();
    S.op_end.clear();
    res.n_sub = res.n_ins = res.n_del = 0;
    int64_t ref = 0;
    size_t ins_from = 0;
    bool ins_open = false;
    int64_t ins_at = 0, del_len = 0, del_at = 0;
    std::string &o = S.ops;
    auto flush_ins = [&](size_t upto) {   // columns ins_from..upto-1 (forward order) are insertions
        o.push_back(':');
        put_num(o, ins_at);
        o.append(":ins(");
        for (size_t q = ins_from; q < upto; ++q) o.push_back(cq[nc - 1 - q]);
        o.push_back(')');
        S.op_end.push_back((uint32_t)o.size());
        res.n_ins += (int64_t)(upto - ins_from);
    };
    auto flush_del = [&]() {
        o.push_back(':');
        put_num(o, del_at);
        o.append(":del(");
        put_num(o, del_len);
        o.push_back(')');
        S.op_end.push_back((uint32_t)o.size());
        res.n_del += del_len;
    };
    const size_t ncols = nc;
    for (size_t q = 0; q < ncols; ++q) {
        const char r = cr[ncols - 1 - q], qq = cq[ncols - 1 - q];
        if (r == '-') {
            if (!ins_open) { ins_at = ref; ins_from = q; ins_open = true; }
            continue;
        }
        if (ins_open) { flush_ins(q); ins_open = false; ins_at = 0; }
        ++ref;
        if (qq == '-') {
            if (del_len == 0) del_at = ref;
            ++del_len;
            continue;
        }
        if (del_len) { flush_del(); del_len = 0; }
        S.obs_idx.push_back(ref - 1);
        S.obs_base.push_back(qq);
        if (r != qq) {
            o.push_back(':');
            put_num(o, ref);
            o.push_back(':');
            o.push_back(r);
            o.push_back('>');
            o.push_back(qq);
            S.op_end.push_back((uint32_t)o.size());
            ++res.n_sub;
        }
    }
    if (ins_open) flush_ins(ncols);
    if (del_len) flush_del();
    if (res.n_sub > tol) return false;
    if (res.n_ins > max_indel || res.n_del > max_indel) return false;
    res.consumed = bj;
    return true;
}

// only the entry counts need clearing: entries at or past pc_k[p] are never read
inline void pc_reset(Scratch &S, int64_t m) {
    if (S.pc_c.size() < (size_t)(m * KIN)) {
        S.pc_c.resize((size_t)(m * KIN));
        S.pc_n.resize((size_t)(m * KIN));
    }
    S.pc_k.assign((size_t)m, 0);
    if ((int64_t)S.pc_over.size() < m) S.pc_over.resize((size_t)m);
    for (int64_t p = 0; p < m; ++p) S.pc_over[(size_t)p].clear();
}

inline void pc_add(Scratch &S, int64_t p, char b, int64_t cnt = 1) {
    char *c = &S.pc_c[(size_t)(p * KIN)];
    int64_t *n = &S.pc_n[(size_t)(p * KIN)];
    const int k = S.pc_k[(size_t)p];
    for (int t = 0; t < k; ++t)
        if (c[t] == b) { n[t] += cnt; return; }
    auto &ov = S.pc_over[(size_t)p];
    for (auto &e : ov)
        if (e.first == b) { e.second += cnt; return; }
    if (k < KIN) { c[k] = b; n[k] = cnt; S.pc_k[(size_t)p] = (uint8_t)(k + 1); }
    else ov.push_back({b, cnt});
}

// Counter.most_common(1): first maximal entry in insertion order
inline bool pc_top(const Scratch &S, int64_t p, char &out) {
    const int k = S.pc_k[(size_t)p];
    if (k == 0) return false;
    const char *c = &S.pc_c[(size_t)(p * KIN)];
    const int64_t *n = &S.pc_n[(size_t)(p * KIN)];
    char b = c[0];
    int64_t best = n[0];
    for (int t = 1; t < k; ++t)
        if (n[t] > best) { best = n[t]; b = c[t]; }
    for (auto &e : S.pc_over[(size_t)p])
        if (e.second > best) { best = e.second; b = e.first; }
    out = b;
    return true;
}

void consensus_from(const Scratch &S, int64_t m, const std::string &fallback, std::string &out) {
    out.resize((size_t)m);
    for (int64_t i = 0; i < m; ++i) {
        char b;
        if (pc_top(S, i, b)) out[(size_t)i] = b;
        else out[(size_t)i] = (size_t)i < fallback.size() ? fallback[(size_t)i] : 'N';
    }
}

}  // namespace

int64_t run_end(const char *s, int64_t pos, int64_t lim, char b) {
    const __m256i vb = _mm256_set1_epi8(b);
    while (pos + 32 <= lim) {
        const uint32_t eq = (uint32_t)_mm256_movemask_epi8(
            _mm256_cmpeq_epi8(_mm256_loadu_si256(reinterpret_cast<const __m256i *>(s + pos)), vb));
        if (eq != 0xFFFFFFFFu) return pos + __builtin_ctz(~eq);
        pos += 32;
    }
    while (pos < lim && s[pos] == b) ++pos;
    return pos;
}

// A walk that stopped at its safety limit, kept for the next call with the
// same region start and template: the walk's states (positions, consensus
// counts, variations) do not depend on the limit, only where it stops does,
// so a call whose limit lies at or past the stop resumes from it instead of
// re-aligning every copy (the merge fold recomputes a growing region from one
// start once per chain step).
struct WalkState {
    bool valid = false;
    const char *seq = nullptr;
    int64_t seq_len = 0, start = 0, max_indel = 0, tol = 0, stop_limit = 0;
    std::string tmpl, cur, variations;
    int64_t pos = 0, copies = 0, tot_ins = 0, tot_del = 0, tot_err = 0, max_err = 0;
    bool any_variation = false, want_copies = false;
    std::vector<int64_t> copy_len, copy_err;
    std::vector<char> pc_c;
    std::vector<int64_t> pc_n;
    std::vector<uint8_t> pc_k;
    std::vector<std::vector<std::pair<char, int64_t>>> pc_over;
};

struct AlignScratch {
    Scratch S;
    std::string cur;
    WalkState saved;
};
AlignScratch *align_scratch_new() { return new AlignScratch(); }
void align_scratch_free(AlignScratch *w) { delete w; }

bool align_repeat_region(const char *seq, int64_t seq_len, int64_t start, int64_t end,
                         const std::string &tmpl, int64_t min_copies, AlignSummary &out, double frac,
                         int64_t max_indel_arg) {
    thread_local AlignScratch tls;
    return align_repeat_region(seq, seq_len, start, end, tmpl, min_copies, out, frac, max_indel_arg, &tls);
}

bool align_repeat_region(const char *seq, int64_t seq_len, int64_t start, int64_t end,
                         const std::string &tmpl, int64_t min_copies, AlignSummary &out, double frac,
                         int64_t max_indel_arg, AlignScratch *ws, bool resume) {
    if (tmpl.empty() || seq_len == 0) return false;
    start = std::max<int64_t>(0, start);
    end = std::min<int64_t>(seq_len, end > start ? end : seq_len);
    const int64_t m = (int64_t)tmpl.size();
    const int64_t tol = std::max<int64_t>(1, (int64_t)std::floor((double)m * frac));
    const int64_t max_indel = max_indel_arg < 0 ? std::max<int64_t>(1, std::min<int64_t>(10, m >= 4 ? m / 2 : 1))
                                                : max_indel_arg;
    if (m == 1 && max_indel >= 1) {
        // One-base motif: a window that differs from the consensus base has
        // the deletion end j = 0 among its best alignments (cost 1, tied with
        // the substitution, first j wins), so _align_unit_to_window reports
        // failure and the walk stops there.  The consensus never changes, so
        // the result is the run of the template base from start (up to limit).
        const int64_t limit = std::min<int64_t>(
            seq_len, std::max<int64_t>(end, start + min_copies) + std::max<int64_t>(3, max_indel * 4));
        const char b = tmpl[0];
        const int64_t pos = start < limit ? run_end(seq, start, limit, b) : start;
        const int64_t copies = pos - start;
        if (copies < min_copies || copies <= 0) return false;
        if (out.want_copies) {
            out.copy_len.assign((size_t)copies, 1);
            out.copy_err.assign((size_t)copies, 0);
        }
        out.variations.clear();
        out.any_variation = false;
        out.consensus.assign(1, b);
        out.at_limit = pos >= limit;
        out.motif_len = 1;
        out.copies = copies;
        out.consumed = copies;
        out.mismatch_rate = 0.0;
        out.max_errors = 0;
        out.tot_err = 0;
        out.tot_ins = 0;
        out.tot_del = 0;
        return true;
    }
    Scratch &S = ws->S;
    int64_t tot_ins = 0, tot_del = 0, tot_err = 0, max_err = 0;
    std::string &cur = ws->cur;
    int64_t pos = start;
    const int64_t limit = std::min<int64_t>(
        seq_len, std::max<int64_t>(end, start + m * min_copies) + std::max<int64_t>(m * 3, max_indel * 4));
    UnitOut res;
    int64_t copies = 0;
    WalkState &W = ws->saved;
    if (resume && W.valid && W.seq == seq && W.seq_len == seq_len && W.start == start && W.max_indel == max_indel &&
        W.tol == tol && W.want_copies == out.want_copies && limit >= W.stop_limit && W.tmpl == tmpl) {
        // the walk up to W.pos is this call's too; it goes on from there (or
        // stops at once when the new limit does not pass W.pos)
        std::swap(S.pc_c, W.pc_c);
        std::swap(S.pc_n, W.pc_n);
        std::swap(S.pc_k, W.pc_k);
        std::swap(S.pc_over, W.pc_over);
        cur.swap(W.cur);
        out.variations.swap(W.variations);
        out.any_variation = W.any_variation;
        out.copy_len.swap(W.copy_len);
        out.copy_err.swap(W.copy_err);
        pos = W.pos;
        copies = W.copies;
        tot_ins = W.tot_ins;
        tot_del = W.tot_del;
        tot_err = W.tot_err;
        max_err = W.max_err;
        W.valid = false;
    } else {
        pc_reset(S, m);
        out.copy_len.clear();
        out.copy_err.clear();
        out.variations.clear();
        out.any_variation = false;
        cur = tmpl;
    }
    // exact copies observe cur[p] at every p; they are counted in bulk before
    // the next count update or read, which keeps first-insertion order
    int64_t pend = 0;
    auto flush = [&]() {
        if (!pend) return;
        for (int64_t p = 0; p < m; ++p) pc_add(S, p, cur[(size_t)p], pend);
        pend = 0;
    };
    while (pos < limit) {
        const int64_t wend = std::min<int64_t>(seq_len, pos + m + max_indel);
        const int64_t wlen = wend - pos;
        if (wlen < m - max_indel) break;
        if (wlen >= m && std::memcmp(cur.data(), seq + pos, (size_t)m) == 0) {
            // exact copy: the DP's unique zero is (m, m) on the all-'M' diagonal,
            // so no ops, consumed m, every base observed; each cur[p] is already
            // its position's first maximal count, so the consensus is unchanged.
            // The copies after it stay exact while the text is m-periodic, so a
            // whole run of them is taken at once: copy j (at pos + j*m) is taken
            // while pos + j*m < limit and pos + (j+1)*m <= seq_len.
            const int64_t top = std::min<int64_t>(seq_len, limit - 1 + m);   // last copy ends by here
            int64_t x = pos + m;
            while (x + 8 <= top) {   // periodic extent, 8 bytes at a time
                uint64_t a, b;
                std::memcpy(&a, seq + x, 8);
                std::memcpy(&b, seq + x - m, 8);
                if (a != b) break;
                x += 8;
            }
            while (x < top && seq[x] == seq[x - m]) ++x;
            const int64_t k = (x - pos) / m;   // >= 1 (the first copy)
            copies += k;
            pend += k;
            if (out.want_copies) {
                out.copy_err.insert(out.copy_err.end(), (size_t)k, 0);
                out.copy_len.insert(out.copy_len.end(), (size_t)k, m);
            }
            pos += k * m;
            continue;
        }
        if (!align_unit(cur.data(), m, seq + pos, wlen, max_indel, tol, S, res) || res.consumed == 0) break;
        flush();
        ++copies;
        // variation pieces "copy:pos:..." in op order (bwt.py:1073-1088)
        uint32_t from = 0;
        for (uint32_t e : S.op_end) {
            if (out.any_variation) out.variations.push_back(';');
            put_num(out.variations, copies);
            out.variations.append(S.ops, from, e - from);
            out.any_variation = true;
            from = e;
        }
        if (out.want_copies) {
            out.copy_err.push_back(res.n_sub + res.n_ins + res.n_del);
            out.copy_len.push_back(res.consumed);
        }
        tot_err += res.n_sub + res.n_ins + res.n_del;
        max_err = std::max<int64_t>(max_err, res.n_sub + res.n_ins + res.n_del);
        tot_ins += res.n_ins;
        tot_del += res.n_del;
        // only the observed positions' counts change, so only their most-common
        // base can (consensus_from over all m positions, incrementally)
        for (size_t q = 0; q < S.obs_idx.size(); ++q) {
            const int64_t idx = S.obs_idx[q];
            if (idx >= 0 && idx < m) {
                pc_add(S, idx, S.obs_base[q]);
                char b;
                if (pc_top(S, idx, b)) cur[(size_t)idx] = b;
            }
        }
        pos += res.consumed;
    }
    out.at_limit = pos >= limit;
    flush();   // the pending exact copies' counts (applied before any later update or read)
    // a walk stopped by its limit is kept for a resume (the counts move, the
    // strings and per-copy vectors are copied: the result still holds them)
    auto save = [&]() {
        if (!resume || !out.at_limit) return;
        W.valid = true;
        W.seq = seq;
        W.seq_len = seq_len;
        W.start = start;
        W.max_indel = max_indel;
        W.tol = tol;
        W.stop_limit = limit;
        W.tmpl = tmpl;
        W.cur = cur;
        W.variations = out.variations;
        W.any_variation = out.any_variation;
        W.want_copies = out.want_copies;
        W.copy_len = out.copy_len;
        W.copy_err = out.copy_err;
        W.pos = pos;
        W.copies = copies;
        W.tot_ins = tot_ins;
        W.tot_del = tot_del;
        W.tot_err = tot_err;
        W.max_err = max_err;
        std::swap(S.pc_c, W.pc_c);
        std::swap(S.pc_n, W.pc_n);
        std::swap(S.pc_k, W.pc_k);
        std::swap(S.pc_over, W.pc_over);
    };
    if (copies < min_copies) {
        save();
        return false;
    }
    const int64_t consumed = pos - start;
    if (consumed <= 0) {
        save();
        return false;
    }
    consensus_from(S, m, cur, out.consensus);
    const int64_t denom = copies * m;
    out.motif_len = m;
    out.copies = copies;
    out.consumed = consumed;
    out.mismatch_rate = denom > 0 ? (double)tot_err / (double)denom : 0.0;
    out.max_errors = max_err;
    out.tot_err = tot_err;
    out.tot_ins = tot_ins;
    out.tot_del = tot_del;
    save();
    return true;
}

}  // namespace bwtmi
