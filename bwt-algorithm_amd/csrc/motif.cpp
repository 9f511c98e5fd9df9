// motif.cpp -- exact host restatement of the MotifUtils pieces on the CLI path.
// Float arithmetic follows the Python expressions operation by operation; the
// library is built with -ffp-contract=off so no FMA changes a rounding.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"

namespace bwtmi {

// Least rotation (Booth).  MotifUtils.get_canonical_motif takes the min over
// all rotations (bwt.py:679-685); the least rotation string is unique, so any
// exact algorithm yields the same string.
std::string min_rotation(const std::string &s) {
    const int64_t n = (int64_t)s.size();
    if (n <= 1) return s;
    std::vector<int64_t> f(2 * n, -1);
    int64_t k = 0;
    auto at = [&](int64_t i) { return (unsigned char)s[(size_t)(i % n)]; };
    for (int64_t j = 1; j < 2 * n; ++j) {
        unsigned char sj = at(j);
        int64_t i = f[j - k - 1];
        while (i != -1 && sj != at(k + i + 1)) {
            if (sj < at(k + i + 1)) k = j - i - 1;
            i = f[i];
        }
        if (sj != at(k + i + 1)) {  // i == -1
            if (sj < at(k)) k = j;
            f[j - k] = -1;
        } else {
            f[j - k] = i + 1;
        }
    }
    return s.substr((size_t)k) + s.substr(0, (size_t)k);
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

void canonical_stranded(const std::string &s, std::string &canon, char &strand) {  // 694-716
    if (s.empty()) {
        canon = s;
        strand = '+';
        return;
    }
    std::string rc(s.rbegin(), s.rend());
    for (auto &c : rc) c = comp_base(c);
    std::string f = min_rotation(s), r = min_rotation(rc);
    if (f <= r) {
        canon.swap(f);
        strand = '+';
    } else {
        canon.swap(r);
        strand = '-';
    }
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
// MotifUtils._align_unit_to_window (bwt.py:829-983), banded storage.
// Cells outside the computed band read as the reference's `inf`; row 0 and
// column 0 hold the reference's initialisation.  Ties keep sub > del > ins.
// ------------------------------------------------------------------------
namespace {

struct Op {
    char kind;      // 's' sub, 'i' ins, 'd' del
    int64_t pos;
    char ref, alt;  // sub
    std::string ins;
    int64_t len = 0;
};

struct UnitResult {
    int64_t consumed = 0;
    int64_t n_sub = 0, n_ins = 0, n_del = 0;
    std::vector<Op> ops;
    std::vector<std::pair<int64_t, char>> observed;
};

struct DPBuf {
    std::vector<int32_t> cost;
    std::vector<char> ptr;
};

bool align_unit(const char *motif, int64_t m, const char *win, int64_t n, int64_t max_indel,
                int64_t tol, DPBuf &buf, UnitResult &res) {
    if (m == 0 || n == 0) return false;
    max_indel = std::max<int64_t>(0, max_indel);
    tol = std::max<int64_t>(0, tol);
    const int64_t lower = std::max<int64_t>(0, m - max_indel);
    const int64_t upper = std::min<int64_t>(n, m + max_indel);
    if (lower > upper) return false;
    const int64_t INF = m + n + 10;
    const int64_t band = max_indel + 2;
    const int64_t W = 2 * band + 1;  // row i stores columns i-band .. i+band
    buf.cost.assign((size_t)((m + 1) * W), (int32_t)INF);
    buf.ptr.assign((size_t)((m + 1) * W), 0);
    auto inb = [&](int64_t i, int64_t j) { return j >= i - band && j <= i + band; };
    auto get = [&](int64_t i, int64_t j) -> int64_t {
        if (i == 0) return j;        // dp[0][j] = j (j <= n)
        if (j == 0) return i;        // dp[i][0] = i
        if (!inb(i, j)) return INF;
        return buf.cost[(size_t)(i * W + (j - i + band))];
    };
    for (int64_t i = 1; i <= m; ++i) {
        const int64_t jmin = std::max<int64_t>(1, i - band), jmax = std::min<int64_t>(n, i + band);
        const char mi = motif[i - 1];
        for (int64_t j = jmin; j <= jmax; ++j) {
            const bool eq = mi == win[j - 1];
            int64_t best = get(i - 1, j - 1) + (eq ? 0 : 1);
            char op = eq ? 'M' : 'S';
            const int64_t dc = get(i - 1, j) + 1;
            if (dc < best) { best = dc; op = 'D'; }
            const int64_t ic = get(i, j - 1) + 1;
            if (ic < best) { best = ic; op = 'I'; }
            buf.cost[(size_t)(i * W + (j - i + band))] = (int32_t)best;
            buf.ptr[(size_t)(i * W + (j - i + band))] = op;
        }
    }
    int64_t bj = -1, bc = INF;
    for (int64_t j = lower; j <= upper; ++j) {
        const int64_t c = get(m, j);
        if (c < bc) { bc = c; bj = j; }
    }
    if (bj <= 0 || bc >= INF) return false;
    auto ptr = [&](int64_t i, int64_t j) -> char {
        if (i == 0 && j == 0) return 0;
        if (i == 0) return 'I';
        if (j == 0) return 'D';
        if (!inb(i, j)) return 0;
        return buf.ptr[(size_t)(i * W + (j - i + band))];
    };
    // traceback into aligned columns (ref, query); '-' = gap
    std::vector<std::pair<char, char>> cols;
    cols.reserve((size_t)(m + n));
    int64_t i = m, j = bj;
    while (i > 0 || j > 0) {
        const char op = ptr(i, j);
        if (op == 'M' || op == 'S') { cols.push_back({motif[i - 1], win[j - 1]}); --i; --j; }
        else if (op == 'D') { cols.push_back({motif[i - 1], '-'}); --i; }
        else if (op == 'I') { cols.push_back({'-', win[j - 1]}); --j; }
        else break;
    }
    std::reverse(cols.begin(), cols.end());
    res.ops.clear();
    res.observed.clear();
    res.n_sub = res.n_ins = res.n_del = 0;
    int64_t ref = 0;
    std::string ins_buf;
    int64_t ins_at = 0, del_len = 0, del_at = 0;
    for (auto &rq : cols) {
        const char r = rq.first, q = rq.second;
        if (r == '-') {
            if (ins_buf.empty()) ins_at = ref;
            ins_buf.push_back(q);
            continue;
        }
        if (!ins_buf.empty()) {
            Op o; o.kind = 'i'; o.pos = ins_at; o.ins = ins_buf;
            res.n_ins += (int64_t)ins_buf.size();
            res.ops.push_back(std::move(o));
            ins_buf.clear();
            ins_at = 0;
        }
        ++ref;
        if (q == '-') {
            if (del_len == 0) del_at = ref;
            ++del_len;
            continue;
        }
        if (del_len) {
            Op o; o.kind = 'd'; o.pos = del_at; o.len = del_len;
            res.n_del += del_len;
            res.ops.push_back(std::move(o));
            del_len = 0;
        }
        res.observed.push_back({ref - 1, q});
        if (r != q) {
            Op o; o.kind = 's'; o.pos = ref; o.ref = r; o.alt = q;
            res.ops.push_back(std::move(o));
            ++res.n_sub;
        }
    }
    if (!ins_buf.empty()) {
        Op o; o.kind = 'i'; o.pos = ins_at; o.ins = ins_buf;
        res.n_ins += (int64_t)ins_buf.size();
        res.ops.push_back(std::move(o));
    }
    if (del_len) {
        Op o; o.kind = 'd'; o.pos = del_at; o.len = del_len;
        res.n_del += del_len;
        res.ops.push_back(std::move(o));
    }
    if (res.n_sub > tol) return false;
    if (res.n_ins > max_indel || res.n_del > max_indel) return false;
    res.consumed = bj;
    return true;
}

// per-position Counter with insertion order (most_common(1) = first max)
struct PosCount {
    std::vector<std::pair<char, int64_t>> v;
    void add(char b) {
        for (auto &p : v)
            if (p.first == b) { ++p.second; return; }
        v.push_back({b, 1});
    }
    bool empty() const { return v.empty(); }
    char top() const {
        char b = v[0].first;
        int64_t c = v[0].second;
        for (size_t k = 1; k < v.size(); ++k)
            if (v[k].second > c) { c = v[k].second; b = v[k].first; }
        return b;
    }
};

void consensus_from(const std::vector<PosCount> &pc, const std::string &fallback, std::string &out) {
    out.resize(pc.size());
    for (size_t i = 0; i < pc.size(); ++i)
        out[i] = !pc[i].empty() ? pc[i].top() : (i < fallback.size() ? fallback[i] : 'N');
}

}  // namespace

bool align_repeat_region(const char *seq, int64_t seq_len, int64_t start, int64_t end,
                         const std::string &tmpl, int64_t min_copies, AlignSummary &out, double frac,
                         int64_t max_indel_arg) {
    if (tmpl.empty() || seq_len == 0) return false;
    start = std::max<int64_t>(0, start);
    end = std::min<int64_t>(seq_len, end > start ? end : seq_len);
    const int64_t m = (int64_t)tmpl.size();
    const int64_t tol = std::max<int64_t>(1, (int64_t)std::floor((double)m * frac));
    const int64_t max_indel = max_indel_arg < 0 ? std::max<int64_t>(1, std::min<int64_t>(10, m >= 4 ? m / 2 : 1))
                                                : max_indel_arg;
    std::vector<PosCount> pc((size_t)m);
    out.copy_len.clear();
    std::vector<std::vector<Op>> ops_by_copy;
    std::vector<int64_t> errs;
    int64_t tot_ins = 0, tot_del = 0;
    std::string cur = tmpl, next;
    int64_t pos = start;
    const int64_t limit = std::min<int64_t>(
        seq_len, std::max<int64_t>(end, start + m * min_copies) + std::max<int64_t>(m * 3, max_indel * 4));
    thread_local DPBuf buf;
    UnitResult res;
    while (pos < limit) {
        const int64_t wend = std::min<int64_t>(seq_len, pos + m + max_indel);
        const int64_t wlen = wend - pos;
        if (wlen < m - max_indel) break;
        if (!align_unit(cur.data(), m, seq + pos, wlen, max_indel, tol, buf, res) || res.consumed == 0)
            break;
        ops_by_copy.push_back(res.ops);
        errs.push_back(res.n_sub + res.n_ins + res.n_del);
        out.copy_len.push_back(res.consumed);
        tot_ins += res.n_ins;
        tot_del += res.n_del;
        for (auto &ob : res.observed)
            if (ob.first >= 0 && ob.first < m) pc[(size_t)ob.first].add(ob.second);
        pos += res.consumed;
        consensus_from(pc, cur, next);
        cur.swap(next);
    }
    const int64_t copies = (int64_t)errs.size();
    if (copies < min_copies) return false;
    const int64_t consumed = pos - start;
    if (consumed <= 0) return false;
    consensus_from(pc, cur, out.consensus);
    int64_t tot = 0, mx = 0;
    for (auto e : errs) { tot += e; mx = std::max(mx, e); }
    const int64_t denom = copies * m;
    out.motif_len = m;
    out.copies = copies;
    out.consumed = consumed;
    out.mismatch_rate = denom > 0 ? (double)tot / (double)denom : 0.0;
    out.max_errors = mx;
    out.tot_ins = tot_ins;
    out.tot_del = tot_del;
    out.copy_err = errs;
    out.variations.clear();
    out.any_variation = false;
    char tmp[64];
    for (size_t k = 0; k < ops_by_copy.size(); ++k) {
        const long long idx = (long long)k + 1;
        for (auto &o : ops_by_copy[k]) {
            std::string piece;
            if (o.kind == 's') {
                snprintf(tmp, sizeof tmp, "%lld:%lld:", idx, (long long)o.pos);
                piece = std::string(tmp) + o.ref + ">" + o.alt;
            } else if (o.kind == 'i') {
                if (o.ins.empty()) continue;
                snprintf(tmp, sizeof tmp, "%lld:%lld:ins(", idx, (long long)o.pos);
                piece = std::string(tmp) + o.ins + ")";
            } else {
                if (o.len <= 0) continue;
                snprintf(tmp, sizeof tmp, "%lld:%lld:del(%lld)", idx, (long long)o.pos, (long long)o.len);
                piece = tmp;
            }
            if (out.any_variation) out.variations.push_back(';');
            out.variations += piece;
            out.any_variation = true;
        }
    }
    return true;
}

}  // namespace bwtmi
