// post.cpp -- exact host restatement of the repeat post-processing
// (TandemRepeatFinder, bwt.py:3144-3944) over the raw strict hits.
//
// Work is organised per "fold unit": the contigs whose natural sort keys are
// equal (normally exactly one contig).  Every stage of the reference either
// groups by chromosome or folds over the globally sorted list with a
// same-chromosome test, so units are independent and run on separate host
// threads; inside a unit the reference's sequential order is kept.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace bwtmi {

int host_threads(const bwtmi_params &p) {
    if (p.threads > 0) return p.threads;
    unsigned hc = std::thread::hardware_concurrency();
    int t = hc ? (int)hc : 4;
    return std::min(t, 16);
}

// ------------------------------------------------------------ natural key
std::vector<NatPart> natural_key(const std::string &s) {      // bwt.py:22-36
    std::vector<NatPart> out;
    size_t i = 0, n = s.size();
    while (i < n) {
        size_t j = i;
        const bool dig = s[i] >= '0' && s[i] <= '9';
        while (j < n && ((s[j] >= '0' && s[j] <= '9') == dig)) ++j;
        NatPart p;
        p.digit = dig;
        if (dig) {
            size_t k = i;
            while (k + 1 < j && s[k] == '0') ++k;  // int(part): strip leading zeros
            p.text = s.substr(k, j - k);
        } else {
            p.text = s.substr(i, j - i);
            for (auto &c : p.text)
                if (c >= 'A' && c <= 'Z') c = (char)(c + 32);
        }
        out.push_back(std::move(p));
        i = j;
    }
    return out;
}

int natural_cmp(const std::vector<NatPart> &a, const std::vector<NatPart> &b) {
    const size_t n = std::min(a.size(), b.size());
    for (size_t i = 0; i < n; ++i) {
        const NatPart &x = a[i], &y = b[i];
        if (x.digit != y.digit) return x.digit ? -1 : 1;  // (0, int) < (1, str)
        if (x.digit) {
            if (x.text.size() != y.text.size()) return x.text.size() < y.text.size() ? -1 : 1;
        }
        int c = x.text.compare(y.text);
        if (c) return c < 0 ? -1 : 1;
    }
    if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
    return 0;
}

void Job::assign_units() {
    natkeys.clear();
    for (auto &c : contigs) natkeys.push_back(natural_key(c.name));
    std::vector<int32_t> order(contigs.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
        return natural_cmp(natkeys[a], natkeys[b]) < 0;
    });
    nunits = 0;
    unit_rank.clear();
    for (size_t k = 0; k < order.size(); ++k) {
        if (k == 0 || natural_cmp(natkeys[order[k - 1]], natkeys[order[k]]) != 0) {
            unit_rank.push_back(nunits);
            ++nunits;
        }
        contigs[order[k]].unit = nunits - 1;   // unit ids are ranks by natural key
    }
}

// ------------------------------------------------------------ strict records
// Record per strict hit: bwt.py:1952-1993 with calculate_trf_statistics
// (1336-1366) at mismatch_rate 0.  Composition/entropy are functions of the
// motif and are evaluated at render time.  Rule 1 (3118-3130) never fires on
// strict hits (mismatch_rate 0, max_mismatches_per_copy 0).
void strict_hits_to_records(const Job &job, int32_t contig, const bwtmi_hit *hits, int64_t n,
                            std::vector<Rec> &out) {
    const Contig &c = job.contigs[(size_t)contig];
    const char *t = c.trimmed();
    out.reserve(out.size() + (size_t)n);
    for (int64_t k = 0; k < n; ++k) {
        const bwtmi_hit &h = hits[k];
        Rec r;
        r.chrom = contig;
        r.tier = 2;
        r.start = h.start;
        r.end = h.end;
        r.length = h.end - h.start;
        r.motif.assign(t + h.start, (size_t)h.prim_len);
        r.copies = (double)h.copies;
        r.confidence = 0.95;
        r.mismatch_rate = 0.0;
        r.max_mm = 0;
        r.n_eval = h.copies;
        r.strand = '+';
        r.pmatch = (1.0 - 0.0) * 100.0;
        r.pindel = 0.0;
        r.score = trf_score(r.length, 0.0);
        r.act_kind = ACT_TRIMMED;
        r.act_off = h.start;
        r.act_len = h.end - h.start;
        out.push_back(std::move(r));
    }
}

namespace {

inline bool key_less(const Rec &a, const Rec &b) {   // (natural(chrom), start, end) in a unit
    if (a.start != b.start) return a.start < b.start;
    return a.end < b.end;
}

// ---------------------------------------------------- nested suppression
// bwt.py:3402-3497.  A repeat is tested only against kept spans of a strictly
// longer motif; the stable sort by (mismatch_rate > 0, -len(motif)) places
// every such span of its class (and the whole perfect class) before it, and
// repeats of equal motif length never test each other.  So each (class,
// length) group is screened against the spans kept so far and appended as a
// whole.  Kept spans live in a bucket grid for the overlap queries; the
// predicate is the reference's, division for division.
std::vector<Rec> suppress_nested_chrom(std::vector<Rec> &rs, double thr) {
    const size_t n = rs.size();
    std::vector<uint32_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        const bool ia = rs[a].mismatch_rate > 0, ib = rs[b].mismatch_rate > 0;
        if (ia != ib) return !ia;
        return rs[a].motif.size() > rs[b].motif.size();
    });
    int64_t maxpos = 1;
    for (auto &r : rs) maxpos = std::max(maxpos, r.end + 1);
    const int64_t B = 2048;
    struct Span { int64_t s, e; int64_t M; };
    std::vector<std::vector<Span>> grid((size_t)(maxpos / B + 2));
    std::vector<uint8_t> keep(n, 0);
    std::vector<Rec> kept;
    kept.reserve(n);
    size_t g = 0;
    while (g < n) {
        const bool cls = rs[order[g]].mismatch_rate > 0;
        const size_t len = rs[order[g]].motif.size();
        size_t h = g;
        while (h < n && (rs[order[h]].mismatch_rate > 0) == cls && rs[order[h]].motif.size() == len) ++h;
        for (size_t k = g; k < h; ++k) {
            const Rec &r = rs[order[k]];
            const int64_t a = r.start, b = r.end, m = (int64_t)r.motif.size();
            const int64_t rl = b - a;
            bool nested = false;
            if (b > a) {
                const int64_t b0 = std::max<int64_t>(0, a) / B, b1 = std::max<int64_t>(0, b - 1) / B;
                for (int64_t bk = b0; bk <= b1 && !nested && bk < (int64_t)grid.size(); ++bk) {
                    for (const Span &sp : grid[(size_t)bk]) {
                        if (sp.M <= m) continue;
                        const int64_t ov = std::max<int64_t>(0, std::min(b, sp.e) - std::max(a, sp.s));
                        if (ov == 0) continue;
                        const double ratio = (double)sp.M / (double)m;
                        const double frac = (double)ov / (double)rl;
                        if (m == 1 && sp.M > 1 && frac >= 0.8) { nested = true; break; }
                        const double t = ratio >= 10 ? 0.1 : (ratio >= 5 ? 0.3 : thr);
                        if (frac >= t) { nested = true; break; }
                    }
                }
            }
            keep[order[k]] = !nested;
        }
        for (size_t k = g; k < h; ++k) {
            const uint32_t idx = order[k];
            if (!keep[idx]) continue;
            Rec &r = rs[idx];
            if (r.end > r.start) {
                Span sp{r.start, r.end, (int64_t)r.motif.size()};
                const int64_t b0 = std::max<int64_t>(0, r.start) / B, b1 = std::max<int64_t>(0, r.end - 1) / B;
                for (int64_t bk = b0; bk <= b1 && bk < (int64_t)grid.size(); ++bk) grid[(size_t)bk].push_back(sp);
            }
            kept.push_back(std::move(r));
        }
        g = h;
    }
    return kept;
}

struct UnitCtx {
    const Job *job;
    int64_t min_copies;
};

// bwt.py:3515-3614 (on the trimmed sequence, before coordinate restore)
Rec recompute(const UnitCtx &u, int32_t chrom, int64_t start, int64_t end, int64_t motif_len, int32_t tier) {
    const Contig &c = u.job->contigs[(size_t)chrom];
    const char *seq = c.trimmed();
    const int64_t L = c.trimmed_len();
    const int64_t m = std::max<int64_t>(1, motif_len);
    start = std::max<int64_t>(0, start);
    end = end > 0 ? std::min(L, end) : L;
    if (end <= start) end = std::min(L, start + m);
    auto slice = [&](int64_t a, int64_t b) {   // Python seq[a:b], a,b >= 0
        a = std::min(a, L);
        b = std::min(b, L);
        return b > a ? std::string(seq + a, (size_t)(b - a)) : std::string();
    };
    std::string tmpl = slice(start, start + m);
    if (tmpl.empty()) {
        const int64_t a = std::max<int64_t>(0, start - m);
        tmpl = slice(a, a + m);
    }
    if (tmpl.empty()) tmpl.assign((size_t)m, 'N');
    AlignSummary s;
    bool ok = align_repeat_region(seq, L, start, end, tmpl, std::max<int64_t>(1, u.min_copies), s);
    if (!ok) ok = align_repeat_region(seq, L, start, end, tmpl, 1, s);
    Rec r;
    r.chrom = chrom;
    r.tier = tier;
    r.start = start;
    int64_t consumed, cint;
    std::string cons;
    double mm, pind;
    int64_t maxe;
    if (!ok) {
        consumed = std::min(L - start, std::max(m, end - start));
        cint = std::max<int64_t>(1, consumed / m);
        cons = tmpl;  // never empty here
        mm = 0.0;
        maxe = 0;
        pind = 0.0;
        r.variations.clear();
    } else {
        consumed = s.consumed;
        cint = s.copies;
        cons = s.consensus.empty() ? tmpl : s.consensus;
        mm = s.mismatch_rate;
        const int64_t tb = s.copies * s.motif_len;
        const double ir = tb > 0 ? (double)(s.tot_ins + s.tot_del) / (double)tb : 0.0;
        pind = ir * 100.0;
        maxe = s.max_errors;
        r.variations = s.any_variation ? s.variations : std::string();
    }
    // actual_sequence = sequence[start:start+consumed]
    const int64_t a0 = std::min(start, L), a1 = std::max(a0, std::min(start + consumed, L));
    const int64_t tl = a1 - a0;
    const int64_t mle = cons.empty() ? m : (int64_t)cons.size();
    double cf = (double)cint;
    if (tl > 0 && mle > 0) {
        const double fr = (double)tl / (double)mle;
        const double rr = std::nearbyint(fr);  // Python round(): half to even
        cf = std::fabs(fr - rr) < 1e-6 ? rr : fr;
    }
    r.end = start + tl;
    r.length = tl;
    r.motif = cons;
    r.copies = cf;
    r.confidence = std::max(0.3, 1.0 - mm);
    r.mismatch_rate = mm;
    r.max_mm = maxe;
    r.n_eval = std::max<int64_t>(1, cint);
    std::string canon;
    canonical_stranded(cons, canon, r.strand);
    r.pmatch = std::max(0.0, 100.0 - mm * 100.0);
    r.pindel = pind;
    r.score = trf_score(tl, mm);
    r.act_kind = ACT_TRIMMED;
    r.act_off = a0;
    r.act_len = tl;
    return r;
}

// canonical of a motif with a tiny cache (adjacent pairs re-ask for the same r1)
struct CanonCache {
    std::string key, val;
    const std::string &get(const std::string &m) {
        if (m != key || val.empty()) {
            char st;
            canonical_stranded(m, val, st);
            key = m;
        }
        return val;
    }
};

// bwt.py:3240-3281
bool should_merge(const UnitCtx &u, const Rec &r1, const Rec &r2, CanonCache &c1, CanonCache &c2) {
    if (r1.chrom != r2.chrom) return false;
    if (r1.motif.empty() || r2.motif.empty()) return false;
    const int64_t ml = (int64_t)std::min(r1.motif.size(), r2.motif.size());
    const int64_t gap = std::max<int64_t>(0, r2.start - r1.end);
    if (gap > ml + 1) return false;   // cheap test first: the result is a conjunction
    if (c1.get(r1.motif) != c2.get(r2.motif)) return false;
    const Rec mg = recompute(u, r1.chrom, std::min(r1.start, r2.start), std::max(r1.end, r2.end),
                             std::max<int64_t>(1, ml), std::min(r1.tier, r2.tier));
    if (mg.copies < (double)u.min_copies) return false;
    const double base = std::max(std::max(r1.mismatch_rate, r2.mismatch_rate), 0.01);
    return mg.mismatch_rate <= base + 0.2;
}

// bwt.py:3327-3354
bool should_collapse(const Rec &r1, const Rec &r2) {
    if (r1.chrom != r2.chrom) return false;
    const int64_t ov = std::min(r1.end, r2.end) - std::max(r1.start, r2.start);
    if (ov <= 0) return false;
    const int64_t sh = std::min(r1.length, r2.length);
    if (sh <= 0) return false;
    const double f = (double)ov / (double)sh;
    if (f < 0.8) return false;
    std::string a, b;
    char st;
    canonical_stranded(r1.motif, a, st);
    canonical_stranded(r2.motif, b, st);
    if (a == b) return true;
    if ((r1.motif.size() == 1 || r2.motif.size() == 1) && f >= 0.95) return true;
    if (r1.motif.size() == r2.motif.size() && f >= 0.9)
        return std::fabs(r1.mismatch_rate - r2.mismatch_rate) >= 0.2;
    return false;
}

// bwt.py:3356-3400 -> true when r1 is preferred
bool prefer_first(const Rec &r1, const Rec &r2) {
    const std::string &m1 = r1.motif, &m2 = r2.motif;
    const size_t l1 = m1.size(), l2 = m2.size();
    if (l1 != l2) {
        if (l1 == 1 && l2 > 1) return false;
        if (l2 == 1 && l1 > 1) return true;
        const std::string &sh = l1 < l2 ? m1 : m2;
        const std::string &lo = l1 < l2 ? m2 : m1;
        if (lo.size() % sh.size() == 0) {
            bool rep = true;
            for (size_t i = 0; i < lo.size() && rep; ++i) rep = lo[i] == sh[i % sh.size()];
            if (rep) return l1 < l2;
        }
        return l1 > l2;
    }
    if (r1.mismatch_rate != r2.mismatch_rate) return r1.mismatch_rate < r2.mismatch_rate;
    if (r1.confidence != r2.confidence) return r1.confidence > r2.confidence;
    if (r1.length != r2.length) return r1.length >= r2.length;
    return true;
}

struct DedupKey {
    int32_t chrom;
    int64_t s, e;
    const std::string *m;
    bool operator==(const DedupKey &o) const {
        return chrom == o.chrom && s == o.s && e == o.e && *m == *o.m;
    }
};
struct DedupHash {
    size_t operator()(const DedupKey &k) const {
        size_t h = std::hash<std::string>()(*k.m);
        h ^= (size_t)k.s * 0x9E3779B97F4A7C15ull + ((size_t)k.e << 7) + (size_t)k.chrom;
        return h;
    }
};

void process_unit(const Job &job, const std::vector<int32_t> &chroms,
                  std::vector<std::vector<Rec>> &raw, std::vector<Rec> &out, double *ms) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    UnitCtx u{&job, job.params.min_copies};
    // 1. nested suppression per chromosome (bwt.py:3928), concatenated in
    //    chromosome order, stable-sorted by (start, end).
    std::vector<Rec> recs;
    for (int32_t c : chroms) {
        std::vector<Rec> kept = suppress_nested_chrom(raw[(size_t)c], 0.5);
        if (recs.empty()) recs.swap(kept);
        else for (auto &r : kept) recs.push_back(std::move(r));
        std::vector<Rec>().swap(raw[(size_t)c]);
    }
    std::stable_sort(recs.begin(), recs.end(), key_less);
    auto t1 = clk::now();
    // 2. dedup (bwt.py:3189-3220)
    {
        std::vector<Rec> d;
        d.reserve(recs.size());
        std::unordered_map<DedupKey, size_t, DedupHash> pos;
        pos.reserve(recs.size() * 2);
        // keys point into `recs`; replaced records keep their slot
        std::vector<size_t> src;
        src.reserve(recs.size());
        for (size_t i = 0; i < recs.size(); ++i) {
            const Rec &r = recs[i];
            DedupKey k{r.chrom, r.start, r.end, &r.motif};
            auto it = pos.find(k);
            if (it == pos.end()) {
                pos.emplace(k, src.size());
                src.push_back(i);
                continue;
            }
            const Rec &ex = recs[src[it->second]];
            bool repl = false;
            if (r.confidence > ex.confidence) repl = true;
            else if (r.confidence == ex.confidence) {
                if (r.mismatch_rate < ex.mismatch_rate) repl = true;
                else if (r.mismatch_rate == ex.mismatch_rate && r.tier < ex.tier) repl = true;
            }
            if (repl) src[it->second] = i;
        }
        for (size_t i : src) d.push_back(std::move(recs[i]));
        recs.swap(d);
        std::stable_sort(recs.begin(), recs.end(), key_less);
    }
    auto t2 = clk::now();
    // 3. merge adjacent (bwt.py:3222-3289) -- sequential fold
    if (!recs.empty()) {
        std::vector<Rec> merged;
        merged.reserve(recs.size());
        Rec cur = std::move(recs[0]);
        CanonCache cc, cn;
        for (size_t i = 1; i < recs.size(); ++i) {
            Rec &nx = recs[i];
            if (should_merge(u, cur, nx, cc, cn)) {
                cur = recompute(u, cur.chrom, std::min(cur.start, nx.start), std::max(cur.end, nx.end),
                                (int64_t)cur.motif.size(), std::min(cur.tier, nx.tier));
            } else {
                merged.push_back(std::move(cur));
                cur = std::move(nx);
                std::swap(cc, cn);
            }
        }
        merged.push_back(std::move(cur));
        recs.swap(merged);
    }
    auto t3 = clk::now();
    // 4. refine (bwt.py:3291-3314)
    for (auto &r : recs) {
        if (r.mismatch_rate == 0.0) continue;
        int64_t m = (int64_t)r.motif.size();
        if (m <= 0) {
            const int64_t rc = (int64_t)std::nearbyint(r.copies);
            m = std::max<int64_t>(1, r.length / std::max<int64_t>(1, rc ? rc : 1));
        }
        r = recompute(u, r.chrom, r.start, r.end, m, r.tier);
    }
    std::stable_sort(recs.begin(), recs.end(), key_less);
    // 5. restore coordinates (bwt.py:3316-3325)
    for (auto &r : recs) {
        const Contig &c = job.contigs[(size_t)r.chrom];
        r.start += c.trim_left;
        r.end += c.trim_left;
        r.length = r.end - r.start;
        if (!c.full.empty()) {
            const int64_t L = (int64_t)c.full.size();
            const int64_t a = std::min(r.start, L), b = std::max(a, std::min(r.end, L));
            r.act_kind = ACT_FULL;
            r.act_off = a;
            r.act_len = b - a;
        }
    }
    // 6. collapse (bwt.py:3499-3513)
    std::stable_sort(recs.begin(), recs.end(), key_less);
    {
        std::vector<Rec> col;
        col.reserve(recs.size());
        for (auto &r : recs) {
            if (!col.empty() && should_collapse(col.back(), r)) {
                if (!prefer_first(col.back(), r)) col.back() = std::move(r);
            } else {
                col.push_back(std::move(r));
            }
        }
        recs.swap(col);
    }
    // 7. final filter (bwt.py:3940-3944)
    out.clear();
    for (auto &r : recs)
        if (r.copies >= (double)job.params.min_copies && r.length >= 6) out.push_back(std::move(r));
    auto t4 = clk::now();
    if (ms) {
        ms[0] += std::chrono::duration<double, std::milli>(t1 - t0).count();
        ms[1] += std::chrono::duration<double, std::milli>(t2 - t1).count();
        ms[2] += std::chrono::duration<double, std::milli>(t3 - t2).count();
        ms[3] += std::chrono::duration<double, std::milli>(t4 - t3).count();
    }
}

}  // namespace

void postprocess(Job &job) {
    job.assign_units();
    std::vector<std::vector<int32_t>> units((size_t)job.nunits);
    for (size_t c = 0; c < job.contigs.size(); ++c) units[(size_t)job.contigs[c].unit].push_back((int32_t)c);
    if (job.raw.size() < job.contigs.size()) job.raw.resize(job.contigs.size());
    std::vector<std::vector<Rec>> res((size_t)job.nunits);
    std::vector<double> ms((size_t)job.nunits * 4, 0.0);
    std::atomic<int32_t> next{0};
    const int nt = std::max(1, std::min(host_threads(job.params), job.nunits));
    auto worker = [&]() {
        for (;;) {
            const int32_t k = next.fetch_add(1);
            if (k >= job.nunits) break;
            process_unit(job, units[(size_t)k], job.raw, res[(size_t)k], &ms[(size_t)k * 4]);
        }
    };
    if (nt == 1) worker();
    else {
        std::vector<std::thread> th;
        for (int i = 0; i < nt; ++i) th.emplace_back(worker);
        for (auto &t : th) t.join();
    }
    job.final_recs.clear();
    for (auto &v : res)
        for (auto &r : v) job.final_recs.push_back(std::move(r));
    for (int s = 0; s < 4; ++s) {
        job.stage_ms[2 + s] = 0;
        for (int32_t k = 0; k < job.nunits; ++k) job.stage_ms[2 + s] += ms[(size_t)k * 4 + s];
    }
    job.postprocessed = true;
}

}  // namespace bwtmi
