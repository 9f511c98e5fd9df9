// post.cpp -- exact host restatement of the repeat post-processing
// (TandemRepeatFinder, bwt.py:3144-3944) over the raw strict hits.
//
// Work is organised per "fold unit": the contigs whose natural sort keys are
// equal (normally exactly one contig).  Every stage of the reference either
// groups by chromosome or folds over the globally sorted list with a
// same-chromosome test, so units are independent.  Inside a unit every stage
// is either data-parallel (record construction, nested-suppression queries,
// refine, restore) or a fold that is parallelised speculatively and then
// repaired to the exact sequential result (merge), so the output is the
// reference's regardless of the thread count.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace bwtmi {

int host_threads(const bwtmi_params &p) {
    if (p.threads > 0) return p.threads;
    unsigned hc = std::thread::hardware_concurrency();
    int t = hc ? (int)hc : 4;
    return std::min(t, 16);
}

// fn(begin, end) over [0, n) in `nt` contiguous chunks
template <class F>
static void parallel_for(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (n + 1023) / 1024));
    if (nt <= 1) {
        fn((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve((size_t)nt);
    for (int t = 0; t < nt; ++t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        th.emplace_back([&fn, a, b] { fn(a, b); });
    }
    for (auto &x : th) x.join();
}

// dynamic scheduling over items (uneven costs)
template <class F>
static void parallel_items(int64_t n, int nt, F &&fn) {
    if (n <= 0) return;
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    std::atomic<int64_t> next{0};
    auto work = [&] {
        for (;;) {
            const int64_t k = next.fetch_add(1);
            if (k >= n) break;
            fn(k);
        }
    };
    if (nt == 1) { work(); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work);
    for (auto &x : th) x.join();
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
        if (x.digit && x.text.size() != y.text.size()) return x.text.size() < y.text.size() ? -1 : 1;
        const int c = x.text.compare(y.text);
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
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return natural_cmp(natkeys[a], natkeys[b]) < 0; });
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
    const size_t base = out.size();
    out.resize(base + (size_t)n);
    parallel_for(n, host_threads(job.params), [&](int64_t a, int64_t b) {
        for (int64_t k = a; k < b; ++k) {
            const bwtmi_hit &h = hits[k];
            Rec &r = out[base + (size_t)k];
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
        }
    });
}

namespace {

// stable sort of records by (start, end): sort compact keys, then permute
void sort_by_pos(std::vector<Rec> &v, int nt) {
    const size_t n = v.size();
    if (n < 2) return;
    bool sorted = true;
    for (size_t i = 1; i < n && sorted; ++i)
        sorted = v[i - 1].start < v[i].start || (v[i - 1].start == v[i].start && v[i - 1].end <= v[i].end);
    if (sorted) return;
    struct K { int64_t s, e; uint32_t i; };
    std::vector<K> k(n);
    for (size_t i = 0; i < n; ++i) k[i] = {v[i].start, v[i].end, (uint32_t)i};
    auto lt = [](const K &a, const K &b) {
        if (a.s != b.s) return a.s < b.s;
        if (a.e != b.e) return a.e < b.e;
        return a.i < b.i;
    };
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, n / 65536 + 1));
    if (T == 1) {
        std::sort(k.begin(), k.end(), lt);
    } else {
        std::vector<size_t> cut(T + 1);
        for (int t = 0; t <= T; ++t) cut[t] = n * (size_t)t / (size_t)T;
        parallel_for(T, T, [&](int64_t a, int64_t b) {
            for (int64_t t = a; t < b; ++t) std::sort(k.begin() + cut[t], k.begin() + cut[t + 1], lt);
        });
        for (int w = 1; w < T; w *= 2) {    // pairwise merges, each level in parallel
            std::vector<std::pair<size_t, std::pair<size_t, size_t>>> jobs;
            for (int t = 0; t + w < T; t += 2 * w)
                jobs.push_back({cut[t], {cut[t + w], cut[std::min(T, t + 2 * w)]}});
            parallel_items((int64_t)jobs.size(), nt, [&](int64_t q) {
                auto &j = jobs[(size_t)q];
                std::inplace_merge(k.begin() + j.first, k.begin() + j.second.first, k.begin() + j.second.second, lt);
            });
        }
    }
    std::vector<Rec> out(n);
    parallel_for((int64_t)n, nt, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) out[(size_t)i] = std::move(v[k[(size_t)i].i]);
    });
    v.swap(out);
}

// ---------------------------------------------------- nested suppression
// bwt.py:3402-3497.  A repeat is tested only against kept spans of a strictly
// longer motif; the stable sort by (mismatch_rate > 0, -len(motif)) places
// every such span of its class (and the whole perfect class) before it, and
// repeats of equal motif length never test each other.  So each (class,
// length) group is screened -- in parallel, against a frozen grid of the
// spans kept so far -- and its survivors are appended as a whole.  The
// predicate is the reference's, division for division.
std::vector<Rec> suppress_nested_chrom(std::vector<Rec> &rs, double thr, int nt) {
    const size_t n = rs.size();
    // stable counting sort by (class, motif length desc)
    size_t maxlen = 0;
    for (auto &r : rs) maxlen = std::max(maxlen, r.motif.size());
    const size_t nb = 2 * (maxlen + 1);
    auto bucket = [&](const Rec &r) { return (r.mismatch_rate > 0 ? (maxlen + 1) : 0) + (maxlen - r.motif.size()); };
    std::vector<uint32_t> cnt(nb + 1, 0), order(n);
    for (auto &r : rs) ++cnt[bucket(r) + 1];
    for (size_t b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
    std::vector<uint32_t> groups(cnt.begin(), cnt.end());
    for (size_t i = 0; i < n; ++i) order[cnt[bucket(rs[i])]++] = (uint32_t)i;

    int64_t maxpos = 1;
    for (auto &r : rs) maxpos = std::max(maxpos, r.end + 1);
    const int64_t B = 256;
    struct Span { int64_t s, e, M; };
    std::vector<std::vector<Span>> grid((size_t)(maxpos / B + 2));
    std::vector<uint8_t> keep(n, 0);
    std::vector<Rec> kept;
    kept.reserve(n);
    for (size_t g = 0; g < nb; ++g) {
        const size_t g0 = groups[g], g1 = groups[g + 1];
        if (g0 == g1) continue;
        parallel_for((int64_t)(g1 - g0), nt, [&](int64_t a, int64_t b) {
            for (int64_t q = a; q < b; ++q) {
                const Rec &r = rs[order[g0 + (size_t)q]];
                const int64_t s0 = r.start, e0 = r.end, m = (int64_t)r.motif.size();
                const int64_t rl = e0 - s0;
                bool nested = false;
                if (e0 > s0) {
                    const int64_t b0 = std::max<int64_t>(0, s0) / B, b1 = std::max<int64_t>(0, e0 - 1) / B;
                    for (int64_t bk = b0; bk <= b1 && !nested && bk < (int64_t)grid.size(); ++bk) {
                        for (const Span &sp : grid[(size_t)bk]) {
                            if (sp.M <= m) continue;
                            const int64_t ov = std::max<int64_t>(0, std::min(e0, sp.e) - std::max(s0, sp.s));
                            if (ov == 0) continue;
                            const double ratio = (double)sp.M / (double)m;
                            const double frac = (double)ov / (double)rl;
                            if (m == 1 && sp.M > 1 && frac >= 0.8) { nested = true; break; }
                            const double t = ratio >= 10 ? 0.1 : (ratio >= 5 ? 0.3 : thr);
                            if (frac >= t) { nested = true; break; }
                        }
                    }
                }
                keep[order[g0 + (size_t)q]] = !nested;
            }
        });
        for (size_t q = g0; q < g1; ++q) {
            const uint32_t idx = order[q];
            if (!keep[idx]) continue;
            Rec &r = rs[idx];
            if (r.end > r.start) {
                const Span sp{r.start, r.end, (int64_t)r.motif.size()};
                const int64_t b0 = std::max<int64_t>(0, r.start) / B, b1 = std::max<int64_t>(0, r.end - 1) / B;
                for (int64_t bk = b0; bk <= b1 && bk < (int64_t)grid.size(); ++bk) grid[(size_t)bk].push_back(sp);
            }
            kept.push_back(std::move(r));
        }
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
    thread_local AlignSummary s;
    bool ok = align_repeat_region(seq, L, start, end, tmpl, std::max<int64_t>(1, u.min_copies), s);
    if (!ok) ok = align_repeat_region(seq, L, start, end, tmpl, 1, s);
    Rec r;
    r.chrom = chrom;
    r.tier = tier;
    r.start = start;
    int64_t consumed, cint, maxe;
    double mm, pind;
    if (!ok) {
        consumed = std::min(L - start, std::max(m, end - start));
        cint = std::max<int64_t>(1, consumed / m);
        r.motif = tmpl;  // never empty here
        mm = 0.0;
        maxe = 0;
        pind = 0.0;
    } else {
        consumed = s.consumed;
        cint = s.copies;
        r.motif = s.consensus.empty() ? tmpl : s.consensus;
        mm = s.mismatch_rate;
        const int64_t tb = s.copies * s.motif_len;
        const double ir = tb > 0 ? (double)(s.tot_ins + s.tot_del) / (double)tb : 0.0;
        pind = ir * 100.0;
        maxe = s.max_errors;
        if (s.any_variation) r.variations = s.variations;
    }
    // actual_sequence = sequence[start:start+consumed]
    const int64_t a0 = std::min(start, L), a1 = std::max(a0, std::min(start + consumed, L));
    const int64_t tl = a1 - a0;
    const int64_t mle = r.motif.empty() ? m : (int64_t)r.motif.size();
    double cf = (double)cint;
    if (tl > 0 && mle > 0) {
        const double fr = (double)tl / (double)mle;
        const double rr = std::nearbyint(fr);  // Python round(): half to even
        cf = std::fabs(fr - rr) < 1e-6 ? rr : fr;
    }
    r.end = start + tl;
    r.length = tl;
    r.copies = cf;
    r.confidence = std::max(0.3, 1.0 - mm);
    r.mismatch_rate = mm;
    r.max_mm = maxe;
    r.n_eval = std::max<int64_t>(1, cint);
    thread_local std::string canon;
    canonical_stranded(r.motif, canon, r.strand);
    r.pmatch = std::max(0.0, 100.0 - mm * 100.0);
    r.pindel = pind;
    r.score = trf_score(tl, mm);
    r.act_kind = ACT_TRIMMED;
    r.act_off = a0;
    r.act_len = tl;
    return r;
}

std::string canon_of(const std::string &m) {
    std::string c;
    char st;
    canonical_stranded(m, c, st);
    return c;
}

// ------------------------------------------------------------ merge fold
// bwt.py:3222-3289.  cur/nxt fold over the sorted list.  should_merge needs
// a recompute only for same-canonical neighbours within min_len+1; when it
// accepts and len(cur.motif) == min_len the merge recompute has identical
// arguments, so that result is reused.
struct MergeState {
    Rec cur;
    std::string canon;
};

// returns true and fills `merged` when cur and nx merge
bool try_merge(const UnitCtx &u, const Rec &r1, const std::string &c1, const Rec &r2, const std::string &c2,
               Rec &merged) {
    if (r1.chrom != r2.chrom) return false;
    if (r1.motif.empty() || r2.motif.empty()) return false;
    const int64_t ml = (int64_t)std::min(r1.motif.size(), r2.motif.size());
    if (std::max<int64_t>(0, r2.start - r1.end) > ml + 1) return false;   // cheap test first
    if (c1 != c2) return false;
    const int64_t s = std::min(r1.start, r2.start), e = std::max(r1.end, r2.end);
    const int32_t tier = std::min(r1.tier, r2.tier);
    Rec mg = recompute(u, r1.chrom, s, e, std::max<int64_t>(1, ml), tier);
    if (mg.copies < (double)u.min_copies) return false;
    const double base = std::max(std::max(r1.mismatch_rate, r2.mismatch_rate), 0.01);
    if (!(mg.mismatch_rate <= base + 0.2)) return false;
    const int64_t m1 = (int64_t)r1.motif.size();     // _merge_repeats uses len(r1.consensus_motif)
    if (m1 == std::max<int64_t>(1, ml)) merged = std::move(mg);
    else merged = recompute(u, r1.chrom, s, e, m1, tier);
    return true;
}

struct SpecOut {
    std::vector<Rec> emitted;           // records emitted by the speculative run
    std::vector<int64_t> emit_step;     // index i at which each was emitted
    Rec pending;
    std::string pending_canon;
};

// speculative run over [b, e): starts with cur = R[b] as if fresh at b
void spec_run(const UnitCtx &u, std::vector<Rec> &R, const std::vector<std::string> &canon, int64_t b, int64_t e,
              std::vector<uint8_t> &fresh, SpecOut &o) {
    Rec cur = R[(size_t)b];
    std::string cc = canon[(size_t)b];
    fresh[(size_t)b] = 1;
    Rec mg;
    for (int64_t i = b + 1; i < e; ++i) {
        if (try_merge(u, cur, cc, R[(size_t)i], canon[(size_t)i], mg)) {
            cur = std::move(mg);
            cc = canon_of(cur.motif);
            fresh[(size_t)i] = 0;
        } else {
            o.emitted.push_back(std::move(cur));
            o.emit_step.push_back(i);
            cur = R[(size_t)i];
            cc = canon[(size_t)i];
            fresh[(size_t)i] = 1;
        }
    }
    o.pending = std::move(cur);
    o.pending_canon = std::move(cc);
}

std::vector<Rec> merge_fold(const UnitCtx &u, std::vector<Rec> &R, int nt) {
    const int64_t n = (int64_t)R.size();
    if (n == 0) return {};
    std::vector<std::string> canon((size_t)n);
    parallel_for(n, nt, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) canon[(size_t)i] = canon_of(R[(size_t)i].motif);
    });
    const int64_t K = std::max<int64_t>(1, std::min<int64_t>(nt * 8, n / 2048 + 1));
    std::vector<int64_t> cut((size_t)K + 1);
    for (int64_t k = 0; k <= K; ++k) cut[(size_t)k] = n * k / K;
    std::vector<uint8_t> fresh((size_t)n, 0);
    std::vector<SpecOut> spec((size_t)K);
    parallel_items(K, nt, [&](int64_t k) { spec_run(u, R, canon, cut[(size_t)k], cut[(size_t)k + 1], fresh, spec[(size_t)k]); });
    // repair: chunk 0 is exact; later chunks are valid once the true run is
    // fresh at an index where the speculative run was fresh too
    std::vector<Rec> out;
    out.reserve((size_t)n);
    for (auto &r : spec[0].emitted) out.push_back(std::move(r));
    Rec cur = std::move(spec[0].pending);
    std::string cc = std::move(spec[0].pending_canon);
    Rec mg;
    for (int64_t k = 1; k < K; ++k) {
        const int64_t b = cut[(size_t)k], e = cut[(size_t)k + 1];
        SpecOut &sp = spec[(size_t)k];
        int64_t i = b;
        int64_t sync = -1;
        for (; i < e; ++i) {
            if (try_merge(u, cur, cc, R[(size_t)i], canon[(size_t)i], mg)) {
                cur = std::move(mg);
                cc = canon_of(cur.motif);
            } else {
                out.push_back(std::move(cur));
                cur = R[(size_t)i];
                cc = canon[(size_t)i];
                if (fresh[(size_t)i]) { sync = i; break; }
            }
        }
        if (sync < 0) continue;   // never re-synchronised: `cur` carries into chunk k+1
        // identical from `sync` on: take the speculative emissions after it
        for (size_t q = 0; q < sp.emitted.size(); ++q)
            if (sp.emit_step[q] > sync) out.push_back(std::move(sp.emitted[q]));
        cur = std::move(sp.pending);
        cc = std::move(sp.pending_canon);
    }
    out.push_back(std::move(cur));
    return out;
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
    if (canon_of(r1.motif) == canon_of(r2.motif)) return true;
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

// bwt.py:3189-3220.  After the (start, end) sort, equal keys (chrom, start,
// end, motif) sit inside runs of equal (start, end); the first occurrence
// keeps its position and takes the preferred content.
void dedup_sorted(std::vector<Rec> &recs) {
    std::vector<Rec> d;
    d.reserve(recs.size());
    size_t i = 0;
    const size_t n = recs.size();
    while (i < n) {
        size_t j = i + 1;
        while (j < n && recs[j].start == recs[i].start && recs[j].end == recs[i].end) ++j;
        const size_t first_out = d.size();
        for (size_t q = i; q < j; ++q) {
            Rec &r = recs[q];
            size_t hit = SIZE_MAX;
            for (size_t x = first_out; x < d.size(); ++x)
                if (d[x].chrom == r.chrom && d[x].motif == r.motif) { hit = x; break; }
            if (hit == SIZE_MAX) { d.push_back(std::move(r)); continue; }
            const Rec &ex = d[hit];
            bool repl = false;
            if (r.confidence > ex.confidence) repl = true;
            else if (r.confidence == ex.confidence) {
                if (r.mismatch_rate < ex.mismatch_rate) repl = true;
                else if (r.mismatch_rate == ex.mismatch_rate && r.tier < ex.tier) repl = true;
            }
            if (repl) d[hit] = std::move(r);
        }
        i = j;
    }
    recs.swap(d);
}

void process_unit(const Job &job, const std::vector<int32_t> &chroms, std::vector<std::vector<Rec>> &raw,
                  std::vector<Rec> &out, double *ms, int nt) {
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    UnitCtx u{&job, job.params.min_copies};
    // 1. nested suppression per chromosome (bwt.py:3928), concatenated in
    //    chromosome order, stable-sorted by (start, end).
    std::vector<Rec> recs;
    for (int32_t c : chroms) {
        std::vector<Rec> kept = suppress_nested_chrom(raw[(size_t)c], 0.5, nt);
        if (recs.empty()) recs.swap(kept);
        else for (auto &r : kept) recs.push_back(std::move(r));
        std::vector<Rec>().swap(raw[(size_t)c]);
    }
    sort_by_pos(recs, nt);
    auto t1 = clk::now();
    // 2. dedup (bwt.py:3189-3220)
    dedup_sorted(recs);
    auto t2 = clk::now();
    // 3. merge adjacent (bwt.py:3222-3289)
    recs = merge_fold(u, recs, nt);
    auto t3 = clk::now();
    // 4. refine (bwt.py:3291-3314)
    parallel_items((int64_t)recs.size(), nt, [&](int64_t k) {
        Rec &r = recs[(size_t)k];
        if (r.mismatch_rate == 0.0) return;
        int64_t m = (int64_t)r.motif.size();
        if (m <= 0) {
            const int64_t rc = (int64_t)std::nearbyint(r.copies);
            m = std::max<int64_t>(1, r.length / std::max<int64_t>(1, rc ? rc : 1));
        }
        r = recompute(u, r.chrom, r.start, r.end, m, r.tier);
    });
    sort_by_pos(recs, nt);
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
    sort_by_pos(recs, nt);
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
    const int T = host_threads(job.params);
    // many small units: one thread per unit; few large units: all threads inside each
    int64_t busy = 0;
    for (auto &v : job.raw) busy += v.empty() ? 0 : 1;
    if (busy >= T) {
        parallel_items(job.nunits, T, [&](int64_t k) {
            process_unit(job, units[(size_t)k], job.raw, res[(size_t)k], &ms[(size_t)k * 4], 1);
        });
    } else {
        for (int32_t k = 0; k < job.nunits; ++k)
            process_unit(job, units[(size_t)k], job.raw, res[(size_t)k], &ms[(size_t)k * 4], T);
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
