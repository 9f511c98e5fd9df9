// render.cpp -- compound detection and the five output writers
// (TandemRepeatFinder.save_results bwt.py:4141-4198, _detect_compound_repeats
// 3995-4139, _simple_kmer_scan 3956-3993, TandemRepeat.to_* 454-641).
// Python's "{x:.Nf}" and C's "%.Nf" both print the exact binary value rounded
// half-to-even, so numeric columns are byte-identical.
#include <algorithm>
#include <map>
#include <thread>
#include <optional>
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "common.h"
#include "fmtnum.h"

namespace bwtmi {
namespace {

struct View {
    const char *p = nullptr;
    int64_t n = 0;
    bool empty() const { return n <= 0; }
};

View act_of(const Job &job, const Rec &r) {
    View v;
    if (r.act_kind == ACT_NONE) return v;
    const Contig &c = job.contigs[(size_t)r.chrom];
    v.p = (r.act_kind == ACT_FULL ? c.full.data() : c.trimmed()) + r.act_off;
    v.n = r.act_len;
    return v;
}

Rec kmer_piece(int32_t chrom, int64_t start, int64_t end, const std::string &motif, int64_t copies,
               int32_t tier, int8_t kind, int64_t off, int64_t len) {
    Rec r;
    r.chrom = chrom;
    r.start = start;
    r.end = end;
    r.length = end - start;
    r.motif = motif;
    r.copies = (double)copies;
    r.tier = tier;
    r.confidence = 1.0;
    r.mismatch_rate = 0.0;
    r.max_mm = 0;
    r.n_eval = copies;
    r.strand = '+';
    r.pmatch = 100.0;
    r.pindel = 0.0;
    r.score = 100;
    r.kmer_stats = true;
    r.act_kind = kind;
    r.act_off = off;
    r.act_len = len;
    return r;
}

// _simple_kmer_scan(chrom, start, end, k=3, use_full_seq=True)
void kmer_scan(const Job &job, int32_t chrom, int64_t start, int64_t end, RecVec &out) {
    const Seq &seq = job.contigs[(size_t)chrom].full;
    const int64_t L = (int64_t)seq.size();
    const int64_t k = 3;
    if (seq.empty() || start >= end || start < 0 || end > L) return;
    const char *reg = seq.data() + start;
    const int64_t rl = end - start;
    int64_t i = 0;
    while (i < rl - k) {
        int64_t c = 1, j = i + k;
        while (j + k <= rl && std::memcmp(reg + j, reg + i, (size_t)k) == 0) {
            ++c;
            j += k;
        }
        if (c >= 5) {
            out.push_back(kmer_piece(chrom, start + i, start + j, std::string(reg + i, (size_t)k), c, 1,
                                     ACT_FULL, start + i, j - i));
            i = j;
        } else {
            ++i;
        }
    }
}

// one output row of the STRfinder writer: a final record or a compound piece,
// with its compound partner (bwt.py:4126-4130)
struct Row {
    const Rec *r;
    const Rec *partner;   // nullptr unless is_compound
    int64_t start, end;   // r's, kept inline so ordering the rows reads no record
    int32_t unit;
};

inline Row row_of(const Job &job, const Rec *r, const Rec *partner) {
    return Row{r, partner, r->start, r->end, job.contigs[(size_t)r->chrom].unit};
}

struct Compound {
    std::deque<Rec> pool;                // k-mer pieces, pointer-stable
    std::deque<std::deque<Rec>> pools;   // split pieces of the walk chunks (a moved deque keeps its
                                         // elements in place; the outer deque never moves its deques)
    std::vector<Row> rows;
};

// rows emitted by a walk over some indices, with the index each was emitted from
struct Walk {
    std::vector<Row> rows;
    std::vector<size_t> at;
    std::deque<Rec> pool;
    size_t next = 0;
    void emit(Row r, size_t i0) {
        rows.push_back(r);
        at.push_back(i0);
    }
};

// _detect_compound_repeats (bwt.py:3995-4139) over the final records; works on
// pointers, so the final records are never copied
void detect_compounds(const Job &job, const RecVec &recs, Compound &out, int nt) {
    auto T0 = std::chrono::steady_clock::now();
    // one pass over the records, in parallel chunks: chromosome of each and the
    // _simple_kmer_scan pieces after every 3-mer record (kept in record order)
    const size_t NR = recs.size();
    const int CK = NR > 8192 ? 4 * std::max(1, nt) : 1;
    struct Chunk {
        int32_t first = -1;
        bool mixed = false;
        std::vector<size_t> bounds;                   // q in the chunk with recs[q].chrom != recs[q - 1].chrom
        std::vector<std::pair<size_t, Rec>> pieces;   // (record index, piece)
    };
    std::vector<Chunk> ck((size_t)CK);
    run_tasks(CK, nt, [&](int64_t t) {
        Chunk &C = ck[(size_t)t];
        RecVec kr;
        for (size_t q = NR * (size_t)t / (size_t)CK; q < NR * (size_t)(t + 1) / (size_t)CK; ++q) {
            const Rec &r = recs[q];
            if (C.first < 0) C.first = r.chrom;
            else if (r.chrom != C.first) C.mixed = true;
            if (q > 0 && r.chrom != recs[q - 1].chrom) C.bounds.push_back(q);
            if (r.motif.size() != 3) continue;
            const Seq &full = job.contigs[(size_t)r.chrom].full;
            if (full.empty()) continue;
            const int64_t a = r.end, b = std::min<int64_t>((int64_t)full.size(), r.end + 50);
            if (a >= b) continue;
            kr.clear();
            kmer_scan(job, r.chrom, a, b, kr);
            for (auto &x : kr)
                if (x.motif != r.motif) C.pieces.emplace_back(q, std::move(x));
        }
    });
    bool single = true;
    for (auto &C : ck) single = single && !C.mixed && (C.first < 0 || C.first == ck[0].first);
    std::vector<int32_t> chrom_order;
    std::vector<std::vector<const Rec *>> by(job.contigs.size());
    if (single && NR > 0) {   // one chromosome: its list is every record, in order
        chrom_order.push_back(recs[0].chrom);
        auto &lst = by[(size_t)recs[0].chrom];
        lst.resize(NR);
        run_tasks(CK, nt, [&](int64_t t) {
            for (size_t q = NR * (size_t)t / (size_t)CK; q < NR * (size_t)(t + 1) / (size_t)CK; ++q) lst[q] = &recs[q];
        });
    } else if (NR > 0) {
        // the usual multi-contig list: each chromosome's records are one contiguous
        // run (the fold units are concatenated), so every list is a range, filled in
        // parallel; otherwise one serial pass
        std::vector<size_t> runs{0};   // start of each run of equal chromosome
        for (auto &C : ck) runs.insert(runs.end(), C.bounds.begin(), C.bounds.end());
        runs.push_back(NR);
        bool contiguous = true;
        {
            std::vector<uint8_t> seen(job.contigs.size(), 0);
            for (size_t k = 0; k + 1 < runs.size() && contiguous; ++k) {
                const size_t ch = (size_t)recs[runs[k]].chrom;
                contiguous = !seen[ch];
                seen[ch] = 1;
            }
        }
        if (contiguous) {
            for (size_t k = 0; k + 1 < runs.size(); ++k) {
                const int32_t ch = recs[runs[k]].chrom;
                chrom_order.push_back(ch);
                by[(size_t)ch].resize(runs[k + 1] - runs[k]);
            }
            run_tasks(CK, nt, [&](int64_t t) {
                const size_t a = NR * (size_t)t / (size_t)CK, b = NR * (size_t)(t + 1) / (size_t)CK;
                size_t k = (size_t)(std::upper_bound(runs.begin(), runs.end(), a) - runs.begin()) - 1;
                for (size_t q = a; q < b; ++q) {
                    while (q >= runs[k + 1]) ++k;
                    by[(size_t)recs[q].chrom][q - runs[k]] = &recs[q];
                }
            });
        } else {
            for (const Rec &r : recs) {
                if (by[(size_t)r.chrom].empty()) chrom_order.push_back(r.chrom);
                by[(size_t)r.chrom].push_back(&r);
            }
        }
    }
    auto T1 = std::chrono::steady_clock::now();
    std::vector<size_t> n_main(job.contigs.size(), 0);
    for (int32_t ch : chrom_order) n_main[(size_t)ch] = by[(size_t)ch].size();
    // pieces go behind their chromosome's records, in record order (bwt.py:4011-4024)
    for (auto &C : ck)
        for (auto &pc : C.pieces) {
            out.pool.push_back(std::move(pc.second));
            by[(size_t)recs[pc.first].chrom].push_back(&out.pool.back());
        }
    auto T2 = std::chrono::steady_clock::now();
    double tsort = 0;
    for (int32_t ch : chrom_order) {
        auto S0 = std::chrono::steady_clock::now();
        std::vector<const Rec *> &rs = by[(size_t)ch];
        // stable sort by start: the final records arrive sorted, only the
        // k-mer pieces appended behind them need ordering and a stable merge
        auto by_start = [](const Rec *a, const Rec *b) { return a->start < b->start; };
        const size_t nmain = n_main[(size_t)ch];
        std::vector<uint8_t> chunk_sorted((size_t)CK, 1);
        run_tasks(CK, nt, [&](int64_t t) {   // chunk t checks the pairs ending in it
            const size_t a = std::max<size_t>(1, nmain * (size_t)t / (size_t)CK), b = nmain * (size_t)(t + 1) / (size_t)CK;
            for (size_t k = a; k < b; ++k)
                if (rs[k]->start < rs[k - 1]->start) { chunk_sorted[(size_t)t] = 0; return; }
        });
        bool main_sorted = true;
        for (auto v : chunk_sorted) main_sorted = main_sorted && v;
        if (main_sorted && rs.size() > nmain) {
            // few k-mer pieces into a long sorted list: each piece goes behind the
            // main records with an equal start (a stable merge), and the main
            // list is copied in parallel segments between the insertion points
            std::stable_sort(rs.begin() + (std::ptrdiff_t)nmain, rs.end(), by_start);
            const size_t np = rs.size() - nmain;
            std::vector<size_t> at(np);
            for (size_t q = 0; q < np; ++q)
                at[q] = (size_t)(std::upper_bound(rs.begin(), rs.begin() + (std::ptrdiff_t)nmain, rs[nmain + q], by_start) -
                                 rs.begin());
            std::vector<const Rec *> merged(rs.size());
            run_tasks((int64_t)np + 1, nt, [&](int64_t q) {   // segment q: main [at[q-1], at[q]) then piece q
                const size_t a0 = q ? at[(size_t)q - 1] : 0, a1 = (size_t)q < np ? at[(size_t)q] : nmain;
                std::copy(rs.begin() + (std::ptrdiff_t)a0, rs.begin() + (std::ptrdiff_t)a1,
                          merged.begin() + (std::ptrdiff_t)(a0 + (size_t)q));
                if ((size_t)q < np) merged[a1 + (size_t)q] = rs[nmain + (size_t)q];
            });
            rs.swap(merged);
        } else if (main_sorted) {
        } else {
            std::stable_sort(rs.begin(), rs.end(), by_start);
        }
        // spans of the > 10 bp motifs in start order, with the prefix max of
        // their ends: the "covered" test visits only those that can overlap
        struct Long { int64_t s, e, pe; };
        std::vector<std::vector<Long>> lpart((size_t)CK);
        const size_t NS = rs.size();
        run_tasks(CK, nt, [&](int64_t t) {
            for (size_t k = NS * (size_t)t / (size_t)CK; k < NS * (size_t)(t + 1) / (size_t)CK; ++k)
                if (rs[k]->motif.size() > 10) lpart[(size_t)t].push_back({rs[k]->start, rs[k]->end, 0});
        });
        std::vector<Long> longs;
        for (auto &lp : lpart)
            for (auto &l : lp) {
                l.pe = longs.empty() ? l.e : std::max(longs.back().pe, l.e);
                longs.push_back(l);
            }
        tsort += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - S0).count();
        const Contig &ctg = job.contigs[(size_t)ch];
        const int64_t TL = ctg.trimmed_len();
        const char *tseq = ctg.trimmed();
        // The walk's only state is the index i; a step may consume 1 or 2
        // records, or more after splits.  Chunks are walked speculatively in
        // parallel as if the walk arrived at their first index; a serial
        // repair walks from the true index until it reaches an index the
        // speculative run also stepped from, after which the two coincide.
        const size_t N = rs.size();
        auto step = [&](size_t i, Walk &w) -> size_t {
            const size_t i0 = i;
            const Rec *cur = rs[i];
            if (cur->motif.size() == 3 && cur->copies >= 10 && TL > 0) {
                // repeat_seq = sequences[chrom][cur.start:cur.end] (trimmed sequence, restored
                // coordinates -- bwt.py:4045-4047)
                const int64_t a = std::min(std::max<int64_t>(cur->start, 0), TL);
                const int64_t b = std::max(a, std::min(std::max<int64_t>(cur->end, 0), TL));
                const char *rsq = tseq + a;
                const int64_t rl = b - a;
                const int64_t k = 3;
                // Every split point sp (k <= sp < rl - k, a multiple of k) sees whole
                // copies only: l1 = l2 = k, c1 = the leading copies equal to copy 0,
                // capped at sp / k, and c2 = the run of copies equal to copy sp/k
                // (exact equality chains), so both come from one pass over the
                // copies instead of a rescan per split point (O(copies), not O(copies^2))
                thread_local std::vector<int32_t> run_from;
                const int64_t nq = rl / k;   // whole copies
                int64_t lead = 0;
                if (rl - k > k) {
                    while (lead < nq && std::memcmp(rsq + lead * k, rsq, (size_t)k) == 0) ++lead;
                    run_from.assign((size_t)nq + 1, 0);
                    for (int64_t q = nq - 1; q >= 0; --q)
                        run_from[(size_t)q] = 1 + (q + 1 < nq && std::memcmp(rsq + q * k, rsq + (q + 1) * k, (size_t)k) == 0
                                                       ? run_from[(size_t)q + 1] : 0);
                }
                for (int64_t sp = k; sp < rl - k; sp += k) {
                    const int64_t l1 = k, l2 = k;
                    if (std::memcmp(rsq, rsq + sp, (size_t)k) == 0) continue;
                    const int64_t c1 = std::min<int64_t>(lead, sp / k);
                    const int64_t c2 = run_from[(size_t)(sp / k)];
                    if (c1 >= 5 && c2 >= 5 && (double)(c1 * l1 + c2 * l2) >= (double)rl * 0.9) {
                        const int64_t e1 = cur->start + c1 * l1;
                        // actual = repeat_seq[:c1*l1], repeat_seq[c1*l1 : c1*l1 + c2*l2]
                        const int64_t x1 = std::min(c1 * l1, rl);
                        const int64_t y0 = std::min(c1 * l1, rl), y1 = std::max(y0, std::min(c1 * l1 + c2 * l2, rl));
                        w.pool.push_back(kmer_piece(ch, cur->start, e1, std::string(rsq, (size_t)l1), c1, cur->tier,
                                                      ACT_TRIMMED, a, x1));
                        Rec *r1 = &w.pool.back();
                        w.pool.push_back(kmer_piece(ch, e1, e1 + c2 * l2, std::string(rsq + sp, (size_t)l2), c2,
                                                      cur->tier, ACT_TRIMMED, a + y0, y1 - y0));
                        r1->is_compound = true;
                        w.emit(row_of(job, r1, &w.pool.back()), i0);
                        ++i;   // the reference advances i inside the split loop (bwt.py:4083)
                    }
                }
            }
            if (i + 1 < N) {
                const Rec *nx = rs[i + 1];
                const int64_t gap = nx->start - cur->end;
                if (gap <= 5 && cur->motif.size() <= 4 && nx->motif.size() <= 4 && cur->motif != nx->motif &&
                    cur->copies >= 5 && nx->copies >= 5) {
                    const int64_t cs = cur->start, ce = nx->end;
                    // any(long overlaps >= 80 %): a long with s >= ce or e <= cs has
                    // ov = 0, so only those before the first s >= ce whose prefix
                    // max end still exceeds cs can qualify
                    bool covered = false;
                    size_t k = (size_t)(std::lower_bound(longs.begin(), longs.end(), ce,
                                                         [](const Long &l, int64_t x) { return l.s < x; }) -
                                        longs.begin());
                    while (k > 0 && !covered) {
                        const Long &lm = longs[--k];
                        if (lm.pe <= cs) break;
                        const int64_t ov = std::max<int64_t>(0, std::min(ce, lm.e) - std::max(cs, lm.s));
                        if ((double)ov / (double)(ce - cs) >= 0.8) covered = true;
                    }
                    if (!covered) {
                        w.emit(row_of(job, cur, nx), i0);
                        return i + 2;
                    }
                }
            }
            w.emit(row_of(job, cur, nullptr), i0);
            return i + 1;
        };
        const int K = N > 8192 ? 4 * std::max(1, nt) : 1;
        std::vector<size_t> cut((size_t)K + 1);
        for (int k = 0; k <= K; ++k) cut[(size_t)k] = N * (size_t)k / (size_t)K;
        std::vector<uint8_t> from(N, 0);   // from[i]: the speculative run of i's chunk stepped from i
        std::vector<Walk> W((size_t)K);
        run_tasks(K, nt, [&](int64_t k) {
            size_t i = cut[(size_t)k];
            Walk &w = W[(size_t)k];
            w.rows.reserve(cut[(size_t)k + 1] - i + 16);
            w.at.reserve(cut[(size_t)k + 1] - i + 16);
            while (i < cut[(size_t)k + 1]) {
                from[i] = 1;
                i = step(i, w);
            }
            w.next = i;
        });
        // the serial repair only decides which rows are taken; they are
        // copied into place afterwards, in parallel
        std::vector<Walk> reps((size_t)K);
        std::vector<std::pair<const Row *, size_t>> seg;
        size_t ti = 0;
        for (int k = 0; k < K; ++k) {
            Walk &sp = W[(size_t)k];
            if (ti >= cut[(size_t)k + 1]) continue;   // the true walk stepped over this chunk
            Walk &rep = reps[(size_t)k];
            while (ti < cut[(size_t)k + 1] && !from[ti]) ti = step(ti, rep);
            if (!rep.rows.empty()) seg.emplace_back(rep.rows.data(), rep.rows.size());
            if (ti >= cut[(size_t)k + 1]) continue;
            size_t q = (size_t)(std::lower_bound(sp.at.begin(), sp.at.end(), ti) - sp.at.begin());
            if (q < sp.rows.size()) seg.emplace_back(sp.rows.data() + q, sp.rows.size() - q);
            ti = sp.next;
        }
        std::vector<size_t> at(seg.size() + 1, out.rows.size());
        for (size_t q = 0; q < seg.size(); ++q) at[q + 1] = at[q] + seg[q].second;
        out.rows.resize(at.back());
        run_tasks((int64_t)seg.size(), nt, [&](int64_t q) {
            std::copy(seg[(size_t)q].first, seg[(size_t)q].first + seg[(size_t)q].second, out.rows.begin() + (std::ptrdiff_t)at[(size_t)q]);
        });
        for (auto &w : reps) out.pools.push_back(std::move(w.pool));
        for (auto &w : W) out.pools.push_back(std::move(w.pool));
    }
    if (stats_on()) {
        auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "  compounds: group+kmer %.1f sort %.1f walk %.1f ms (%zu pieces)\n", d(T0, T1), tsort,
                     d(T2, std::chrono::steady_clock::now()) - tsort, out.pool.size());
    }
}

// ---------------------------------------------------------------- formatting
struct Out {
    // rows are written through a raw cursor into s (sized ahead, grown by
    // doubling); finish() cuts s to what was written
    Text s;
    char *w = nullptr, *e = nullptr;
    std::string built, fc;   // per-chunk scratch of the row formatters (no thread-local lookups per row)
    void reserve(size_t n) {
        const size_t used = w ? (size_t)(w - s.data()) : 0;
        s.set_size(used);
        s.grow(used + n);
        w = s.data() + used;
        e = s.data() + s.capacity();
    }
    void need(size_t n) {
        if ((size_t)(e - w) < n) reserve(std::max(n, s.capacity()));
    }
    Text finish() {
        s.set_size(w ? (size_t)(w - s.data()) : 0);
        w = e = nullptr;
        return std::move(s);
    }
    void put(const char *p, int64_t n) {
        if (n <= 0) return;
        need((size_t)n);
        std::memcpy(w, p, (size_t)n);
        w += n;
    }
    void put(const std::string &x) { put(x.data(), (int64_t)x.size()); }
    void put(View v) { put(v.p, v.n); }
    void c(char ch) {
        need(1);
        *w++ = ch;
    }
    void f(const char *fmt, double x) {   // printf keeps Python's exact-value rounding
        if (fmt[1] == '.' && fmt[2] == '0' && fmt[3] == 'f' && std::fabs(x) < 1e15 && !std::signbit(x)) {
            // %.0f rounds the exact binary value to nearest, ties to even --
            // nearbyint in the default rounding mode, without printf
            i((int64_t)std::nearbyint(x));
            return;
        }
        if (fmt[1] == '.' && fmt[2] >= '1' && fmt[2] <= '3' && fmt[3] == 'f') {   // exact, no printf (fmtnum.h)
            need(40);
            if (char *end = fixed_dec(x, fmt[2] - '0', w)) {
                w = end;
                return;
            }
        }
        char b[64];
        int n = snprintf(b, sizeof b, fmt, x);
        put(b, n);
    }
    void i(int64_t x) {   // decimal (std::to_chars took a third of the rows' time)
        need(24);
        w = int_dec(x, w);
    }
    void rep(const std::string &m, int64_t times) {
        for (int64_t k = 0; k < times; ++k) put(m);
    }
};

inline int64_t py_round(double x) { return (int64_t)std::nearbyint(x); }

void comp_entropy(const Rec &r, double comp[4], double &ent) {
    if (r.kmer_stats) {
        comp[0] = comp[1] = comp[2] = comp[3] = 0.0;
        ent = 1.5;
        return;
    }
    if (r.stats_none) {   // to_trf_table/to_trf_dat: composition or 25 % each (bwt.py:485, 505)
        comp[0] = comp[1] = comp[2] = comp[3] = 25.0;
        ent = 0.0;
        return;
    }
    composition_of(r.motif.data(), (int64_t)r.motif.size(), comp);
    ent = entropy_of(r.motif.data(), (int64_t)r.motif.size());
}

void row_strfinder(Out &o, const Job &job, const Rec &r, const Rec *partner) {
    const Contig &c = job.contigs[(size_t)r.chrom];
    const Seq &full = c.full;
    const int64_t FL = (int64_t)full.size();
    View fl, fr;
    if (!full.empty()) {   // full[max(0,start-30):start], full[end:end+30]
        int64_t a = std::min(std::max<int64_t>(0, r.start - 30), FL), b = std::min(std::max<int64_t>(r.start, 0), FL);
        if (b > a) { fl.p = full.data() + a; fl.n = b - a; }
        a = std::min(std::max<int64_t>(r.end, 0), FL);
        b = std::min(std::max<int64_t>(r.end + 30, 0), FL);
        if (b > a) { fr.p = full.data() + a; fr.n = b - a; }
    }
    const bool flanks = !fl.empty() || !fr.empty();
    o.put("STR_");
    o.put(c.name);
    o.c('\t');
    if (partner) {
        const Rec &p = *partner;
        const int64_t k1 = py_round(r.copies), k2 = py_round(p.copies);
        std::string core;
        View a1 = act_of(job, r), a2 = act_of(job, p);
        if (!a1.empty()) core.append(a1.p, (size_t)a1.n);
        else for (int64_t k = 0; k < k1; ++k) core += r.motif;
        if (!a2.empty()) core.append(a2.p, (size_t)a2.n);
        else for (int64_t k = 0; k < k2; ++k) core += p.motif;
        o.put(c.name); o.c(':'); o.i(r.start + 1); o.c('-'); o.i(p.end); o.c('\t');
        o.c('['); o.put(r.motif); o.put("]n+["); o.put(p.motif); o.put("]n\t");
        o.i((int64_t)r.motif.size()); o.c('['); o.put(r.motif); o.c(']'); o.i(k1); o.c(';');
        o.i((int64_t)p.motif.size()); o.c('['); o.put(p.motif); o.c(']'); o.i(k2); o.put(",0\t");
        o.i(k1); o.c('/'); o.i(k2); o.c('\t');
        o.put(core); o.put("\t100%\t-\t");
        o.i(k1); o.c(':'); o.i(k2); o.c('\t'); o.i(k1 + k2); o.c('\t');
        if (flanks) { o.put(fl); o.put(core); o.put(fr); } else o.put(core);
        o.put("\t-\n");
        return;
    }
    const std::string &cons = r.motif;
    const int64_t ml = (int64_t)cons.size();
    const int64_t cc = (int64_t)std::floor(r.copies + 1e-6);
    o.put(c.name); o.c(':'); o.i(r.start + 1); o.c('-'); o.i(r.end); o.c('\t');
    o.c('['); o.put(cons); o.put("]n\t");
    o.i(ml); o.c('['); o.put(cons); o.c(']'); o.i(cc); o.c(','); o.i((r.end - r.start) - ml * cc); o.c('\t');
    if (std::fabs(r.copies - std::nearbyint(r.copies)) < 1e-6) {
        o.i(py_round(r.copies));
    } else {
        char b[64];
        char *e = fixed_dec(r.copies, 2, b);
        const int n = e ? (int)(e - b) : snprintf(b, sizeof b, "%.2f", r.copies);
        int m = n;
        while (m > 0 && b[m - 1] == '0') --m;
        while (m > 0 && b[m - 1] == '.') --m;
        o.put(b, m);
    }
    o.c('\t');
    // core sequence: the actual-sequence slice, or the motif repeated int(copies) times
    std::string &built = o.built;
    View core = act_of(job, r);
    if (core.empty()) {
        built.clear();
        for (int64_t k = 0; k < (int64_t)r.copies; ++k) built += cons;
        core.p = built.data();
        core.n = (int64_t)built.size();
    }
    if (core.n > 150) {
        o.put(core.p, 70);
        o.put("... (x"); o.i(cc); o.c(')');
    } else {
        o.put(core);
    }
    o.c('\t');
    o.f("%.0f", r.pmatch);
    o.put("%\t-\t");
    o.i(cc); o.c(':'); o.i(r.n_eval); o.c('\t'); o.i(r.n_eval); o.c('\t');
    const int64_t tot = (flanks ? fl.n + fr.n : 0) + core.n;
    if (tot > 500) {   // full_seq[:250] + "..." + full_seq[-200:] of fl + core + fr, without building it
        const View parts[3] = {flanks ? fl : View{}, core, flanks ? fr : View{}};
        auto put_range = [&](int64_t a, int64_t b) {   // bytes [a, b) of the concatenation
            int64_t base = 0;
            for (const View &v : parts) {
                const int64_t lo = std::max(a, base), hi = std::min(b, base + v.n);
                if (hi > lo) o.put(v.p + (lo - base), hi - lo);
                base += v.n;
            }
        };
        put_range(0, 250);
        o.put("...");
        put_range(tot - 200, tot);
    } else {
        if (flanks) { o.put(fl); o.put(core); o.put(fr); } else o.put(core);
    }
    o.c('\t');
    if (!r.variations.empty()) o.put(r.variations); else o.c('-');
    o.c('\n');
}

const char *kVcfHeader =
    "##fileformat=VCFv4.2\n"
    "##INFO=<ID=MOTIF,Number=1,Type=String,Description=\"Original seed motif\">\n"
    "##INFO=<ID=CONS_MOTIF,Number=1,Type=String,Description=\"Consensus motif from all copies\">\n"
    "##INFO=<ID=COPIES,Number=1,Type=Float,Description=\"Number of copies\">\n"
    "##INFO=<ID=TIER,Number=1,Type=Integer,Description=\"Detection tier (1=short, 2=medium/long, 3=very long)\">\n"
    "##INFO=<ID=CONF,Number=1,Type=Float,Description=\"Confidence score\">\n"
    "##INFO=<ID=MM_RATE,Number=1,Type=Float,Description=\"Overall mismatch rate across all copies\">\n"
    "##INFO=<ID=MAX_MM_PER_COPY,Number=1,Type=Integer,Description=\"Maximum mismatches in any single copy\">\n"
    "##INFO=<ID=N_COPIES_EVAL,Number=1,Type=Integer,Description=\"Number of copies evaluated for consensus\">\n"
    "##INFO=<ID=STRAND,Number=1,Type=String,Description=\"Strand of canonical motif (+/-)\">\n"
    "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n";

}  // namespace

// Rows are formatted in parallel, in chunks of consecutive rows; each chunk is
// one part of the output, so concatenating the parts gives the file.
void render_rows(Job &job, int fmt, const int64_t *row_base, Rendered &out,
                 const std::function<void(size_t)> *on_part) {
    auto t0 = std::chrono::steady_clock::now();
    job.assign_units();
    Compound comp;
    std::vector<Row> rows;
    if (fmt == BWTMI_FMT_STRFINDER) {
        BWTMI_STAGE("bwtmi:compounds");
        detect_compounds(job, job.final_recs, comp, host_threads(job.params));
        rows.swap(comp.rows);
    } else {
        rows.reserve(job.final_recs.size());
        for (const Rec &r : job.final_recs) rows.push_back(row_of(job, &r, nullptr));
    }
    // sorted(all_repeats, key=lambda r: (natural_sort_key(r.chrom), r.start, r.end)) (bwt.py:4150)
    // The rows arrive ordered by (unit, start) in the usual case (one contig
    // per unit): then only runs of equal (unit, start) need a stable order by
    // end, which equals the full stable sort.
    auto unit_start_lt = [](const Row &a, const Row &b) {
        if (a.unit != b.unit) return a.unit < b.unit;
        return a.start < b.start;
    };
    const int nt = host_threads(job.params);
    const size_t NR = rows.size();
    const int RC = NR > 8192 ? 4 * nt : 1;
    std::vector<uint8_t> chunk_ok((size_t)RC, 1);
    run_tasks(RC, nt, [&](int64_t t) {   // sorted by (unit, start)?  chunk t checks pairs ending in it
        const size_t a = std::max<size_t>(1, NR * (size_t)t / (size_t)RC), b = NR * (size_t)(t + 1) / (size_t)RC;
        for (size_t k = a; k < b; ++k)
            if (unit_start_lt(rows[k], rows[k - 1])) { chunk_ok[(size_t)t] = 0; return; }
    });
    bool by_unit_start = true;
    for (auto v : chunk_ok) by_unit_start = by_unit_start && v;
    if (by_unit_start) {
        run_tasks(RC, nt, [&](int64_t t) {   // chunk t orders the equal-(unit, start) runs that begin in it
            size_t i = NR * (size_t)t / (size_t)RC;
            const size_t b = NR * (size_t)(t + 1) / (size_t)RC;
            while (i > 0 && i < b && !unit_start_lt(rows[i - 1], rows[i])) ++i;
            while (i < b) {
                size_t j = i + 1;
                while (j < NR && !unit_start_lt(rows[i], rows[j])) ++j;   // equal (unit, start)
                for (size_t a = i + 1; a < j; ++a) {   // stable insertion sort by end (runs are short)
                    const Row x = rows[a];
                    size_t q = a;
                    while (q > i && rows[q - 1].end > x.end) {
                        rows[q] = rows[q - 1];
                        --q;
                    }
                    rows[q] = x;
                }
                i = j;
            }
        });
    } else {
        std::stable_sort(rows.begin(), rows.end(), [](const Row &a, const Row &b) {
            if (a.unit != b.unit) return a.unit < b.unit;
            if (a.start != b.start) return a.start < b.start;
            return a.end < b.end;
        });
    }
    auto t1 = std::chrono::steady_clock::now();
    std::string head;
    switch (fmt) {
        case BWTMI_FMT_BED:
            head = "# Tandem Repeats (BED format with imperfect repeat support)\n"
                   "# chrom\tstart\tend\tconsensus_motif\tcopies\ttier\tmismatch_rate\tstrand\n";
            break;
        case BWTMI_FMT_VCF: head = kVcfHeader; break;
        case BWTMI_FMT_TRF_TABLE:
            head = "# Tandem Repeats Finder Compatible Table Format\n"
                   "# Indices\tPeriod\tCopyNumber\tConsensusSize\tPercentMatches\tPercentIndels\t"
                   "Score\tA\tC\tG\tT\tEntropy\n";
            break;
        case BWTMI_FMT_TRF_DAT: break;
        case BWTMI_FMT_STRFINDER:
            head = "STR_marker\tSTR_position\tSTR_motif\tSTR_genotype_structure\tSTR_genotype\t"
                   "STR_core_seq\tAllele_coverage\tAlleles_ratio\tReads_Distribution(consensused)\t"
                   "STR_depth\tFull_seq\tVariations\n";
            break;
        default:
            fail(BWTMI_E_ARG, "unknown output format %d", fmt);
    }
    // chunks of <= CH consecutive rows that never span two fold units; VCF row
    // ids are row_base[unit] + rank within the unit (global index when the
    // caller renders only its own shard), else the local index
    const int64_t n = (int64_t)rows.size();
    // >= 8 chunks per thread while that keeps them >= 256 rows (a 40k-row shard
    // in 8192-row chunks kept 5 of 16 threads busy; in 1024-row chunks, 2 or 3
    // chunks a thread, the last wave left threads idle)
    const int64_t CH = std::max<int64_t>(256, std::min<int64_t>(8192, n / (8 * (int64_t)host_threads(job.params)) + 1));
    auto unit_of = [&](int64_t k) { return rows[(size_t)k].unit; };
    struct Chunk { int64_t a, b, id0; int32_t unit; };
    std::vector<Chunk> chunks;
    for (int64_t a = 0; a < n;) {
        const int32_t un = unit_of(a);
        int64_t e = a;
        if (by_unit_start)   // rows ordered by unit: the unit's run ends at the first larger unit
            e = (int64_t)(std::partition_point(rows.begin() + (std::ptrdiff_t)a, rows.end(),
                                               [un](const Row &x) { return x.unit == un; }) - rows.begin());
        else
            while (e < n && unit_of(e) == un) ++e;
        const int64_t base = row_base ? row_base[un] : a;
        for (int64_t c = a; c < e; c += CH) chunks.push_back({c, std::min(e, c + CH), base + (c - a), un});
        a = e;
    }
    out.header = std::move(head);
    out.parts.clear();
    out.parts.resize(chunks.size());
    out.part_unit.resize(chunks.size());
    for (size_t q = 0; q < chunks.size(); ++q) out.part_unit[q] = chunks[q].unit;
    auto t2 = std::chrono::steady_clock::now();
    std::optional<StageRange> fr;
    fr.emplace("bwtmi:format");
    // BWTMI_STATS=3: per-chunk timeline (thread, formatting, on_part) of this stage
    struct Tl { double a, b, c; size_t th; };
    std::vector<Tl> tl(stats_on(3) ? chunks.size() : 0);
    auto now_ms = [t2] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t2).count(); };
    run_tasks((int64_t)chunks.size(), host_threads(job.params), [&](int64_t ck) {
        if (!tl.empty()) { tl[(size_t)ck].a = now_ms(); tl[(size_t)ck].th = std::hash<std::thread::id>()(std::this_thread::get_id()); }
        Out o;
        const Chunk &C = chunks[(size_t)ck];
        const int64_t a = C.a, b = C.b;
        o.reserve((size_t)(b - a) * 256);
        double cp[4], ent;
        // a row's flanks and core are bytes of its contig at random distances
        // from the last row's: their lines are requested a few rows ahead
        constexpr int64_t kAhead = 6;
        auto prefetch_row = [&](int64_t k) {
            const Rec &r = *rows[(size_t)k].r;
            const Seq &full = job.contigs[(size_t)r.chrom].full;
            if (full.empty()) return;
            const int64_t FL = (int64_t)full.size();
            const int64_t s0 = std::min(std::max<int64_t>(0, r.start - 30), FL - 1), e0 = std::min(std::max<int64_t>(0, r.end), FL - 1);
            __builtin_prefetch(full.data() + s0);
            __builtin_prefetch(full.data() + s0 + 64);
            __builtin_prefetch(full.data() + e0);
        };
        if (fmt == BWTMI_FMT_STRFINDER)
            for (int64_t k = a; k < std::min(b, a + kAhead); ++k) prefetch_row(k);
        for (int64_t k = a; k < b; ++k) {
            if (fmt == BWTMI_FMT_STRFINDER && k + kAhead < b) prefetch_row(k + kAhead);
            const Rec &r = *rows[(size_t)k].r;
            const int64_t row_id = C.id0 + (k - a);
            switch (fmt) {
                case BWTMI_FMT_BED:
                    o.put(job.contigs[(size_t)r.chrom].name); o.c('\t'); o.i(r.start); o.c('\t'); o.i(r.end);
                    o.c('\t'); o.put(r.motif); o.c('\t'); o.f("%.1f", r.copies); o.c('\t'); o.i(r.tier); o.c('\t');
                    o.f("%.3f", r.mismatch_rate); o.c('\t'); o.c(r.strand); o.c('\n');
                    break;
                case BWTMI_FMT_VCF:
                    o.put(job.contigs[(size_t)r.chrom].name); o.c('\t'); o.i(r.start + 1); o.put("\tTR"); o.i(row_id);
                    o.put("\t.\t<TR>\t.\tPASS\tMOTIF="); o.put(r.motif); o.put(";CONS_MOTIF="); o.put(r.motif);
                    o.put(";COPIES="); o.f("%.1f", r.copies); o.put(";TIER="); o.i(r.tier);
                    o.put(";CONF="); o.f("%.2f", r.confidence); o.put(";MM_RATE="); o.f("%.3f", r.mismatch_rate);
                    o.put(";MAX_MM_PER_COPY="); o.i(r.max_mm); o.put(";N_COPIES_EVAL="); o.i(r.n_eval);
                    o.put(";STRAND="); o.c(r.strand); o.c('\n');
                    break;
                case BWTMI_FMT_TRF_TABLE: {
                    comp_entropy(r, cp, ent);
                    const int64_t ml = (int64_t)r.motif.size();
                    o.i(r.start); o.put("--"); o.i(r.end); o.c('\t'); o.i(ml); o.c('\t'); o.f("%.1f", r.copies);
                    o.c('\t'); o.i(ml); o.c('\t'); o.f("%.0f", r.pmatch); o.c('\t'); o.f("%.0f", r.pindel); o.c('\t');
                    o.i(r.score); o.c('\t'); o.f("%.0f", cp[0]); o.c('\t'); o.f("%.0f", cp[1]); o.c('\t');
                    o.f("%.0f", cp[2]); o.c('\t'); o.f("%.0f", cp[3]); o.c('\t'); o.f("%.2f", ent); o.c('\n');
                    break;
                }
                case BWTMI_FMT_TRF_DAT: {
                    comp_entropy(r, cp, ent);
                    const int64_t ml = (int64_t)r.motif.size();
                    o.i(r.start); o.c(' '); o.i(r.end); o.c(' '); o.i(ml); o.c(' '); o.f("%.1f", r.copies); o.c(' ');
                    o.i(ml); o.c(' '); o.f("%.0f", r.pmatch); o.c(' '); o.f("%.0f", r.pindel); o.c(' ');
                    o.i(r.score); o.c(' '); o.f("%.0f", cp[0]); o.c(' '); o.f("%.0f", cp[1]); o.c(' ');
                    o.f("%.0f", cp[2]); o.c(' '); o.f("%.0f", cp[3]); o.c(' '); o.f("%.2f", ent); o.c(' ');
                    o.put(r.motif); o.c(' ');
                    View av = act_of(job, r);
                    if (!av.empty()) o.put(av); else o.rep(r.motif, (int64_t)r.copies);
                    o.c('\n');
                    break;
                }
                default:   // STRfinder
                    row_strfinder(o, job, r, rows[(size_t)k].partner);
            }
        }
        out.parts[(size_t)ck] = o.finish();
        if (!tl.empty()) tl[(size_t)ck].b = now_ms();
        if (on_part) (*on_part)((size_t)ck);
        if (!tl.empty()) tl[(size_t)ck].c = now_ms();
    });
    fr.reset();
    auto t3 = std::chrono::steady_clock::now();
    if (!tl.empty()) {
        std::map<size_t, std::pair<double, double>> busy;   // thread -> (formatting, on_part)
        double first = 1e30, last = 0, lastfmt = 0;
        for (const Tl &x : tl) {
            busy[x.th].first += x.b - x.a;
            busy[x.th].second += x.c - x.b;
            first = std::min(first, x.a);
            last = std::max(last, x.c);
            lastfmt = std::max(lastfmt, x.b);
        }
        std::string per;
        for (auto &kv : busy) per += " " + std::to_string((int)(kv.second.first * 100) / 100.0).substr(0, 4) + "/" +
                                     std::to_string((int)(kv.second.second * 100) / 100.0).substr(0, 4);
        std::fprintf(stderr, "  format timeline: %zu chunks, first start %.2f, last format end %.2f, last end %.2f ms; "
                     "threads (format/on_part ms):%s\n", tl.size(), first, lastfmt, last, per.c_str());
    }
    job.stage_ms[6] = std::chrono::duration<double, std::milli>(t3 - t0).count();
    if (stats_on()) {
        auto d = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        std::fprintf(stderr, "  render: compounds+sort %.1f chunking %.1f format %.1f ms (%zu rows)\n", d(t0, t1),
                     d(t1, t2), d(t2, t3), rows.size());
    }
}

std::vector<Text> render_parts(Job &job, int fmt) {
    Rendered r;
    render_rows(job, fmt, nullptr, r);
    std::vector<Text> parts;
    parts.reserve(r.parts.size() + 1);
    parts.emplace_back(r.header.data(), r.header.size());
    for (auto &p : r.parts) parts.push_back(std::move(p));
    return parts;
}

std::string render(Job &job, int fmt) {
    std::vector<Text> parts = render_parts(job, fmt);
    size_t tot = 0;
    for (auto &p : parts) tot += p.size();
    std::string s;
    s.reserve(tot);
    for (auto &p : parts) s.append(p.data(), p.size());
    return s;
}

}  // namespace bwtmi
