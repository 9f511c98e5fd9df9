// recompute.hip -- MotifUtils.align_repeat_region (bwt.py:998-1102, with
// _align_unit_to_window 829-983 and _consensus_from_counts 986-995) on the
// device, one wavefront per region: the DP recomputes that
// _merge_adjacent_repeats (bwt.py:3222-3289) needs for neighbour pairs whose
// current record is still the fresh one (~80 % of them), batched per fold
// unit.  Both attempts of _recompute_repeat (min_copies, then 1;
// bwt.py:3530-3534) run here.
//
// The restatement follows the host's scalar path (motif.cpp align_repeat_region
// / align_unit / finish_unit) decision for decision:
//  * the band DP row by row, lane l holding column j = i - band - 1 + l:
//    substitution/match from the previous row's lane l, deletion from lane
//    l + 1 (sub preferred on ties), then the insertion pass as a prefix
//    minimum of c0[l'] + (l - l') over the row (a wave scan); 'I' only where
//    the left neighbour's final value + 1 is strictly smaller, as the host's
//    left-to-right pass decides it.  The host's INF (m + n + 10) is kept for the
//    boundary column and the column past the previous row's band;
//  * the best end column is the first minimum on row m in [lower, upper];
//  * traceback, the copy tests, the variation pieces and the observed bases
//    on lane 0 (serial, a few dozen steps);
//  * exact copies by a wave compare and the periodic extent 64 bytes a step;
//  * the consensus Counter per motif position in first-insertion order
//    (Counter.most_common(1): first maximal entry); the observed positions of
//    one copy are distinct, so lanes update them in parallel.
// Bounds: motifs of 2..kRcMaxMotif bases, kKin distinct symbols per consensus
// position, kVarCap variation bytes per region -- past any of them (rare) the
// region comes back with status -1 and the host recomputes it.
#include <hip/hip_runtime.h>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kMaxM = kRcMaxMotif;
constexpr int kMaxIndel = 10;                   // max_indel = max(1, min(10, m // 2)) (m >= 4), 1 below
constexpr int kBandMax = kMaxIndel + 2;
constexpr int kWMax = 2 * kBandMax + 1;
constexpr int kWinCap = kMaxM + kMaxIndel;      // window: m + max_indel bases
constexpr int kColCap = kMaxM + kWinCap + 2;    // alignment columns <= m + n
constexpr int kKin = 6;                         // distinct symbols per consensus position
constexpr int kOpsCap = 1024, kPieceCap = 256;  // one copy's ops
constexpr int kVarCap = 2048;                   // a region's variation string
constexpr int32_t kBig = 1 << 29;               // lanes outside the row's band (never read)

struct Lds {
    char ptr[(kMaxM + 1) * kWMax];
    char cur[kMaxM];
    char win[kWinCap + 2];
    char cr[kColCap], cq[kColCap];
    int16_t obs_idx[kMaxM];
    char obs_base[kMaxM];
    char ops[kOpsCap];
    int16_t op_end[kPieceCap];
    char var[kVarCap];
    char pc_c[kMaxM * kKin];
    int32_t pc_n[kMaxM * kKin];
    uint8_t pc_k[kMaxM];
    int64_t r[4];     // lane 0 -> wave: unit result (consumed, n_sub, n_ins, n_del)
    int32_t ok;       // lane 0 -> wave: unit accepted
    int32_t nobs, npieces, nvar, overflow;
    unsigned long long off;
};

__device__ inline int put_num(char *d, int cap, int at, int64_t v) {   // v >= 0
    char b[24];
    int k = 0;
    do {
        b[k++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    if (at + k > cap) return -1;
    for (int q = 0; q < k; ++q) d[at + q] = b[k - 1 - q];
    return at + k;
}

// one copy's formatted ops on lane 0: pieces end at op_end[]
struct Ops {
    Lds &S;
    int n = 0, np = 0;
    bool bad = false;
    __device__ explicit Ops(Lds &s) : S(s) {}
    __device__ void ch(char c) {
        if (n < kOpsCap) S.ops[n++] = c;
        else bad = true;
    }
    __device__ void str(const char *s) {
        while (*s) ch(*s++);
    }
    __device__ void num(int64_t v) {
        const int r = put_num(S.ops, kOpsCap, n, v);
        if (r < 0) bad = true;
        else n = r;
    }
    __device__ void end_piece() {
        if (np < kPieceCap) S.op_end[np++] = (int16_t)n;
        else bad = true;
    }
};

// Counter[p][b] += cnt; false past kKin distinct symbols
__device__ inline bool pc_add(Lds &S, int p, char b, int32_t cnt) {
    char *c = S.pc_c + p * kKin;
    int32_t *n = S.pc_n + p * kKin;
    const int k = S.pc_k[p];
    for (int t = 0; t < k; ++t)
        if (c[t] == b) {
            n[t] += cnt;
            return true;
        }
    if (k == kKin) return false;
    c[k] = b;
    n[k] = cnt;
    S.pc_k[p] = (uint8_t)(k + 1);
    return true;
}

__device__ inline bool pc_top(const Lds &S, int p, char &out) {
    const int k = S.pc_k[p];
    if (k == 0) return false;
    const char *c = S.pc_c + p * kKin;
    const int32_t *n = S.pc_n + p * kKin;
    char b = c[0];
    int32_t best = n[0];
    for (int t = 1; t < k; ++t)
        if (n[t] > best) {
            best = n[t];
            b = c[t];
        }
    out = b;
    return true;
}

__device__ inline int32_t wave_min(int32_t v) {
    for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d));
    return __builtin_amdgcn_readfirstlane(v);
}

// traceback, copy tests, ops and observed bases of one unit (finish_unit), on
// lane 0; the ptr rows are complete and bj is the end column
__device__ void finish_unit_lane0(Lds &S, int m, int band, int W, int tol, int max_indel, int bj) {
    S.ok = 0;
    int nc = 0, i = m, j = bj;
    int ns = 0, ni = 0, nd = 0;
    while (i > 0 || j > 0) {
        char op;
        if (i == 0) op = 'I';
        else if (j == 0) op = 'D';
        else if (j < i - band || j > i + band) op = 0;
        else op = S.ptr[i * W + (j - i + band)];
        if (op == 'M' || op == 'S') {
            S.cr[nc] = S.cur[i - 1];
            S.cq[nc++] = S.win[j - 1];
            ns += op == 'S';
            --i;
            --j;
        } else if (op == 'D') {
            S.cr[nc] = S.cur[i - 1];
            S.cq[nc++] = '-';
            ++nd;
            --i;
        } else if (op == 'I') {
            S.cr[nc] = '-';
            S.cq[nc++] = S.win[j - 1];
            ++ni;
            --j;
        } else {
            break;
        }
    }
    if (ns > tol || ni > max_indel || nd > max_indel) return;
    Ops o(S);
    int nobs = 0;
    int64_t n_sub = 0, n_ins = 0, n_del = 0;
    int ref = 0, ins_from = 0, ins_at = 0, del_len = 0, del_at = 0;
    bool ins_open = false;
    auto flush_ins = [&](int upto) {
        o.ch(':');
        o.num(ins_at);
        o.str(":ins(");
        for (int q = ins_from; q < upto; ++q) o.ch(S.cq[nc - 1 - q]);
        o.ch(')');
        o.end_piece();
        n_ins += upto - ins_from;
    };
    auto flush_del = [&]() {
        o.ch(':');
        o.num(del_at);
        o.str(":del(");
        o.num(del_len);
        o.ch(')');
        o.end_piece();
        n_del += del_len;
    };
    for (int q = 0; q < nc; ++q) {
        const char r = S.cr[nc - 1 - q], qq = S.cq[nc - 1 - q];
        if (r == '-') {
            if (!ins_open) {
                ins_at = ref;
                ins_from = q;
                ins_open = true;
            }
            continue;
        }
        if (ins_open) {
            flush_ins(q);
            ins_open = false;
            ins_at = 0;
        }
        ++ref;
        if (qq == '-') {
            if (del_len == 0) del_at = ref;
            ++del_len;
            continue;
        }
        if (del_len) {
            flush_del();
            del_len = 0;
        }
        S.obs_idx[nobs] = (int16_t)(ref - 1);
        S.obs_base[nobs++] = qq;
        if (r != qq) {
            o.ch(':');
            o.num(ref);
            o.ch(':');
            o.ch(r);
            o.ch('>');
            o.ch(qq);
            o.end_piece();
            ++n_sub;
        }
    }
    if (ins_open) flush_ins(nc);
    if (del_len) flush_del();
    if (o.bad) {
        S.overflow = 1;
        return;
    }
    if (n_sub > tol) return;
    if (n_ins > max_indel || n_del > max_indel) return;
    S.nobs = nobs;
    S.npieces = o.np;
    S.r[0] = bj;
    S.r[1] = n_sub;
    S.r[2] = n_ins;
    S.r[3] = n_del;
    S.ok = 1;
}

// _align_unit_to_window of the consensus S.cur (m) against S.win (n): true
// with S.r / S.obs_* / S.ops filled when the copy is accepted
__device__ bool align_unit_wave(Lds &S, int m, int n, int max_indel, int tol, int lane) {
    if (m == 0 || n == 0) return false;
    const int lower = m - max_indel > 0 ? m - max_indel : 0;
    const int upper = n < m + max_indel ? n : m + max_indel;
    if (lower > upper) return false;
    const int32_t INF = m + n + 10;
    const int band = max_indel + 2;
    const int W = 2 * band + 1;
    const int32_t reject = tol + 2 * max_indel;
    int32_t q;   // previous row, lane form: column j = (i - 1) - band - 1 + lane
    {
        const int j = lane - band - 1;   // row 0: prev[j] = j, prev[n + 1] = INF
        q = (j >= 0 && j <= n) ? j : (j == n + 1 ? INF : kBig);
    }
    for (int i = 1; i <= m; ++i) {
        const int jmin = i - band > 1 ? i - band : 1, jmax = n < i + band ? n : i + band;
        const int j = i - band - 1 + lane;
        const char mi = S.cur[i - 1];
        const int32_t qn = __shfl_down(q, 1);   // prev[j]; prev[j - 1] is q
        const bool valid = j >= jmin && j <= jmax;
        int32_t c0 = kBig;
        char op = 0;
        if (valid) {
            const bool eq = mi == S.win[j - 1];
            const int32_t sub = q + (eq ? 0 : 1), dc = qn + 1;
            c0 = dc < sub ? dc : sub;
            op = dc < sub ? 'D' : (eq ? 'M' : 'S');
        } else if (j == jmin - 1) {
            c0 = j == 0 ? i : INF;
        }
        int32_t g = c0 - lane;   // prefix min of c0[l'] + (lane - l')
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t o = __shfl_up(g, d);
            if (lane >= d) g = min(g, o);
        }
        const int32_t f = g + lane;
        const int32_t left = __shfl_up(f, 1);
        if (valid) {
            if (left + 1 < c0) op = 'I';
            S.ptr[i * W + lane - 1] = op;
        }
        const int32_t rowmin = wave_min(valid ? f : INF);
        if (rowmin > reject && (jmin > 1 || i > reject)) return false;
        q = (valid || j == jmin - 1) ? f : ((j == jmax + 1 && j <= n) ? INF : kBig);
    }
    // first minimal end column on row m in [lower, upper] (j == 0 costs m)
    const int j = m - band - 1 + lane;
    const bool inr = j >= lower && j <= upper;
    const int32_t cost = j == 0 ? m : q;
    const int32_t bc = wave_min(inr ? cost : kBig);
    const uint64_t hit = __ballot(inr && cost == bc);
    if (!hit) return false;
    const int bj = m - band - 1 + (__ffsll((unsigned long long)hit) - 1);
    if (bj <= 0 || bc >= INF) return false;
    if (bc > tol + 2 * max_indel) return false;
    __syncthreads();   // ptr rows complete
    if (lane == 0) finish_unit_lane0(S, m, band, W, tol, max_indel, bj);
    __syncthreads();
    return S.ok != 0;
}

struct RegionOut {
    int64_t copies, consumed, tot_err, max_err, tot_ins, tot_del;
};

// align_repeat_region(text, start, end, text[start : start + m], min_copies), m >= 2,
// on the whole wave: 1 aligned (consensus in S.cr[0, m), variations S.var[0, S.nvar)),
// 0 not aligned, -1 past a bound
__device__ int align_region_wave(Lds &S, const char *__restrict__ text, int64_t L, int64_t start, int64_t end,
                                 int m, int64_t min_copies, RegionOut &out, int lane) {
    start = start > 0 ? start : 0;
    end = end > start ? (end < L ? end : L) : L;
    const int tol = (int)floor((double)m * 0.1) > 1 ? (int)floor((double)m * 0.1) : 1;
    const int max_indel = m >= 4 ? (m / 2 < 10 ? m / 2 : 10) : 1;
    for (int p = lane; p < m; p += 64) {
        S.pc_k[p] = 0;
        S.cur[p] = text[start + p];
    }
    if (lane == 0) {
        S.nvar = 0;
        S.overflow = 0;
    }
    __syncthreads();
    int64_t tot_ins = 0, tot_del = 0, tot_err = 0, max_err = 0, copies = 0, pend = 0;
    int64_t pos = start;
    const int64_t ext = (int64_t)m * 3 > (int64_t)max_indel * 4 ? (int64_t)m * 3 : (int64_t)max_indel * 4;
    const int64_t base = end > start + (int64_t)m * min_copies ? end : start + (int64_t)m * min_copies;
    const int64_t limit = L < base + ext ? L : base + ext;
    auto flush = [&]() {   // pend exact copies observe every cur[p]
        if (!pend) return;
        bool bad = false;
        for (int p = lane; p < m; p += 64) bad |= !pc_add(S, p, S.cur[p], (int32_t)pend);
        if (bad) S.overflow = 1;
        pend = 0;
        __syncthreads();
    };
    while (pos < limit) {
        const int64_t wend = L < pos + m + max_indel ? L : pos + m + max_indel;
        const int64_t wlen = wend - pos;
        if (wlen < m - max_indel) break;
        bool exact = wlen >= m;
        if (exact) {
            bool mis = false;
            for (int p = lane; p < m; p += 64) mis |= S.cur[p] != text[pos + p];
            exact = __ballot(mis) == 0;
        }
        if (exact) {   // a run of exact copies: copy j at pos + j*m while pos + j*m < limit
            const int64_t top = L < limit - 1 + m ? L : limit - 1 + m;
            int64_t x = pos + m;
            for (;;) {
                const int64_t k = x + lane;
                const bool stop = k >= top || text[k] != text[k - m];
                const uint64_t b = __ballot(stop);
                if (b) {
                    x += __ffsll((unsigned long long)b) - 1;
                    break;
                }
                x += 64;
            }
            const int64_t k = (x - pos) / m;
            copies += k;
            pend += k;
            pos += k * m;
            continue;
        }
        for (int t = lane; t < wlen; t += 64) S.win[t] = text[pos + t];
        __syncthreads();
        if (!align_unit_wave(S, m, (int)wlen, max_indel, tol, lane)) break;
        const int64_t consumed = S.r[0];
        if (consumed == 0) break;
        flush();
        ++copies;
        if (lane == 0) {   // "copy:pos:..." pieces in op order
            const int np = S.npieces;
            int nv = S.nvar, from = 0;
            for (int q = 0; q < np; ++q) {
                if (nv > 0) {
                    if (nv >= kVarCap) { S.overflow = 1; break; }
                    S.var[nv++] = ';';
                }
                const int r = put_num(S.var, kVarCap, nv, copies);
                const int e = S.op_end[q];
                if (r < 0 || r + (e - from) > kVarCap) { S.overflow = 1; break; }
                nv = r;
                for (int c = from; c < e; ++c) S.var[nv++] = S.ops[c];
                from = e;
            }
            S.nvar = nv;
        }
        const int64_t err = S.r[1] + S.r[2] + S.r[3];
        tot_err += err;
        max_err = max_err > err ? max_err : err;
        tot_ins += S.r[2];
        tot_del += S.r[3];
        const int nobs = S.nobs;
        bool bad = false;
        for (int q = lane; q < nobs; q += 64) {   // distinct positions: independent updates
            const int idx = S.obs_idx[q];
            if (idx >= 0 && idx < m) {
                bad |= !pc_add(S, idx, S.obs_base[q], 1);
                char b;
                if (pc_top(S, idx, b)) S.cur[idx] = b;
            }
        }
        if (bad) S.overflow = 1;
        __syncthreads();
        if (S.overflow) return -1;
        pos += consumed;
    }
    if (S.overflow) return -1;
    if (copies < min_copies) return 0;
    const int64_t consumed = pos - start;
    if (consumed <= 0) return 0;
    flush();
    if (S.overflow) return -1;
    for (int p = lane; p < m; p += 64) {   // _consensus_from_counts, else the running consensus
        char b;
        S.cr[p] = pc_top(S, p, b) ? b : S.cur[p];
    }
    __syncthreads();
    out.copies = copies;
    out.consumed = consumed;
    out.tot_err = tot_err;
    out.max_err = max_err;
    out.tot_ins = tot_ins;
    out.tot_del = tot_del;
    return 1;
}

__global__ __launch_bounds__(64) void k_recompute(const RcReq *__restrict__ req, int64_t nreq,
                                                  RcOut *__restrict__ out, char *__restrict__ arena,
                                                  int64_t arena_cap, unsigned long long *__restrict__ top) {
    __shared__ Lds S;
    const int lane = threadIdx.x;
    const int64_t r = blockIdx.x;
    if (r >= nreq) return;
    const RcReq q = req[r];
    RcOut o{};
    RegionOut ro{};
    int st = -1;
    if (q.m >= 2 && q.m <= kMaxM && q.start >= 0 && q.start + q.m <= q.text_len) {
        st = align_region_wave(S, q.text, q.text_len, q.start, q.end, q.m, q.min_copies, ro, lane);
        if (st == 0) st = align_region_wave(S, q.text, q.text_len, q.start, q.end, q.m, 1, ro, lane);
    }
    if (st == 1) {
        const int len = q.m + S.nvar;
        if (lane == 0) S.off = atomicAdd(top, (unsigned long long)len);
        __syncthreads();
        const int64_t off = (int64_t)S.off;
        if (off + len > arena_cap) {
            st = -1;
        } else {
            for (int t = lane; t < q.m; t += 64) arena[off + t] = S.cr[t];
            for (int t = lane; t < S.nvar; t += 64) arena[off + q.m + t] = S.var[t];
            o.str_off = off;
            o.str_len = len;
            o.copies = ro.copies;
            o.consumed = ro.consumed;
            o.tot_err = (int32_t)ro.tot_err;
            o.max_err = (int32_t)ro.max_err;
            o.tot_ins = (int32_t)ro.tot_ins;
            o.tot_del = (int32_t)ro.tot_del;
        }
    }
    o.status = st;
    if (lane == 0) out[r] = o;
}

}  // namespace

void recompute_batch_device(Ctx &c, const RcReq *h_req, int64_t nreq, RcOut *h_out, std::vector<char> &arena) {
    arena.clear();
    if (nreq <= 0) return;
    hipStream_t st = c.stream;
    const int64_t cap = std::max<int64_t>(1 << 20, nreq * 64);   // consensus + variations: typically < 64 B
    c.slot[S_MISC0].ensure((size_t)nreq * sizeof(RcReq));
    c.slot[S_MISC1].ensure((size_t)nreq * sizeof(RcOut) + 64);
    c.slot[S_MISC2].ensure((size_t)cap);
    RcOut *d_out = c.slot[S_MISC1].as<RcOut>();
    auto *d_top = (unsigned long long *)(c.slot[S_MISC1].as<char>() + (size_t)nreq * sizeof(RcOut));
    HIPCHECK(hipMemcpyAsync(c.slot[S_MISC0].p, h_req, (size_t)nreq * sizeof(RcReq), hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemsetAsync(d_top, 0, sizeof(unsigned long long), st));
    KLAUNCH("k_recompute", 0.0, k_recompute, dim3((unsigned)nreq), dim3(64), 0, st, c.slot[S_MISC0].as<RcReq>(),
            nreq, d_out, c.slot[S_MISC2].as<char>(), cap, d_top);
    HIPCHECK(hipGetLastError());
    unsigned long long used = 0;
    HIPCHECK(hipMemcpyAsync(h_out, d_out, (size_t)nreq * sizeof(RcOut), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipMemcpyAsync(&used, d_top, sizeof(used), hipMemcpyDeviceToHost, st));
    HIPCHECK(hipStreamSynchronize(st));
    const size_t got = (size_t)std::min<unsigned long long>(used, (unsigned long long)cap);
    arena.resize(got);
    if (got) {
        HIPCHECK(hipMemcpyAsync(arena.data(), c.slot[S_MISC2].p, got, hipMemcpyDeviceToHost, st));
        HIPCHECK(hipStreamSynchronize(st));
    }
    c.kresolve();
}

}  // namespace bwtmi
