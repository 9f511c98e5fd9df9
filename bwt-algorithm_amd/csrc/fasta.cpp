// fasta.cpp -- TandemRepeatFinder.load_reference (bwt.py:3713-3756), native and
// parallel.
//
// Python reads the file in text mode: universal newlines (\n, \r\n, \r end a
// line), each line .strip()-ed (ASCII whitespace incl. \x1c-\x1f), headers
// '>' take line[1:].split()[0], other non-empty lines are upper-cased and
// appended (inner whitespace kept); lines before the first header are
// dropped.  A repeated name keeps its first position and the last content.
// Trim: 30+30 flanks when len > 2*flank_trim.
//
// The file is cut into chunks at line starts (empty lines are skipped, so a
// cut between '\r' and '\n' is harmless).  Pass 1 measures, per chunk, the
// stripped content before its first header and after each header; a serial
// stitch turns those into contig lengths and the destination offset of every
// chunk piece; pass 2 writes the upper-cased bytes straight into the contig
// buffers.  With world > 1 only this rank's fold units (shard_units) are
// written -- the others keep their names and lengths for the shard layout.
#include <fcntl.h>
#include <immintrin.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace bwtmi {

static std::atomic<uint64_t> g_gen{0};
uint64_t next_contig_gen() { return ++g_gen; }

namespace {

inline bool py_space(unsigned char c) { return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f); }
inline bool eol(char c) { return c == '\n' || c == '\r'; }

struct Hdr {
    int64_t name_a, name_b;   // name bytes in the file buffer
    int64_t len;              // stripped content after the header, inside the chunk
    int64_t line = 0;         // the header's '>' in the buffer
};
struct Chunk {
    int64_t a = 0, b = 0;     // [a, b): whole lines
    int64_t bad = -1;         // first non-ASCII byte of a sequence line, or of an invalid header
    int64_t pre = 0;          // content before the chunk's first header
    bool plain = false;       // only '\n' and bytes 0x21..0x7f, no '>': lines need no strip
    std::vector<Hdr> hdrs;
    // pass 2 destinations (nullptr: not written), with their contig and the
    // content offset there (the device placement of a whole-file load)
    char *pre_dst = nullptr;
    int32_t pre_cid = -1;
    int64_t pre_off = 0;
    std::vector<char *> dst;
    std::vector<int32_t> dcid;
    // a chunk with a header (or other irregular lines) whose bytes after the
    // last '>' line are plain: [tail_a, b) holds tail_len content bytes that
    // continue the chunk's last destination (-1: no such tail)
    int64_t tail_a = -1, tail_len = 0;
};

// calls line(a, b) with the stripped bounds of every non-empty line in [a, e)
template <class F>
void for_lines(const char *p, int64_t a, int64_t e, F &&line) {
    int64_t i = a;
    // the per-line '\r' search only runs when the range holds one at all
    const bool has_cr = std::memchr(p + a, '\r', (size_t)(e - a)) != nullptr;
    while (i < e) {
        // line end: the next '\n' (memchr), or an earlier '\r'
        const char *nl = (const char *)std::memchr(p + i, '\n', (size_t)(e - i));
        int64_t j = nl ? (int64_t)(nl - p) : e;
        if (has_cr)
            if (const char *cr = (const char *)std::memchr(p + i, '\r', (size_t)(j - i))) j = (int64_t)(cr - p);
        int64_t s = i, t = j;
        while (s < t && py_space((unsigned char)p[s])) ++s;
        while (t > s && py_space((unsigned char)p[t - 1])) --t;
        if (t > s) line(s, t);
        i = j + 1;   // "\r\n": the '\n' becomes an empty line
    }
}

// a header line the reference reads like we do: ASCII, or valid UTF-8 without
// the Unicode whitespace that str.split() / strip() would also cut at
bool header_ok(const char *h, int64_t n) {
    int64_t i = 0;
    while (i < n) {
        const unsigned char c = (unsigned char)h[i];
        if (c < 0x80) { ++i; continue; }
        int len = c >= 0xF0 && c < 0xF5 ? 4 : c >= 0xE0 ? 3 : c >= 0xC2 && c < 0xE0 ? 2 : 0;
        if (!len || i + len > n) return false;
        uint32_t cp = c & (len == 2 ? 0x1F : len == 3 ? 0x0F : 0x07);
        for (int k = 1; k < len; ++k) {
            const unsigned char d = (unsigned char)h[i + k];
            if ((d & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (d & 0x3F);
        }
        if ((len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) || (cp >= 0xD800 && cp <= 0xDFFF))
            return false;
        if (cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 ||
            cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000)
            return false;
        i += len;
    }
    return true;
}

// index of the first byte >= 0x80 in [s, s + n), or -1 (8 bytes per step)
inline int64_t first_high(const char *s, int64_t n) {
    int64_t q = 0;
    for (; q + 32 <= n; q += 32) {
        uint64_t w[4];
        std::memcpy(w, s + q, 32);
        if ((w[0] | w[1] | w[2] | w[3]) & 0x8080808080808080ull) break;
    }
    for (; q < n; ++q)
        if ((unsigned char)s[q] >= 0x80) return q;
    return -1;
}

// A chunk whose bytes are all '\n' or 0x21..0x7f other than '>' has no header,
// no CR, no strippable whitespace and no non-ASCII byte: its content is every
// byte but the newlines.  Returns the newline count, or -1 if not plain.
// (AVX2, 32 bytes per step; a signed compare also flags bytes >= 0x80.)
int64_t plain_newlines(const char *p, int64_t n) {
    const __m256i vnl = _mm256_set1_epi8('\n'), vgt = _mm256_set1_epi8('>'), v21 = _mm256_set1_epi8(0x21);
    int64_t q = 0, nl = 0;
    for (; q + 32 <= n; q += 32) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(p + q));
        const __m256i isnl = _mm256_cmpeq_epi8(v, vnl);
        const __m256i low = _mm256_cmpgt_epi8(v21, v);   // v < 0x21 or v >= 0x80
        const __m256i bad = _mm256_or_si256(_mm256_andnot_si256(isnl, low), _mm256_cmpeq_epi8(v, vgt));
        if (!_mm256_testz_si256(bad, bad)) return -1;
        nl += __builtin_popcount((unsigned)_mm256_movemask_epi8(isnl));
    }
    for (; q < n; ++q) {
        const unsigned char c = (unsigned char)p[q];
        if (c == '\n') ++nl;
        else if (c < 0x21 || c >= 0x80 || c == '>') return -1;
    }
    return nl;
}

// upper-cased copy (ASCII a-z), vectorised
inline void upper_copy(char *__restrict d, const char *__restrict s, int64_t n) {
    for (int64_t q = 0; q < n; ++q) {
        const unsigned char ch = (unsigned char)s[q];
        d[q] = (char)(ch - ((unsigned char)(ch - 'a') < 26u ? 32 : 0));
    }
}

// the content of plain lines [i, e) ('\n' ends every line) upper-cased to d; returns the end
inline char *plain_copy(const char *p, int64_t i, int64_t e, char *d) {
    while (i < e) {
        const char *nl = (const char *)std::memchr(p + i, '\n', (size_t)(e - i));
        const int64_t j = nl ? (int64_t)(nl - p) : e;
        upper_copy(d, p + i, j - i);
        d += j - i;
        i = j + 1;
    }
    return d;
}

// where the chunk's plain tail goes (host pointer, or nullptr), its contig and content offset
inline char *tail_dst(const Chunk &C, int32_t &cid, int64_t &off) {
    if (!C.hdrs.empty()) {
        cid = C.dcid.back();
        off = C.hdrs.back().len - C.tail_len;
        return C.dst.back() ? C.dst.back() + off : nullptr;
    }
    cid = C.pre_cid;
    off = C.pre_off + C.pre - C.tail_len;
    return C.pre_dst ? C.pre_dst + (C.pre - C.tail_len) : nullptr;
}

// pass 2 of one chunk: its upper-cased content into place (head: the lines
// before a plain tail; tail: the plain tail only)
enum Part { P_ALL, P_HEAD, P_TAIL };
void pass2(const char *p, const Chunk &C, Part part = P_ALL) {
    char *d = C.pre_dst;
    if (C.plain) {   // lines end at '\n' only and need no strip
        if (d && part != P_HEAD) plain_copy(p, C.a, C.b, d);
        return;
    }
    const int64_t e = C.tail_a >= 0 ? C.tail_a : C.b;
    if (part != P_TAIL) {
        size_t h = 0;
        for_lines(p, C.a, e, [&](int64_t s, int64_t t) {
            if (p[s] == '>') {
                d = C.dst[h++];
                return;
            }
            if (!d) return;
            upper_copy(d, p + s, t - s);
            d += t - s;
        });
    }
    if (C.tail_a >= 0 && part != P_HEAD) {
        int32_t cid;
        int64_t off;
        if (char *td = tail_dst(C, cid, off)) plain_copy(p, C.tail_a, C.b, td);
    }
}

void read_file(const char *path, Seq &data, int nt, FastaDev *dev = nullptr) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) fail(BWTMI_E_IO, "cannot open %s", path);
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        ::close(fd);
        fail(BWTMI_E_IO, "cannot stat %s", path);
    }
    const int64_t n = (int64_t)st.st_size;
    char *buf = data.resize_uninit((size_t)n);
    if (dev) dev->image(buf, n);   // each piece goes to the device as soon as it is read
    std::atomic<bool> bad{false};
    const int64_t piece = int64_t(4) << 20;
    run_tasks((n + piece - 1) / piece, nt, [&](int64_t k) {
        const int64_t o0 = k * piece;
        int64_t o = o0;
        const int64_t e = std::min(n, o + piece);
        while (o < e) {
            const ssize_t r = ::pread(fd, buf + o, (size_t)(e - o), (off_t)o);
            if (r <= 0) { bad = true; return; }
            o += r;
        }
        if (dev) dev->image_part(o0, e - o0);
    });
    ::close(fd);
    if (bad) fail(BWTMI_E_IO, "read error on %s", path);
}

}  // namespace

void load_fasta(Job &job, const char *path, int32_t flank_trim, int32_t world, int32_t rank, FastaDev *dev) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    job.text_join();   // a deferred pass 2 of the previous load still writes the old buffers
    const int nt = host_threads(job.params);
    thread_local Seq data;   // the file image (kept for the next load)
    read_file(path, data, nt, dev);   // with a device: the image is copied up while it is read
    const auto t1 = clk::now();
    const char *p = data.data();
    const int64_t N = (int64_t)data.size();

    // chunks at line starts
    const int64_t T = std::max<int64_t>(1, std::min<int64_t>(4 * (int64_t)nt, N / (int64_t(1) << 20) + 1));
    std::vector<Chunk> ck((size_t)T);
    std::vector<int64_t> cut((size_t)T + 1, N);
    cut[0] = 0;
    run_tasks(T - 1, nt, [&](int64_t q) {
        int64_t i = N * (q + 1) / T;
        while (i < N && !eol(p[i - 1])) ++i;
        cut[(size_t)q + 1] = i;
    });
    for (int64_t t = 1; t <= T; ++t) cut[(size_t)t] = std::max(cut[(size_t)t], cut[(size_t)t - 1]);

    // pass 1: lengths
    run_tasks(T, nt, [&](int64_t t) {
        Chunk &C = ck[(size_t)t];
        C.a = cut[(size_t)t];
        C.b = cut[(size_t)t + 1];
        const bool no_plain = knob(KN_NO_PLAIN) != 0;   // A/B switch: every chunk line by line
        if (const int64_t nl = no_plain ? -1 : plain_newlines(p + C.a, C.b - C.a); nl >= 0) {   // no header: all content
            C.plain = true;
            C.pre = (C.b - C.a) - nl;
            return;
        }
        // the bytes after the line of the chunk's last '>' may be plain: they
        // are then content of the last destination, counted without line work
        int64_t e_lines = C.b;
        if (!no_plain) {
            if (const char *gt = (const char *)memrchr(p + C.a, '>', (size_t)(C.b - C.a))) {
                const int64_t g = (int64_t)(gt - p);
                const char *nl = (const char *)std::memchr(p + g, '\n', (size_t)(C.b - g));
                int64_t t = nl ? (int64_t)(nl - p) + 1 : C.b;
                if (const char *cr = (const char *)std::memchr(p + g, '\r', (size_t)((nl ? t - 1 : C.b) - g)))
                    t = (int64_t)(cr - p) + 1 + ((int64_t)(cr - p) + 1 < C.b && cr[1] == '\n');
                if (t < C.b)
                    if (const int64_t nl2 = plain_newlines(p + t, C.b - t); nl2 >= 0) {
                        C.tail_a = t;
                        C.tail_len = (C.b - t) - nl2;
                        e_lines = t;
                    }
            }
        }
        for_lines(p, C.a, e_lines, [&](int64_t s, int64_t e) {
            if (p[s] == '>') {
                int64_t x = s + 1;
                while (x < e && py_space((unsigned char)p[x])) ++x;
                int64_t y = x;
                while (y < e && !py_space((unsigned char)p[y])) ++y;
                C.hdrs.push_back(Hdr{x, y, 0, s});
                if (C.bad < 0 && !header_ok(p + s, e - s)) C.bad = s;
                return;
            }
            if (C.bad < 0)
                if (const int64_t q = first_high(p + s, e - s); q >= 0) C.bad = s + q;
            if (C.hdrs.empty()) C.pre += e - s;
            else C.hdrs.back().len += e - s;
        });
        if (C.tail_a >= 0) (C.hdrs.empty() ? C.pre : C.hdrs.back().len) += C.tail_len;
    });

    // Non-ASCII text: the reference reads the file as UTF-8 str (bwt.py:3719), so an
    // invalid byte raises UnicodeDecodeError there, and a valid multi-byte character
    // in a sequence makes BWTCore's text_arr (seq.encode('utf-8'), bwt.py:121) longer
    // than the str, which aborts its parent-side index build (ValueError from
    // np.lexsort, bwt.py:3782; tests/golden/expected_edge.json).  Either way the
    // reference writes no output: fail likewise, before touching the job.
    for (const Chunk &C : ck)
        if (C.bad >= 0)
            fail(BWTMI_E_IO, "non-ASCII text at byte %lld of %s: the reference (bwt.py:3719, 121) fails on it",
                 (long long)C.bad, path);

    // stitch: header instances in file order -> contigs (a repeated name reuses its slot)
    struct Inst {
        int32_t contig;
        int64_t len;
    };
    std::vector<Inst> inst;
    std::unordered_map<std::string, int32_t> index;
    for (size_t i = 0; i < job.contigs.size(); ++i) index[job.contigs[i].name] = (int32_t)i;
    std::vector<int32_t> last_inst;   // per contig: the instance whose content it keeps
    for (int64_t t = 0; t < T; ++t) {
        Chunk &C = ck[(size_t)t];
        if (!inst.empty()) inst.back().len += C.pre;
        for (auto &h : C.hdrs) {
            if (h.name_b == h.name_a) fail(BWTMI_E_IO, "empty FASTA header in %s", path);   // split()[0]
            std::string name(p + h.name_a, (size_t)(h.name_b - h.name_a));
            auto it = index.find(name);
            int32_t cid;
            if (it == index.end()) {
                cid = (int32_t)job.contigs.size();
                index.emplace(name, cid);
                Contig c;
                c.name = std::move(name);
                job.contigs.push_back(std::move(c));
            } else {
                cid = it->second;
            }
            inst.push_back(Inst{cid, h.len});
        }
    }
    last_inst.assign(job.contigs.size(), -1);
    for (size_t k = 0; k < inst.size(); ++k) last_inst[(size_t)inst[k].contig] = (int32_t)k;
    const int64_t flank = flank_trim < 0 ? 0 : flank_trim;
    for (size_t cid = 0; cid < job.contigs.size(); ++cid) {
        const int32_t k = last_inst[cid];
        if (k < 0) continue;   // registered before this call and not in the file
        Contig &c = job.contigs[cid];
        const int64_t L = inst[(size_t)k].len;
        c.trim_left = c.trim_right = (L <= 2 * flank) ? 0 : flank;
        c.weight = L - c.trim_left - c.trim_right;
        c.gen = next_contig_gen();
    }

    // this rank's contigs
    std::vector<uint8_t> mine(job.contigs.size(), 1);
    if (world > 1) {
        std::fill(mine.begin(), mine.end(), 0);
        for (int32_t c : shard_units(job, world, rank)) mine[(size_t)c] = 1;
        job.selected.assign(mine.begin(), mine.end());
    } else {
        job.selected.clear();   // a whole load: every contig (a restriction from an earlier shard load goes)
    }
    // buffers (allocation only; pass 2 fills them in parallel)
    std::vector<char *> base(job.contigs.size(), nullptr);
    for (size_t cid = 0; cid < job.contigs.size(); ++cid) {
        const int32_t k = last_inst[cid];
        if (k < 0) continue;
        Contig &c = job.contigs[cid];
        if (!mine[cid]) {   // another rank's contig: name and weight only
            c.full.clear();
            c.trim_left = c.trim_right = 0;
            continue;
        }
        base[cid] = c.full.resize_uninit((size_t)inst[(size_t)k].len);   // filled by pass 2
    }
    // destinations of every chunk piece
    {
        size_t k = 0;
        int64_t off = 0;   // offset inside the current instance
        bool have = false;
        auto dst_of = [&](size_t kk, int64_t o) -> char * {
            const Inst &I = inst[kk];
            if (last_inst[(size_t)I.contig] != (int32_t)kk || !base[(size_t)I.contig]) return nullptr;
            return base[(size_t)I.contig] + o;
        };
        for (int64_t t = 0; t < T; ++t) {
            Chunk &C = ck[(size_t)t];
            if (have) {
                C.pre_dst = C.pre ? dst_of(k - 1, off) : nullptr;
                C.pre_cid = inst[k - 1].contig;
                C.pre_off = off;
                off += C.pre;
            }
            C.dst.resize(C.hdrs.size());
            C.dcid.resize(C.hdrs.size());
            for (size_t h = 0; h < C.hdrs.size(); ++h) {
                C.dst[h] = C.hdrs[h].len ? dst_of(k, 0) : nullptr;
                C.dcid[h] = inst[k].contig;
                off = C.hdrs[h].len;
                ++k;
                have = true;
            }
        }
    }
    const auto t2 = clk::now();
    auto stats = [&](const char *what) {
        if (stats_on()) {
            auto d = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
            std::fprintf(stderr, "  load_fasta: read %.1f pass1+stitch %.1f %s %.1f ms (%d threads, %lld chunks)\n",
                         d(t0, t1), d(t1, t2), what, d(t2, clk::now()), nt, (long long)T);
        }
    };
    if (!dev) {
        // pass 2: upper-cased content into place
        run_tasks(T, nt, [&](int64_t t) { pass2(p, ck[(size_t)t]); });
        stats("pass2");
        return;
    }
    // Device placement: the plain chunks are compacted on the device from the
    // file image (already on its way); the other chunks (headers, CR, spaces)
    // are written on the host now and their pieces copied up; the host copy of
    // the plain chunks is written behind the device work (Job::text_join).
    dev->contigs();
    std::vector<int64_t> rest;   // chunks whose head is written now
    std::vector<FastaPiece> pcs;
    for (int64_t t = 0; t < T; ++t) {
        const Chunk &C = ck[(size_t)t];
        if (!C.plain) rest.push_back(t);
        else if (C.pre_dst) pcs.push_back(FastaPiece{C.a, C.b, C.pre_off, C.pre_cid});
        if (C.tail_a >= 0) {
            int32_t cid;
            int64_t off;
            if (tail_dst(C, cid, off)) pcs.push_back(FastaPiece{C.tail_a, C.b, off, cid});
        }
    }
    run_tasks((int64_t)rest.size(), nt, [&](int64_t q) { pass2(p, ck[(size_t)rest[(size_t)q]], P_HEAD); });
    for (int64_t t : rest) {   // the head's pieces (a plain tail is not among them)
        const Chunk &C = ck[(size_t)t];
        const bool tail_pre = C.tail_a >= 0 && C.hdrs.empty();
        if (C.pre_dst) dev->piece(C.pre_cid, C.pre_off, C.pre_dst, C.pre - (tail_pre ? C.tail_len : 0));
        for (size_t h = 0; h < C.hdrs.size(); ++h) {
            const bool tail_here = C.tail_a >= 0 && h + 1 == C.hdrs.size();
            if (C.dst[h]) dev->piece(C.dcid[h], 0, C.dst[h], C.hdrs[h].len - (tail_here ? C.tail_len : 0));
        }
    }
    dev->plain(pcs);
    // the deferred pass owns the image (another load on this thread starts a
    // fresh one); the device layer keeps it until its copy has completed
    auto img = std::make_shared<Seq>();
    img->swap(data);
    auto keep = std::make_shared<std::vector<Chunk>>(std::move(ck));
    dev->defer(
        [keep, img, nt] {
            const std::vector<Chunk> &K = *keep;
            const char *q = img->data();
            run_tasks((int64_t)K.size(), nt, [&](int64_t t) {
                const Chunk &C = K[(size_t)t];
                if (C.plain || C.tail_a >= 0) pass2(q, C, P_TAIL);
            });
        },
        img);
    stats("non-plain pass2 + device launch");
}

// ------------------------------------------------------------------ split load
// Multi-rank load with an exchange (bwtmi_job_fasta_scan_part +
// bwtmi_job_load_fasta_parts): rank r runs pass 1 over its 1/world of the
// file only, the ranks exchange the resulting header tables (a few words per
// contig), and each rank then reads and copies only its own contigs' bytes.
// Every rank sees every header and every bad byte, so names, lengths, trims,
// the shard layout and a non-ASCII failure come out identical everywhere.
namespace {

// the first line start >= x (0, or the byte after '\n' / '\r'), N if none
int64_t line_start_from(int fd, int64_t N, int64_t x) {
    if (x <= 0) return 0;
    if (x >= N) return N;
    char buf[1 << 16];
    int64_t pos = x - 1;
    while (pos < N) {
        const ssize_t r = ::pread(fd, buf, (size_t)std::min<int64_t>((int64_t)sizeof buf, N - pos), (off_t)pos);
        if (r <= 0) fail(BWTMI_E_IO, "read error");
        for (ssize_t k = 0; k < r; ++k)
            if (eol(buf[k])) return pos + k + 1;
        pos += r;
    }
    return N;
}

// read pieces and line-start chunks of a split load: a rank's share of a
// file is small (12.5 MB of C4 at 8 ranks), so pieces shrink to keep every
// thread busy (4 MB pieces gave a 12.7 MB range 4 tasks for 16 threads)
inline int64_t split_piece(int64_t n, int nt) {
    return std::max<int64_t>(int64_t(256) << 10, std::min<int64_t>(int64_t(4) << 20, n / (2 * std::max(1, nt)) + 1));
}
inline int64_t split_chunks(int64_t n, int nt) {
    return std::max<int64_t>(1, std::min<int64_t>(4 * (int64_t)nt, n / (int64_t(256) << 10) + 1));
}

void pread_range(int fd, char *dst, int64_t a, int64_t b, int nt) {
    std::atomic<bool> bad{false};
    const int64_t piece = split_piece(b - a, nt);
    run_tasks((b - a + piece - 1) / piece, nt, [&](int64_t k) {
        int64_t o = a + k * piece;
        const int64_t e = std::min(b, o + piece);
        while (o < e) {
            const ssize_t r = ::pread(fd, dst + (o - a), (size_t)(e - o), (off_t)o);
            if (r <= 0) { bad = true; return; }
            o += r;
        }
    });
    if (bad) fail(BWTMI_E_IO, "read error");
}

struct Fd {
    int fd;
    explicit Fd(const char *path) : fd(::open(path, O_RDONLY)) {
        if (fd < 0) fail(BWTMI_E_IO, "cannot open %s", path);
    }
    ~Fd() { ::close(fd); }
    int64_t size() const {
        struct stat st;
        if (::fstat(fd, &st) != 0) fail(BWTMI_E_IO, "cannot stat");
        return (int64_t)st.st_size;
    }
    void stamp(int64_t out[2]) const {   // size and modification time (ns)
        struct stat st;
        if (::fstat(fd, &st) != 0) fail(BWTMI_E_IO, "cannot stat");
        out[0] = (int64_t)st.st_size;
        out[1] = (int64_t)st.st_mtim.tv_sec * 1000000000 + (int64_t)st.st_mtim.tv_nsec;
    }
};

// [a, b) of the buffer p cut into T chunks at line starts
std::vector<int64_t> cut_lines(const char *p, int64_t a, int64_t b, int64_t T, int nt) {
    std::vector<int64_t> cut((size_t)T + 1, b);
    cut[0] = a;
    run_tasks(T - 1, nt, [&](int64_t q) {
        int64_t i = a + (b - a) * (q + 1) / T;
        while (i < b && !eol(p[i - 1])) ++i;
        cut[(size_t)q + 1] = i;
    });
    for (int64_t t = 1; t <= T; ++t) cut[(size_t)t] = std::max(cut[(size_t)t], cut[(size_t)t - 1]);
    return cut;
}

}  // namespace

// blob (int64 words): N, A, B, bad, pre, nh, then per header: line, len,
// name bytes, name words (the name's bytes, zero-padded to 8)
// Header lines ('>' at the file start or right after '\n' / '\r') of a FASTA
// file, counted up to `limit`, in parallel 8 MiB pieces (each also reads the
// byte before it): the CLI's launch decision reads a 100 MB one-record file in
// ~2 ms instead of two mmap scans (~30 ms).  -1 if the file cannot be read.
int64_t fasta_count_records(const char *path, int64_t limit) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return -1;
    struct stat st;
    if (::fstat(fd, &st) != 0) {
        ::close(fd);
        return -1;
    }
    const int64_t size = (int64_t)st.st_size;
    constexpr int64_t kPiece = int64_t(8) << 20;
    const int64_t np = (size + kPiece - 1) / kPiece;
    std::atomic<int64_t> total{0};
    std::atomic<bool> bad{false};
    run_tasks(np, host_cpu_budget(nullptr, nullptr), [&](int64_t k) {
        if (bad.load(std::memory_order_relaxed) || total.load(std::memory_order_relaxed) >= limit) return;
        const int64_t a = k * kPiece, b = std::min(size, a + kPiece);
        const int64_t from = a > 0 ? a - 1 : 0;   // the byte before the piece decides its first '>'
        std::vector<char> buf((size_t)(b - from));   // this call's only: freed when the task ends
        int64_t got = 0;
        while (got < b - from) {
            const ssize_t r = ::pread(fd, buf.data() + got, (size_t)(b - from - got), (off_t)(from + got));
            if (r <= 0) {
                bad.store(true);
                return;
            }
            got += r;
        }
        const char *p = buf.data(), *e = p + got;
        int64_t c = 0;
        const char *q = p + (a > 0 ? 1 : 0);   // first byte of the piece
        if (a == 0 && q < e && *q == '>') ++c;
        while (q < e) {
            const char *g = (const char *)std::memchr(q, '>', (size_t)(e - q));
            if (!g) break;
            if (g > p && (g[-1] == '\n' || g[-1] == '\r')) ++c;
            q = g + 1;
        }
        total.fetch_add(c, std::memory_order_relaxed);
    });
    ::close(fd);
    if (bad.load()) return -1;
    return std::min<int64_t>(total.load(), limit);
}

void fasta_scan_part(Job &job, const char *path, int32_t world, int32_t rank, std::vector<int64_t> &blob) {
    const int nt = host_threads(job.params);
    Fd f(path);
    const int64_t N = f.size();
    const int64_t A = line_start_from(f.fd, N, N * rank / world), B = line_start_from(f.fd, N, N * (rank + 1) / world);
    Seq &part = job.part;
    job.part_settle();   // a device copy of the previous part has left it; its tag no longer names these bytes
    char *p = part.resize_uninit((size_t)std::max<int64_t>(0, B - A));
    job.part_path = path;
    job.part_a = A;
    job.part_b = B;
    f.stamp(job.part_stamp);
    if (B > A) pread_range(f.fd, p, A, B, nt);
    const int64_t n = B - A;
    const int64_t T = split_chunks(n, nt);
    const std::vector<int64_t> cut = cut_lines(p, 0, n, T, nt);
    std::vector<Chunk> ck((size_t)T);
    run_tasks(T, nt, [&](int64_t t) {
        Chunk &C = ck[(size_t)t];
        C.a = cut[(size_t)t];
        C.b = cut[(size_t)t + 1];
        if (const int64_t nl = plain_newlines(p + C.a, C.b - C.a); nl >= 0) {   // no header: all content
            C.plain = true;
            C.pre = (C.b - C.a) - nl;
            return;
        }
        for_lines(p, C.a, C.b, [&](int64_t s, int64_t e) {
            if (p[s] == '>') {
                int64_t x = s + 1;
                while (x < e && py_space((unsigned char)p[x])) ++x;
                int64_t y = x;
                while (y < e && !py_space((unsigned char)p[y])) ++y;
                C.hdrs.push_back(Hdr{x, y, 0, s});
                if (C.bad < 0 && !header_ok(p + s, e - s)) C.bad = s;
                return;
            }
            if (C.bad < 0)
                if (const int64_t q = first_high(p + s, e - s); q >= 0) C.bad = s + q;
            if (C.hdrs.empty()) C.pre += e - s;
            else C.hdrs.back().len += e - s;
        });
    });
    int64_t bad = -1, pre = 0, nh = 0;
    for (const Chunk &C : ck) {
        if (bad < 0 && C.bad >= 0) bad = A + C.bad;
        nh += (int64_t)C.hdrs.size();
    }
    blob.assign({N, A, B, bad, 0, nh});
    bool have = false;   // content after the last header so far lands in blob[last_at]
    size_t last_at = 0;
    for (const Chunk &C : ck) {
        if (have) blob[last_at] += C.pre;
        else pre += C.pre;
        for (const Hdr &h : C.hdrs) {
            const int64_t nb = h.name_b - h.name_a;
            blob.push_back(A + h.line);
            last_at = blob.size();
            blob.push_back(h.len);
            have = true;
            blob.push_back(nb);
            const size_t w0 = blob.size();
            blob.resize(w0 + (size_t)((nb + 7) / 8), 0);
            std::memcpy(blob.data() + w0, p + h.name_a, (size_t)nb);
        }
    }
    blob[4] = pre;
}

void fasta_load_parts(Job &job, const char *path, int32_t flank_trim, int32_t world, int32_t rank,
                      const int64_t *blob, int64_t nwords, FastaDev *dev) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    job.text_join();
    const int nt = host_threads(job.params);
    struct Inst {
        int32_t contig;
        int64_t len, line;
    };
    std::vector<Inst> inst;
    std::unordered_map<std::string, int32_t> index;
    for (size_t i = 0; i < job.contigs.size(); ++i) index[job.contigs[i].name] = (int32_t)i;
    int64_t N = -1, bad = -1, q = 0;
    for (int32_t r = 0; r < world; ++r) {
        if (q + 6 > nwords) fail(BWTMI_E_ARG, "truncated FASTA part table");
        const int64_t n = blob[q], b = blob[q + 3], pre = blob[q + 4], nh = blob[q + 5];
        if (N >= 0 && n != N) fail(BWTMI_E_ARG, "FASTA part tables of different files");
        N = n;
        if (b >= 0 && (bad < 0 || b < bad)) bad = b;
        if (!inst.empty()) inst.back().len += pre;
        q += 6;
        for (int64_t h = 0; h < nh; ++h) {
            if (q + 3 > nwords) fail(BWTMI_E_ARG, "truncated FASTA part table");
            const int64_t line = blob[q], len = blob[q + 1], nb = blob[q + 2];
            q += 3;
            if (nb < 0 || q + (nb + 7) / 8 > nwords) fail(BWTMI_E_ARG, "truncated FASTA part table");
            if (nb == 0) fail(BWTMI_E_IO, "empty FASTA header in %s", path);   // split()[0]
            std::string name((const char *)(blob + q), (size_t)nb);
            q += (nb + 7) / 8;
            auto it = index.find(name);
            int32_t cid;
            if (it == index.end()) {
                cid = (int32_t)job.contigs.size();
                index.emplace(name, cid);
                Contig c;
                c.name = std::move(name);
                job.contigs.push_back(std::move(c));
            } else {
                cid = it->second;
            }
            inst.push_back(Inst{cid, len, line});
        }
    }
    if (bad >= 0)
        fail(BWTMI_E_IO, "non-ASCII text at byte %lld of %s: the reference (bwt.py:3719, 121) fails on it",
             (long long)bad, path);
    std::vector<int32_t> last_inst(job.contigs.size(), -1);
    for (size_t k = 0; k < inst.size(); ++k) last_inst[(size_t)inst[k].contig] = (int32_t)k;
    const int64_t flank = flank_trim < 0 ? 0 : flank_trim;
    for (size_t cid = 0; cid < job.contigs.size(); ++cid) {
        const int32_t k = last_inst[cid];
        if (k < 0) continue;
        Contig &c = job.contigs[cid];
        const int64_t L = inst[(size_t)k].len;
        c.trim_left = c.trim_right = (L <= 2 * flank) ? 0 : flank;
        c.weight = L - c.trim_left - c.trim_right;
        c.gen = next_contig_gen();
    }
    std::vector<uint8_t> mine(job.contigs.size(), 1);
    if (world > 1) {
        std::fill(mine.begin(), mine.end(), 0);
        for (int32_t c : shard_units(job, world, rank)) mine[(size_t)c] = 1;
        job.selected.assign(mine.begin(), mine.end());
    } else {
        job.selected.clear();   // a whole load: every contig (a restriction from an earlier shard load goes)
    }
    const auto t1 = clk::now();
    Fd f(path);
    // this rank's contigs: their byte ranges read into one buffer by one
    // parallel read, then cut into line-start chunks that the count and copy
    // passes process as one flat list (not contig by contig: a 12.5 Mbp
    // contig alone gave the pool three read pieces and short regions)
    struct Own {
        size_t cid;
        int64_t a, b, off;   // file range [a, b) at off in the buffer
        size_t c0, c1;       // its chunks [c0, c1) of the flat list
    };
    std::vector<Own> own;
    int64_t tot = 0;
    for (size_t cid = 0; cid < job.contigs.size(); ++cid) {
        const int32_t k = last_inst[cid];
        if (k < 0) continue;
        Contig &c = job.contigs[cid];
        if (!mine[cid]) {   // another rank's contig: name and weight only
            c.full.clear();
            c.trim_left = c.trim_right = 0;
            continue;
        }
        const int64_t a = inst[(size_t)k].line;
        const int64_t b = (size_t)k + 1 < inst.size() ? inst[(size_t)k + 1].line : N;
        own.push_back(Own{cid, a, b, tot, 0, 0});
        tot += b - a;
    }
    // own contigs inside the range this rank's pass 1 read (the common case:
    // equal contigs, one per rank) are taken from those bytes in place; only
    // the others are read again
    int64_t st_now[2] = {-2, -2};
    f.stamp(st_now);
    const bool same_file = job.part_path == path && st_now[0] == job.part_stamp[0] && st_now[1] == job.part_stamp[1] &&
                           (int64_t)job.part.size() == job.part_b - job.part_a;
    bool inside = same_file && !own.empty();
    for (const Own &w : own) inside = inside && w.a >= job.part_a && w.b <= job.part_b;
    thread_local Seq raw;
    char *p = nullptr;
    if (inside) {
        p = job.part.data();
        for (Own &w : own) w.off = w.a - job.part_a;
    } else {
        p = raw.resize_uninit((size_t)tot);
    }
    int64_t span = 0;   // own bytes lie in p[0, span)
    for (const Own &w : own) span = std::max(span, w.off + (w.b - w.a));
    if (dev) dev->image(p, span);
    if (!inside) {
        const int64_t piece = split_piece(tot, nt);
        std::vector<std::pair<size_t, int64_t>> rd;   // (own index, piece start in its range)
        for (size_t u = 0; u < own.size(); ++u)
            for (int64_t o = 0; o < own[u].b - own[u].a; o += piece) rd.push_back({u, o});
        std::atomic<bool> bad{false};
        run_tasks((int64_t)rd.size(), nt, [&](int64_t q) {
            const Own &w = own[rd[(size_t)q].first];
            int64_t o = w.a + rd[(size_t)q].second;
            const int64_t e = std::min(w.b, o + piece);
            const int64_t o0 = o;
            while (o < e) {
                const ssize_t r = ::pread(f.fd, p + w.off + (o - w.a), (size_t)(e - o), (off_t)o);
                if (r <= 0) { bad = true; return; }
                o += r;
            }
            if (dev) dev->image_part(w.off + (o0 - w.a), e - o0);
        });
        if (bad) fail(BWTMI_E_IO, "read error");
    } else if (dev) {
        for (const Own &w : own) dev->image_part(w.off, w.b - w.a);   // already read by pass 1
    }
    std::vector<int64_t> ca, cb;   // chunk [ca, cb) in the buffer
    for (Own &w : own) {
        const int64_t n = w.b - w.a;
        const int64_t T = split_chunks(n, nt);
        const std::vector<int64_t> cut = cut_lines(p, w.off, w.off + n, T, nt);
        w.c0 = ca.size();
        for (int64_t t = 0; t < T; ++t) {
            ca.push_back(cut[(size_t)t]);
            cb.push_back(cut[(size_t)t + 1]);
        }
        w.c1 = ca.size();
    }
    const size_t NC = ca.size();
    std::vector<int64_t> cnt(NC, 0);
    std::vector<uint8_t> plain(NC, 0);
    run_tasks((int64_t)NC, nt, [&](int64_t t) {   // content bytes per chunk (the header line is skipped)
        const int64_t a0 = ca[(size_t)t], b0 = cb[(size_t)t];
        if (const int64_t nl = plain_newlines(p + a0, b0 - a0); nl >= 0) {   // lines need no per-line work
            plain[(size_t)t] = 1;
            cnt[(size_t)t] = (b0 - a0) - nl;
            return;
        }
        int64_t m = 0;
        for_lines(p, a0, b0, [&](int64_t s, int64_t e) {
            if (p[s] != '>') m += e - s;
        });
        cnt[(size_t)t] = m;
    });
    std::vector<char *> dst(NC, nullptr);   // where each chunk's content goes
    for (const Own &w : own) {
        int64_t len = 0;
        for (size_t t = w.c0; t < w.c1; ++t) len += cnt[t];
        Contig &c = job.contigs[w.cid];
        if (len != inst[(size_t)last_inst[w.cid]].len)
            fail(BWTMI_E_IO, "%s changed while it was read (contig %s)", path, c.name.c_str());
        char *d = c.full.resize_uninit((size_t)len);
        for (size_t t = w.c0; t < w.c1; ++t) {
            dst[t] = d;
            d += cnt[t];
        }
    }
    auto copy_chunk = [](const char *q, int64_t a0, int64_t b0, bool pl, char *d) {
        if (pl) {   // runs between newlines, as load_fasta's pass 2
            plain_copy(q, a0, b0, d);
            return;
        }
        for_lines(q, a0, b0, [&](int64_t s, int64_t e) {
            if (q[s] == '>') return;
            upper_copy(d, q + s, e - s);
            d += e - s;
        });
    };
    auto stats = [&] {
        if (stats_on()) {
            auto d = [](clk::time_point x, clk::time_point y) { return std::chrono::duration<double, std::milli>(y - x).count(); };
            std::fprintf(stderr, "  load_fasta_parts: stitch %.1f own contigs %.1f ms%s\n", d(t0, t1), d(t1, clk::now()),
                         dev ? " (device placement)" : "");
        }
    };
    if (!dev) {
        run_tasks((int64_t)NC, nt, [&](int64_t t) { copy_chunk(p, ca[(size_t)t], cb[(size_t)t], plain[(size_t)t], dst[(size_t)t]); });
        stats();
        return;
    }
    // device placement (load_fasta's): plain chunks rebuilt on the device from
    // the uploaded bytes, the others written here and copied up, the host copy
    // of the plain chunks written behind the scan
    dev->contigs();
    std::vector<int32_t> cid_of(NC, -1);
    for (const Own &w : own)
        for (size_t t = w.c0; t < w.c1; ++t) cid_of[t] = (int32_t)w.cid;
    std::vector<int64_t> rest;
    std::vector<FastaPiece> pcs;
    for (size_t t = 0; t < NC; ++t) {
        if (!dst[t] || !cnt[t]) continue;
        const int64_t off = dst[t] - job.contigs[(size_t)cid_of[t]].full.data();
        if (plain[t]) pcs.push_back(FastaPiece{ca[t], cb[t], off, cid_of[t]});
        else rest.push_back((int64_t)t);
    }
    run_tasks((int64_t)rest.size(), nt, [&](int64_t q) {
        const size_t t = (size_t)rest[(size_t)q];
        copy_chunk(p, ca[t], cb[t], false, dst[t]);
    });
    for (int64_t t : rest) {
        const Contig &c = job.contigs[(size_t)cid_of[(size_t)t]];
        dev->piece(cid_of[(size_t)t], dst[(size_t)t] - c.full.data(), dst[(size_t)t], cnt[(size_t)t]);
    }
    dev->plain(pcs);
    // the deferred pass holds the bytes: the thread-local read buffer moves into
    // it; the pass-1 bytes stay in the job (the next load joins this pass first)
    std::shared_ptr<Seq> hold = std::make_shared<Seq>();
    if (!inside) hold->swap(raw);
    struct Cp {
        int64_t a, b;
        char *d;
    };
    auto work = std::make_shared<std::vector<Cp>>();
    for (size_t t = 0; t < NC; ++t)
        if (plain[t] && dst[t] && cnt[t]) work->push_back(Cp{ca[t], cb[t], dst[t]});
    const char *src = inside ? p : hold->data();
    dev->defer(
        [work, src, nt] {
            const std::vector<Cp> &W = *work;
            run_tasks((int64_t)W.size(), nt, [&](int64_t k) { plain_copy(src, W[(size_t)k].a, W[(size_t)k].b, W[(size_t)k].d); });
        },
        hold);
    stats();
}

}  // namespace bwtmi
