// fasta.cpp -- TandemRepeatFinder.load_reference (bwt.py:3713-3756), native.
// Python reads the file in text mode: universal newlines (\n, \r\n, \r end a
// line), each line .strip()-ed (ASCII whitespace incl. \x1c-\x1f), headers
// '>' take line[1:].split()[0], other non-empty lines are upper-cased and
// appended (inner whitespace kept).  A repeated name keeps its first position
// and the last content.  Trim: 30+30 flanks when len > 2*flank_trim.
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace bwtmi {

static inline bool py_space(unsigned char c) {
    return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f);
}

void load_fasta(Job &job, const char *path, int32_t flank_trim) {
    FILE *f = std::fopen(path, "rb");
    if (!f) fail(BWTMI_E_IO, "cannot open %s", path);
    std::string data;
    {
        std::fseek(f, 0, SEEK_END);
        long sz = std::ftell(f);
        std::fseek(f, 0, SEEK_SET);
        if (sz < 0) sz = 0;
        data.resize((size_t)sz);
        if (sz && std::fread(&data[0], 1, (size_t)sz, f) != (size_t)sz) {
            std::fclose(f);
            fail(BWTMI_E_IO, "read error on %s", path);
        }
        std::fclose(f);
    }
    const int64_t flank = flank_trim < 0 ? 0 : flank_trim;
    std::unordered_map<std::string, size_t> index;
    for (size_t i = 0; i < job.contigs.size(); ++i) index[job.contigs[i].name] = i;
    std::string name;
    bool have = false;
    std::string seq;
    auto flush = [&]() {
        Contig c;
        c.name = name;
        c.full.swap(seq);
        const int64_t L = (int64_t)c.full.size();
        if (L <= 2 * flank) {
            c.trim_left = c.trim_right = 0;
        } else {
            c.trim_left = c.trim_right = flank;
        }
        auto it = index.find(c.name);
        if (it != index.end()) {
            job.contigs[it->second] = std::move(c);
        } else {
            index[c.name] = job.contigs.size();
            job.contigs.push_back(std::move(c));
        }
        seq.clear();
    };
    const char *p = data.data();
    const size_t n = data.size();
    size_t i = 0;
    while (i < n) {
        size_t j = i;
        while (j < n && p[j] != '\n' && p[j] != '\r') ++j;
        size_t a = i, b = j;
        while (a < b && py_space((unsigned char)p[a])) ++a;
        while (b > a && py_space((unsigned char)p[b - 1])) --b;
        if (b > a) {
            if (p[a] == '>') {
                if (have) flush();
                size_t x = a + 1;
                while (x < b && py_space((unsigned char)p[x])) ++x;
                size_t y = x;
                while (y < b && !py_space((unsigned char)p[y])) ++y;
                if (y == x) fail(BWTMI_E_IO, "empty FASTA header in %s", path);  // split()[0] IndexError
                name.assign(p + x, y - x);
                have = true;
                seq.clear();
            } else {
                const size_t o = seq.size();
                seq.append(p + a, b - a);
                for (size_t k = o; k < seq.size(); ++k)
                    if (seq[k] >= 'a' && seq[k] <= 'z') seq[k] = (char)(seq[k] - 32);
            }
        }
        // line end: \r\n counts once
        if (j < n && p[j] == '\r' && j + 1 < n && p[j + 1] == '\n') ++j;
        i = j + 1;
    }
    if (have) flush();
}

}  // namespace bwtmi
