// fasta_dev.hip -- the analysed sequences of a FASTA file built on the device
// from the raw file image (load_reference, bwt.py:3713-3756; fasta.cpp pass 2).
//
// The host loader's pass 1 finds the "plain" chunks (whole lines of bytes
// 0x21..0x7f other than '>', ended by '\n': no header, no CR, nothing to
// strip) and where their content lands in each contig.  Their content is every
// byte but the newlines, upper-cased, so the device rebuilds it from the image
// while the host writes its own copy behind the scan:
//   k_fa_count    per 8 KB segment of every piece: its newlines
//   exclusive scan of the segment counts (the content offset of each segment
//                 inside its piece is its byte offset minus the newlines before)
//   k_fa_compact  per segment: 256 threads x 32 bytes, newline-free bytes
//                 upper-cased into LDS at their block prefix, then one
//                 coalesced copy into the trimmed contig window
// Image bytes are read once (counts) + once (compact), the text written once.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "device.h"

namespace bwtmi {
namespace {

constexpr int kFaThreads = 256;
constexpr int kFaPer = 32;                          // bytes per thread
constexpr int64_t kFaSeg = kFaThreads * kFaPer;     // 8192 bytes per segment

struct DPiece {
    int64_t a, b;      // image bytes
    int64_t off;       // content offset of byte a in the contig
    int64_t tl, tn;    // the contig's trimmed window [tl, tl + tn)
    char *dst;         // device copy of the trimmed contig
    int64_t seg0;      // first segment of the piece
};

__global__ __launch_bounds__(kFaThreads) void k_fa_count(const uint8_t *__restrict__ img,
                                                         const DPiece *__restrict__ pc,
                                                         const int32_t *__restrict__ segp, int64_t nseg,
                                                         uint32_t *__restrict__ cnt) {
    __shared__ uint32_t ws[kFaThreads / 64];
    const int64_t s = blockIdx.x;
    if (s >= nseg) return;
    const DPiece P = pc[segp[s]];
    const int64_t lo = P.a + (s - P.seg0) * kFaSeg, hi = min(P.b, lo + kFaSeg);
    uint32_t c = 0;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kFaThreads) c += img[i] == '\n';
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[s] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(kFaThreads) void k_fa_compact(const uint8_t *__restrict__ img,
                                                           const DPiece *__restrict__ pc,
                                                           const int32_t *__restrict__ segp, int64_t nseg,
                                                           const uint32_t *__restrict__ nl_before) {
    __shared__ char buf[kFaSeg];
    __shared__ uint32_t wsum[kFaThreads / 64];
    const int64_t s = blockIdx.x;
    if (s >= nseg) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const DPiece P = pc[segp[s]];
    const int64_t lo = P.a + (s - P.seg0) * kFaSeg, hi = min(P.b, lo + kFaSeg);
    // this thread's 32 bytes
    const int64_t x0 = lo + (int64_t)t * kFaPer;
    char v[kFaPer];
    uint32_t keep = 0;   // bit k: byte k is content
#pragma unroll
    for (int k = 0; k < kFaPer; ++k) {
        const int64_t i = x0 + k;
        const uint8_t ch = i < hi ? img[i] : (uint8_t)'\n';
        v[k] = (char)(ch - ((uint8_t)(ch - 'a') < 26u ? 32 : 0));
        keep |= (uint32_t)(ch != '\n') << k;
    }
    const uint32_t c = (uint32_t)__popc(keep);
    // block exclusive prefix of the per-thread counts
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    uint32_t at = base + incl - c;
#pragma unroll
    for (int k = 0; k < kFaPer; ++k)
        if (keep >> k & 1u) buf[at++] = v[k];
    __syncthreads();
    // content offset of the segment's first byte in the contig
    const int64_t seg_in_piece = (s - P.seg0) * kFaSeg;
    const int64_t o0 = P.off + seg_in_piece - (int64_t)(nl_before[s] - nl_before[P.seg0]);
    for (uint32_t j = (uint32_t)t; j < tot; j += kFaThreads) {
        const int64_t idx = o0 + j - P.tl;
        if (idx >= 0 && idx < P.tn) P.dst[idx] = buf[j];
    }
}

__global__ void k_wake() {}

}  // namespace

void device_wake(Ctx &c) {
    k_wake<<<1, 64, 0, c.stream>>>();
    HIPCHECK(hipGetLastError());
}

void fasta_build_device(Ctx &c, const uint8_t *d_img, const FastaDevPiece *pieces, int64_t npieces) {
    if (npieces <= 0) return;
    hipStream_t st = c.stream;
    std::vector<DPiece> hp((size_t)npieces);
    std::vector<int32_t> segp;
    int64_t nseg = 0;
    for (int64_t k = 0; k < npieces; ++k) {
        const FastaDevPiece &q = pieces[k];
        DPiece &d = hp[(size_t)k];
        d.a = q.a;
        d.b = q.b;
        d.off = q.off;
        d.tl = q.tl;
        d.tn = q.tn;
        d.dst = q.dst;
        d.seg0 = nseg;
        const int64_t ns = (q.b - q.a + kFaSeg - 1) / kFaSeg;
        for (int64_t x = 0; x < ns; ++x) segp.push_back((int32_t)k);
        nseg += ns;
    }
    if (nseg == 0) return;
    // table: pieces, segment -> piece, counts (nseg + 1 for the scan)
    const size_t tb = hp.size() * sizeof(DPiece), sb = segp.size() * 4;
    c.slot[S_MISC3].ensure(tb + sb + (size_t)(nseg + 1) * 8 + 256);
    char *base = c.slot[S_MISC3].as<char>();
    DPiece *d_pc = (DPiece *)base;
    int32_t *d_segp = (int32_t *)(base + ((tb + 15) & ~size_t(15)));
    uint32_t *d_cnt = (uint32_t *)((char *)d_segp + ((sb + 15) & ~size_t(15)));
    // pinned staging: the copies run behind this call, so the previous load's
    // table copies (another job may share this context) must have read it
    HBuf &hs = c.host[3];
    hs.ensure(tb + sb + 64);   // settles the previous copies first
    std::memcpy(hs.p, hp.data(), tb);
    std::memcpy((char *)hs.p + tb, segp.data(), sb);
    HIPCHECK(hipMemcpyAsync(d_pc, hs.p, tb, hipMemcpyHostToDevice, st));
    HIPCHECK(hipMemcpyAsync(d_segp, (char *)hs.p + tb, sb, hipMemcpyHostToDevice, st));
    hs.arm(st);
    KLAUNCH("k_fa_count", 0.0, k_fa_count, dim3((unsigned)nseg), dim3(kFaThreads), 0, st, d_img, d_pc, d_segp, nseg,
            d_cnt);
    exclusive_scan<uint32_t>(c, d_cnt, d_cnt, nseg);
    KLAUNCH("k_fa_compact", 0.0, k_fa_compact, dim3((unsigned)nseg), dim3(kFaThreads), 0, st, d_img, d_pc, d_segp,
            nseg, d_cnt);
    HIPCHECK(hipGetLastError());
}

}  // namespace bwtmi
