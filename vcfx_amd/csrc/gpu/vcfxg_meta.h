// vcfxg_meta.h -- the head pass of one data line (k_line_meta, k_af_stream): its first 160
// bytes decide the kind -- empty (after the mmap-mode '\r' strip), '#', GT-first data line
// (FORMAT's first sub-field is GT: the reference's findGTIndex == 0, VCFX_allele_freq_calc
// .cpp:298-316) with its sample region start S, first separator and row prefix length, or
// the full per-line path for anything else.  Templated on the byte source: global memory
// or an LDS ring holding the line.
#pragma once
#include "vcfxg_device.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

struct GlobalSrc {
    const char *buf;
    __device__ __forceinline__ uint4 load16(int64_t x) const { return vcfxg::load16(buf, x); }
    __device__ __forceinline__ uint32_t load4(int64_t x) const { return vcfxg::load4(buf, x); }
    __device__ __forceinline__ uint32_t byte(int64_t x) const { return byte_at(buf, x); }
};

template <class Src>
__device__ __forceinline__ LineMeta head_meta(const Src &src, int64_t ls, int64_t le, int strip_cr) {
    LineMeta m{};
    m.kind = kMetaFull;
    if (le <= ls) {
        m.kind = kMetaEmpty;
        return m;
    }
    const int64_t a = ls & ~(int64_t)15;
    constexpr int kB = 10;  // 160 bytes of head
    uint4 v[kB];
#pragma unroll
    for (int b = 0; b < kB; b++) v[b] = src.load16(a + 16 * b);
    const uint32_t last = src.byte(le - 1);
    int64_t ae = le;
    if (strip_cr && last == '\r') {
        ae--;
        m.cr = 1;
    }
    const uint32_t first = src.byte(ls);
    if (ae <= ls || first == '#') {
        m.kind = ae <= ls ? kMetaEmpty : kMetaHeader;
        return m;
    }
    int nt = 0;
    int64_t t4 = 0, t7 = 0, t8 = 0;
#pragma unroll
    for (int b = 0; b < kB; b++) {
        uint32_t mk = eq_mask16(v[b], kRepTab) & range_mask16(a + 16 * b, ls, ae);
        while (mk && nt < 9) {
            const int j = __builtin_ctz(mk);
            mk &= mk - 1u;
            const int64_t p = a + 16 * b + j;
            nt++;
            if (nt == 5) t4 = p;
            if (nt == 8) t7 = p;
            if (nt == 9) t8 = p;
        }
    }
    if (nt == 9 && t8 - t7 >= 3 && src.byte(t7 + 1) == 'G' && src.byte(t7 + 2) == 'T' &&
        (t8 - t7 == 3 || src.byte(t7 + 3) == ':')) {
        m.kind = kMetaGt;
        m.S = (uint64_t)(t8 + 1);
        m.rowpre = (uint32_t)(t4 - ls + 1);
        m.sep = t8 + 2 < ae ? (uint8_t)src.byte(t8 + 2) : 0;
    }
    return m;
}

}  // namespace vcfxg
