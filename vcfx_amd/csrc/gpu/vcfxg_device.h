// vcfxg_device.h -- device-side building blocks shared by the record kernels (gfx950,
// wave64).  Byte classification is SWAR on 32-bit words loaded 16 B per lane; cross-lane
// work uses wave64 ballots and shuffles; nothing here assumes a 32-wide warp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcfxg {

constexpr int kWave = 64;
constexpr int kBlockBytes = 16;                 // bytes per lane per load
constexpr int kWaveStep = kWave * kBlockBytes;  // 1 KiB per wave-wide load
constexpr uint32_t kRepTab = 0x09090909u, kRepNl = 0x0A0A0A0Au, kRepColon = 0x3A3A3A3Au;

__device__ __forceinline__ int lane() { return (int)__lane_id(); }

// 0x80 in every zero byte of x, exact per byte (no borrow false positives)
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
// compress a 0x80-per-byte mask to 4 bits (bit j = byte j)
__device__ __forceinline__ uint32_t pack4(uint32_t m) { return (((m >> 7) * 0x00204081u) >> 21) & 0xFu; }

// bytes of a 4-bit mask (bit j -> byte j = 0xFF)
__device__ __forceinline__ uint32_t nib_bytes(uint32_t nib) { return ((nib * 0x00204081u) & 0x01010101u) * 0xFFu; }
// 16-bit mask of the bytes of v equal to the byte replicated in rep
__device__ __forceinline__ uint32_t eq_mask16(const uint4 v, uint32_t rep) {
    return pack4(zero_bytes(v.x ^ rep)) | (pack4(zero_bytes(v.y ^ rep)) << 4) |
           (pack4(zero_bytes(v.z ^ rep)) << 8) | (pack4(zero_bytes(v.w ^ rep)) << 12);
}

// bits j of a 16-byte block at `base` with lo <= base + j < hi
__device__ __forceinline__ uint32_t range_mask16(int64_t base, int64_t lo, int64_t hi) {
    int64_t a = lo - base, b = hi - base;
    a = a < 0 ? 0 : (a > 16 ? 16 : a);
    b = b < 0 ? 0 : (b > 16 ? 16 : b);
    if (b <= a) return 0u;
    return ((1u << b) - 1u) & ~((1u << a) - 1u);
}

// bits j of a 16-byte block at relative offset b with lo <= b + j < hi (32-bit offsets)
__device__ __forceinline__ uint32_t range16(int b, int lo, int hi) {
    int a = lo - b, e = hi - b;
    a = a < 0 ? 0 : (a > 16 ? 16 : a);
    e = e < 0 ? 0 : (e > 16 ? 16 : e);
    return e <= a ? 0u : ((1u << e) - 1u) & ~((1u << a) - 1u);
}

__device__ __forceinline__ uint4 load16(const char *buf, int64_t off) {
    return *reinterpret_cast<const uint4 *>(buf + off);
}
// a raw buffer resource over [p, p + bytes) (bytes < 2^31, p wave-uniform): a load whose
// offset is past the end returns 0 without touching memory, so a sweep's lanes past its
// record need no clamped addresses -- the load is one instruction on a per-lane 32-bit offset
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, int off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return uint4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ uint32_t bload4(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t load4(const char *buf, int64_t off) {
    return *reinterpret_cast<const uint32_t *>(buf + off);
}
__device__ __forceinline__ uint32_t byte_at(const char *buf, int64_t off) {
    return (uint32_t)(uint8_t)buf[off];
}

// DPP move of x within the wave (lanes the pattern gives no source, or rows row_mask leaves
// out, read 0): the building block of the 32-bit scans and sums below, which take six DPP
// adds where the shuffle forms took six LDS permutes, each a round trip the wave waits for
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, kRowMask, 0xF, false);
}
// inclusive prefix sum over the 64 lanes: Hillis-Steele inside each row of 16 (row_shr 1, 2,
// 4, 8), then row 0's total into row 1 and row 2's into row 3 (row_bcast:15), then rows
// 0..1's total into rows 2 and 3 (row_bcast:31).  EVERY LANE MUST BE ACTIVE (a DPP source
// lane outside EXEC holds a stale value): the walkers' uniform per-record code calls it.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    x += dpp0<0x111>(x);
    x += dpp0<0x112>(x);
    x += dpp0<0x114>(x);
    x += dpp0<0x118>(x);
    x += dpp0<0x142, 0xA>(x);
    x += dpp0<0x143, 0xC>(x);
    return x;
}
// the sum over the wave (every lane active), wave-uniform in scalar registers
__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
    return __builtin_amdgcn_readlane(wave_incl_scan32(x), kWave - 1);
}
template <typename T>
__device__ __forceinline__ T wave_incl_scan(T v) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        T t = __shfl_up(v, o);
        if (lane() >= o) v += t;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_bcast(T v, int src) { return __shfl(v, src); }
// acc + popcount(x) as the one v_bcnt_u32_b32 with its accumulator operand
__device__ __forceinline__ uint32_t popc_acc(uint32_t x, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}
// lane k's 32-bit x (k wave-uniform), in scalar registers
__device__ __forceinline__ uint32_t lane_get(uint32_t x, int k) { return __builtin_amdgcn_readlane(x, k); }
// lane i gets lane i - 1's x, lane 0 gets 0: one DPP move (wave_shr:1), no LDS permute
__device__ __forceinline__ uint32_t lane_prev(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x138, 0xF, 0xF, false);
}
// the last lane's x, wave-uniform (v_readlane into a scalar register)
__device__ __forceinline__ uint32_t lane_last(uint32_t x) { return __builtin_amdgcn_readlane(x, 63); }

// a value known to be equal in all lanes, moved to scalar registers
__device__ __forceinline__ int64_t uniform64(int64_t v) {
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int uniform32(int v) { return (int)__builtin_amdgcn_readfirstlane((uint32_t)v); }

// j-th (0-based) set bit of m (m has > j bits set)
__device__ __forceinline__ int nth_bit(uint32_t m, int j) {
    for (int k = 0; k < j; k++) m &= m - 1u;
    return __builtin_ctz(m);
}

// ---------------------------------------------------------------------------------------
// head parse: absolute offsets of the first `want` (<= 10) tabs of the line [ls, le)
// (wave-cooperative; results uniform across the wave).  Returns the number found.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int head_tabs(const char *buf, int64_t ls, int64_t le, int want, int64_t *t,
                                         int64_t *lds /* per-wave scratch of >= 10 */) {
    int nt = 0;
    for (int64_t w = ls & ~(int64_t)15; w < le && nt < want; w += kWaveStep) {
        int64_t blk = w + (int64_t)lane() * kBlockBytes;
        uint32_t m = 0;
        if (blk < le) m = eq_mask16(load16(buf, blk), kRepTab) & range_mask16(blk, ls, le);
        int c = __popc(m);
        int incl = wave_incl_scan(c);
        int excl = incl - c;
        int total = wave_bcast(incl, kWave - 1);
        // each lane deposits its tabs whose running index is < want
        int idx = nt + excl;
        uint32_t mm = m;
        while (mm && idx < want) {
            int j = __builtin_ctz(mm);
            mm &= mm - 1u;
            lds[idx] = blk + j;
            idx++;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        nt += total;
    }
    if (nt > want) nt = want;
    // wave-uniform: keep the offsets in SGPRs
    for (int k = 0; k < nt; k++) t[k] = uniform64(lds[k]);
    __builtin_amdgcn_wave_barrier();
    return nt;
}

// ---------------------------------------------------------------------------------------
// index of the first "GT" sub-field of FORMAT [fs, fe) (colon separated), -1 if none.
// Semantics of findGTIndex, VCFX_allele_freq_calc.cpp:298-316 / VCFX_genotype_query.cpp:
// 176-194 (both return the same index whenever one exists).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int gt_index(const char *buf, int64_t fs, int64_t fe) {
    int before = 0;
    for (int64_t w = fs; w < fe; w += kWave) {
        int64_t p = w + lane();
        bool in = p < fe;
        uint32_t c = in ? byte_at(buf, p) : 0u;
        bool start = in && (p == fs || byte_at(buf, p - 1) == ':');
        bool match = start && c == 'G' && p + 1 < fe && byte_at(buf, p + 1) == 'T' &&
                     (p + 2 == fe || byte_at(buf, p + 2) == ':');
        uint64_t mm = __ballot(match);
        uint64_t cm = __ballot(in && c == ':');
        if (mm) {
            int L = __builtin_ctzll(mm);
            uint64_t below = L ? (cm & ((1ull << L) - 1ull)) : 0ull;
            return before + __popcll(below);
        }
        before += __popcll(cm);
    }
    return -1;
}

}  // namespace vcfxg
