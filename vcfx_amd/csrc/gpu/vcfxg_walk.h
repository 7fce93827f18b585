// vcfxg_walk.h -- building blocks of the walk kernels (vcfxg_af_walk.hip, vcfxg_fq_walk.hip):
// one wave ("walker") per chunk of the data region walks the chunk's lines one after the
// other, each line's head analysed out of an LDS window that was fetched (LDS-DMA) while the
// previous line's sample sweep ran.
#pragma once
#include <algorithm>

#include "vcfxg_device.h"

namespace vcfxg {

#ifndef VCFXG_WALK_THREADS
#define VCFXG_WALK_THREADS 256
#endif
constexpr int kWalkThreads = VCFXG_WALK_THREADS;  // walkers (waves) per block x 64
constexpr int kWalkWaves = kWalkThreads / kWave;
// a walker's search for its first line start reads the tail of the previous chunk's last
// line, which that chunk's walker reads too (much later, so from HBM again): small steps
#ifndef VCFXG_FIRST_SCAN_U
#define VCFXG_FIRST_SCAN_U 4
#endif
constexpr int kFirstScanU = VCFXG_FIRST_SCAN_U;

// The walker block of this workgroup.  The dispatcher hands workgroup b to XCD b mod 8; with
// VCFXG_WALK_XCD each XCD takes one contiguous eighth of the blocks instead, in order, so the
// two walkers either side of a block boundary run at about the same time on one XCD and the
// bytes both read at their starts (the straddling line's head, the backward scans) come from
// one L2 rather than from HBM twice.  Bijective for any grid.
#ifndef VCFXG_WALK_XCD
#define VCFXG_WALK_XCD 1
#endif
__device__ __forceinline__ uint32_t walk_block() {
    const uint32_t b = blockIdx.x;
    if (!VCFXG_WALK_XCD) return b;
    const uint32_t n = gridDim.x, q = n / 8, r = n % 8, x = b % 8, k = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + k;
}

// first '\n' in [p, hi), else hi (wave-uniform; kU KiB per step, lane offsets 32-bit)
template <int kU = 4>
__device__ __forceinline__ int64_t scan_nl(const char *__restrict__ buf, int64_t p, int64_t hi) {
    const int lo16 = 16 * lane();
    for (int64_t w = p & ~(int64_t)15; w < hi; w += kU * kWaveStep) {
        const char *__restrict__ wb = buf + w;
        const int pr = (int)std::max<int64_t>(p - w, 0), hr = (int)std::min<int64_t>(hi - w, kU * kWaveStep);
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {  // branch-free: lanes past hi re-read the last block
            const int b = u * kWaveStep + lo16;
            v[u] = load16(wb, b < hr ? b : ((hr - 1) & ~15));
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int b = u * kWaveStep + lo16;
            const uint32_t m = eq_mask16(v[u], kRepNl) & range16(b, pr, hr);
            const uint64_t any = __ballot(m != 0u);
            if (any) {
                const int k = __builtin_ctzll(any);
                const uint32_t mk = lane_get(m, k);
                return uniform64(w + (int64_t)u * kWaveStep + 16 * k + __builtin_ctz(mk));
            }
        }
    }
    return hi;
}

// true iff [a, b) holds no '\n' (a 16-aligned, a < b, wave-uniform): the rest of a record whose
// sweep stopped early (a match), checked before a predicted end is accepted.  A step of kU KiB
// through a buffer resource, tested with the exact zero-byte test ANDed over the lane's dwords
// (one ballot a step); only the last step, whose blocks may hold bytes at or past b, takes the
// exact per-byte masks
template <int kU = 4>
__device__ __forceinline__ bool nl_free(const char *__restrict__ buf, int64_t a, int64_t b) {
    const int lo16 = kBlockBytes * lane();
    constexpr uint32_t K = 0x7F7F7F7Fu;
    for (int64_t w = a; w < b; w += (int64_t)kU * kWaveStep) {
        const int hr = (int)std::min<int64_t>(b - w, (int64_t)kU * kWaveStep);
        const __amdgpu_buffer_rsrc_t rs = buf_rsrc(buf + w, (uint32_t)((hr + 15) & ~15));
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) v[u] = bload16(rs, u * kWaveStep + lo16);
        if (hr == kU * kWaveStep) {  // every byte of the step is below b
            uint32_t t = ~0u;
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const uint32_t x0 = v[u].x ^ kRepNl, x1 = v[u].y ^ kRepNl, x2 = v[u].z ^ kRepNl, x3 = v[u].w ^ kRepNl;
                t &= (((x0 & K) + K) | x0) & (((x1 & K) + K) | x1) & (((x2 & K) + K) | x2) & (((x3 & K) + K) | x3);
            }
            if (__ballot((~t & 0x80808080u) != 0u)) return false;
        } else {
            uint32_t m = 0;
#pragma unroll
            for (int u = 0; u < kU; u++) m |= eq_mask16(v[u], kRepNl) & range16(u * kWaveStep + lo16, 0, hr);
            if (__ballot(m != 0u)) return false;
        }
    }
    return true;
}

// last '\n' in [lo, p), else lo - 1 (wave-uniform; kU KiB per step, backwards from p: lane 0
// holds the highest block of a step, so the first lane with a '\n' holds the last one)
template <int kU = 4>
__device__ __forceinline__ int64_t scan_nl_back(const char *__restrict__ buf, int64_t p, int64_t lo) {
    if (p <= lo) return lo - 1;
    const int64_t tb = (p - 1) & ~(int64_t)15, lb = lo & ~(int64_t)15;
    for (int64_t top = tb; top >= lb; top -= (int64_t)kU * kWaveStep) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {  // branch-free: lanes below lo re-read the lowest block
            const int64_t bb = top - (int64_t)kBlockBytes * (u * kWave + lane());
            v[u] = load16(buf, bb >= lb ? bb : lb);
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int64_t bb = top - (int64_t)kBlockBytes * (u * kWave + lane());
            const uint32_t m = bb >= lb ? eq_mask16(v[u], kRepNl) & range_mask16(bb, lo, p) : 0u;
            const uint64_t any = __ballot(m != 0u);
            if (any) {
                const int k = __builtin_ctzll(any);
                const uint32_t mk = lane_get(m, k);  // (nonzero: lane k's exact mask)
                return uniform64(top - (int64_t)kBlockBytes * (u * kWave + k) + 31 - __builtin_clz(mk));
            }
        }
    }
    return lo - 1;
}

// A walker's lines: those starting in [b(cs), b(ce)), b(x) = the byte after the last '\n'
// before x (b = lo for the first chunk, hi past the last): the line across a chunk boundary
// belongs to the walker after it, which reads that line first, right after its backward
// scans over the line's head (the walker before stops at the same b).  With lines owned by the
// chunk of their first byte, a walker's forward search for its first line read the tail of
// the previous chunk's last line, which that chunk's walker read again only at its end (from
// HBM: the walk's 3.9 % over-fetch).
#ifndef VCFXG_WALK_SCAN_U
// KiB per backward-scan step.  r05: 1 (from 3): a step reads past the '\n' it finds into the
// previous line, which that line's walker reads again much later -- PMC fetch 4.61 -> 4.56 GB per
// AF walk launch (a plain stream of the same bytes: 4.45), walk time unchanged or 0.3 % better
// (profiles/r05_walk_scan_step_ab.txt, r05_pmc_calibration.json)
#define VCFXG_WALK_SCAN_U 1
#endif
template <int kU>
__device__ __forceinline__ void walker_lines_u(const char *__restrict__ buf, int64_t lo, int64_t hi, int64_t cs,
                                               int64_t ce, int64_t &b0, int64_t &b1) {
    // both backward scans in one loop: each step issues the loads of both before either is
    // examined (one round trip for the two where two scans in sequence took two)
    // (kU KiB per step; 4: the prologue pushed the walks over an occupancy step)
    bool da = cs <= lo, db = ce >= hi;
    int64_t ra = lo - 1, rb = lo - 1;
    const int64_t lb = lo & ~(int64_t)15;
    int64_t ta = (cs - 1) & ~(int64_t)15, tb = (ce - 1) & ~(int64_t)15;
    if (ta < lb) da = true;
    if (tb < lb) db = true;
    // a step's blocks descend from top: block (u, lane) at top - 16 (64 u + lane).  Each scan's
    // loads go through a buffer based at its iteration's lowest block (no lower than lb), so a
    // block below lb -- or any block of a finished scan (an empty buffer) -- reads zeros with
    // no clamped 64-bit address: its offset is negative, i.e. far past the buffer's end.
    constexpr int kSpan = kU * kWave * kBlockBytes;
    const int off16 = kBlockBytes * lane();
    while (!(da && db)) {
        const int64_t ba = std::max<int64_t>(lb, ta + kBlockBytes - kSpan), bb0 = std::max<int64_t>(lb, tb + kBlockBytes - kSpan);
        const __amdgpu_buffer_rsrc_t rsa = buf_rsrc(buf + ba, da ? 0u : (uint32_t)(ta + kBlockBytes - ba));
        const __amdgpu_buffer_rsrc_t rsb = buf_rsrc(buf + bb0, db ? 0u : (uint32_t)(tb + kBlockBytes - bb0));
        uint4 va[kU], vb[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            va[u] = bload16(rsa, (int)(ta - ba) - (u * kWaveStep + off16));
            vb[u] = bload16(rsb, (int)(tb - bb0) - (u * kWaveStep + off16));
        }
        // per step: any '\n' at all (exact per byte: ((x & 0x7F..) + 0x7F..) | x has bit 7 clear
        // only in a zero byte; the four dwords' words ANDed), then, in the rare step that has
        // one, the exact masks inside [lo, p) (a hit outside them -- header bytes below lo, bytes
        // at or past p in the top block -- is dropped there and the scan goes on)
        auto look = [&](const uint4 *v, int64_t top, int64_t p, bool &done, int64_t &r) {
            if (done) return;
#pragma unroll
            for (int u = 0; u < kU; u++) {
                const uint32_t x0 = v[u].x ^ kRepNl, x1 = v[u].y ^ kRepNl, x2 = v[u].z ^ kRepNl, x3 = v[u].w ^ kRepNl;
                const uint32_t K = 0x7F7F7F7Fu;
                const uint32_t t = (((x0 & K) + K) | x0) & (((x1 & K) + K) | x1) & (((x2 & K) + K) | x2) &
                                   (((x3 & K) + K) | x3);
                if (!__ballot((~t & 0x80808080u) != 0u)) continue;
                const int64_t bb = top - (int64_t)kBlockBytes * (u * kWave + lane());
                const uint32_t m = bb >= lb ? eq_mask16(v[u], kRepNl) & range_mask16(bb, lo, p) : 0u;
                const uint64_t any = __ballot(m != 0u);
                if (any) {
                    const int k = __builtin_ctzll(any);
                    const uint32_t mk = lane_get(m, k);  // (nonzero: lane k's exact mask)
                    r = uniform64(top - (int64_t)kBlockBytes * (u * kWave + k) + 31 - __builtin_clz(mk));
                    done = true;
                    return;
                }
            }
        };
        look(va, ta, cs, da, ra);
        look(vb, tb, ce, db, rb);
        ta -= (int64_t)kU * kWaveStep;
        tb -= (int64_t)kU * kWaveStep;
        if (ta < lb) da = true;
        if (tb < lb) db = true;
    }
    b0 = cs <= lo ? lo : ra + 1;
    b1 = ce >= hi ? hi : rb + 1;
}
// the step by chunk size: long-record chunks (> 256 KiB: ~12 records of > 16 KiB, the boundary
// ~half a record back) take 3 KiB steps -- 1 KiB steps cost the GT:AD:DP walk 3 % (r05)
__device__ __forceinline__ void walker_lines(const char *__restrict__ buf, int64_t lo, int64_t hi, int64_t cs,
                                             int64_t ce, int64_t &b0, int64_t &b1, int64_t chunk) {
    if (chunk > ((int64_t)256 << 10)) walker_lines_u<3>(buf, lo, hi, cs, ce, b0, b1);
    else walker_lines_u<VCFXG_WALK_SCAN_U>(buf, lo, hi, cs, ce, b0, b1);
}

// The head analysis classifies the window SWAR and then walks the matches in scalar code:
// the lanes holding a match come from one ballot, each one's mask from one v_readlane, and
// the positions in ascending order from s_ff1 -- no wave scan, no LDS permute, no per-lane
// bit loop.  Two lane layouts: kBytes = 4 (lane l holds window bytes [4l, 4l + 4), a mask
// with 0x80 per matching byte; the kWin window) or 16 (bytes [16l, 16l + 16), one bit per
// byte; the 1 KiB window of a long head).
template <int kBytes>
__device__ __forceinline__ int match_pos(int k, uint32_t m) {
    return kBytes == 4 ? 4 * k + (__builtin_ctz(m) >> 3) : 16 * k + __builtin_ctz(m);
}
// the first match of the per-lane masks (relative position, wave-uniform), -1 if none
template <int kBytes>
__device__ __forceinline__ int first_match(uint32_t mk) {
    const uint64_t any = __ballot(mk != 0u);
    if (!any) return -1;
    const int k = __builtin_ctzll(any);
    return match_pos<kBytes>(k, lane_get(mk, k));
}
// the window bytes [lo, hi) among this lane's four (kBytes = 4 layout), 0x80 per byte
__device__ __forceinline__ uint32_t range4(int lo, int hi) {
    const int b = 4 * lane(), t = lo - b, u = hi - b;
    const uint32_t mlo = t <= 0 ? 0x80808080u : t >= 4 ? 0u : (0x80808080u << (8 * t));
    const uint32_t mhi = u >= 4 ? 0x80808080u : u <= 0 ? 0u : (0x80808080u >> (32 - 8 * u));
    return mlo & mhi;
}
// the first (up to) 9 tabs of the per-lane masks below position lim: rt[0..n), returns n
// (entries past n are unspecified).
// kBytes = 4, VCFXG_TABS_LANE (default): lane-parallel -- each lane's tab index from the four
// byte-slot ballots (v_mbcnt), its tabs' byte slots as 2-bit fields; tab r is then one ballot
// ("r falls in my range"), one s_ff1 and one v_readlane.  The scalar form walked the matches
// with a branch and an early break per tab, and the compiler copied the whole rt[] array of
// SGPRs at every exit (~40 SALU per tab: with the sweep's mask logic, 856 SALU per record in
// the pipeline walk, r05 SQ pass, against one scalar issue per CU per cycle).
#ifndef VCFXG_TABS_LANE
#define VCFXG_TABS_LANE 1
#endif
__device__ __forceinline__ uint32_t first_tabs_lane4(uint32_t tm, int lim, int (&rt)[9]) {
    tm &= range4(0, lim);
    uint32_t P = 0, t = tm;  // byte slot of this lane's j-th tab in bits [2j, 2j + 2)
#pragma unroll
    for (int j = 0; j < 3; j++) {
        P |= ((uint32_t)__builtin_ctz(t | 0x80000000u) >> 3) << (2 * j);
        t &= t - 1u;
    }
    P |= 3u << 6;  // (a fourth tab can only be in slot 3)
    const uint32_t cnt = (uint32_t)__builtin_popcount(tm);
    uint32_t excl = 0, total = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint64_t bj = __ballot((tm & (0x80u << (8 * j))) != 0u);
        excl = __builtin_amdgcn_mbcnt_hi((uint32_t)(bj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bj, excl));
        total += (uint32_t)__builtin_popcountll(bj);
    }
#pragma unroll
    for (int r = 0; r < 9; r++) {
        const uint32_t d = (uint32_t)r - excl;  // (wraps for lanes past tab r: d >= cnt)
        const uint64_t own = __ballot(d < cnt);
        const int k = (int)__builtin_ctzll(own | (1ull << 63));
        const uint32_t slot = lane_get((P >> (2 * (d & 3u))) & 3u, k);
        rt[r] = 4 * k + (int)slot;
    }
    return total < 9u ? total : 9u;
}
template <int kBytes>
__device__ __forceinline__ uint32_t first_tabs(uint32_t tm, int lim, int (&rt)[9]) {
    if constexpr (kBytes == 4 && VCFXG_TABS_LANE) return first_tabs_lane4(tm, lim, rt);
    uint64_t lanes = __ballot(tm != 0u);
    uint32_t m = 0, n = 0;
    int k = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        if (m == 0u) {
            if (lanes == 0ull) break;
            k = __builtin_ctzll(lanes);
            lanes &= lanes - 1ull;
            m = lane_get(tm, k);
        }
        const int p = match_pos<kBytes>(k, m);
        if (p >= lim) break;
        rt[r] = p;
        n = (uint32_t)r + 1u;
        m &= m - 1u;
    }
    return n;
}
// window byte o (wave-uniform) out of the kBytes = 4 layout's registers
__device__ __forceinline__ uint32_t dword_byte(uint32_t w, int o) {
    return (lane_get(w, o >> 2) >> (8 * (o & 3))) & 0xFFu;
}

// the window at A (16 B per lane) -> the wave's LDS slot by LDS-DMA: issued before the
// current record's sweep, it lands while the sweep runs (lanes past hi re-read the last
// block; those bytes are masked by the analysis)
// The window is kWin bytes (the first kWin / 16 lanes; a line head is rarely longer and the
// sweep re-reads the bytes after it from HBM anyway), or the full 1 KiB for a long head.
#ifndef VCFXG_WALK_WIN
#define VCFXG_WALK_WIN 256
#endif
constexpr int kWin = VCFXG_WALK_WIN;
__device__ __forceinline__ void prefetch_window(const char *__restrict__ buf, int64_t A, int64_t hi, uint4 *slot,
                                                int bytes = kWin) {
    if (16 * lane() >= bytes) return;
    const int b = 16 * lane(), hr = (int)std::min<int64_t>(hi - A, bytes);
    const char *src = buf + A + (b < hr ? b : ((hr - 1) & ~15));
    // inline asm, so the compiler tracks no pending write for it: with the intrinsic it
    // waited for the DMA (vmcnt(0)) before reusing the address registers inside the sweep.
    // Nothing reads the slot before read_window / slot_check wait for vmcnt(0) themselves;
    // the compiler's own counted waits only over-wait for this older load.
    const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void *)slot);
    uint32_t m0_saved;  // M0 is the DMA's LDS base; whatever the compiler kept there is restored
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(m0_saved)
                 : "v"(src), "s"(lds)
                 : "memory");
}
// the slot after its LDS-DMA landed (every earlier vector-memory op of this wave done)
__device__ __forceinline__ uint4 read_window(const uint4 *slot) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return slot[lane()];
}
// byte at relative offset o (uniform) of a landed slot
__device__ __forceinline__ uint32_t slot_byte(const uint4 *slot, int o) {
    return __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<const uint8_t *>(slot)[o]);
}

}  // namespace vcfxg
