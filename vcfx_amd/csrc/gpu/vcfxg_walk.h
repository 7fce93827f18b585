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
                const uint32_t mk = (uint32_t)__shfl((int)m, k);
                return uniform64(w + (int64_t)u * kWaveStep + 16 * k + __builtin_ctz(mk));
            }
        }
    }
    return hi;
}

// relative position of the tab with 0-based rank r (< total) given per-lane tab masks and
// their exclusive per-lane counts (wave-uniform result)
__device__ __forceinline__ int tab_at(uint32_t tm, uint32_t excl, uint32_t c, int r, int b) {
    const bool mine = (uint32_t)r >= excl && (uint32_t)r < excl + c;
    const uint64_t who = __ballot(mine);
    const int k = __builtin_ctzll(who);
    const int p = mine ? b + nth_bit(tm, r - (int)excl) : 0;
    return __builtin_amdgcn_readfirstlane(__shfl(p, k));
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
