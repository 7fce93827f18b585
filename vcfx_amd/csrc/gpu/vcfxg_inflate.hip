// vcfxg_inflate.hip -- BGZF members inflated on the device (the GPU form).
//
// The reference reads .vcf.gz through zlib (StreamingGzipReader, src/vcfx_core.cpp:144-354: one
// inflate stream, inflateReset at each gzip member).  A BGZF file is a chain of independent gzip
// members of <= 64 KiB output each, whose sizes are in their headers (BSIZE) and trailers (ISIZE),
// so the host knows every member's input span and output offset before a byte is inflated: one
// wave per member inflates it straight into the device input buffer, and the record kernels then
// run on it unchanged.  The compressed file crosses PCIe instead of the text (17x less on the
// bench shard).
//
// k_inflate (one 64-lane wave per member; the DEFLATE decode of RFC 1951 is serial per stream, so
// the wave's scalar unit decodes and its lanes do the parallel parts).  Every CU's scalar unit
// issues one instruction per cycle for all its waves, so the decode is built to spend as few
// scalar instructions per symbol as it can:
//   - the input is a 64-byte window held in one VGPR, lane i holding the 32 stream bits that start
//     at byte B + i: the next bits at bit position bp are one v_readlane + one shift (>= 25 valid
//     bits), consuming bits is one add to bp, and the window moves (one unaligned dword load per
//     lane) only when a symbol could reach past it;
//   - each block's Huffman codes (fixed, or the dynamic header's) are built by the whole wave:
//     per-length counts and each symbol's canonical rank from ballots, then lookup tables of 2^9
//     (literal/length) and 2^8 (distance) entries held in VGPRs (entry e is register e >> 6 of lane
//     e & 63: a uniform-indexed register move and a v_readlane), filled by all lanes and decoded
//     canonically; a length or distance code whose extra bits fit in the table's index carries its
//     final value, so most matches need no extra-bit reads; the rare longer codes take a per-length
//     canonical walk over LDS tables; the code-length code's table is in LDS;
//   - the output goes through an 8 KiB LDS window: a match of <= 64 bytes is one LDS read (all 64
//     lanes, the period-d pattern out[p + i] = out[p - d + i mod d] for overlapping copies) whose
//     write waits until after the next symbol's decode; a match from further back than 4 KiB reads
//     the member's own output, already in HBM;
//   - the window goes to HBM in aligned 16 B blocks as it fills (byte stores only at the member's
//     two ends, which neighbouring members share).
// Every condition under which zlib's inflate fails (zlib inflate.c / inftrees.c: invalid block
// type, stored LEN != ~NLEN, more than 286 / 30 symbols, an over-subscribed or incomplete code --
// incomplete only allowed for a single code of length 1, and never for the code-length code --,
// a bit-length repeat with nothing before it or past the end, no end-of-block code, literal /
// length symbols 286-287 and distance symbols 30-31, a distance past the member's start) marks the
// member bad; so does a stream that does not end exactly before the member's 8-byte trailer or
// whose output is not ISIZE bytes.  k_crc32 then checks each member's CRC-32 against its trailer
// (zlib's gzip check).  A bad member makes the whole ingest fail and the caller inflates on the
// host, which reproduces the reference's behaviour on a damaged stream.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "vcfxg_kernels.h"

namespace vcfxg {
namespace {

// the LDS output window: the last 8 KiB (deflate reaches back 32 KiB: a match from further back
// than kFar reads the member's own output, already written to HBM, instead)
constexpr uint32_t kWin = 1u << 13, kWinMask = kWin - 1;
constexpr uint32_t kFar = 4096;
// lookup-table bits: lit/len, distance, code lengths.  The VGPR tables are one 16-register array
// (the compiler keeps one such array in registers with uniform-indexed moves; a second array went
// to scratch): lit/len entries in registers 0-7, distance entries in 8-11, distance values in 12-15
constexpr int kLB = 9, kDB = 8, kCB = 7;
constexpr uint32_t kFlushStep = 1024;  // HBM writes in 1 KiB-aligned steps

// table entries: bits 0-4 `cons` (bits the entry consumes: the code, plus its extra bits when they
// were folded into the value), 5-8 flags, 9-13 `tot` (cons + the extra bits still to read), 16-19
// `unf` (those extra bits; with cons this is the s_bfe field of the extra value), 23-31 the value
// (literal byte, length, code-length symbol; a distance value is in the value table)
constexpr uint32_t kLit = 1u << 5, kEob = 1u << 6, kExc = 1u << 7, kBad = 1u << 8;

// RFC 1951 §3.2.5: length codes 257..285 and distance codes 0..29 (base, extra bits)
__constant__ uint16_t c_lbase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                     31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
// the order of the code-length code's lengths in a dynamic block header (RFC 1951 §3.2.7)
__constant__ uint8_t c_clorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// three codes per block: 0 literal/length (288 symbols), 1 distance (32), 2 code-length code (19)
constexpr int kLensOff[3] = {0, 288, 320};
constexpr int kNsym[3] = {288, 32, 19};
constexpr int kBits[3] = {kLB, kDB, kCB};

struct InfLds {
    uint8_t win[kWin];
    uint32_t far[80];  // a far match's source dwords (staging)
    uint32_t cl[1 << kCB];  // the code-length code's table (dynamic headers only)
    uint32_t lim[3][16];  // per code and length L: end of the length-L codes, left-justified to 15 bits
    int32_t base[3][16];  // per code and length: sorted index = base + (the code's L-bit value)
    int32_t offs[3][16];  // per code and length: first sorted index of that length
    uint16_t sorted[340];  // per code: its symbols ordered by (length, symbol)
    uint8_t lens[340];     // code lengths: lit/len [0, 288), dist [288, 320), code-length code [320, 339)
};

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// s_bfe_u32 with the entry as the field spec: the `unf` extra bits that follow the entry's `cons`
__device__ __forceinline__ uint32_t sbfe(uint32_t p, uint32_t e) {
    uint32_t r;
    asm volatile("s_bfe_u32 %0, %1, %2" : "=s"(r) : "s"(p), "s"(e) : "scc");
    return r;
}
__device__ __forceinline__ uint32_t tot_of(uint32_t e) { return (e >> 9) & 31; }

__device__ __forceinline__ uint32_t make(uint32_t cons, uint32_t unf, uint32_t v9, uint32_t flags) {
    return cons | flags | ((cons + unf) << 9) | (unf << 16) | (v9 << 23);
}

// the entry of symbol `sym` with an L-bit code; idx = the table index (stream bits, first in bit
// 0) when the entry is a table slot (the extra bits after the code are idx >> L when L + extra <=
// bits), bits = 0 for the canonical walk (no folding).  k 1: the distance value goes to `val`
__device__ __forceinline__ uint32_t make_entry(int k, uint32_t sym, uint32_t L, uint32_t idx, int bits, uint32_t &val) {
    val = 0;
    if (k == 0) {
        if (sym < 256) return make(L, 0, sym, kLit);
        if (sym == 256) return make(L, 0, 0, kEob);
        if (sym < 286) {
            const uint32_t b = c_lbase[sym - 257], ex = c_lext[sym - 257];
            if (L + ex <= (uint32_t)bits) return make(L + ex, 0, b + ((idx >> L) & ((1u << ex) - 1)), 0);
            return make(L, ex, b, 0);
        }
        return make(L, 0, 0, kExc | kBad);  // 286, 287: "invalid literal/length code"
    }
    if (k == 1) {
        if (sym >= 30) return make(L, 0, 0, kExc | kBad);  // "invalid distance code"
        const uint32_t b = c_dbase[sym], ex = c_dext[sym];
        if (L + ex <= (uint32_t)bits) {
            val = b + ((idx >> L) & ((1u << ex) - 1));
            return make(L + ex, 0, 0, 0);
        }
        val = b;
        return make(L, ex, 0, 0);
    }
    return make(L, 0, sym, 0);
}

// Builds code k from S.lens (wave-wide): the sorted symbol list, the per-length limits and the
// lookup table.  false: zlib's inflate_table would refuse the lengths (over-subscribed, or
// incomplete other than one code of length 1; the code-length code must be complete and non-empty).
// k 0: the table goes to registers 0-7 of lut; k 1: entries to 8-11, values to 12-15; k 2: to S.cl
template <int K>
__device__ bool build_code(InfLds &S, uint32_t (&lut)[16]) {
    const int lane = threadIdx.x;
    constexpr int nsym = kNsym[K], bits = kBits[K];
    const uint8_t *lens = S.lens + kLensOff[K];
    uint32_t cnt[16];
#pragma unroll
    for (int L = 0; L < 16; L++) cnt[L] = 0;
    int rk[5], ln[5];
#pragma unroll
    for (int ch = 0; ch < 5; ch++) {
        rk[ch] = 0;
        ln[ch] = 0;
        if (ch * 64 >= nsym) continue;
        const int s = ch * 64 + lane;
        const int l = s < nsym ? lens[s] : 0;
        int r = 0;
#pragma unroll
        for (int L = 1; L < 16; L++) {
            const uint64_t m = __ballot(l == L);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
            if (l == L) r = (int)(cnt[L] + below);
            cnt[L] += (uint32_t)__popcll(m);
        }
        rk[ch] = r;
        ln[ch] = l;
    }
    int left = 1, maxl = 0;
    bool over = false;
#pragma unroll
    for (int L = 1; L < 16; L++) {
        left = 2 * left - (int)cnt[L];
        over = over || left < 0;
        if (cnt[L]) maxl = L;
    }
    if (over) return false;
    if (K == 2 && (maxl == 0 || left > 0)) return false;
    if (maxl > 1 && left > 0) return false;
    // canonical first codes (RFC 1951 §3.2.2), limits, offsets
    uint32_t first = 0, o = 0;
    uint32_t limv[16];
    if (lane < 16) {
        S.lim[K][lane] = 0;
        S.base[K][lane] = 0;
        S.offs[K][lane] = 0;
    }
    limv[0] = 0;
#pragma unroll
    for (int L = 1; L < 16; L++) {
        first = (first + cnt[L - 1]) << 1;
        if (L == 1) first = 0;
        limv[L] = (first + cnt[L]) << (15 - L);
        if (lane == L) {
            S.lim[K][L] = limv[L];
            S.base[K][L] = (int32_t)o - (int32_t)first;
            S.offs[K][L] = (int32_t)o;
        }
        o += cnt[L];
    }
    __syncthreads();
#pragma unroll
    for (int ch = 0; ch < 5; ch++) {
        if (ch * 64 >= nsym) continue;
        if (ln[ch] > 0) S.sorted[kLensOff[K] + S.offs[K][ln[ch]] + rk[ch]] = (uint16_t)(ch * 64 + lane);
    }
    __syncthreads();
    // the lookup table: entry e = the next `bits` stream bits (first bit in bit 0) is register
    // e >> 6 of lane e & 63 (a lookup is a uniform-indexed register move + readlane)
    constexpr int NR = (1 << bits) / 64;
#pragma unroll
    for (int r = 0; r < NR; r++) {
        const uint32_t e = 64 * r + lane;
        const uint32_t rev = __brev(e) >> (32 - bits);  // the bits MSB-first (code order)
        int Lf = 0;
#pragma unroll
        for (int L = 1; L < 16; L++)
            if (L <= bits && Lf == 0 && rev < (limv[L] >> (15 - bits))) Lf = L;
        uint32_t ent, val = 0;
        if (Lf == 0) {
            ent = maxl > bits ? kExc : (kExc | kBad);  // a longer code, or none (incomplete code / empty)
        } else {
            const int idx = S.base[K][Lf] + (int)(rev >> (bits - Lf));
            ent = make_entry(K, S.sorted[kLensOff[K] + idx], (uint32_t)Lf, e, bits, val);
        }
        if (K == 2) S.cl[e] = ent;
        else if (K == 0) lut[r] = ent;
        else {
            lut[8 + r] = ent;
            lut[12 + r] = val;
        }
    }
    __syncthreads();
    return true;
}

// a code longer than the table's bits: the canonical walk over lengths bits+1 .. 15 (p: the next
// >= 15 stream bits); the entry carries the code's length as cons and its extra bits as unf
__device__ __forceinline__ uint32_t slow_decode(InfLds &S, int k, uint32_t p, uint32_t &val) {
    const uint32_t rev = __brev(p) >> 17;  // next 15 bits, code order
    for (int L = kBits[k] + 1; L < 16; L++) {
        if (rev < S.lim[k][L]) {
            const int idx = S.base[k][L] + (int)(rev >> (15 - L));
            return make_entry(k, S.sorted[kLensOff[k] + idx], (uint32_t)L, 0, 0, val);
        }
    }
    val = 0;
    return kExc | kBad;
}

// the lane decoder's verdict for a member it hands to the wave decoder (mstat)
constexpr uint32_t kDefer = 0xFFFFu;
// the lane decoder's token count of a member it hands over
constexpr uint32_t kTokNone = 0xFFFFFFFFu;

// One member inflated by the whole wave (the wave decoder): every member the lane decoder below
// hands over (kDefer), which includes every member that zlib would refuse.
__device__ __forceinline__ void inflate_wave(InfLds &S, const uint8_t *__restrict__ comp, const BgzfMember *__restrict__ mem,
                                             const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                             uint32_t *__restrict__ mstat, unsigned long long *__restrict__ first_bad,
                                             uint64_t mbase, const uint32_t m) {
    const int lane = threadIdx.x;
    const BgzfMember M = mem[m];
    const uint64_t src = M.src_off;
    const uint32_t olen = M.out_len;
    uint32_t why = 0;  // 0 ok, else the first failing check (diagnostic)
    // gzip header: 10 bytes + XLEN + the extra field (the host checked FLG == FEXTRA)
    // (byte loads land in VGPRs: readfirstlane keeps every offset derived from them -- the whole
    // reader state -- in scalar registers and the decode loop in scalar branches)
    const uint32_t xlen = uni((uint32_t)comp[src + 10] | ((uint32_t)comp[src + 11] << 8));
    const uint64_t pay0 = src + 12 + xlen;
    const uint64_t pend = src + M.src_len - 8;  // the deflate stream ends where the trailer starts
    uint8_t *const dst = out + out_off[m];
    const uint64_t A = (uint64_t)(uintptr_t)dst;  // absolute output address of byte 0
    const uint64_t Ab = A & ~15ull;               // the window holds byte p at (A - Ab + p) & mask
    const uint32_t ph = (uint32_t)(A - Ab);
    // output position x = ph + the member's byte index; xend = ph + ISIZE
    uint32_t x = ph;
    const uint32_t xend = ph + olen;
    uint32_t fl = ph;  // output written to HBM up to x = fl
    uint32_t fnext = (ph & ~(kFlushStep - 1)) + 2 * kFlushStep;  // flush when x reaches this
    if (pay0 + 2 > pend || olen > 65536) why = 1;
    // the bit reader: stream bytes relative to gb; lane i of pk holds the dword at byte B + i (past
    // plen_end + 2 KiB it holds zeros, so loads stay within the buffer's pad; a stream that runs
    // past its end is caught at its block's end, and every loop ends since each symbol consumes
    // bits and adds output or ends its block)
    const uint64_t gb = pay0;
    const uint32_t plen_end = (uint32_t)(pend - gb);  // stream end, relative to gb
    uint32_t bp = 0, B = 0;
    uint32_t pk = 0;
    auto advance = [&]() {  // the window to start at the byte holding bit bp
        B = bp >> 3;
        uint32_t v = 0;
        if (B + (uint32_t)lane < plen_end + 2048) __builtin_memcpy(&v, comp + gb + B + lane, 4);
        pk = v;
    };
    auto peek = [&]() -> uint32_t {  // >= 25 valid stream bits from bp (the window must hold them)
        return (uint32_t)__builtin_amdgcn_readlane((int)pk, (int)((bp >> 3) - B)) >> (bp & 7);
    };
    auto room = [&]() {  // the window holds >= 6 more bytes past bp's byte (a whole match)
        if ((bp >> 3) - B > 57) advance();
    };
    auto getb = [&](uint32_t n) -> uint32_t {  // n <= 16 bits
        room();
        const uint32_t v = peek() & ((1u << n) - 1);
        bp += n;
        return v;
    };
    auto consumed_bytes = [&]() -> uint32_t { return (bp + 7) >> 3; };  // (a partial byte counts)
    if (!why) advance();
    // the window up to x = `to` goes to HBM: the member's first partial 16 B block (shared with the
    // previous member) by byte stores, aligned 16 B blocks from LDS, the last partial block only
    // when `fin`
    uint8_t *const gout = dst - ph;  // (from the kernel argument: global, not flat, accesses)
    // The pending write: the bytes of the last literal or match of <= 64 bytes, read into pv (a byte
    // per lane) and written at x0 + lane only after the next symbol's decode, whose table lookups
    // need no LDS, hides the read's latency.  All 64 lanes write: the lanes past the symbol's length
    // write bytes ahead of the output, which later symbols overwrite before anything reads or
    // flushes them (and which land on window slots that are flushed and out of match reach).  Every
    // window access commits the pending write first, so the window sees the writes in stream order.
    uint32_t pv = 0, pa = 0;  // pending byte and window slot (per lane)
    auto commit = [&]() { S.win[pa] = (uint8_t)pv; };
    pa = (x + lane) & kWinMask;
    pv = 0;  // (the first commit writes zeros ahead of the output)
    auto flush = [&](uint32_t to, bool fin) {
        if (to <= fl) return;
        uint32_t a = fl;
        const uint32_t a16 = (a + 15) & ~15u;
        if (a != a16) {
            const uint32_t e = a16 < to ? a16 : to;
            if ((uint32_t)lane < e - a) gout[a + lane] = S.win[(a + lane) & kWinMask];
            a = e;
        }
        const uint32_t b16 = to & ~15u;
        for (uint32_t y = a + 16 * lane; y + 16 <= b16; y += 16 * 64)
            *reinterpret_cast<uint4 *>(gout + y) = *reinterpret_cast<const uint4 *>(S.win + (y & kWinMask));
        if (fin && b16 >= a && to > b16)
            if ((uint32_t)lane < to - b16) gout[b16 + lane] = S.win[(b16 + lane) & kWinMask];
        fl = fin ? to : (b16 > a ? b16 : a);
        fnext = (fl & ~(kFlushStep - 1)) + 2 * kFlushStep;
    };
    auto maybe_flush = [&]() {
        if (x >= fnext) {
            commit();
            flush(x & ~(kFlushStep - 1), false);
        }
    };
    uint32_t lut[16];  // lit/len entries in registers 0-7, distance entries 8-11, distance values 12-15
    auto lookL = [&](uint32_t p) -> uint32_t {  // entry p & 511 (readlane takes the lane as p & 63)
        return (uint32_t)__builtin_amdgcn_readlane((int)lut[(p >> 6) & 7], (int)(p & 63));
    };
    auto lookD = [&](uint32_t p, uint32_t &val) -> uint32_t {
        const uint32_t r = (p >> 6) & 3;
        val = (uint32_t)__builtin_amdgcn_readlane((int)lut[12 + r], (int)(p & 63));
        return (uint32_t)__builtin_amdgcn_readlane((int)lut[8 + r], (int)(p & 63));
    };
    const float lanef = (float)lane + 0.5f;
    bool fixed_built = false;
    bool last = false;
    // (the decoder state is wave-uniform and lives in scalar registers: the code builder's verdict
    // is readfirstlane'd -- the compiler cannot see it is uniform, and one divergent `why` made the
    // whole decode loop run on exec masks and VGPR copies of its state, 2.5x the instructions)
    while (!why && !last) {
        last = getb(1) != 0;
        const uint32_t bt = getb(2);
        commit();
        if (bt == 0) {  // stored block: to a byte boundary, LEN, NLEN, LEN raw bytes
            bp = (bp + 7) & ~7u;
            const uint32_t ln = getb(16);
            const uint32_t nl = getb(16);
            if (ln != (~nl & 0xFFFFu)) {
                why = 2;
                break;
            }
            const uint32_t q = bp >> 3;  // the next stream byte (relative to gb)
            if ((uint64_t)q + ln > plen_end) {
                why = 3;
                break;
            }
            if (x + ln > xend) {
                why = 4;
                break;
            }
            for (uint32_t c = 0; c < ln; c += 1024) {  // through the window, 1 KiB at a time
                const uint32_t take = ln - c < 1024 ? ln - c : 1024;
                for (uint32_t i = lane; i < take; i += 64) S.win[(x + i) & kWinMask] = comp[gb + q + c + i];
                __syncthreads();
                x += take;
                pa = (x + lane) & kWinMask;  // (the next commit writes ahead of the output)
                maybe_flush();
            }
            bp = (q + ln) * 8;
            advance();
            continue;
        }
        if (bt == 3) {
            why = 5;
            break;
        }
        if (bt == 1) {  // fixed codes (RFC 1951 §3.2.6)
            if (!fixed_built) {
                for (int s = lane; s < 320; s += 64) S.lens[s] = s < 144 ? 8 : (s < 256 ? 9 : (s < 280 ? 7 : (s < 288 ? 8 : 5)));
                __syncthreads();
                build_code<0>(S, lut);
                build_code<1>(S, lut);
                fixed_built = true;
            }
        } else {  // dynamic: HLIT, HDIST, HCLEN, the code-length code, then the two codes' lengths
            fixed_built = false;
            const uint32_t nlen = getb(5) + 257, ndist = getb(5) + 1, ncl = getb(4) + 4;
            if (nlen > 286 || ndist > 30) {
                why = 6;
                break;
            }
            for (int s = lane; s < 340; s += 64) S.lens[s] = 0;
            __syncthreads();
            for (uint32_t i = 0; i < ncl; i++) {
                const uint32_t v = getb(3);
                if (lane == 0) S.lens[320 + c_clorder[i]] = (uint8_t)v;
            }
            __syncthreads();
            if (!uni((uint32_t)build_code<2>(S, lut))) {
                why = 7;
                break;
            }
            const uint32_t tot = nlen + ndist;
            uint32_t n = 0, prev = 0;
            while (n < tot) {
                room();
                const uint32_t p = peek();
                const uint32_t e = uni(S.cl[p & ((1u << kCB) - 1)]);
                if (e & kExc) {
                    why = 8;
                    break;
                }
                bp += e & 31;
                const uint32_t sym = e >> 23;
                uint32_t rep = 1, val = sym;
                if (sym == 16) {
                    if (n == 0) {
                        why = 9;
                        break;
                    }
                    rep = 3 + getb(2);
                    val = prev;
                } else if (sym == 17) {
                    rep = 3 + getb(3);
                    val = 0;
                } else if (sym == 18) {
                    rep = 11 + getb(7);
                    val = 0;
                }
                if (n + rep > tot) {
                    why = 9;
                    break;
                }
                for (uint32_t i = lane; i < rep; i += 64) {
                    const uint32_t at = n + i;
                    S.lens[at < nlen ? at : 288 + (at - nlen)] = (uint8_t)val;
                }
                n += rep;
                prev = val;
            }
            if (why) break;
            __syncthreads();
            if (uni(S.lens[256]) == 0) {  // "invalid code -- missing end-of-block"
                why = 10;
                break;
            }
            if (!uni((uint32_t)build_code<0>(S, lut))) {
                why = 11;
                break;
            }
            if (!uni((uint32_t)build_code<1>(S, lut))) {
                why = 12;
                break;
            }
        }
        // the block's symbols
        for (;;) {
            room();
            uint32_t p = peek();
            uint32_t e = lookL(p);
            if (e & (kLit | kEob | kExc)) {
                if (e & kExc) {
                    if (e & kBad) {
                        why = 13;
                        break;
                    }
                    uint32_t unused;
                    e = uni(slow_decode(S, 0, p, unused));
                    if (e & kBad) {
                        why = 13;
                        break;
                    }
                }
                if (e & kLit) {
                    if (x >= xend) {
                        why = 14;
                        break;
                    }
                    commit();
                    pv = e >> 23;
                    pa = (x + lane) & kWinMask;
                    x++;
                    bp += tot_of(e);
                    maybe_flush();
                    continue;
                }
                if (e & kEob) {
                    bp += tot_of(e);
                    commit();
                    break;
                }
            }
            const uint32_t len = (e >> 23) + sbfe(p, e);
            bp += tot_of(e);
            p = peek();
            uint32_t dv;
            uint32_t d = lookD(p, dv);
            uint32_t dist;
            if (d & kExc) {
                if (d & kBad) {
                    why = 15;
                    break;
                }
                d = uni(slow_decode(S, 1, p, dv));
                if (d & kBad) {
                    why = 15;
                    break;
                }
                dv = uni(dv);
                bp += d & 31;  // the code, then its extra bits from a fresh peek (they may be 13)
                dist = dv + (peek() & ((1u << ((d >> 16) & 15)) - 1));
                bp += (d >> 16) & 15;
            } else {
                dist = dv + sbfe(p, d);
                bp += tot_of(d);
            }
            if (dist > x - ph) {  // "invalid distance too far back"
                why = 16;
                break;
            }
            if (x + len > xend) {
                why = 14;
                break;
            }
            commit();  // (this match may read the previous symbol's bytes)
            if (dist > kFar) {
                // further back than the window keeps: the member's own output, already in HBM (x - fl
                // stays below 3.3 KiB between flushes, so every source byte went out earlier).  Every
                // store of this wave has completed (s_waitcnt 0); the dwords are read at agent scope
                // (from L2, never an older L1 line), staged in LDS, then placed bytewise.
                __builtin_amdgcn_s_waitcnt(0);
                const uint32_t sx = x - dist, s4 = sx & ~3u, nb = len + (sx - s4);
                uint32_t *const src32 = reinterpret_cast<uint32_t *>(gout + s4);
                for (uint32_t k = lane; 4 * k < nb; k += 64)
                    S.far[k] = __hip_atomic_load(src32 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __syncthreads();
                const uint8_t *far8 = reinterpret_cast<const uint8_t *>(S.far) + (sx - s4);
                for (uint32_t i = lane; i < len; i += 64) S.win[(x + i) & kWinMask] = far8[i];
                __syncthreads();
                x += len;
                pa = (x + lane) & kWinMask;
                pv = 0;
                maybe_flush();
                continue;
            }
            // source byte of output byte i: sbase + (i mod dist) (the period-dist pattern, which is
            // also the plain copy when dist > i); (i + 0.5) / dist through an approximate reciprocal
            // stays within 0.5 / dist of the exact quotient's distance to an integer, so the floor
            // is exact for i < 258 and dist <= 4096
            const float rd = __builtin_amdgcn_rcpf((float)dist);
            const uint32_t sbase = x - dist;
            const uint32_t q0 = (uint32_t)(lanef * rd);
            const uint32_t s0 = (sbase + (uint32_t)lane - q0 * dist) & kWinMask;
            if (len <= 64) {  // read now, written after the next symbol's decode
                pv = S.win[s0];
                pa = (x + lane) & kWinMask;
            } else {
                for (uint32_t c = 0; c < len; c += 64) {
                    const uint32_t i = c + lane;
                    const uint32_t q = (uint32_t)(((float)c + lanef) * rd);
                    const uint8_t v = S.win[(sbase + i - q * dist) & kWinMask];
                    if (i < len) S.win[(x + i) & kWinMask] = v;
                }
                pa = (x + len + lane) & kWinMask;
                pv = 0;
            }
            x += len;
            maybe_flush();
        }
        if (!why && consumed_bytes() > plen_end) why = 17;  // (a block ran into the trailer)
    }
    if (!why && (uint64_t)consumed_bytes() != plen_end) why = 18;  // the trailer follows the stream
    if (!why && x != xend) why = 19;                                 // ISIZE
    if (!why) {
        commit();
        __syncthreads();
        flush(x, true);
    }
    if (lane == 0) {
        mstat[m] = why;
        if (why) atomicMin(first_bad, (unsigned long long)(mbase + m));
    }
}

// The members the lane decoder handed over (2.6 in 10,000 on the bench shard: a code whose tables
// pass the lane's slice, a stored or fixed block, damage): the wave decoder, one member per wave,
// from the list the lane decoder appends them to (hlist[0] their count, then their token slots),
// on a second stream beside the copy, its waves at raised priority.  (A scan of the token slots
// for them, one wave per 256 slots, serialised the members that sort together: 15 ms.)
constexpr uint32_t kHandGrid = 256;
__global__ void __launch_bounds__(64) k_inflate_handover(const uint8_t *__restrict__ comp, const BgzfMember *__restrict__ mem,
                                                         const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                         uint32_t *__restrict__ mstat, unsigned long long *__restrict__ first_bad,
                                                         uint64_t mbase, const uint32_t *__restrict__ perm,
                                                         const uint32_t *__restrict__ hlist) {
    __shared__ InfLds S;
    __builtin_amdgcn_s_setprio(3);
    const uint32_t cnt = uni(hlist[0]);
    for (uint32_t k = blockIdx.x; k < cnt; k += gridDim.x) {
        __syncthreads();  // (the previous member's last reads of S)
        inflate_wave(S, comp, mem, out_off, out, mstat, first_bad, mbase, uni(perm[uni(hlist[1 + k])]));
    }
}

// the wave decoder over every member, one per wave (VCFX_INFLATE_LANES=0: the A/B baseline)
__global__ void __launch_bounds__(64) k_inflate(const uint8_t *__restrict__ comp, const BgzfMember *__restrict__ mem,
                                                const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                uint32_t *__restrict__ mstat, unsigned long long *__restrict__ first_bad,
                                                uint64_t mbase) {
    __shared__ InfLds S;
    inflate_wave(S, comp, mem, out_off, out, mstat, first_bad, mbase, blockIdx.x);
}

// ---- the lane decoder: one member per lane -------------------------------------------------------
// The wave decoder above decodes on the CU's one scalar unit: on the bench shard (65,834 members of
// level-1 bgzip output, each ~2,200 symbols, mostly matches of ~35 B) it spends ~23 ms.  The
// Huffman decode moves to the vector lanes, one member per lane, and the copy keeps the wave:
//   k_inflate_decode: the Huffman decode of a member per lane, to a token list per member (a
//     literal byte, or a match's length and distance: 4 B each, in a per-launch token buffer).  The
//     tables live in the lane's own 848-byte slice of LDS (three waves per CU): a 2^7-entry
//     literal/length root table and a 2^6-entry distance root table of 16-bit entries (fewer root
//     bits when the tables would not fit), with zlib's
//     sub-tables (inftrees.c: a root entry points to a table indexed by the bits past the root) for
//     longer codes, built per lane from the code lengths (which the header decode writes into the
//     token slot's spare tail).  The stream comes through a 64-byte LDS window per lane: a symbol's
//     64 bits are one ds_read2 + ds_read and two funnel shifts.  The window is reloaded once per
//     trip of four symbols from registers loaded a whole trip ahead, and every trip makes the same
//     loads and one 16-byte token store whatever its lanes decoded: the vector-memory counter is
//     per wave and in order, so a load one lane needs now must not sit behind loads other lanes
//     issued just before.  The lanes of a wave take members of similar compressed size (the host
//     orders them, largest first): a wave runs as long as its longest member.
//   k_inflate_copy (below): the LZ77 copy of a member's tokens per wave.
// Only what zlib accepts is accepted: dynamic-Huffman blocks whose codes are complete (no
// over-subscribed or incomplete code, an end-of-block code), repeats within bounds, no distance
// past the member's start, output exactly ISIZE and a stream ending exactly at the trailer.
// Everything else -- stored and fixed blocks, the single-code and empty distance codes zlib allows,
// tables past the slice, members over the token capacity, and every damaged stream -- is handed to
// the wave decoder (mstat kDefer), which decides it exactly as before.  k_crc32 then checks every
// member.
constexpr int kLT = 424;         // 16-bit table entries per lane (848 B: 3 waves per CU in 160 KiB)
constexpr int kCtr = kLT - 32;   // the builder's 16 32-bit counters at the slice's tail
// the copy's window (k_inflate_copy): 8 KiB of LDS per wave; a match from further back than
// kCReach, or longer than 64 bytes, takes its slow path
constexpr uint32_t kCW = 8192, kCWMask = kCW - 1;
constexpr uint32_t kCReach = kCW - 258;
constexpr uint32_t kCFlush = 1024;  // the window goes out in 1 KiB steps
// a token: bits 16-24 its length (a literal: 1), bits 0-14 a match's distance - 1 (a literal: its
// byte), bit 15 the copy's slow path, bit 25 a literal
constexpr uint32_t kTLit = 1u << 25, kTSlow = 1u << 15;

// entries: bits 0-3 the code length, 4-12 the value (literal byte, length symbol - 257, distance
// symbol, code-length symbol), 14-15 the kind; a root entry of kind kKPtr holds its sub-table's
// offset in the slice (bits 0-8) and index bits (9-12)
constexpr uint32_t kKLit = 0, kKLen = 1, kKPtr = 2, kKEob = 3;

__device__ __forceinline__ uint32_t brev_n(uint32_t c, uint32_t n) { return __brev(c) >> (32 - n); }
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_inflate_decode(const uint8_t *__restrict__ comp, const BgzfMember *__restrict__ mem, const uint64_t *__restrict__ out_off,
                 uint8_t *__restrict__ out, uint32_t *__restrict__ mstat, uint32_t *__restrict__ ndefer,
                 uint32_t *__restrict__ tok, uint32_t tok_cap, const uint32_t *__restrict__ perm, uint32_t n_lanes,
                 uint32_t *__restrict__ hlist) {
    __shared__ __attribute__((aligned(16))) uint16_t T[64 * kLT];
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x * 64 + lane;  // the lane's slot; its member perm[i]
    if (i >= n_lanes) return;  // (no barrier below: lanes never share LDS)
    const uint32_t m = perm[i];
    const uint32_t lt = lane * kLT;
    // the slice's last 64 bytes: the builder's counters, and otherwise the stream window
    uint32_t *const C = reinterpret_cast<uint32_t *>(&T[lt + kCtr]);
    uint32_t *const Wd = C;
    uint32_t *const tk = tok + (size_t)i * tok_cap;  // [0] the count, then the tokens
    const BgzfMember M = mem[m];
    const uint32_t olen = M.out_len;
    // the code lengths' scratch: the token slot's last 512 bytes (past every token)
    uint8_t *const lp = reinterpret_cast<uint8_t *>(tk + tok_cap - 128);
    const uint8_t *const cp = comp + M.src_off;
    const uint32_t xlen = (uint32_t)cp[10] | ((uint32_t)cp[11] << 8);
    const int64_t plen = (int64_t)M.src_len - 8 - 12 - (int64_t)xlen;  // the deflate stream's bytes
    if (plen < 2 || olen > 65536) {
        tk[0] = kTokNone;
        mstat[m] = kDefer;
        hlist[1 + atomicAdd(hlist, 1u)] = i;
        atomicAdd(ndefer, 1u);
        atomicAdd(ndefer + 1, 1u);
        return;
    }
    bool bad = false;
    uint32_t why = 0;  // the first refusal (a diagnostic: ndefer[1 + why - 1] counts them)
    // The bit reader: bpos = the next stream bit, counted from qp (the stream's first byte rounded
    // down to a dword; the first sh bits are not the stream's).  The window holds stream dwords
    // [wb, wb + 16) in LDS: a symbol's 64 bits are one ds_read2 + ds_read and two funnel shifts.
    const uint32_t a3 = (uint32_t)((uintptr_t)(cp + 12 + xlen) & 3);
    const uint32_t *const qp = reinterpret_cast<const uint32_t *>(cp + 12 + xlen - a3);  // (global: no int casts)
    const uint32_t sh = a3 * 8;
    const uint32_t bend = (uint32_t)(plen * 8) + sh;  // the stream's end bit
    uint32_t bpos = sh, wb = 0;
    uint4 N0, N1, N2, N3;  // the next trip's window, loaded a trip ahead (from dword nbase)
    uint32_t nbase = 0;
    auto qdw = [&]() -> uint32_t {  // the dword a window load starts at (a stream run past its end stops)
        return bad ? 0u : (bpos >> 5);
    };
    auto read64 = [&](uint32_t &lo, uint32_t &hi) {
        const uint32_t k = (bpos >> 5) - wb;
        const uint32_t d0 = Wd[k], d1 = Wd[k + 1], d2 = Wd[k + 2];
        lo = __builtin_amdgcn_alignbit(d1, d0, bpos & 31);
        hi = __builtin_amdgcn_alignbit(d2, d1, bpos & 31);
    };
    auto put_window = [&](const uint4 &a, const uint4 &b, const uint4 &c, const uint4 &d, uint32_t base) {
        reinterpret_cast<uint4 *>(Wd)[0] = a;
        reinterpret_cast<uint4 *>(Wd)[1] = b;
        reinterpret_cast<uint4 *>(Wd)[2] = c;
        reinterpret_cast<uint4 *>(Wd)[3] = d;
        wb = base;
    };
    auto sync_window = [&]() {  // the window from the current dword, now (block headers)
        const uint32_t q = qdw();
        const uint4 *p = reinterpret_cast<const uint4 *>(qp + q);
        put_window(p[0], p[1], p[2], p[3], q);
    };
    auto hread = [&](uint32_t &lo, uint32_t &hi) {  // a header's read: the window moved when needed
        if ((bpos >> 5) - wb > 13) sync_window();
        read64(lo, hi);
    };

    // Builds the code of `nsym` lengths at lens (bytes) into the slice at `base` with `R` root
    // bits; kind 0 literal/length, 1 distance or code-length.  Returns the entries used, or -1: a
    // code zlib refuses or allows only as a special case (incomplete, over-subscribed, empty), or
    // one whose tables pass the counters.  (The counters overwrite the stream window.)
    auto build = [&](uint32_t base, const uint8_t *lens, uint32_t nsym, uint32_t R, int kind) -> int {
#pragma unroll
        for (int L = 0; L < 16; L++) C[L] = 0;
        uint4 v = make_uint4(0, 0, 0, 0);
        for (uint32_t s = 0; s < nsym; s++) {
            if ((s & 15) == 0) v = ld16(lens + s);
            atomicAdd(&C[v.x & 15], 1u);
            v.x = __builtin_amdgcn_alignbit(v.y, v.x, 8);
            v.y = __builtin_amdgcn_alignbit(v.z, v.y, 8);
            v.z = __builtin_amdgcn_alignbit(v.w, v.z, 8);
            v.w >>= 8;
        }
        uint32_t cnt[16];
#pragma unroll
        for (int L = 0; L < 16; L++) cnt[L] = C[L];
        cnt[0] = 0;
        int left = 1;
        uint32_t maxl = 0;
        bool over = false;
#pragma unroll
        for (int L = 1; L < 16; L++) {
            left = 2 * left - (int)cnt[L];
            over = over || left < 0;
            if (cnt[L]) maxl = L;
        }
        if (over || left != 0) return -1;
        uint32_t first[16];
        uint32_t code = 0;
        first[0] = 0;
#pragma unroll
        for (int L = 1; L < 16; L++) {
            code = (code + cnt[L - 1]) << 1;
            first[L] = code;
        }
        uint32_t size = 1u << R;
        if (base + size > (uint32_t)kCtr) return -2;
        if (maxl > R) {
            // zlib's sub-tables, from the counts alone: the long codes in canonical order fill one
            // root prefix after another; a prefix's table has the fewest index bits its codes fill
            // (inftrees.c "determine length of next table"); C holds the counts not yet placed
            uint32_t p = 0;
#pragma unroll
            for (int L = 1; L < 16; L++)
                if ((uint32_t)L == R) p = first[L] + cnt[L];  // the first prefix of a long code
            uint32_t len = R + 1;
            while (C[len] == 0) len++;
            while (len <= maxl) {
                uint32_t curr = len - R;
                int lf = 1 << curr;
                while (curr + R < maxl) {
                    lf -= (int)C[curr + R];
                    if (lf <= 0) break;
                    curr++;
                    lf <<= 1;
                }
                if (p >= (1u << R)) return -1;
                if (base + size + (1u << curr) > (uint32_t)kCtr) return -2;
                T[lt + base + brev_n(p, R)] = (uint16_t)((base + size) | (curr << 9) | (kKPtr << 14));
                size += 1u << curr;
                uint32_t space = 1u << curr;
                while (space) {
                    const uint32_t s2 = R + curr - len;
                    const uint32_t r = C[len], k = min(r, space >> s2);
                    C[len] = r - k;
                    space -= k << s2;
                    if (r == k) {
                        do len++;
                        while (len <= maxl && C[len] == 0);
                        if (len > maxl) break;
                    }
                }
                p++;
            }
        }
#pragma unroll
        for (int L = 0; L < 16; L++) C[L] = first[L];
        for (uint32_t s = 0; s < nsym; s++) {
            if ((s & 15) == 0) v = ld16(lens + s);
            const uint32_t L = v.x & 15;
            v.x = __builtin_amdgcn_alignbit(v.y, v.x, 8);
            v.y = __builtin_amdgcn_alignbit(v.z, v.y, 8);
            v.z = __builtin_amdgcn_alignbit(v.w, v.z, 8);
            v.w >>= 8;
            if (!L) continue;
            const uint32_t c = atomicAdd(&C[L], 1u);
            uint32_t e;
            if (kind == 0)
                e = s < 256 ? (L | (s << 4)) : (s == 256 ? (L | (kKEob << 14)) : (L | ((s - 257) << 4) | (kKLen << 14)));
            else
                e = L | (s << 4);
            if (L <= R) {
                for (uint32_t i = brev_n(c, L); i < (1u << R); i += 1u << L) T[lt + base + i] = (uint16_t)e;
            } else {
                const uint32_t pe = T[lt + base + brev_n(c >> (L - R), R)];
                const uint32_t so = pe & 511, cb = (pe >> 9) & 15;
                for (uint32_t i = brev_n(c & ((1u << (L - R)) - 1), L - R); i < (1u << cb); i += 1u << (L - R))
                    T[lt + so + i] = (uint16_t)e;
            }
        }
        return (int)size;
    };
    // a lookup: the root entry of the next R bits, or its sub-table's entry
    auto look = [&](uint32_t tb, uint32_t R, uint32_t bits) -> uint32_t {
        uint32_t e = T[lt + tb + (bits & ((1u << R) - 1))];
        if ((e >> 14) == kKPtr) e = T[lt + (e & 511) + ((bits >> R) & ((1u << ((e >> 9) & 15)) - 1))];
        return e;
    };

    uint32_t xd = 0;      // output bytes decoded so far
    uint32_t st = 0;      // 0 block header next, 1 in a block, 2 after the last block
    bool last = false;
    uint32_t dbase = 0;   // the distance table's offset in the slice
    constexpr uint32_t kLR = 7, kDR = 6;  // the root bits of the two tables
    // A block header: the code lengths into lp (the code-length code's at lp[320, 339)), then the
    // tables; the window follows the reads.  Any refusal sets bad.
    auto header = [&]() {
        sync_window();
        uint32_t lo, hi;
        hread(lo, hi);
        last = lo & 1;
        const uint32_t bt = (lo >> 1) & 3;
        if (bt != 2) {
            bad = true, why = why ? why : 2u;
            return;
        }
        const uint32_t nlen = ((lo >> 3) & 31) + 257, ndist = ((lo >> 8) & 31) + 1, ncl = ((lo >> 13) & 15) + 4;
        bpos += 17;
        if (nlen > 286 || ndist > 30) {
            bad = true, why = why ? why : 3u;
            return;
        }
        const uint4 z = make_uint4(0, 0, 0, 0);
        __builtin_memcpy(lp + 320, &z, 16);
        __builtin_memcpy(lp + 336, &z, 16);
        hread(lo, hi);  // (at most 19 x 3 = 57 bits: one read)
        const uint64_t cl = (uint64_t)hi << 32 | lo;
        for (uint32_t i = 0; i < ncl; i++) lp[320 + c_clorder[i]] = (uint8_t)((cl >> (3 * i)) & 7);
        bpos += 3 * ncl;
        if (bad || build(0, lp + 320, 19, 7, 1) < 0) {
            bad = true, why = why ? why : 4u;
            return;
        }
        sync_window();  // (the counters took the window's place)
        const uint32_t tot = nlen + ndist;
        uint32_t n = 0, prev = 0;
        while (!bad && n < tot) {
            hread(lo, hi);
            const uint32_t e = look(0, 7, lo);
            const uint32_t L = e & 15, sym = (e >> 4) & 31;
            if (sym < 16) {
                bpos += L;
                lp[n++] = (uint8_t)sym;
                prev = sym;
                continue;
            }
            uint32_t rep, val = 0;
            if (sym == 16) {
                rep = 3 + __builtin_amdgcn_ubfe(lo, L, 2);
                bpos += L + 2;
                val = prev;
                if (n == 0) bad = true, why = why ? why : 5u;
            } else if (sym == 17) {
                rep = 3 + __builtin_amdgcn_ubfe(lo, L, 3);
                bpos += L + 3;
            } else {
                rep = 11 + __builtin_amdgcn_ubfe(lo, L, 7);
                bpos += L + 7;
            }
            if (n + rep > tot) bad = true, why = why ? why : 5u;
            if (bad) break;
            for (uint32_t i = 0; i < rep; i++) lp[n + i] = (uint8_t)val;
            n += rep;
            prev = val;
        }
        if (bad || lp[256] == 0) {  // (no end-of-block code)
            bad = true, why = why ? why : 6u;
            return;
        }
        // (one loop for the two codes: one copy of the builder in the code)
        int used = 0;
#pragma nounroll
        for (int j = 0; j < 2 && used >= 0; j++) {
            const int r = build(j ? (uint32_t)used : 0u, j ? lp + nlen : lp, j ? ndist : nlen, j ? kDR : kLR, j);
            if (j == 0) dbase = (uint32_t)r;
            used = r;
        }
        if (used < 0) bad = true, why = why ? why : 7u;
        st = 1;
        // the window from here, and the next trip's from here too
        sync_window();
        N0 = reinterpret_cast<uint4 *>(Wd)[0];
        N1 = reinterpret_cast<uint4 *>(Wd)[1];
        N2 = reinterpret_cast<uint4 *>(Wd)[2];
        N3 = reinterpret_cast<uint4 *>(Wd)[3];
        nbase = wb;
    };

    uint32_t ti = 0;  // tokens stored (the first trip starts with the first block's header)
    // (a trip's store reaches 4 slots past the count; the code-length scratch is the last 128)
    const uint32_t tmax = tok_cap - 1 - 128 - 8;
    for (;;) {
        const bool act = !bad && st != 2;
        if (!__builtin_amdgcn_ballot_w64(act)) break;
        // every lane makes a trip's window write, load and token store, decoding or not: the
        // window loaded a trip ago into LDS, the next trip's from where this one starts
        put_window(N0, N1, N2, N3, nbase);
        {
            const uint32_t q = qdw();
            const uint4 *p = reinterpret_cast<const uint4 *>(qp + q);
            N0 = p[0], N1 = p[1], N2 = p[2], N3 = p[3];
            nbase = q;
        }
        uint4 tg = make_uint4(0, 0, 0, 0);
        uint32_t pc = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            if (!bad && st == 1) {
                uint32_t lo, hi;
                read64(lo, hi);
                const uint32_t e = look(0, kLR, lo);
                const uint32_t L = e & 15, kind = e >> 14;
                uint32_t t = 0;
                if (kind == kKLit) {
                    bpos += L;
                    if (xd >= olen) bad = true, why = why ? why : 8u;
                    t = kTLit | (1u << 16) | ((e >> 4) & 255);
                    xd++;
                } else if (kind == kKLen) {
                    const uint32_t v = (e >> 4) & 31;
                    uint32_t ext = 0, base = v + 3;
                    if (v == 28) base = 258;
                    else if (v >= 8) {
                        ext = (v - 4) >> 2;
                        base = ((4 + (v & 3)) << ext) + 3;
                    }
                    const uint32_t len = base + __builtin_amdgcn_ubfe(lo, L, ext);
                    const uint32_t s1 = L + ext;
                    const uint32_t db = __builtin_amdgcn_alignbit(hi, lo, s1);
                    const uint32_t d = look(dbase, kDR, db);
                    const uint32_t dl = d & 15, ds = (d >> 4) & 31;
                    const uint32_t dext = ds < 4 ? 0 : (ds >> 1) - 1;
                    const uint32_t dbs = ds < 4 ? ds + 1 : ((2u | (ds & 1)) << dext) + 1;
                    const uint32_t dist = dbs + __builtin_amdgcn_ubfe(db, dl, dext);
                    bpos += s1 + dl + dext;
                    if (dist > xd || xd + len > olen) bad = true, why = why ? why : 8u;
                    t = (len << 16) | (dist - 1) | (len > 64 || dist > kCReach ? kTSlow : 0u);
                    xd += len;
                } else {  // end of block
                    bpos += L;
                    st = last ? 2 : 0;
                }
                if (kind != kKEob) {
                    tg.x = pc == 0 ? t : tg.x;
                    tg.y = pc == 1 ? t : tg.y;
                    tg.z = pc == 2 ? t : tg.z;
                    tg.w = pc == 3 ? t : tg.w;
                    pc++;
                }
                if (bpos > bend + 64) bad = true, why = why ? why : 9u;  // (ran past the stream)
            }
            if (!bad && st == 0) header();  // (the first block's, or a block after it)
        }
        // the trip's tokens (slots past them are rewritten by the next trip)
        const uint32_t at = ti <= tmax ? ti : tmax;
        __builtin_memcpy(tk + 1 + at, &tg, 16);
        ti += pc;
        if (ti > tmax) bad = true, why = why ? why : 10u;
    }
    if (!bad && (((bpos - sh) + 7) >> 3 != (uint32_t)plen || xd != olen)) bad = true, why = why ? why : 11u;
    tk[0] = bad ? kTokNone : ti;
    mstat[m] = bad ? kDefer : 0u;
    if (bad) {
        hlist[1 + atomicAdd(hlist, 1u)] = i;
        atomicAdd(ndefer, 1u);
        atomicAdd(ndefer + (why ? why : 12u), 1u);
    }
}

// k_inflate_copy: the LZ77 copy of the decoded tokens, one member per wave.  The lane decoder's
// tokens make the copy a loop of wave-uniform steps (no Huffman work left in it):
//   - the member's tokens come 64 at a time, one per lane (a coalesced load, the next group in
//     flight behind the current), and each step broadcasts the next one (v_readlane);
//   - the output goes through an 8 KiB LDS window: a token's bytes are one LDS read and one write
//     per lane per 64 bytes (the period-d pattern out[x + i] = out[x - d + i mod d], which is also
//     the plain copy when d > i: every byte read lies before the match);
//   - the window goes to memory in aligned, coalesced 16-byte blocks every 1 KiB (byte stores only
//     at the member's two ends, whose 16-byte blocks it shares with its neighbours);
//   - a match further back than the window holds (7,934 bytes: 2 % of the bench shard's) reads
//     the member's output in memory, already written (every store of the wave waited for, the
//     dwords read at agent scope: from L2, never an older L1 line).
// Eight KiB of LDS a wave: 20 waves on a CU hide each other's LDS round trips.
__global__ void __launch_bounds__(64) k_inflate_copy(const BgzfMember *__restrict__ mem, const uint64_t *__restrict__ out_off,
                                                     uint8_t *__restrict__ out, const uint32_t *__restrict__ tok,
                                                     uint32_t tok_cap, const uint32_t *__restrict__ perm, uint32_t n_lanes) {
    __shared__ __attribute__((aligned(16))) uint8_t W[kCW];
    const uint32_t lane = threadIdx.x;
    const uint32_t i = blockIdx.x;  // the member's token slot (perm order)
    if (i >= n_lanes) return;
    const uint32_t *const tk = tok + (size_t)i * tok_cap;
    const uint32_t ntok = uni(tk[0]);
    if (ntok == kTokNone) return;  // (handed over: k_inflate_handover's)
    const uint32_t m = uni(perm[i]);
    uint8_t *const ob = out + out_off[m];
    const uint32_t olen = uni(mem[m].out_len);
    // output byte p is at window slot (ph + p) & mask, ph = its address mod 16: aligned 16-byte
    // blocks of the window go to aligned 16-byte blocks of memory
    const uint32_t ph = (uint32_t)((uintptr_t)ob & 15);
    uint8_t *const gout = ob - ph;
    uint32_t x = ph, fl = ph;  // the next byte (window coordinates), the first byte not yet out
    const uint32_t xend = ph + olen;
    auto flush = [&](uint32_t to, bool fin) {
        if (to <= fl) return;
        uint32_t a = fl;
        const uint32_t a16 = (a + 15) & ~15u;
        if (a != a16) {  // (the first block: shared with the member before)
            const uint32_t e = a16 < to ? a16 : to;
            if (lane < e - a) gout[a + lane] = W[(a + lane) & kCWMask];
            a = e;
        }
        const uint32_t b16 = to & ~15u;
        for (uint32_t y = a + 16 * lane; y + 16 <= b16; y += 16 * 64)
            *reinterpret_cast<uint4 *>(gout + y) = *reinterpret_cast<const uint4 *>(W + (y & kCWMask));
        if (fin && b16 >= a && to > b16)  // (the last block: shared with the member after)
            if (lane < to - b16) gout[b16 + lane] = W[(b16 + lane) & kCWMask];
        fl = fin ? to : (b16 > a ? b16 : a);
    };
    const float lanef = (float)lane + 0.5f;
    // A token of at most 64 bytes from within the window (all literals, nearly all matches) is one
    // branch-free step: every lane reads its byte of the period-d pattern (a literal's lanes take
    // its byte) and writes it at x + lane; the lanes past the length write ahead of the output,
    // into slots of bytes long flushed and out of reach, which the next tokens rewrite before
    // anything reads or flushes them.  Longer or further matches (the slow flag) take the loops
    // of slow() below.  The fields of a group's 64 tokens are unpacked once, a token per lane
    // (length, distance, its reciprocal, a literal's byte); a fast step takes them by v_readlane,
    // which is vector work: the CU's one scalar unit, which a step of scalar field extraction and
    // branching kept busy (~15 scalar instructions a token), now counts steps only.
    uint32_t nxt = tk[1 + lane];
    for (uint32_t tb = 0; tb < ntok; tb += 64) {
        const uint32_t cur = nxt;
        {
            const uint32_t q = tb + 64 + lane;  // (the next group: a token slot's spare tail past the count)
            nxt = tk[1 + (q < tok_cap - 1 ? q : tok_cap - 2)];
        }
        const uint32_t nt = ntok - tb < 64 ? ntok - tb : 64;
        const uint32_t tlen = (cur >> 16) & 511, tdist = (cur & 0x7FFF) + 1;
        const float trcp = __builtin_amdgcn_rcpf((float)tdist);
        const uint32_t tlit = (cur & kTLit) ? (cur & 255) : 256u;  // < 256: a literal's byte
        uint64_t slowm = __builtin_amdgcn_ballot_w64(lane < nt && (cur & kTSlow));
        auto fast = [&](uint32_t j) {
            const uint32_t dist = (uint32_t)__builtin_amdgcn_readlane((int)tdist, (int)j);
            const uint32_t lit = (uint32_t)__builtin_amdgcn_readlane((int)tlit, (int)j);
            const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((int)tlen, (int)j);
            const float rd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(trcp), (int)j));
            const uint32_t q = (uint32_t)(lanef * rd);
            uint32_t v = W[(x + lane - __umul24(q + 1u, dist)) & kCWMask];
            v = lit < 256 ? lit : v;
            W[(x + lane) & kCWMask] = (uint8_t)v;
            x += len;
        };
        auto slow = [&](uint32_t j) {
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)cur, (int)j);
            const uint32_t len = (t >> 16) & 511, dist = (t & 0x7FFF) + 1;
            const float rd = __builtin_amdgcn_rcpf((float)dist);
            if (dist <= kCReach) {
                for (uint32_t c = 0; c < len; c += 64) {
                    const uint32_t q = (uint32_t)(((float)c + lanef) * rd);
                    const uint8_t v = W[(x - dist + c + lane - __mul24(q, dist)) & kCWMask];
                    W[(x + c + lane) & kCWMask] = v;
                }
            } else {
                // from memory: [x - dist, x - dist + len) went out long ago (no period: dist > len)
                __builtin_amdgcn_s_waitcnt(0);
                for (uint32_t c = 0; c < len; c += 64) {
                    const uint32_t p = x - dist + c + lane;
                    const uint32_t w = __hip_atomic_load(reinterpret_cast<uint32_t *>(gout + (p & ~3u)), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    W[(x + c + lane) & kCWMask] = (uint8_t)(w >> (8 * (p & 3)));
                }
            }
            x += len;
        };
        // runs of fast tokens up to the next slow one; a flush check every 16 fast tokens (x moves
        // at most 1 KiB between checks) and after each slow one
        uint32_t j = 0;
        while (j < nt) {
            const uint32_t stop = slowm ? min((uint32_t)__builtin_ctzll(slowm), nt) : nt;
            while (j < stop) {
                const uint32_t e = min(stop, j + 16);
                for (; j + 4 <= e; j += 4) {
                    fast(j);
                    fast(j + 1);
                    fast(j + 2);
                    fast(j + 3);
                }
                for (; j < e; j++) fast(j);
                if (x - fl >= 2 * kCFlush) flush(x & ~(kCFlush - 1), false);
            }
            if (j < nt) {
                slow(j++);
                slowm &= slowm - 1;
                if (x - fl >= 2 * kCFlush) flush(x & ~(kCFlush - 1), false);
            }
        }
    }
    flush(xend, true);
}

// ---- CRC-32 (zlib's gzip trailer check) ----------------------------------------------------------
// Per member (one wave): the output is cut at its end into 1 KiB segments, the first one partial;
// lane j computes the raw CRC register of segment j (slice-by-4 tables in LDS; the first segment
// starts from 0xFFFFFFFF, the others from 0), then lane 0 folds them in order with the linear map
// "through 1 KiB of zero bytes" (four 256-entry tables built from its 32 basis images, which the
// host computes): acc = Z(acc) ^ R_j.  ~acc is the member's CRC-32.
__global__ void __launch_bounds__(64) k_crc32(const uint8_t *__restrict__ comp, const BgzfMember *__restrict__ mem,
                                              const uint64_t *__restrict__ out_off, const uint8_t *__restrict__ out,
                                              Crc1k z1k, uint32_t *__restrict__ mstat,
                                              unsigned long long *__restrict__ first_bad, uint64_t mbase) {
    __shared__ uint32_t T[4][256];
    __shared__ uint32_t Z[4][256];
    const int lane = threadIdx.x;
    const uint32_t m = blockIdx.x;
    for (int i = lane; i < 256; i += 64) {
        uint32_t c = (uint32_t)i;
#pragma unroll
        for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1)));
        T[0][i] = c;
        uint32_t zz[4] = {0, 0, 0, 0};
#pragma unroll
        for (int b = 0; b < 8; b++)
#pragma unroll
            for (int t = 0; t < 4; t++)
                if ((i >> b) & 1) zz[t] ^= z1k.v[8 * t + b];
#pragma unroll
        for (int t = 0; t < 4; t++) Z[t][i] = zz[t];
    }
    __syncthreads();
    for (int i = lane; i < 256; i += 64) {
        const uint32_t c0 = T[0][i];
        const uint32_t c1 = (c0 >> 8) ^ T[0][c0 & 0xFF];
        const uint32_t c2 = (c1 >> 8) ^ T[0][c1 & 0xFF];
        const uint32_t c3 = (c2 >> 8) ^ T[0][c2 & 0xFF];
        T[1][i] = c1;
        T[2][i] = c2;
        T[3][i] = c3;
    }
    __syncthreads();
    const BgzfMember M = mem[m];
    const uint32_t n = M.out_len;
    const uint8_t *p = out + out_off[m];
    const uint32_t head = n & 1023u, nseg = (n >> 10) + (head ? 1 : 0);
    uint32_t r = 0;
    if ((uint32_t)lane < nseg) {
        const uint32_t s0 = lane == 0 ? 0 : head + ((uint32_t)lane - (head ? 1 : 0)) * 1024;
        const uint32_t s1 = lane == 0 ? (head ? head : 1024) : s0 + 1024;
        uint32_t c = lane == 0 ? 0xFFFFFFFFu : 0u;
        const uint8_t *q = p + s0, *qe = p + s1;
        auto step4 = [&](uint32_t w) {
            c ^= w;
            c = T[3][c & 0xFF] ^ T[2][(c >> 8) & 0xFF] ^ T[1][(c >> 16) & 0xFF] ^ T[0][c >> 24];
        };
        while (q < qe && (((uintptr_t)q) & 15)) c = (c >> 8) ^ T[0][(c ^ *q++) & 0xFF];
        // 64 B per step from 16 B-aligned loads, the next step's four loads in flight while this
        // step's 16 dwords go through the tables (a serial chain of loads was the kernel's cost)
        // (named registers, not arrays: the arrays' loop-carried copies went to scratch)
        if (q + 64 <= qe) {
            const uint4 *q4 = reinterpret_cast<const uint4 *>(q);
            uint4 v0 = q4[0], v1 = q4[1], v2 = q4[2], v3 = q4[3];
            for (; q + 64 <= qe; q += 64) {
                uint4 n0 = v0, n1 = v1, n2 = v2, n3 = v3;
                if (q + 128 <= qe) {
                    const uint4 *p4 = reinterpret_cast<const uint4 *>(q + 64);
                    n0 = p4[0], n1 = p4[1], n2 = p4[2], n3 = p4[3];
                }
                step4(v0.x), step4(v0.y), step4(v0.z), step4(v0.w);
                step4(v1.x), step4(v1.y), step4(v1.z), step4(v1.w);
                step4(v2.x), step4(v2.y), step4(v2.z), step4(v2.w);
                step4(v3.x), step4(v3.y), step4(v3.z), step4(v3.w);
                v0 = n0, v1 = n1, v2 = n2, v3 = n3;
            }
        }
        for (; q + 4 <= qe; q += 4) step4(*reinterpret_cast<const uint32_t *>(q));
        while (q < qe) c = (c >> 8) ^ T[0][(c ^ *q++) & 0xFF];
        r = c;
    }
    // fold in order on lane 0 (the other lanes' registers through LDS)
    __shared__ uint32_t R[64];
    R[lane] = r;
    __syncthreads();
    if (lane == 0) {
        uint32_t acc = n ? R[0] : 0xFFFFFFFFu;
        for (uint32_t j = 1; j < nseg; j++)
            acc = Z[0][acc & 0xFF] ^ Z[1][(acc >> 8) & 0xFF] ^ Z[2][(acc >> 16) & 0xFF] ^ Z[3][acc >> 24] ^ R[j];
        const uint64_t t = M.src_off + M.src_len - 8;
        const uint32_t want = (uint32_t)comp[t] | ((uint32_t)comp[t + 1] << 8) | ((uint32_t)comp[t + 2] << 16) |
                              ((uint32_t)comp[t + 3] << 24);
        if (~acc != want && mstat[m] == 0) {
            mstat[m] = 20;
            atomicMin(first_bad, (unsigned long long)(mbase + m));
        }
    }
}

}  // namespace

void crc32_zero1k_basis(Crc1k *z) {
    uint32_t t[256];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int b = 0; b < 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1)));
        t[i] = c;
    }
    for (int k = 0; k < 32; k++) {
        uint32_t c = 1u << k;
        for (int i = 0; i < 1024; i++) c = (c >> 8) ^ t[c & 0xFF];
        z->v[k] = c;
    }
}

hipError_t launch_inflate(int which, const uint8_t *comp, const BgzfMember *mem, const uint64_t *out_off,
                          uint64_t n_members, uint8_t *out, uint32_t *mstat, unsigned long long *first_bad,
                          const Crc1k &z1k, hipStream_t s, uint64_t mbase, uint32_t *tok, uint64_t tok_members,
                          const uint32_t *perm, const InflateSide *side) {
    // (mem, out_off, mstat: the arrays' entries for members mbase ..; first_bad: a global index,
    // followed by the 32-bit count of members the lane decoder handed to the wave decoder)
    static const int lanes_env = [] {
        const char *e = getenv("VCFX_INFLATE_LANES");  // 0: every member on the wave decoder (A/B)
        return e && *e == '0' ? 0 : 1;
    }();
    const int lanes = lanes_env && tok && tok_members && perm && side && side->aux;
    uint32_t *const ndefer = reinterpret_cast<uint32_t *>(first_bad + 1);
    if (which == 0 && !lanes) {
        for (uint64_t m0 = 0; m0 < n_members; m0 += (1u << 30)) {
            const uint64_t nm = n_members - m0 < (1u << 30) ? n_members - m0 : (1u << 30);
            hipLaunchKernelGGL(k_inflate, dim3((unsigned)nm), dim3(64), 0, s, comp, mem + m0, out_off + m0, out,
                               mstat + m0, first_bad, mbase + m0);
            const hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (which == 0) {
        hipStream_t aux = side->aux;
        hipEvent_t ev_dec = side->ev[0], ev_fb = side->ev[1];
        // the hand-over list follows the tokens
        uint32_t *const hl0 = tok + (size_t)tok_members * kTokCap;
        hipError_t e;
        auto decode = [&](hipStream_t st, uint64_t b, uint32_t nb, uint32_t *hl) -> hipError_t {
            hipError_t r;
            if ((r = hipMemsetAsync(hl, 0, 4, st)) != hipSuccess) return r;
            hipLaunchKernelGGL(k_inflate_decode, dim3((nb + 63) / 64), dim3(64), 0, st, comp, mem, out_off, out, mstat,
                               ndefer, tok + (size_t)(b % tok_members) * kTokCap, kTokCap, perm + b, nb, hl);
            return hipGetLastError();
        };
        auto handover = [&](uint64_t b, const uint32_t *hl) -> hipError_t {
            hipLaunchKernelGGL(k_inflate_handover, dim3(kHandGrid), dim3(64), 0, aux, comp, mem, out_off, out, mstat,
                               first_bad, mbase, perm + b, hl);
            return hipGetLastError();
        };
        auto copy = [&](hipStream_t st, uint64_t b, uint32_t nb) -> hipError_t {
            hipLaunchKernelGGL(k_inflate_copy, dim3(nb), dim3(64), 0, st, mem, out_off, out,
                               tok + (size_t)(b % tok_members) * kTokCap, kTokCap, perm + b, nb);
            return hipGetLastError();
        };
        // the lane decoder, then its hand-overs on `aux` beside the copy on `s`, in pieces of at
        // most tok_members (the token buffer's members).  (Two pieces on two streams -- one round of
        // decode waves, the rest on a low-priority stream so that the first piece's copy starts
        // while the rest decodes -- measured 8.64-8.75 ms against 8.70: not kept.)
        for (uint64_t b = 0; b < n_members; b += tok_members) {
            const uint32_t nb = (uint32_t)(n_members - b < tok_members ? n_members - b : tok_members);
            if (b && (e = hipStreamWaitEvent(s, ev_fb, 0)) != hipSuccess) return e;  // (the list is reused)
            if ((e = decode(s, b, nb, hl0)) != hipSuccess || (e = hipEventRecord(ev_dec, s)) != hipSuccess ||
                (e = hipStreamWaitEvent(aux, ev_dec, 0)) != hipSuccess || (e = handover(b, hl0)) != hipSuccess ||
                (e = hipEventRecord(ev_fb, aux)) != hipSuccess || (e = copy(s, b, nb)) != hipSuccess)
                return e;
        }
        return hipStreamWaitEvent(s, ev_fb, 0);
    }
    for (uint64_t m0 = 0; m0 < n_members; m0 += (1u << 30)) {
        const uint64_t nm = n_members - m0 < (1u << 30) ? n_members - m0 : (1u << 30);
        hipLaunchKernelGGL(k_crc32, dim3((unsigned)nm), dim3(64), 0, s, comp, mem + m0, out_off + m0, out, z1k,
                           mstat + m0, first_bad, mbase + m0);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace vcfxg
