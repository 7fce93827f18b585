// vcfxg_dose.hip -- VCFX_dosage_calculator's per-record pass (a per-sample
// GT map on the record path).
//
// Output per data record: "CHROM\tPOS\tID\tREF\tALT\t" + one dosage per sample ('0' / '1' /
// '2', or "NA"), comma separated, + '\n' -- about 2 bytes per sample, so the output is half
// the input.  Two passes over the indexed lines, one wave per line:
//   k_dose_len  the record's head (tabs, the FORMAT's GT index) and its row length: on the
//               fixed-stride layout (GT-only, single-digit diploid) the sweep counts the NA
//               samples (gt_fast); GT-first records of any width go through gt_first;
//               anything else through the exact per-sample parse (gt_general);
//   k_dose_fmt  after a scan of the row lengths: the prefix and the dosages, each lane's
//               samples placed by a wave scan of their output bytes (the fixed-stride sweep
//               on fixed-stride records, a lane per sample start otherwise).
// Semantics (VCFX_dosage_calculator.cpp): processFileMmap :426-577 (mode 0: '\r' stripped) /
// calculateDosage :229-353 (mode 1: no strip); fields split up to 10 (< 10: the warning);
// findGTIndexRaw :160-178 (GT not in FORMAT: "NA" for the record); extractGTFromSample
// :182-203 and parseDosageInline :111-156 per sample (samples run to the line end: a
// trailing tab adds no sample).
#include <algorithm>

#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

constexpr int kDoseThreads = 256;
constexpr int kDoseWaves = kDoseThreads / kWave;

// parseDosageInline on [g, g + n): -1 NA, else the dosage (an allele counts when its number,
// accumulated modulo 2^32, is non-zero: the reference build's `> 0` on a non-negative int)
__device__ __forceinline__ int dose_parse(const char *__restrict__ buf, int64_t g, int64_t n) {
    if (n <= 0) return -1;
    int dose = 0, count = 0;
    int64_t p = g, e = g + n;
    while (p < e) {
        while (p < e && (byte_at(buf, p) == '/' || byte_at(buf, p) == '|')) p++;
        if (p >= e) break;
        if (byte_at(buf, p) == '.') return -1;
        uint32_t a = 0;
        bool dig = false;
        while (p < e && is_digit(byte_at(buf, p))) {
            a = a * 10u + (byte_at(buf, p) - '0');
            dig = true;
            p++;
        }
        if (!dig) return -1;
        dose += a != 0u;
        if (++count > 2) return -1;
    }
    return count == 2 ? dose : -1;
}

// extractGTFromSample(gi) + parseDosageInline for the sample starting at st (ends at the next
// tab or E)
__device__ __forceinline__ int dose_sample(const char *__restrict__ buf, int64_t st, int64_t E, int gi) {
    const int64_t se = sample_end(buf, st, E);
    int cur = 0;
    int64_t fs = st;
    for (int64_t q = st; q <= se; q++) {
        if (q == se || byte_at(buf, q) == ':') {
            if (cur == gi) return dose_parse(buf, fs, q - fs);
            cur++;
            fs = q + 1;
        }
    }
    return -1;
}

// pass-1 reducer: samples and NA samples (NA = 2 output bytes)
struct DoseCountOp {
    const char *buf;
    int64_t E;
    int gi;
    uint32_t ns = 0, na = 0;
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &v) {  // "a s b": NA unless both are digits
        ns += v.real;
        na += v.real && v.dig != 0x01000100u;
    }
    __device__ void gt3(uint32_t c0, uint32_t c2) {
        ns++;
        na += !(c0 - '0' < 10u && c2 - '0' < 10u);
    }
    __device__ void sample(int64_t st) {
        ns++;
        na += dose_sample(buf, st, E, gi) < 0;
    }
    __device__ void finish() {
        ns = wave_sum(ns);
        na = wave_sum(na);
    }
};

enum : uint8_t { kDoseSkip = 0, kDoseRow = 1, kDoseWarn = 3, kDosePend = 0xFE };
enum : uint8_t { kDoseFast = 1, kDoseGeneral = 2, kDoseNA = 3, kDoseNoSamples = 4 };

// per line: status, row length, and how pass 2 writes it (kind, GT index, sample start)
struct DoseMeta {
    uint64_t S;     // sample region start
    uint32_t pre;   // bytes of "CHROM\t..ALT\t"
    uint32_t ae;    // line end (after the mode's '\r' strip) - S
    int32_t gi;     // GT index in FORMAT
    uint8_t kind;   // kDose*
    uint8_t plain;  // kDoseFast without an "NA": 2 output bytes per sample
    uint8_t sep;    // kDoseFast: the separator (the byte at S + 1)
    uint8_t pad;
};

// kFast: the first pass -- fixed-stride records (and the head-only kinds) only; any other
// record is left kDosePend for the second pass (kFast = false, which skips every other line),
// so the first pass carries none of the general parsers' registers (occupancy)
template <bool kFast>
__global__ __launch_bounds__(kDoseThreads) void k_dose_len(const char *__restrict__ buf, int64_t data_start,
                                                           const uint64_t *__restrict__ line_end,
                                                           const uint64_t *n_lines_p, int mode,
                                                           uint8_t *__restrict__ status, uint64_t *__restrict__ len,
                                                           DoseMeta *__restrict__ meta,
                                                           unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kDoseWaves][16];
    __shared__ uint32_t red[5][kDoseWaves];
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t rows = 0, warns = 0, gen = 0, slow = 0, napl = 0;  // (wave-uniform; slow: rows not kDoseFast)
    for (uint64_t li = wid; li < n_lines; li += nw) {
        if (!kFast && status[li] != kDosePend) continue;  // (wave-uniform)
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
        int64_t ae = le;
        if (mode == 0 && ae > ls && byte_at(buf, ae - 1) == '\r') ae--;
        uint8_t st = kDoseSkip;
        uint64_t L = 0;
        DoseMeta m{};
        if (ae > ls && byte_at(buf, ls) != '#') {
            int64_t t[10];
            const int nt = head_tabs(buf, ls, ae, 10, t, lds);
            if (nt < 9) st = kDoseWarn;
            else {
                st = kDoseRow;
                m.pre = (uint32_t)(t[4] - ls + 1);
                m.S = (uint64_t)(t[8] + 1);
                m.ae = (uint32_t)(ae - (t[8] + 1));
                const int gi = gt_index(buf, t[7] + 1, t[8]);
                if (gi < 0) {
                    m.kind = kDoseNA;
                    L = m.pre + 3u;  // "NA\n"
                } else if (t[8] + 1 >= ae) {
                    m.kind = kDoseNoSamples;
                    L = m.pre + 1u;  // "\n"
                } else {
                    m.gi = gi;
                    const int64_t S = t[8] + 1;
                    DoseCountOp op{buf, ae, gi};
                    bool fast = gi == 0 && gt_fast(buf, S, ae, op);
                    m.kind = kDoseFast;
                    m.plain = fast && op.na == 0;
                    m.sep = fast ? (uint8_t)byte_at(buf, S + 1) : 0;
                    if (kFast && !fast) st = kDosePend;
                    else if (!fast) {
                        m.kind = kDoseGeneral;
                        op = DoseCountOp{buf, ae, gi};
                        if (!(gi == 0 && gt_first_known(buf, S, ae, op))) {
                            op = DoseCountOp{buf, ae, gi};
                            gt_general(buf, S, ae, op);
                        }
                        gen++;
                    }
                    if (st != kDosePend) L = (uint64_t)m.pre + 2u * op.ns + op.na;  // dosages + separators / '\n'
                }
            }
        }
        rows += st == kDoseRow;
        slow += st == kDoseRow && m.kind != kDoseFast;
        napl += st == kDoseRow && m.kind == kDoseFast && !m.plain;
        warns += st == kDoseWarn;
        if (lane() == 0) {
            status[li] = st;
            len[li] = L;
            meta[li] = m;
        }
    }
    // one atomic per block and counter (same-address atomics serialise in L2)
    if (lane() == 0) {
        red[0][threadIdx.x / kWave] = rows;
        red[1][threadIdx.x / kWave] = warns;
        red[2][threadIdx.x / kWave] = gen;
        red[3][threadIdx.x / kWave] = slow;
        red[4][threadIdx.x / kWave] = napl;
    }
    __syncthreads();
    if (threadIdx.x < 5) {  // counters: rows, rows of k_dose_fmt<kFmtOther>, warnings, general, rows of kFmtNa
        uint32_t t = 0;
        for (int k = 0; k < kDoseWaves; k++) t += red[threadIdx.x][k];
        const int slot = threadIdx.x == 0 ? 0 : threadIdx.x == 1 ? 2 : threadIdx.x == 2 ? 3 : threadIdx.x == 3 ? 1 : 4;
        if (t) atomicAdd(&counters[slot], (unsigned long long)t);
    }
}

__device__ __forceinline__ void put_dose(char *o, int d, bool last) {
    if (d < 0) {
        o[0] = 'N';
        o[1] = 'A';
        o[2] = last ? '\n' : ',';
    } else {
        o[0] = (char)('0' + d);
        o[1] = last ? '\n' : ',';
    }
}

// one launch per row kind, so each carries only its own registers and code: kFmtPlain the
// fixed-stride rows without "NA" (every row of a clean GT-only input), kFmtNa the fixed-stride
// rows with some "NA" (launched when k_dose_len / k_dose_from_walk counted any), kFmtOther every
// other row kind (likewise)
enum : int { kFmtOther = 0, kFmtNa = 1, kFmtPlain = 2 };
template <int kMode>
__global__ __launch_bounds__(kDoseThreads) void k_dose_fmt(const char *__restrict__ buf, int64_t data_start,
                                                           const uint64_t *__restrict__ line_end,
                                                           const uint64_t *n_lines_p,
                                                           const uint8_t *__restrict__ status,
                                                           const DoseMeta *__restrict__ meta,
                                                           const uint64_t *__restrict__ off, char *__restrict__ out,
                                                           uint64_t cap, unsigned *__restrict__ bad) {
    // kFmtNa: a wave-step's text (512 samples, at most 3 bytes each) composed in LDS
    __shared__ __attribute__((aligned(16))) unsigned char na_tile[kMode == kFmtNa ? kDoseThreads / kWave : 1]
                                                                 [kMode == kFmtNa ? 3 * 8 * kWave + 32 : 16];
    const uint64_t n_lines = *n_lines_p;
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t li = wid; li < n_lines; li += nw) {
        if (status[li] != kDoseRow || off[li + 1] > cap) continue;  // (wave-uniform)
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start;
        const DoseMeta m = meta[li];
        if ((m.kind != kDoseFast ? kFmtOther : m.plain ? kFmtPlain : kFmtNa) != kMode) continue;  // (wave-uniform)
        char *o = out + off[li];
        for (uint32_t k = lane(); k < m.pre; k += kWave) o[k] = buf[ls + k];
        o += m.pre;
        if (m.kind == kDoseNA) {
            if (lane() == 0) {
                o[0] = 'N';
                o[1] = 'A';
                o[2] = '\n';
            }
            continue;
        }
        if (m.kind == kDoseNoSamples) {
            if (lane() == 0) o[0] = '\n';
            continue;
        }
        const int64_t S = (int64_t)uniform64((int64_t)m.S), E = S + (int64_t)m.ae;
        // the samples' output bytes (pass 1's row length less the prefix): the sample whose
        // bytes end there is the last, and ends with '\n' instead of ','
        const uint64_t tot = off[li + 1] - off[li] - m.pre;
        uint64_t run = 0;  // output bytes of the samples before this wave-step
        if (kMode == kFmtPlain) {
            // fixed-stride, no "NA": sample k ("a s b\t" at S + 4k) is output bytes 2k, 2k + 1
            // of the dosage text (the digit, then ',' -- the row's last byte '\n').  Lane c takes
            // samples 8c..8c+7 (32 input bytes, realigned by S mod 4 from 36 bytes at a 4-aligned address) and
            // builds the aligned 16 B output block that starts inside its 16 bytes' span: the
            // previous lane's last (ob mod 16) bytes, then its own first ones -- one store per block.
            // Every sample is checked while it is read (a row the head walk took on its predicted
            // end alone may turn out otherwise -- the call is then redone): with e = dword ^
            // "0 s 0 \t" (s = m.sep), the separator and tab bytes of e are 0 and each allele
            // field of e is below 10; the dosage is the number of non-zero allele fields.
            const int64_t ns = (E - S + 1) / 4;
            const uint64_t ob = (uint64_t)(o - out), oe = ob + 2 * (uint64_t)ns;
            const uint32_t osh = (uint32_t)(ob & 15);
            const uint32_t ib = (uint32_t)(S & 3), wq = (16u - osh) >> 2, wb = (16u - osh) & 3;
            const int64_t nch = (ns + 7) / 8;  // chunks of 8 samples; chunk nch holds only the tail block
            uint32_t carry[4] = {0u, 0u, 0u, 0u};  // the previous wave-step's last chunk
            const uint32_t exp = 0x09300030u | ((uint32_t)m.sep << 8);
            uint32_t err = m.sep == '/' || m.sep == '|' ? 0u : 1u;
            for (int64_t c0 = 0; c0 <= nch; c0 += kWave) {
                const int64_t c = c0 + lane(), k0 = 8 * c;
                const bool edge = c0 + kWave > nch - 1;  // (wave-uniform) the step holds the last sample
                uint32_t od[4] = {0u, 0u, 0u, 0u};
                if (c < nch) {
                    // 36 bytes from the 4-aligned address at or before the lane's first sample:
                    // the samples are then the byte rotation ib (= S mod 4) of consecutive words,
                    // with no word-level select (a select on the uniform word offset compiled to
                    // branches around the loads: 1.38 -> 1.58 ms for this pass with the checks)
                    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
                    const uint32_t *ip = reinterpret_cast<const uint32_t *>(buf + ((S + 4 * k0) & ~(int64_t)3));
                    const u32x4a4 v0 = *reinterpret_cast<const u32x4a4 *>(ip), v1 = *reinterpret_cast<const u32x4a4 *>(ip + 4);
                    const uint32_t w[9] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, ip[8]};
                    uint32_t e[8];
#pragma unroll
                    for (int i = 0; i < 8; i++) e[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], ib);
#pragma unroll
                    for (int t = 0; t < 8; t++) e[t] ^= exp;
                    if (edge) {  // samples past the record: nothing; the last one's tab byte is the line end
                        const int rem = (int)std::min<int64_t>(ns - k0, 8);
#pragma unroll
                        for (int t = 0; t < 8; t++) e[t] = t < rem ? (t == rem - 1 ? e[t] & 0x00FFFFFFu : e[t]) : 0u;
                    }
                    uint32_t dd[8];
#pragma unroll
                    for (int t = 0; t < 8; t++) {
                        const uint32_t f = e[t] & 0x00FF00FFu;
                        err |= (e[t] & 0xFF00FF00u) | ((f + 0x00F600F6u) & 0x01000100u);  // field >= 10
                        dd[t] = __popc((f + 0x00FF00FFu) & 0x01000100u);                  // field >= 1
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) od[j] = 0x2C302C30u + dd[2 * j] + (dd[2 * j + 1] << 16);  // "d,d,"
                }
                // the previous chunk's bytes: the lane before, or the carry for lane 0
                uint32_t pv[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t up = lane_prev(od[j]);
                    pv[j] = lane() ? up : carry[j];
                    carry[j] = lane_last(od[j]);
                }
                // the block = bytes [16 - osh, 32 - osh) of (pv ++ od): word wq + i, byte wb
                const uint32_t X[9] = {pv[0], pv[1], pv[2], pv[3], od[0], od[1], od[2], od[3], 0u};
                uint32_t bw[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {  // (wq wave-uniform)
                    const uint32_t lo_ = wq == 0 ? X[i] : wq == 1 ? X[i + 1] : wq == 2 ? X[i + 2] : wq == 3 ? X[i + 3] : X[i + 4];
                    const uint32_t hi_ = wq == 0 ? X[i + 1] : wq == 1 ? X[i + 2] : wq == 2 ? X[i + 3] : wq == 3 ? X[i + 4] : X[i + 5];
                    bw[i] = __builtin_amdgcn_alignbyte(hi_, lo_, wb);
                }
                const uint64_t base = (ob & ~15ull) + 16ull * (uint64_t)c;
                if (edge && oe - 1 >= base && oe - 1 < base + 16) {  // the row's last byte: '\n'
                    const uint32_t q = (uint32_t)(oe - 1 - base);
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if ((q >> 2) == (uint32_t)i) bw[i] = (bw[i] & ~(0xFFu << (8 * (q & 3)))) | (0x0Au << (8 * (q & 3)));
                }
                if (c <= nch && base < oe) {
                    if (base >= ob && base + 16 <= oe)
                        *reinterpret_cast<uint4 *>(out + base) = make_uint4(bw[0], bw[1], bw[2], bw[3]);
                    else
#pragma unroll
                        for (int j = 0; j < 16; j++)
                            if (base + j >= ob && base + j < oe) out[base + j] = (char)(bw[j >> 2] >> (8 * (j & 3)));
                }
            }
            if (__any(err != 0u) && lane() == 0 && bad) atomicOr(bad, 1u);
            continue;
        }
        if (kMode == kFmtNa) {
            // the fixed-stride layout with some "NA" (k_dose_len / the walk validated it: every
            // allele a digit or '.'): lane c of a wave-step reads samples 8c..8c+7 as the plain
            // rows do (36 bytes from the 4-aligned address, rotated by S mod 4); a sample is "NA"
            // when an allele field of e = dword ^ "0 s 0 \t" is >= 10 ('.'), else its dosage is the
            // number of non-zero allele fields.  The lanes' texts (2 or 3 bytes per sample) are
            // placed by a wave scan of their lengths into the wave's LDS tile (offset = output
            // offset - the 16 B boundary below the step's first byte) and the tile goes out as
            // aligned 16 B stores -- byte stores only for its two partial blocks.
            const int64_t ns = (E - S + 1) / 4;
            const int64_t nch = (ns + 7) / 8;
            const uint32_t ib = (uint32_t)(S & 3);
            const uint32_t exp = 0x09300030u | ((uint32_t)m.sep << 8);
            unsigned char *tile = na_tile[threadIdx.x / kWave];
            const uint64_t ob = (uint64_t)(o - out);
            for (int64_t c0 = 0; c0 < nch; c0 += kWave) {
                const int64_t c = c0 + lane(), k0 = 8 * c;
                uint32_t na = 0, dg = 0, bytes = 0;  // bit t: sample k0 + t is "NA" / its dosage digit (2 bits)
                const int rem = c < nch ? (int)std::min<int64_t>(ns - k0, 8) : 0;
                if (rem > 0) {
                    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
                    const uint32_t *ip = reinterpret_cast<const uint32_t *>(buf + ((S + 4 * k0) & ~(int64_t)3));
                    const u32x4a4 v0 = *reinterpret_cast<const u32x4a4 *>(ip), v1 = *reinterpret_cast<const u32x4a4 *>(ip + 4);
                    const uint32_t w[9] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, ip[8]};
#pragma unroll
                    for (int t = 0; t < 8; t++) {
                        const uint32_t f = (__builtin_amdgcn_alignbyte(w[t + 1], w[t], ib) ^ exp) & 0x00FF00FFu;
                        const bool isna = ((f + 0x00F600F6u) & 0x01000100u) != 0u;  // an allele field >= 10: '.'
                        const uint32_t d = __popc((f + 0x00FF00FFu) & 0x01000100u);
                        if (t < rem) {
                            na |= (isna ? 1u : 0u) << t;
                            dg |= d << (2 * t);
                            bytes += isna ? 3u : 2u;
                        }
                    }
                }
                const uint32_t incl = wave_incl_scan(bytes);
                const uint32_t step = (uint32_t)wave_bcast(incl, kWave - 1);
                const uint64_t sb = ob + run;  // the step's first output byte
                const uint64_t tb = sb & ~15ull;
                uint32_t q = (uint32_t)(sb - tb) + incl - bytes;  // this lane's tile offset
                for (int t = 0; t < rem; t++) {
                    const unsigned char sepc = k0 + t == ns - 1 ? '\n' : ',';
                    if ((na >> t) & 1u) {
                        tile[q] = 'N';
                        tile[q + 1] = 'A';
                        tile[q + 2] = sepc;
                        q += 3;
                    } else {
                        tile[q] = (unsigned char)('0' + ((dg >> (2 * t)) & 3u));
                        tile[q + 1] = sepc;
                        q += 2;
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const uint64_t se = sb + step;
                const int nblk = (int)((se - tb + 15) >> 4);
                for (int j = lane(); j < nblk; j += kWave) {
                    const uint64_t gb = tb + 16u * (uint64_t)j;
                    if (gb >= sb && gb + 16 <= se) {
                        *reinterpret_cast<uint4 *>(out + gb) = reinterpret_cast<const uint4 *>(tile)[j];
                    } else {
                        const uint64_t b0 = gb > sb ? gb : sb, b1 = gb + 16 < se ? gb + 16 : se;
                        for (uint64_t b = b0; b < b1; b++) out[b] = (char)tile[b - tb];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                run += step;
            }
            continue;
        }
        // any other layout: a lane per 16 B block, its sample starts in order
        const int gi = m.gi;
        for (int64_t w = S & ~(int64_t)15; w < E; w += kWaveStep) {
            const int64_t blk = w + (int64_t)lane() * kBlockBytes;
            uint32_t starts = 0;
            if (blk < E) {
                const uint32_t tm = eq_mask16(load16(buf, blk), kRepTab);
                starts = (tm << 1) & 0xFFFFu;
                if (blk > 0 && byte_at(buf, blk - 1) == '\t') starts |= 1u;
                starts &= range_mask16(blk, S + 1, E);
                if (S >= blk && S < blk + 16) starts |= 1u << (S - blk);
            }
            int8_t dd[16];
            uint32_t bytes = 0, mm = starts;
            for (int c = 0; mm; c++) {
                const int j = __builtin_ctz(mm);
                mm &= mm - 1u;
                dd[c] = (int8_t)dose_sample(buf, blk + j, E, gi);
                bytes += dd[c] < 0 ? 3u : 2u;
            }
            const uint32_t incl = wave_incl_scan(bytes);
            uint64_t pos = run + incl - bytes;
            mm = starts;
            for (int c = 0; mm; c++) {
                mm &= mm - 1u;
                const uint32_t nb = dd[c] < 0 ? 3u : 2u;
                put_dose(o + pos, dd[c], pos + nb == tot);
                pos += nb;
            }
            run += wave_bcast(incl, kWave - 1);
        }
    }
}

static unsigned dose_grid(int64_t n, int64_t per, unsigned cap) {
    int64_t g = (n + per - 1) / per;
    if (g < 1) g = 1;
    return (unsigned)(g > cap ? cap : g);
}

size_t dose_meta_bytes() { return sizeof(DoseMeta); }

// the walk's lines -> dose statuses (thread per line): a fixed-stride GT-only record (walk
// status 1) is a kDoseFast row of pre + 2 ns + na bytes; '#' / empty lines are skipped; the
// rest (fewer than 9 tabs, other FORMATs, GT records off the fixed-stride layout) pending
__global__ void k_dose_from_walk(const uint64_t *__restrict__ line_end, const uint64_t *n_lines_p,
                                 const LineMeta *__restrict__ wm, const int32_t *__restrict__ ns,
                                 const int32_t *__restrict__ na, uint8_t *__restrict__ status,
                                 uint64_t *__restrict__ len, DoseMeta *__restrict__ meta,
                                 unsigned long long *__restrict__ counters) {
    const uint64_t n_lines = *n_lines_p;
    uint32_t rows = 0, napl = 0;
    for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < n_lines;
         li += (uint64_t)gridDim.x * blockDim.x) {
        const LineMeta w = wm[li];
        DoseMeta m{};
        uint8_t st = kDosePend;
        uint64_t L = 0;
        if (w.kind == kMetaEmpty || w.kind == kMetaHeader) st = kDoseSkip;
        else if (w.kind == kMetaGt && status[li] == 1) {
            const uint64_t ae = line_end[li] - w.cr;
            m.S = w.S;
            m.pre = w.rowpre;
            m.ae = (uint32_t)(ae - w.S);
            m.gi = 0;
            m.kind = kDoseFast;
            m.plain = na[li] == 0;
            m.sep = w.sep;
            napl += !m.plain;
            st = kDoseRow;
            L = (uint64_t)m.pre + 2u * (uint64_t)ns[li] + (uint64_t)na[li];
            rows++;
        }
        status[li] = st;
        len[li] = L;
        meta[li] = m;
    }
    rows = wave_sum(rows);
    napl = wave_sum(napl);
    if (lane() == 0 && rows) atomicAdd(&counters[0], (unsigned long long)rows);
    if (lane() == 0 && napl) atomicAdd(&counters[4], (unsigned long long)napl);
}

hipError_t launch_dose_from_walk(const uint64_t *line_end, const uint64_t *n_lines_dev, uint64_t n_lines_host,
                                 const void *walk_meta, const int32_t *ns, const int32_t *na, uint8_t *status,
                                 uint64_t *len, void *meta, unsigned long long *counters, hipStream_t s) {
    if (!n_lines_host) return hipSuccess;
    const unsigned g = (unsigned)std::min<uint64_t>((n_lines_host + 255) / 256, 4096);
    hipLaunchKernelGGL(k_dose_from_walk, dim3(g), dim3(256), 0, s, line_end, n_lines_dev,
                       static_cast<const LineMeta *>(walk_meta), ns, na, status, len, static_cast<DoseMeta *>(meta),
                       counters);
    return hipGetLastError();
}

hipError_t launch_dose_len(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, int mode, uint8_t *status, uint64_t *len, void *meta,
                           unsigned long long *counters, hipStream_t s, bool pending_only) {
    if (!n_lines_host) return hipSuccess;
    const dim3 g(dose_grid((int64_t)n_lines_host, kDoseWaves, 2048));
    if (!pending_only)
        hipLaunchKernelGGL(k_dose_len<true>, g, dim3(kDoseThreads), 0, s, buf, data_start, line_end, n_lines_dev, mode,
                           status, len, static_cast<DoseMeta *>(meta), counters);
    hipLaunchKernelGGL(k_dose_len<false>, g, dim3(kDoseThreads), 0, s, buf, data_start, line_end, n_lines_dev, mode,
                       status, len, static_cast<DoseMeta *>(meta), counters);
    return hipGetLastError();
}

hipError_t launch_dose_fmt(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, const uint8_t *status, const void *meta, const uint64_t *off,
                           char *out, uint64_t cap, uint64_t slow_rows, hipStream_t s, unsigned *bad,
                           uint64_t na_rows) {
    if (!n_lines_host) return hipSuccess;
    const dim3 g(dose_grid((int64_t)n_lines_host, kDoseWaves, 2048));
    hipLaunchKernelGGL(k_dose_fmt<kFmtPlain>, g, dim3(kDoseThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                       status, static_cast<const DoseMeta *>(meta), off, out, cap, bad);
    // (k_dose_len / k_dose_from_walk counted these rows: no pass over every line for nothing)
    if (na_rows)
        hipLaunchKernelGGL(k_dose_fmt<kFmtNa>, g, dim3(kDoseThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                           status, static_cast<const DoseMeta *>(meta), off, out, cap, bad);
    if (slow_rows)
        hipLaunchKernelGGL(k_dose_fmt<kFmtOther>, g, dim3(kDoseThreads), 0, s, buf, data_start, line_end, n_lines_dev,
                           status, static_cast<const DoseMeta *>(meta), off, out, cap, bad);
    return hipGetLastError();
}

}  // namespace vcfxg
