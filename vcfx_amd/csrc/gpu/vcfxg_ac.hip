// vcfxg_ac.hip -- VCFX_allele_counter's per-record, per-sample pass (a
// per-sample GT reducer on the record path whose output is a row per (record, sample)).
//
// Output per data record (no '\r' handling anywhere, as in the reference), for the selected
// samples in selection order:
//   text:      "CHROM\tPOS\tID\tREF\tALT\t" + name + "\t" + ref + "\t" + alt + "\n" per sample
//   aggregate: "CHROM\tPOS\tID\tREF\tALT\t" + Σref + "\t" + Σalt + "\t" + rows + "\n"
//   binary:    the two counts as int8 bytes per sample
// Two selection semantics (VCFX_allele_counter.cpp):
//   all (countAllelesMmapMT / processChunk :550-642): every selected sample gets a row; a sample
//       index past the record's last tab counts 0 / 0; the counts print as int8_t;
//   seq (countAllelesUnified :1371-1465, countAllelesStream :1188-1246): a forward-only cursor
//       (slot i reads the running maximum of the indices so far), rows stop at the first slot
//       whose sample starts at or past the line end; counts print as int.
// parseGenotypeRaw :267-294 per GT (the sample up to its first ':' or tab): digit runs count,
// 0 (modulo 2^32) as REF and anything else as ALT.
//
// Two passes, one wave per indexed line:
//   k_ac_len  head (prefix length, sample start), then either the fixed-stride sweep (gt_fast:
//             every GT is "a s b", so every count is one digit and a sample's bytes sit at
//             S + 4k) or the general path (the line's sample starts into a per-wave table in
//             global scratch, then a lane per output slot parses its sample); the row bytes;
//   k_ac_fmt  after a scan of the row bytes: the rows.  Fixed-stride text rows are composed
//             64 at a time in LDS (a lane per row) and written out as aligned 16 B stores.
#include "vcfxg_device.h"
#include "vcfxg_gt.h"
#include "vcfxg_kernels.h"

namespace vcfxg {

// VCFXG_AC_EXPT (diagnostic builds only, output invalid): bit 0 skips the text rows' composition
// in LDS, bit 1 their copy to the output
#ifndef VCFXG_AC_EXPT
#define VCFXG_AC_EXPT 0
#endif
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kAcThreads = 512;  // 8 waves share one LDS copy of the selection (r02: 256 -> 512)
constexpr int kAcWaves = kAcThreads / kWave;
constexpr int kAcTile = 3072;  // LDS bytes per wave for one tile of 64 text rows (longer: straight out)
constexpr int kAcPre = 256;    // LDS bytes per wave for the record's prefix

enum : uint8_t { kAcFast = 1, kAcGeneral = 2 };

struct AcMeta {
    uint64_t S;        // sample region start
    uint64_t sr, sa;   // aggregate: Σref, Σalt
    uint32_t P;        // prefix bytes ("CHROM\t..ALT\t", missing fields as empty)
    uint32_t rows;     // output rows
    uint32_t ns;       // fast: samples in the record
    uint32_t lim;      // prefix bytes taken from the line (the rest are tabs)
    uint8_t kind;
    uint8_t pad[7];
};

struct AcArgs {
    const uint32_t *eff;   // per slot: the sample index it reads
    const uint64_t *noff;  // per slot: name offsets (m + 1)
    const char *names;
    uint32_t *scratch;     // per wave: scap sample starts (relative to S)
    uint32_t m, scap;      // slots; sample starts a line needs (max index + 1)
    int seq, kind;
    uint32_t sel_lds;      // k_ac_fmt: the selection (eff, name offsets, names) copied to LDS (its bytes; 0: read from global memory)
    uint32_t ident;        // k_ac_fmt: eff[i] == i for every slot (no index array in LDS)
    uint32_t direct;       // text rows: k_ac_rows writes the records ac_direct_rec accepts (k_ac_fmt skips them)
    uint32_t ntile;        // direct: tiles per record in the nibble array (ceil(m / 64), 8 dwords each)
};

// the direct rows (k_ac_rows): a fixed-stride record whose prefix is 16..64 bytes, under a text
// selection whose names all have one length L <= 11 (the host's check, A.direct)
constexpr uint32_t kAcDirectP = 64;
__device__ __forceinline__ bool ac_direct_rec(const AcArgs &A, const AcMeta &m) {
    return A.direct && m.kind == kAcFast && m.P >= 16 && m.P <= kAcDirectP;
}

struct AcNullOp {
    __device__ void begin(uint32_t, uint32_t) {}
    __device__ bool done() const { return false; }
    __device__ void dword(const DwordView &) {}
    __device__ void finish() {}
};

__device__ __forceinline__ uint32_t dec_digits(uint64_t v) {
    uint32_t d = 1;
    while (v >= 10) {
        v /= 10;
        d++;
    }
    return d;
}
__device__ __forceinline__ uint32_t int_bytes(int64_t v) { return v < 0 ? 1u + dec_digits((uint64_t)(-v)) : dec_digits((uint64_t)v); }

// parseGenotypeRaw over [g, e)
__device__ __forceinline__ void ac_parse(const char *__restrict__ buf, int64_t g, int64_t e, int &r, int &a) {
    r = a = 0;
    uint32_t v = 0;
    bool dig = false;
    for (int64_t p = g; p <= e; p++) {
        const uint32_t c = p < e ? byte_at(buf, p) : (uint32_t)'/';
        if (c - '0' < 10u) {
            v = v * 10u + (c - '0');
            dig = true;
        } else {
            if (dig) {
                if (v == 0u) r++;
                else a++;
            }
            dig = false;
            v = 0u;
        }
    }
}

// the GT of the sample starting at st: up to its first ':' or tab (or the line end)
__device__ __forceinline__ void ac_sample(const char *__restrict__ buf, int64_t st, int64_t le, int &r, int &a) {
    int64_t e = st;
    while (e < le) {
        const uint32_t c = byte_at(buf, e);
        if (c == ':' || c == '\t') break;
        e++;
    }
    ac_parse(buf, st, e, r, a);
}

// the line's sample starts in [S, le] into the wave's table: tab[k] = start of sample k - S
// for k < min(ns, scap), sample 0 at S and one after every tab (a trailing tab's sample starts
// at le); returns ns capped at scap
__device__ __forceinline__ uint32_t ac_starts(const char *__restrict__ buf, int64_t S, int64_t le, uint32_t *tab,
                                              uint32_t scap) {
    if (lane() == 0) tab[0] = 0u;
    uint32_t cnt = 0;  // tabs seen (wave-uniform)
    for (int64_t w = S & ~(int64_t)15; w < le && cnt + 1 < scap; w += kWaveStep) {
        const int64_t blk = w + (int64_t)lane() * kBlockBytes;
        uint32_t tm = blk < le ? eq_mask16(load16(buf, blk), kRepTab) & range_mask16(blk, S, le) : 0u;
        const uint32_t c = (uint32_t)__popc(tm);
        const uint32_t incl = wave_incl_scan(c);
        uint32_t k = cnt + incl - c + 1;
        while (tm) {
            const int j = __builtin_ctz(tm);
            tm &= tm - 1u;
            if (k < scap) tab[k] = (uint32_t)(blk + j + 1 - S);
            k++;
        }
        cnt += wave_bcast(incl, kWave - 1);
    }
    // the table is read back by other lanes of the wave (through a fresh L1)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t ns = cnt + 1;
    return ns < scap ? ns : scap;
}

// slot counts on the general path for sample e (ns = ac_starts' count): valid = the slot
// produces a row (seq: its sample starts before the line end; all: always, 0 / 0 past the
// last sample)
__device__ __forceinline__ void ac_slot_general(const char *__restrict__ buf, int64_t S, int64_t le, const uint32_t *tab,
                                                uint32_t ns, uint32_t e, bool seq, bool &valid, int &r, int &a) {
    r = a = 0;
    const bool has = e < ns;
    const int64_t st = has ? S + tab[e] : le;
    valid = seq ? st < le : true;
    if (has) ac_sample(buf, st, le, r, a);
}

// slot counts on the fixed-stride path: sample e's GT is the 3 bytes at S + 4e
__device__ __forceinline__ void ac_slot_fast(const char *__restrict__ buf, int64_t S, uint32_t ns, uint32_t e, int &r,
                                             int &a) {
    r = a = 0;
    if (e < ns) {
        const uint32_t c0 = byte_at(buf, S + 4 * (int64_t)e), c2 = byte_at(buf, S + 4 * (int64_t)e + 2);
        r = (c0 == '0') + (c2 == '0');
        a = (c0 - '1' < 9u) + (c2 - '1' < 9u);
    }
}

__global__ __launch_bounds__(kAcThreads) void k_ac_len(const char *__restrict__ buf, int64_t data_start,
                                                       const uint64_t *__restrict__ line_end, uint64_t l0, uint64_t l1,
                                                       AcArgs A, uint8_t *__restrict__ status, uint64_t *__restrict__ len,
                                                       AcMeta *__restrict__ meta,
                                                       unsigned long long *__restrict__ counters) {
    __shared__ int64_t scratch[kAcWaves][16];
    __shared__ unsigned long long red[5][kAcWaves];
    int64_t *lds = scratch[threadIdx.x / kWave];
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t *tab = A.scratch + wid * (uint64_t)A.scap;
    unsigned long long rows_all = 0;
    uint32_t data = 0, chrom = 0, gen = 0, slow = 0;  // (wave-uniform)
    for (uint64_t li = l0 + wid; li < l1; li += nw) {
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
        uint8_t st = 0;
        uint64_t L = 0;
        AcMeta m{};
        if (le > ls) {
            if (byte_at(buf, ls) == '#') {
                const bool c = le - ls >= 6 && byte_at(buf, ls + 1) == 'C' && byte_at(buf, ls + 2) == 'H' &&
                               byte_at(buf, ls + 3) == 'R' && byte_at(buf, ls + 4) == 'O' && byte_at(buf, ls + 5) == 'M';
                st = c ? 4 : 0;
                chrom += c;
            } else {
                st = 1;
                data++;
                int64_t t[9];
                const int nt = head_tabs(buf, ls, le, 9, t, lds);
                m.P = nt >= 5 ? (uint32_t)(t[4] - ls + 1) : (uint32_t)(le - ls) + (uint32_t)(5 - nt);
                m.lim = nt >= 5 ? m.P : (uint32_t)(le - ls);
                const int64_t S = nt >= 9 ? t[8] + 1 : le;
                m.S = (uint64_t)S;
                AcNullOp nop;
                const bool fast = S < le && gt_fast(buf, S, le, nop);
                uint32_t rows = 0;
                uint64_t text = 0, sr = 0, sa = 0;
                if (fast) {
                    m.kind = kAcFast;
                    const uint32_t ns = (uint32_t)((le - S + 1) / 4);
                    m.ns = ns;
                    if (A.kind != 1 && (!A.seq || A.ident)) {
                        // no per-slot work: every slot is a row, or (seq, slot i reads sample i)
                        // the slots below the record's sample count
                        rows = A.seq ? min(A.m, ns) : A.m;
                    } else {
                        uint32_t cnt = 0;
                        for (uint32_t i = lane(); i < A.m; i += kWave) {
                            const uint32_t e = A.eff[i];
                            const bool valid = !A.seq || e < ns;
                            cnt += valid;
                            if (A.kind == 1 && valid) {
                                int r, a;
                                ac_slot_fast(buf, S, ns, e, r, a);
                                sr += (uint64_t)r;
                                sa += (uint64_t)a;
                            }
                        }
                        rows = wave_sum(cnt);
                    }
                    if (A.kind == 0) text = (uint64_t)rows * (m.P + 5u) + A.noff[rows];
                } else {
                    m.kind = kAcGeneral;
                    gen++;
                    const uint32_t nsa = ac_starts(buf, S, le, tab, A.scap);
                    uint32_t cnt = 0;
                    for (uint32_t i = lane(); i < A.m; i += kWave) {
                        const uint32_t e = A.eff[i];
                        bool valid;
                        int r, a;
                        ac_slot_general(buf, S, le, tab, nsa, e, A.seq, valid, r, a);
                        if (!valid) continue;
                        cnt++;
                        if (A.kind == 0) {
                            const int pr = A.seq ? r : (int)(int8_t)r, pa = A.seq ? a : (int)(int8_t)a;
                            text += m.P + (A.noff[i + 1] - A.noff[i]) + 3u + int_bytes(pr) + int_bytes(pa);
                        } else if (A.kind == 1) {
                            sr += (uint64_t)r;
                            sa += (uint64_t)a;
                        }
                    }
                    rows = wave_sum(cnt);
                    text = wave_sum(text);
                }
                m.rows = rows;
                slow += !ac_direct_rec(A, m);  // (k_ac_nib then packs the direct records' counts)
                if (A.kind == 1) {
                    sr = wave_sum(sr);
                    sa = wave_sum(sa);
                    m.sr = sr;
                    m.sa = sa;
                    text = m.P + dec_digits(sr) + dec_digits(sa) + dec_digits(rows) + 3u;
                } else if (A.kind == 2)
                    text = 2ull * rows;
                L = text;
                rows_all += A.kind == 1 ? 1u : rows;
            }
        }
        if (lane() == 0) {
            status[li] = st;
            len[li - l0] = L;
            meta[li] = m;
        }
    }
    if (lane() == 0) {
        red[0][threadIdx.x / kWave] = rows_all;
        red[1][threadIdx.x / kWave] = data;
        red[2][threadIdx.x / kWave] = chrom;
        red[3][threadIdx.x / kWave] = gen;
        red[4][threadIdx.x / kWave] = slow;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        unsigned long long t = 0;
        for (int k = 0; k < kAcWaves; k++) t += red[threadIdx.x][k];
        if (t) atomicAdd(&counters[threadIdx.x], t);
    }
}

// writes the decimal text of v (bytes already known) at o
__device__ __forceinline__ void put_int(char *o, int64_t v, uint32_t nb) {
    uint64_t x = v < 0 ? (uint64_t)(-v) : (uint64_t)v;
    if (v < 0) o[0] = '-';
    for (uint32_t k = nb; k-- > (v < 0 ? 1u : 0u);) {
        o[k] = (char)('0' + x % 10);
        x /= 10;
    }
}

// kSel: the selection sits in LDS (A.sel_lds != 0).  A compile-time choice: with both forms in one
// body the tile loop's name offsets came from an LDS read or a global load, and the join waited
// vmcnt(0) every tile -- on the previous tile's stores (loads and stores share vmcnt)
template <bool kSel>
__global__ __launch_bounds__(kAcThreads) void k_ac_fmt(const char *__restrict__ buf, int64_t data_start,
                                                       const uint64_t *__restrict__ line_end, uint64_t l0, uint64_t l1,
                                                       AcArgs A, const uint8_t *__restrict__ status,
                                                       const AcMeta *__restrict__ meta, const uint64_t *__restrict__ off,
                                                       char *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) char tile_all[kAcWaves][kAcTile + 16];
    __shared__ char pre_all[kAcWaves][kAcPre];
    // the selection in LDS when it fits (the text rows read a slot's sample index, name offset and
    // name bytes for every row: LDS reads instead of chains of dependent global loads)
    extern __shared__ __attribute__((aligned(16))) char sel_all[];
    uint32_t *s_eff = reinterpret_cast<uint32_t *>(sel_all), *s_noff = s_eff + (A.ident ? 0u : A.m);
    char *s_names = reinterpret_cast<char *>(s_noff + A.m + 1);
    if (kSel) {
        for (uint32_t k = threadIdx.x; k <= A.m; k += blockDim.x) {
            if (k < A.m && !A.ident) s_eff[k] = A.eff[k];
            s_noff[k] = (uint32_t)A.noff[k];
        }
        for (uint64_t k = threadIdx.x; k < A.noff[A.m]; k += blockDim.x) s_names[k] = A.names[k];
        __syncthreads();
    }
    auto EFF = [&](uint32_t i) -> uint32_t { return A.ident ? i : kSel ? s_eff[i] : A.eff[i]; };
    auto NOFF = [&](uint32_t i) -> uint64_t { return kSel ? (uint64_t)s_noff[i] : A.noff[i]; };
    auto NAME = [&](uint64_t k) -> char { return kSel ? s_names[k] : A.names[k]; };
    char *tile = tile_all[threadIdx.x / kWave];
    char *pre = pre_all[threadIdx.x / kWave];
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    uint32_t *tab = A.scratch + wid * (uint64_t)A.scap;
    for (uint64_t li = l0 + wid; li < l1; li += nw) {
        if (status[li] != 1) continue;  // (wave-uniform)
        const int64_t ls = li ? (int64_t)line_end[li - 1] + 1 : data_start, le = (int64_t)line_end[li];
        const AcMeta m = meta[li];
        if (ac_direct_rec(A, m)) continue;  // (k_ac_rows' record)
        char *o = out + off[li - l0];
        const int64_t S = (int64_t)m.S;
        const uint32_t P = m.P;
        auto pre_byte = [&](uint32_t k) -> char { return k < m.lim ? buf[ls + k] : '\t'; };
        if (A.kind == 1) {  // aggregate: one row
            if (lane() == 0) {
                for (uint32_t k = 0; k < P; k++) o[k] = pre_byte(k);
                uint32_t p = P, nb = dec_digits(m.sr);
                put_int(o + p, (int64_t)m.sr, nb);
                p += nb;
                o[p++] = '\t';
                nb = dec_digits(m.sa);
                put_int(o + p, (int64_t)m.sa, nb);
                p += nb;
                o[p++] = '\t';
                nb = dec_digits(m.rows);
                put_int(o + p, (int64_t)m.rows, nb);
                p += nb;
                o[p] = '\n';
            }
            continue;
        }
        const uint32_t nsa = m.kind == kAcGeneral ? ac_starts(buf, S, le, tab, A.scap) : 0u;
        if (A.kind == 2) {  // binary: two int8 bytes per row
            for (uint32_t i = lane(); i < m.rows; i += kWave) {
                int r, a;
                bool valid;
                if (m.kind == kAcFast) ac_slot_fast(buf, S, m.ns, A.eff[i], r, a);
                else ac_slot_general(buf, S, le, tab, nsa, A.eff[i], A.seq, valid, r, a);
                o[2 * i] = (char)(int8_t)r;
                o[2 * i + 1] = (char)(int8_t)a;
            }
            continue;
        }
        if (m.kind == kAcGeneral || P > kAcPre) {
            // any layout: a lane per row, rows placed by a wave scan of their bytes
            uint64_t run = 0;
            for (uint32_t i0 = 0; i0 < m.rows; i0 += kWave) {
                const uint32_t i = i0 + lane();
                int r = 0, a = 0;
                uint32_t nb = 0, br = 0, ba = 0;
                if (i < m.rows) {
                    bool valid;
                    if (m.kind == kAcFast) ac_slot_fast(buf, S, m.ns, A.eff[i], r, a);
                    else ac_slot_general(buf, S, le, tab, nsa, A.eff[i], A.seq, valid, r, a);
                    if (!A.seq) {
                        r = (int8_t)r;
                        a = (int8_t)a;
                    }
                    br = int_bytes(r);
                    ba = int_bytes(a);
                    nb = P + (uint32_t)(A.noff[i + 1] - A.noff[i]) + 3u + br + ba;
                }
                const uint64_t incl = wave_incl_scan((uint64_t)nb);
                if (i < m.rows) {
                    char *q = o + run + incl - nb;
                    for (uint32_t k = 0; k < P; k++) q[k] = pre_byte(k);
                    q += P;
                    for (uint64_t k = A.noff[i]; k < A.noff[i + 1]; k++) *q++ = A.names[k];
                    *q++ = '\t';
                    put_int(q, r, br);
                    q += br;
                    *q++ = '\t';
                    put_int(q, a, ba);
                    q[ba] = '\n';
                }
                run += wave_bcast(incl, kWave - 1);
            }
            continue;
        }
        // fixed-stride text rows: P + name + 5 bytes each; the prefix staged once in LDS
        for (uint32_t k = lane(); k < P; k += kWave) pre[k] = pre_byte(k);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t rl = P + 5u;
        // the counts of 32 tiles at a time (a nibble r | a << 2 per tile in pk0 / pk1), loaded
        // before any of those tiles' rows is stored: a count loaded between two tiles' stores made
        // every tile wait for the previous tile's stores (loads and stores share vmcnt, and the
        // varying store count leaves the compiler vmcnt(0))
        uint64_t pk0 = 0, pk1 = 0;
        bool lo_valid = false;  // tile[0, ga & 15) holds the previous tile's last partial block
        for (uint32_t i0 = 0; i0 < m.rows; i0 += kWave) {
            const uint32_t i1 = min(m.rows, i0 + (uint32_t)kWave);
            const uint64_t g0 = (uint64_t)i0 * rl + NOFF(i0);                // tile start in the line's text
            const uint64_t B = (uint64_t)(i1 - i0) * rl + NOFF(i1) - NOFF(i0);  // tile bytes
            const uint32_t i = i0 + lane();
            const uint32_t t = i0 / kWave;
            if ((t & 31) == 0) {
                pk0 = pk1 = 0;
#pragma unroll 4
                for (uint32_t kk = 0; kk < 32; kk++) {
                    const uint32_t ii = i + kk * kWave;
                    uint32_t nib = 0;
                    if (ii < m.rows) {
                        int rr, aa;
                        ac_slot_fast(buf, S, m.ns, EFF(ii), rr, aa);
                        nib = (uint32_t)rr | ((uint32_t)aa << 2);
                    }
                    if (kk < 16) pk0 |= (uint64_t)nib << (4 * kk);
                    else pk1 |= (uint64_t)nib << (4 * (kk - 16));
                }
            }
            const uint32_t nib = (uint32_t)(((t & 16) ? pk1 : pk0) >> (4 * (t & 15))) & 15u;
            const int r = (int)(nib & 3u), a = (int)(nib >> 2);
            const uint64_t ga = (uint64_t)(o - out) + g0;  // absolute text offset of the tile
            const uint64_t lo = lo_valid ? (ga & ~(uint64_t)15) : ga;  // first byte this tile stores
            if (B + 32 > (uint64_t)kAcTile) {             // long names: straight to global memory
                if (lo_valid && (uint32_t)lane() < (uint32_t)(ga - lo)) out[lo + lane()] = tile[lane()];  // the carry
                lo_valid = false;
                if (i < i1) {
                    char *q = o + (uint64_t)i * rl + NOFF(i);
                    for (uint32_t k = 0; k < P; k++) q[k] = pre[k];
                    q += P;
                    for (uint64_t k = NOFF(i); k < NOFF(i + 1); k++) *q++ = NAME(k);
                    q[0] = '\t';
                    q[1] = (char)('0' + r);
                    q[2] = '\t';
                    q[3] = (char)('0' + a);
                    q[4] = '\n';
                }
                continue;
            }
            const uint32_t sh = (uint32_t)(ga & 15);  // LDS position = text position mod 16
            if (i < i1 && !(VCFXG_AC_EXPT & 1)) {
                char *q = tile + sh + ((uint64_t)i * rl + NOFF(i) - g0);
                for (uint32_t k = 0; k < P; k++) q[k] = pre[k];
                q += P;
                for (uint64_t k = NOFF(i), ke = NOFF(i + 1); k < ke; k++) *q++ = NAME(k);
                q[0] = '\t';
                q[1] = (char)('0' + r);
                q[2] = '\t';
                q[3] = (char)('0' + a);
                q[4] = '\n';
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // copy out: the aligned 16 B blocks of [lo, ga + B); a tile's last partial block is
            // not stored but carried to the front of the next tile's LDS image (text position mod
            // 16 again), so only the record's first and last blocks take byte stores (a block
            // holding another record's bytes is never written whole)
            const uint64_t a0 = ga & ~(uint64_t)15, aend = ga + B;
            const bool last = i1 == m.rows;
            const uint64_t cend = last ? aend : (aend & ~(uint64_t)15);
            for (uint64_t blk = a0 + 16ull * lane(); blk < cend && !(VCFXG_AC_EXPT & 2); blk += 16ull * kWave) {
                const char *src = tile + (blk - a0);
                if (blk >= lo && blk + 16 <= cend)
                    *reinterpret_cast<v4u *>(out + blk) = *reinterpret_cast<const v4u *>(src);
                else
                    for (int k = 0; k < 16; k++)
                        if (blk + k >= lo && blk + k < cend) out[blk + k] = src[k];
            }
            __builtin_amdgcn_wave_barrier();  // the tile is rewritten by the next iteration
            lo_valid = !last;
            if (!last) {  // the carry: bytes [cend, aend) to the front
                const uint32_t nc = (uint32_t)(aend - cend);
                const uint32_t cv = (uint32_t)lane() < nc ? (uint32_t)(uint8_t)tile[(cend - a0) + lane()] : 0u;
                __builtin_amdgcn_wave_barrier();
                if ((uint32_t)lane() < nc) tile[lane()] = (char)cv;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
    }
}

// k_ac_nib: k_ac_rows' counts, for the records ac_direct_rec accepts (k_ac_len's meta), a wave per
// line.  A kernel of its own: inside k_ac_len (149 VGPRs, 3 waves per SIMD) the pass cost 1.5 ms,
// latency-bound per record; here a wave holds 4 groups' loads with few registers.
constexpr int kAcNibThreads = 256;
__global__ __launch_bounds__(kAcNibThreads) void k_ac_nib(const char *__restrict__ buf, uint64_t l0, uint64_t l1,
                                                          AcArgs A, const AcMeta *__restrict__ meta,
                                                          uint32_t *__restrict__ nib) {
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    for (uint64_t lv = l0 + wid; lv < l1; lv += nw) {
        const uint64_t li = (uint64_t)uniform64((int64_t)lv);
        AcMeta m;
        {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(meta + li);
            m.S = (uint64_t)w[0] | (uint64_t)w[1] << 32;
            m.P = w[6];
            m.rows = w[7];
            m.ns = w[8];
            m.lim = w[9];
            m.kind = (uint8_t)w[10];
        }
        const uint32_t rows = (uint32_t)__builtin_amdgcn_readfirstlane((int)m.rows);
        if (!ac_direct_rec(A, m) || rows == 0) continue;
        const int64_t S = (int64_t)m.S;
        // k_ac_rows' counts: per tile of 64 rows 8 dwords, row i's nibble r | a << 2 at
        // bits 4 (i & 7) of dword (i & 63) / 8 (a lane past the last row: the last row's).
        // A lane makes one dword, rows 8 k .. 8 k + 7 of 512 (8 tiles' dwords are
        // contiguous: dword 8 t + j of the record is rows 64 t + 8 j ..): 8 loads, then a
        // store, no cross-lane step
        uint32_t *nb = nib + (li - l0) * (uint64_t)A.ntile * 8u;
        const uint32_t ns = m.ns;
        auto nib8 = [](const v4u &u) -> uint32_t {  // 4 GT dwords -> 4 nibbles
            uint32_t x = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t c0 = u[q] & 255u, c2 = (u[q] >> 16) & 255u;
                const uint32_t r = (c0 == '0') + (c2 == '0'), a = (c0 - '1' < 9u) + (c2 - '1' < 9u);
                x |= (r | a << 2) << (4 * q);
            }
            return x;
        };
        // the identity selection over whole groups of 512 rows below the sample count:
        // a lane's 8 GT dwords are 32 contiguous bytes, 4 groups' loads in flight at once
        const uint32_t full = A.ident ? min(rows, ns) / (8 * kWave) * (8 * kWave) : 0u;
        uint32_t r0 = 0;
        for (; r0 + 4 * 8 * kWave <= full; r0 += 4 * 8 * kWave) {
            v4u u[8];
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const char *p = buf + S + 4 * (uint64_t)(r0 + h * 8 * kWave + 8u * lane());
                __builtin_memcpy(&u[2 * h], p, 16);  // (unaligned)
                __builtin_memcpy(&u[2 * h + 1], p + 16, 16);
            }
#pragma unroll
            for (int h = 0; h < 4; h++)
                nb[(r0 + h * 8 * kWave) / 8u + lane()] = nib8(u[2 * h]) | nib8(u[2 * h + 1]) << 16;
        }
        for (; r0 < rows; r0 += 8 * kWave) {
            const uint32_t b = r0 + 8u * lane();
            uint32_t g[8], ev[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t i = min(b + q, rows - 1);
                ev[q] = A.ident ? i : A.eff[i];
                g[q] = __hip_atomic_load(
                    reinterpret_cast<const uint32_t *>(buf + S + 4 * (uint64_t)(ev[q] < ns ? ev[q] : 0u)),
                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);  // (unaligned: S + 4 e)
            }
            uint32_t x = 0;
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const uint32_t gc = ev[q] < ns ? g[q] : 0u;  // (a slot past the samples: 0 / 0)
                const uint32_t c0 = gc & 255u, c2 = (gc >> 16) & 255u;
                const uint32_t r = (c0 == '0') + (c2 == '0'), a = (c0 - '1' < 9u) + (c2 - '1' < 9u);
                x |= (r | a << 2) << (4 * q);
            }
            if (b < ((rows + 63u) & ~63u)) nb[r0 / 8u + lane()] = x;  // (the last tile whole)
        }
    }
}

// k_ac_rows: the text rows of the records ac_direct_rec accepts, straight from registers to the
// output -- no LDS image, no copy-out.  Every row is P + L + 5 bytes: the record's prefix, the
// slot's name, "\t" r "\t" a "\n".  A lane per row writes it as unaligned 16 B stores:
//   prefix [0, 16) (and [16, 32), [32, 48) when P exceeds them), prefix [P - 16, P), and the
//   row's last 16 bytes: 11 - L prefix bytes, the name, '\t', r, '\t', a, '\n'.
// The pieces overlap only where they carry the same bytes, so their order does not matter, and
// none leaves the row (P >= 16).  The last piece comes from the slot's entry in LDS (etab: the
// name right-aligned before "\t0\t0\n", zeros in front), the record's prefix bytes ORed into
// its zeros and the counts into its last dword.
// The kernel issues no vector load: the record's metadata, prefix bytes and counts (k_ac_len's
// nibbles, 32 B a tile) come by scalar loads (lgkmcnt).  Vector loads and stores share vmcnt, so
// any vector load among the rows' stores waits for all of them: a load batch every 16 tiles made
// the same stores 8.9 -> 11.1 ms (tools/microbench/store_fronts.hip), and this kernel with its
// counts loaded per record 12.9 ms.  r02-r06 composed the rows in an LDS image and copied it
// out; the image's round trips, not the stores, bounded that kernel.
constexpr int kAcRowsThreads = 1024;  // 16 waves share one LDS copy of etab
constexpr int kAcRowsWaves = kAcRowsThreads / kWave;
#define AC_CONST __attribute__((address_space(4)))  // (uniform loads through it are scalar loads)
typedef unsigned int v8u __attribute__((ext_vector_type(8)));
typedef unsigned int v16u __attribute__((ext_vector_type(16)));
// (whole vectors: a select among the dwords of separate loads became one per-lane vector load)
__global__ __launch_bounds__(kAcRowsThreads, 8) void k_ac_rows(const char *__restrict__ buf, int64_t data_start,
                                                            const uint64_t *__restrict__ line_end, uint64_t l0,
                                                            uint64_t l1, AcArgs A, const v4u *__restrict__ etab,
                                                            uint32_t L, const uint32_t *__restrict__ nib,
                                                            const AcMeta *__restrict__ meta,
                                                            const uint64_t *__restrict__ off, char *__restrict__ out) {
    extern __shared__ v4u s_e[];  // (ac_rows_lds) the m entries
    __shared__ __attribute__((aligned(16))) uint32_t pre_all[kAcRowsWaves][(kAcDirectP + 16) / 4 + 4];
    for (uint32_t k = threadIdx.x; k < A.m; k += blockDim.x) s_e[k] = etab[k];
    __syncthreads();
    uint32_t *prew = pre_all[threadIdx.x / kWave];
    const uint64_t wid = (uint64_t)uniform64((int64_t)((blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave));
    const uint64_t nw = (gridDim.x * (uint64_t)blockDim.x) / kWave;
    const uint32_t kp = 11u - L;  // prefix bytes in an entry's front
    const uint32_t sub = lane() >> 3, shn = 4u * (lane() & 7u);  // this lane's nibble in a tile's 8 dwords
    for (uint64_t lv = l0 + wid; lv < l1; lv += nw) {
        const uint64_t li = (uint64_t)uniform64((int64_t)lv);  // (so that the loads below are scalar)
        AcMeta m;  // (its dwords: a byte field alone would be a vector load)
        {
            const v8u a = *(const AC_CONST v8u *)(meta + li);
            const v4u b = *(const AC_CONST v4u *)((const char *)(meta + li) + 32);
            m.S = (uint64_t)a[0] | (uint64_t)a[1] << 32;
            m.P = a[6];
            m.rows = a[7];
            m.ns = b[0];
            m.lim = b[1];
            m.kind = (uint8_t)b[2];
        }
        if (!ac_direct_rec(A, m)) continue;  // (every other line: k_ac_fmt or no row)
        const uint32_t R = m.rows;
        if (R == 0) continue;
        const int64_t ls = li ? (int64_t)*(const AC_CONST uint64_t *)(line_end + li - 1) + 1 : data_start;
        char *o = out + *(const AC_CONST uint64_t *)(off + li - l0);
        const uint32_t P = m.P, rl = P + L + 5u;
        // the prefix: 17 dwords from ls rounded down (P <= 64; the input has 256 zeroed bytes past
        // its end) into the wave's LDS, tabs for the fields the line lacks, then the pieces
        const AC_CONST uint32_t *pw = (const AC_CONST uint32_t *)(buf + (ls & ~(int64_t)3));
        const v16u pv = *(const AC_CONST v16u *)pw;
        uint32_t w = pw[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w = lane() == j ? pv[j] : w;
        if (lane() < 17) prew[lane()] = w;
        char *pre = reinterpret_cast<char *>(prew) + (ls & 3);
        if ((uint32_t)lane() >= m.lim && (uint32_t)lane() < P) pre[lane()] = '\t';
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        v4u c0v, c1, c2v, cl, pm;
        __builtin_memcpy(&c0v, pre, 16);
        __builtin_memcpy(&c1, pre + 16, 16);
        __builtin_memcpy(&c2v, pre + 32, 16);
        __builtin_memcpy(&cl, pre + P - 16, 16);
        __builtin_memcpy(&pm, pre + P - kp, 16);
        pm.x &= kp >= 4 ? ~0u : (1u << (8 * kp)) - 1u;
        pm.y &= kp >= 8 ? ~0u : kp <= 4 ? 0u : (1u << (8 * (kp - 4))) - 1u;
        pm.z &= kp <= 8 ? 0u : (1u << (8 * (kp - 8))) - 1u;  // (kp <= 11)
        const AC_CONST uint32_t *nt = (const AC_CONST uint32_t *)(nib + (li - l0) * (uint64_t)A.ntile * 8u);
        // kNp: the prefix pieces before [P - 16, P) (1: P <= 32, 2: P <= 48, 3: P <= 64); a loop per
        // count, so that no store in it is conditional; lanes past the last row repeat it (same
        // bytes to the same places; k_ac_len gave them its nibble)
        auto rows = [&](auto np) {
            constexpr int kNp = decltype(np)::value;
            for (uint32_t i0 = 0, t = 0; i0 < R; i0 += kWave, t++) {
                const v8u nd = *(const AC_CONST v8u *)(nt + 8u * t);
                uint32_t d = nd[0];
#pragma unroll
                for (int j = 1; j < 8; j++) d = sub == (uint32_t)j ? nd[j] : d;
                const uint32_t nb = (d >> shn) & 15u;
                const uint32_t i = min(i0 + (uint32_t)lane(), R - 1);
                char *q = o + (uint64_t)(i * rl);  // (a record's text is < 4 GiB)
                __builtin_memcpy(q, &c0v, 16);
                if (kNp > 1) __builtin_memcpy(q + 16, &c1, 16);
                if (kNp > 2) __builtin_memcpy(q + 32, &c2v, 16);
                __builtin_memcpy(q + P - 16, &cl, 16);
                v4u e = s_e[i];
                e.x |= pm.x;
                e.y |= pm.y;
                e.z |= pm.z;
                e.w = 0x0A000900u | ('0' + (nb & 3u)) | (('0' + (nb >> 2)) << 16);
                __builtin_memcpy(q + rl - 16, &e, 16);
            }
        };
        if (P <= 32) rows(std::integral_constant<int, 1>{});
        else if (P <= 48) rows(std::integral_constant<int, 2>{});
        else rows(std::integral_constant<int, 3>{});
        __builtin_amdgcn_wave_barrier();  // (the prefix buffer is rewritten by the next record)
    }
}
#undef AC_CONST

size_t ac_meta_bytes() { return sizeof(AcMeta); }

static AcArgs ac_args(const uint32_t *eff, const uint64_t *noff, const char *names, uint32_t *scratch, uint32_t m,
                      uint32_t scap, int seq, int kind, uint32_t sel_lds = 0, int ident = 0, int direct = 0) {
    // (direct: ntile for the nibble array)
    AcArgs A;
    A.ident = ident ? 1u : 0u;
    A.eff = eff;
    A.noff = noff;
    A.names = names;
    A.scratch = scratch;
    A.m = m;
    A.scap = scap;
    A.seq = seq;
    A.kind = kind;
    A.sel_lds = sel_lds;
    A.direct = direct ? 1u : 0u;
    A.ntile = (m + 63u) / 64u;
    return A;
}

hipError_t launch_ac_len(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                         unsigned blocks, const uint32_t *eff, const uint64_t *noff, const char *names,
                         uint32_t *scratch, uint32_t m, uint32_t scap, int seq, int kind, int ident, int direct,
                         uint32_t *nib, uint8_t *status, uint64_t *len, void *meta, unsigned long long *counters,
                         hipStream_t s) {
    if (l1 <= l0) return hipSuccess;
    if (direct && !nib) return hipErrorInvalidValue;
    const AcArgs A = ac_args(eff, noff, names, scratch, m, scap, seq, kind, 0, ident, direct);
    hipLaunchKernelGGL(k_ac_len, dim3(blocks), dim3(kAcThreads), 0, s, buf, data_start, line_end, l0, l1, A, status,
                       len, static_cast<AcMeta *>(meta), counters);
    if (direct) {
        const uint64_t w = (l1 - l0 + (kAcNibThreads / kWave) - 1) / (kAcNibThreads / kWave);
        hipLaunchKernelGGL(k_ac_nib, dim3((unsigned)std::min<uint64_t>(w, 8192)), dim3(kAcNibThreads), 0, s, buf, l0,
                           l1, A, static_cast<const AcMeta *>(meta), nib);
    }
    return hipGetLastError();
}

hipError_t launch_ac_fmt(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                         unsigned blocks, const uint32_t *eff, const uint64_t *noff, const char *names,
                         uint32_t *scratch, uint32_t m, uint32_t scap, int seq, int kind, uint32_t sel_lds,
                         int ident, int direct, const uint8_t *status, const void *meta, const uint64_t *off,
                         char *out, hipStream_t s) {
    if (l1 <= l0) return hipSuccess;
    const AcArgs A = ac_args(eff, noff, names, scratch, m, scap, seq, kind, sel_lds, ident, direct);
    if (sel_lds)
        hipLaunchKernelGGL(k_ac_fmt<true>, dim3(blocks), dim3(kAcThreads), sel_lds, s, buf, data_start, line_end, l0,
                           l1, A, status, static_cast<const AcMeta *>(meta), off, out);
    else
        hipLaunchKernelGGL(k_ac_fmt<false>, dim3(blocks), dim3(kAcThreads), 0, s, buf, data_start, line_end, l0, l1, A,
                           status, static_cast<const AcMeta *>(meta), off, out);
    return hipGetLastError();
}

hipError_t launch_ac_rows(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                          unsigned blocks, const uint32_t *eff, uint32_t m, int ident, const void *etab, uint32_t L,
                          const uint32_t *nib, const void *meta, const uint64_t *off, char *out, hipStream_t s) {
    if (l1 <= l0) return hipSuccess;
    const size_t lds = ac_rows_lds(m, ident);
    if (L > 11 || m > 4096 || lds > ac_rows_lds_max()) return hipErrorInvalidValue;
    const AcArgs A = ac_args(eff, nullptr, nullptr, nullptr, m, 0, 0, 0, 0, ident, 1);
    hipLaunchKernelGGL(k_ac_rows, dim3(blocks), dim3(kAcRowsThreads), lds, s, buf, data_start, line_end, l0, l1,
                       A, static_cast<const v4u *>(etab), L, nib, static_cast<const AcMeta *>(meta), off, out);
    return hipGetLastError();
}

size_t ac_rows_lds(uint32_t m, int) { return 16 * (size_t)m; }
size_t ac_rows_lds_max() { return 131072; }
int ac_rows_threads() { return kAcRowsThreads; }
int ac_threads() { return kAcThreads; }

}  // namespace vcfxg
