// vcfxg_kernels.h -- host-visible launchers of the record kernels (vcfxg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcfxg {

// per-line head summary shared by the AF / GQ head passes (k_line_meta, k_af_combine)
enum : uint8_t { kMetaEmpty = 0, kMetaGt = 1, kMetaFull = 2, kMetaHeader = 3, kMetaGated = 4 };
struct LineMeta {
    uint64_t S;       // sample region start (kMetaGt)
    uint32_t rowpre;  // bytes of "CHROM\tPOS\tID\tREF\tALT\t" (kMetaGt)
    uint8_t kind;     // kMeta*: empty (after the '\r' strip), GT-first data line, full
                      // per-line path, '#' line, gated out (fused RF|GQ: RF dropped it)
    uint8_t sep;      // byte at S + 1 (kMetaGt)
    uint8_t cr;       // a trailing '\r' was stripped
    uint8_t pad;
};
constexpr uint8_t kAfPending = 0xFF;  // AF status of a kMetaGt line whose fast sweep failed
constexpr uint8_t kGqPending = 0xFE;  // GQ: a kMetaGt line whose fast sweep failed (general sweep)
constexpr uint8_t kRfPending = 0xFD;  // RF walk: head beyond the window (k_fq_finish filters it)
constexpr uint8_t kGqFull = 0xFC;     // GQ walk: a kMetaFull line for k_gq_complex's gq_line
// HWE walk: LineMeta::pad of a kMetaGt line -- ALT holds a ',' / CHROM, POS or ALT is empty
constexpr uint8_t kHweAltComma = 1, kHweEmptyField = 2;
// dosage HEAD walk: LineMeta::pad of a GT-only record taken on its predicted end, unswept
constexpr uint8_t kWalkUnswept = 4;

// single-sweep index over 16 KiB wave-chunks (idx_wchunks of them): counts + the first
// idx_pos_cap() newline offsets per chunk, then a compaction into line_end (overflow != 0:
// some chunk needs the emit sweep launch_idx_emit instead)
int idx_pos_cap();
// BGZF members inflated on the device (vcfxg_inflate.hip): one wave per member into
// out + out_off[m]; mstat[m] = 0 or the first failing check, *first_bad = the lowest bad member
// (initialise to ~0); then each member's CRC-32 against its trailer.  z1k: the images of the 32
// CRC register bits through 1 KiB of zero bytes (crc32_zero1k_basis).
struct BgzfMember {  // = vcfxg_bgzf_member
    uint64_t src_off;
    uint32_t src_len;
    uint32_t out_len;
};
struct Crc1k {
    uint32_t v[32];
};
void crc32_zero1k_basis(Crc1k *z);
// the lane decoder's side stream (the hand-overs') and the events that join it
struct InflateSide {
    hipStream_t aux = nullptr;
    hipEvent_t ev[2] = {};  // decoded, hand-overs done
};
// which: 0 = the inflate (k_inflate_decode; k_inflate_handover, the wave decoder on the members the
// lane decoder hands over, on side->aux beside k_inflate_copy), 1 = k_crc32.  first_bad[0]: the
// first bad member; the 32-bit word after it counts the hand-overs.
hipError_t launch_inflate(int which, const uint8_t *comp, const BgzfMember *mem, const uint64_t *out_off,
                          uint64_t n_members, uint8_t *out, uint32_t *mstat, unsigned long long *first_bad,
                          const Crc1k &z1k, hipStream_t s, uint64_t mbase = 0, uint32_t *tok = nullptr,
                          uint64_t tok_members = 0, const uint32_t *perm = nullptr, const InflateSide *side = nullptr);
// the lane decoder's token buffer: kTokCap 32-bit slots per member, tok_members members (launches
// of more members run in pieces), then the hand-over list of tok_members + 1 words; perm: the
// members in the order the lanes take them (largest compressed first: a wave's lanes then decode
// similar amounts).  No side: every member on the wave decoder.
constexpr uint32_t kTokCap = 6144;
// occurrences of `byte` in buf[lo, hi) added to *out (k_count_byte)
hipError_t launch_count_byte(const uint8_t *buf, uint64_t lo, uint64_t hi, uint8_t byte, unsigned long long *out,
                             hipStream_t s);
int64_t idx_wchunks(int64_t lo, int64_t hi);
hipError_t launch_idx_count(const char *buf, int64_t lo, int64_t hi, uint32_t *counts, uint64_t *pos,
                            unsigned *overflow, hipStream_t s);
hipError_t launch_idx_emit(const char *buf, int64_t lo, int64_t hi, const uint64_t *offs, uint64_t *line_end,
                           hipStream_t s);
hipError_t launch_nl_compact(int64_t lo, int64_t hi, const uint32_t *counts, const uint64_t *offs, const uint64_t *pos,
                             uint64_t *line_end, hipStream_t s);
hipError_t launch_af_records(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, int32_t *alt, int32_t *tot, uint32_t *rowpre,
                             uint8_t *status, unsigned long long *counters, hipStream_t s);
// AF head pass (k_af_meta, meta = af_meta_bytes() per line) + sample sweep (k_af_sweep)
size_t af_meta_bytes();
hipError_t launch_af_meta_sweep(const char *buf, int64_t data_start, const uint64_t *line_end,
                                const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, void *meta, int32_t *alt,
                                int32_t *tot, uint32_t *rowpre, uint8_t *status, unsigned long long *counters,
                                hipStream_t s);
hipError_t launch_af_meta_sweep_range(const char *buf, int64_t data_start, const uint64_t *line_end,
                                      const uint64_t *range, uint64_t max_lines, int mode, void *meta, int32_t *alt,
                                      int32_t *tot, uint32_t *rowpre, uint8_t *status, unsigned long long *counters,
                                      hipStream_t s);
int64_t idx_wchunk_bytes();
// AF record pass without a separate index (vcfxg_af_walk.hip): one wave per `chunk` bytes
// walks its lines (predicted fixed-stride ends validated by the sweep); per-walker regions
// of cap_w lines, then k_walk_compact (offs = exclusive scan of wcount)
int64_t af_walkers(int64_t lo, int64_t hi, int64_t chunk);
// the AF walk's region tail (all null: the walk only fills its regions): per walker its row
// bytes (GT lines) and first line start, and the list of region slots left to the exact
// per-line path (kMetaFull lines, GT lines off the fixed-stride sweep)
struct WalkTail {
    uint64_t *wtext = nullptr;
    uint64_t *wstart = nullptr;
    uint64_t *cx_list = nullptr;
    unsigned long long *cx_n = nullptr;
    uint64_t cx_cap = 0;
    // AF: each walker's rows as text, composed by the walk itself into its stage_cap bytes of
    // stage (k_af_format_w then copies them out whole); wdirty[w] = 1 when the walker left a
    // line to k_af_cx or its rows outgrew its stage (its rows are formatted from the arrays)
    char *stage = nullptr;
    uint32_t stage_cap = 0;
    uint8_t *wdirty = nullptr;
};
hipError_t launch_af_walk(const char *buf, int64_t lo, int64_t hi, int64_t chunk, int mode, int64_t span0,
                          uint64_t cap_w, uint64_t *le_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b,
                          uint8_t *status_b, void *meta_b, uint64_t *wcount, uint32_t *wgt, unsigned *overflow,
                          hipStream_t s, int32_t *hwe_aux_b = nullptr, const WalkTail *tail = nullptr,
                          bool dose = false, bool gt_first_walk = false, bool dose_head = false);
// AF region tail without the dense per-line arrays (vcfxg_kernels.hip):
//   launch_af_cx       the walk's leftover slots: af_line / the general sweep, new rows' bytes
//                      added to their walker's total (counters as k_af_complex)
//   launch_walker_scan one block: exclusive scans of the walkers' line counts and row bytes,
//                      GT-line totals into counters[0..1], the line count to *n_lines and the
//                      7-value call summary (lines, text bytes, counters[0..3], *fail); with
//                      reset: summary[7] = reset[1] (the leftover count), then reset[0..5] = 0
//   launch_af_format_w one wave per walker region: rows into out (rows ending past cap skipped)
hipError_t launch_af_cx(const char *buf, int mode, uint64_t cap_w, const uint64_t *list, const unsigned long long *list_n,
                        uint64_t list_cap, uint64_t list_cap_host, const uint64_t *wstart, const uint64_t *le_b,
                        const void *meta_b, int32_t *alt_b, int32_t *tot_b, uint32_t *rowpre_b, uint8_t *status_b,
                        uint64_t *wtext, unsigned long long *counters, hipStream_t s);
// walker offsets are block-local: woff[w] + bpre[w / kWalkerScanBlock] (bsum: 3 per block,
// bpre_*: blocks + 1 entries; *done zero before the launch)
constexpr int kWalkerScanBlock = 1024;
hipError_t launch_walker_scan(int64_t nw, const uint64_t *wcount, const uint64_t *wtext, const uint32_t *wgt,
                              uint64_t *woff, uint64_t *wtoff, uint64_t *bpre_a, uint64_t *bpre_b, uint64_t *bsum,
                              unsigned *done, unsigned long long *counters, const unsigned *fail, uint64_t *n_lines,
                              uint64_t *summary, hipStream_t s, uint64_t *reset = nullptr);
hipError_t launch_af_format_w(const char *buf, int mode, int64_t nw, uint64_t cap_w, const uint64_t *wcount,
                              const uint64_t *wtoff, const uint64_t *bpre_b, const uint64_t *wstart,
                              const uint64_t *le_b, const int32_t *alt_b, const int32_t *tot_b, const uint32_t *rowpre_b,
                              const uint8_t *status_b, char *out, uint64_t cap, hipStream_t s, const WalkTail *tail = nullptr);
hipError_t launch_walk_compact(int64_t n_walkers, uint64_t cap_w, const uint64_t *offs, const uint32_t *wgt,
                               const uint64_t *le_b, const int32_t *alt_b, const int32_t *tot_b,
                               const uint32_t *rowpre_b, const uint8_t *status_b, const void *meta_b,
                               uint64_t *line_end, int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                               void *meta, uint64_t *n_lines, unsigned long long *counters, hipStream_t s,
                               const int32_t *aux_b = nullptr, int32_t *aux = nullptr, const uint64_t *bpre = nullptr);
hipError_t launch_af_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, const void *meta,
                             int32_t *alt, int32_t *tot, uint32_t *rowpre, uint8_t *status,
                             unsigned long long *counters, hipStream_t s);
// VCFX_nonref_filter per line (mode 0 mmap, 1 stdin): status 1 keep / 2 drop / 4 '#' / 0 empty;
// counters: [0] kept, [1] data lines, [3] lines off the fixed-stride sweep
// after the nonref walk: nr_line for the lines it left (kGqPending / kGqFull), counters as above
hipError_t launch_nr_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                             unsigned long long *counters, hipStream_t s);
hipError_t launch_nr_records(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                             unsigned long long *counters, hipStream_t s);
hipError_t launch_gq_records(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int strip_cr, const char *q_dev,
                             int qlen, int strict, int qa, int qb, uint8_t *status, unsigned long long *counters,
                             hipStream_t s, const uint8_t *gate, void *meta = nullptr);
// k_gq_complex alone (the query's general lines after the filter / query walk): lines of
// kind kMetaFull (gq_line) and kMetaGt lines with status kGqPending (general sweep)
hipError_t launch_gq_complex(const char *buf, int64_t data_start, const uint64_t *line_end,
                             const uint64_t *n_lines_dev, uint64_t n_lines_host, int strip_cr, const char *q_dev,
                             int qlen, int strict, int qa, int qb, const void *meta, uint8_t *status,
                             unsigned long long *counters, const uint8_t *gate, hipStream_t s);
// asynchronous AF region path: capacity-guarded compaction, device-side line count and
// a one-record summary for the single host synchronisation
hipError_t launch_nl_compact_cap(int64_t lo, int64_t hi, const uint32_t *counts, const uint64_t *offs,
                                 const uint64_t *pos, uint64_t *line_end, uint64_t cap, hipStream_t s);
hipError_t launch_idx_finish(const uint64_t *offs, int64_t nchunks, const unsigned *idx_overflow, int tail, int64_t hi,
                             uint64_t cap, uint64_t *line_end, uint64_t *n_lines, unsigned *fail, hipStream_t s);
hipError_t launch_af_summary(const uint64_t *n_lines, const uint64_t *rowoff, const unsigned long long *counters,
                             const unsigned *fail, uint64_t *out, hipStream_t s);
hipError_t launch_af_rowlen(const uint32_t *rowpre, const uint8_t *status, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, uint64_t *len, hipStream_t s);
// VCFX_hwe_tester (vcfxg_hwe.hip): the exact per-line pass (meta == nullptr: every line;
// else the walk's kMetaFull / kAfPending lines), the row lengths (the walk's CHROM..ALT flags
// applied when meta != nullptr; counters[0] += rows), and the rows (rechecks: vcfxg_hwe_recheck entries, *rc_n counted)
hipError_t launch_hwe_lines(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, int mode, const void *meta, int32_t *c0, int32_t *c1, int32_t *c2,
                            uint32_t *rowpre, uint8_t *status, unsigned long long *counters, hipStream_t s);
hipError_t launch_hwe_rowlen(const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, const void *meta,
                             const uint32_t *rowpre, uint8_t *status, uint64_t *len, unsigned long long *counters,
                             hipStream_t s);
hipError_t launch_hwe_format(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, int mode, const int32_t *c0, const int32_t *c1, const int32_t *c2,
                             const uint32_t *rowpre, const uint8_t *status, const uint64_t *off, char *out,
                             uint64_t text_cap, int64_t ulps, void *rc, unsigned long long *rc_n, uint64_t rc_cap,
                             hipStream_t s);
// VCFX_dosage_calculator (vcfxg_dose.hip) over the indexed lines: per line status (1 row,
// 3 "< 10 fields", 0 skip), row length and meta (dose_meta_bytes() each; counters[0] rows,
// [2] warnings, [3] lines off the fixed-stride sweep); then the rows at their offsets
size_t dose_meta_bytes();
hipError_t launch_dose_len(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, int mode, uint8_t *status, uint64_t *len, void *meta,
                           unsigned long long *counters, hipStream_t s, bool pending_only = false);
// after the dosage walk (launch_af_walk dose, compacted): the walk's fixed-stride GT-only lines
// become rows (ns = alt, na = tot), '#' / empty lines are skipped, every other line is left
// pending for launch_dose_len(pending_only); status is rewritten in place, meta is the dose meta
hipError_t launch_dose_from_walk(const uint64_t *line_end, const uint64_t *n_lines_dev, uint64_t n_lines_host,
                                 const void *walk_meta, const int32_t *ns, const int32_t *na, uint8_t *status,
                                 uint64_t *len, void *meta, unsigned long long *counters, hipStream_t s);
hipError_t launch_dose_fmt(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, const uint8_t *status, const void *meta, const uint64_t *off,
                           char *out, uint64_t cap, uint64_t slow_rows, hipStream_t s, unsigned *bad = nullptr,
                           uint64_t na_rows = ~0ull);
// VCFX_missing_detector (vcfxg_md.hip) over the indexed lines: per line status (0 empty, 4 '#',
// 1 kept as is, kMdFlag flagged) and the flagged lines' INFO span relative to the line start;
// counters [0] data lines, [1] flagged, [2] lines ending in '\n' with a '.' in their samples;
// walk: the statuses hold the missing-detector walk's decisions (1 / kMdFlag taken as they are)
constexpr uint8_t kMdFlag = 6;
hipError_t launch_md_lines(const char *buf, int64_t data_start, int64_t n_input, const uint64_t *line_end,
                           const uint64_t *n_lines_dev, uint64_t n_lines_host, int mode, uint8_t *status,
                           int32_t *info_s, int32_t *info_e, unsigned long long *counters, hipStream_t s,
                           int walk = 0);
// VCFX_allele_counter (vcfxg_ac.hip) over indexed lines [l0, l1): per line status (1 data,
// 4 '#CHROM', 0 other), row bytes (len[li - l0]) and meta (ac_meta_bytes() each); counters
// [0] rows, [1] data lines, [2] '#CHROM' lines, [3] lines off the fixed-stride sweep.  eff:
// per output slot the sample index it reads; scratch: ac_threads() / 64 * blocks * scap u32;
// sel_lds: LDS bytes for the selection in k_ac_fmt (4 m + 4 (m + 1) + name bytes), 0 = global
size_t ac_meta_bytes();
int ac_threads();
hipError_t launch_ac_len(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                         unsigned blocks, const uint32_t *eff, const uint64_t *noff, const char *names,
                         uint32_t *scratch, uint32_t m, uint32_t scap, int seq, int kind, int ident, int direct,
                         uint32_t *nib, uint8_t *status, uint64_t *len, void *meta, unsigned long long *counters,
                         hipStream_t s);
// direct != 0 (text rows, every name L <= 11 bytes, m <= 4096, ac_rows_lds <= ac_rows_lds_max()): k_ac_rows writes
// the fixed-stride records whose prefix is 16..64 bytes (etab: per slot 16 B, the name at bytes
// [11 - L, 11), then "\t0\t0\n", zeros in front; nib: k_ac_len's counts, per line li - l0
// ceil(m / 64) tiles of 8 dwords) and k_ac_fmt the others; k_ac_len counts the others' data lines
// in counters[4] (0: no k_ac_fmt launch needed)
hipError_t launch_ac_fmt(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                         unsigned blocks, const uint32_t *eff, const uint64_t *noff, const char *names,
                         uint32_t *scratch, uint32_t m, uint32_t scap, int seq, int kind, uint32_t sel_lds,
                         int ident, int direct, const uint8_t *status, const void *meta, const uint64_t *off,
                         char *out, hipStream_t s);
hipError_t launch_ac_rows(const char *buf, int64_t data_start, const uint64_t *line_end, uint64_t l0, uint64_t l1,
                          unsigned blocks, const uint32_t *eff, uint32_t m, int ident, const void *etab, uint32_t L,
                          const uint32_t *nib, const void *meta, const uint64_t *off, char *out, hipStream_t s);
size_t ac_rows_lds(uint32_t m, int ident);  // k_ac_rows' dynamic LDS bytes (m <= 4096)
size_t ac_rows_lds_max();
int ac_rows_threads();
// VCFX_haplotype_phaser (vcfxg_ph.hip): per line status (kPh*), the variants' genotype codes
// (row = line, kpad bytes; counters[3] = the largest sample count past kpad), the variant ->
// line compaction, per variant the pair flags with its predecessor (bit 0 the block rule
// passes, bit 1 same CHROM) + r^2 + entry length, and the entries "v:(chrom:pos)"
enum : uint8_t { kPhSkip = 0, kPhVar = 1, kPhFew = 3, kPhHeader = 4, kPhPos = 7, kPhNoGt = 8 };
size_t ph_line_bytes();
// walk_meta (nullable): the head walk's LineMeta per line (its index); a line taken unswept
// (kWalkUnswept) that the parse does not validate by the fixed-stride sweep sets *bad
hipError_t launch_ph_lines(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                           uint64_t n_lines_host, int mode, uint32_t kpad, int8_t *G, uint8_t *status, uint32_t *isvar,
                           void *info, unsigned long long *counters, hipStream_t s, const void *walk_meta = nullptr,
                           unsigned *bad = nullptr);
hipError_t launch_ph_compact(const uint32_t *isvar, const uint64_t *vnum, const uint64_t *n_lines_dev,
                             uint64_t n_lines_host, uint64_t *vline, uint64_t *n_var, hipStream_t s);
hipError_t launch_ph_pairs(const char *buf, const uint64_t *vline, const uint64_t *n_var_dev, uint64_t n_var_host,
                           const void *info, const int8_t *G, uint32_t kpad, double thr, uint8_t *flags, uint64_t *len,
                           double *r2, hipStream_t s);
hipError_t launch_ph_fmt(const char *buf, const uint64_t *vline, const uint64_t *n_var_dev, uint64_t n_var_host,
                         const void *info, const uint64_t *off, char *out, hipStream_t s);
// text_cap: rows whose end passes it are not written (the caller checks the total)
hipError_t launch_af_format(const char *buf, int64_t data_start, const uint64_t *line_end, const uint64_t *n_lines_dev,
                            uint64_t n_lines_host, int mode, const int32_t *alt, const int32_t *tot,
                            const uint32_t *rowpre, const uint8_t *status, const uint64_t *off, char *out,
                            hipStream_t s, uint64_t text_cap = ~0ull);

}  // namespace vcfxg
