// hostio.h -- host-side plumbing shared by the VCFX_<tool> drop-ins: whole-input staging
// (mmap of a file = the reference's MappedFile; or all of stdin), fd writers, the per-
// process GPU context, and the '#CHROM' gate scan that runs on the host before the
// device takes the record region.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "gz.h"
#include "vcfx_gpu.h"

namespace vcfxh {

struct Out;
struct BgzfShard;

struct Input {
    // the input bytes [p, p + host_n) on the host; n = all input bytes.  host_n < n only for
    // a stdin pipe read with host_copy = false: the bytes past the header then exist only on
    // the device (already ingested; see load_input).
    const char *p = nullptr;
    size_t n = 0;
    size_t host_n = 0;
    // a shard view (VCFX_INPUT_VIEW): input bytes [host_n, n) are at tail[0, n - host_n) on the
    // host (another part of the same mapping), not after p
    const char *tail = nullptr;
    bool mapped = false;
    // mapping to release: [map_base, map_base + map_len)
    void *map_base = nullptr;
    size_t map_len = 0;
    // pipe path: bytes [0, streamed) were appended to stream_ctx's device input while stdin
    // was read (vcfxg_ingest, final chunk outstanding); see load_input
    vcfxg_ctx *stream_ctx = nullptr;
    size_t streamed = 0;
    std::vector<void *> ring;  // pinned staging slots of a device-only stream (freed with ring_ctx)
    vcfxg_ctx *ring_ctx = nullptr;
    // compressed input: set by the tools that read .vcf.gz (the record
    // tools; not VCFX_variant_counter, whose own gzip handling is the reference's) before
    // open_file / read_fd; decompress() then inflates gzip / BGZF input in place
    bool gzip_ok = false;
    // BGZF input may be inflated on the device (vcfxg_ingest_bgzf) into a device-only input (the
    // host keeps the inflated head through the '#CHROM' line): set by the tools whose record
    // phase reads only the header on the host and fetches kept records from the device
    bool bgzf_device = false;
    bool gz = false;          // the input was inflated
    int read_errno = 0;       // read_fd stopped on a read(2) error (decompress() reports it)
    size_t source_n = 0;      // bytes of the file / stream as read (compressed size for gz)
    Input() = default;
    Input(const Input &) = delete;
    Input &operator=(const Input &) = delete;
    ~Input();
    // MappedFile::open semantics (VCFX_allele_freq_calc.cpp:52-63): false if open/stat
    // fails; a 0-byte file is a successful empty map.  Inputs of 1 MiB and more start the
    // GPU context opening on a background thread (gpu_prefetch).
    bool open_file(const char *path);
    // open_file for a tool that needs only the header on the host (AF: the device formats every
    // row).  A regular file of 256 MiB and more (VCFX_FILE_STREAM_MIN) is not mapped: its head
    // (through the '#CHROM' line) is read into host memory, the rest by reader threads into a
    // pinned staging ring (kept per context) from which it is copied to the device in order
    // (vcfxg_ingest, DMA overlapping the reads): no page-table population, no unmapping of the
    // whole input afterwards.  Views, gzip input, smaller files and VCFX_FILE_STREAM=0 take
    // open_file.  Afterwards host_n < n and load_input completes the device input.
    bool open_file_device(const char *path);
    // open_file_device's BGZF branch (bgzf_device tools): the compressed file through the pinned
    // ring to the device, the members inflated there; first[0, fn): its first bytes as read
    bool stream_bgzf_device(int fd, size_t total, const char *first, size_t fn);
    // VCFX_INPUT_VIEW="H:LO:HI" in the environment (set by the multi-GPU runner,
    // vcfx_amd/shard.py): the input is the file's header bytes [0, H) followed by its records
    // [LO, HI) -- one rank's shard, without a copy.  The device input is ingested from those
    // two host ranges (load_input); host-side line access goes through LineSource.
    // VCFX_VIEW_SKIP_HEADER=1: the tool writes nothing for the header part (ranks > 0).
    void apply_view();
    // All of fd's remaining bytes (the stream path's input).  A regular file (`< file`) is
    // mapped from the current offset, with no copy.  A pipe is read into a reserved,
    // transparently-huge-page region that a helper thread pre-faults ahead of the reader,
    // while a second thread streams each complete 64 MiB to the device (vcfxg_ingest): the
    // H2D copy overlaps the read.  host_copy = false (a tool that needs only the header on
    // the host): once the head holds the '#CHROM' line the rest of the pipe is read into a
    // pinned staging ring and copied to the device from there, never kept on the host.
    void read_fd(int fd, bool host_copy = true);
    // A read error of read_fd first: false after "Error: vcfx_amd: reading the input failed".
    // gzip / BGZF input (magic 1f 8b) and gzip_ok, unless VCFX_GZIP=0: inflate it (BGZF members
    // on every host thread) into a reserved region that becomes the input.  false (after an
    // "Error: ..." line on err_fd) when the stream is truncated or corrupt.
    bool decompress(int err_fd);
    // decompress()'s device path (bgzf_device, a BGZF chain of >= VCFX_BGZF_DEVICE_MIN inflated
    // bytes, 64 MiB by default; VCFX_BGZF_DEVICE=0 turns it off): false leaves the input as it was
    bool device_bgzf();
    // decompress() on a rank of a multi-GPU run over a BGZF file (ShardRank::bgz, or
    // VCFX_INPUT_VIEW="bgzf:H:LO:HI" from vcfx_amd/shard.py): the header [0, h) and the rank's
    // records [lo, hi) of the inflated stream, on the rank's device (the members wholly inside
    // inflated there; the two cut members' parts on the host); false after an "Error: ..." line
    bool bgzf_view(int err_fd, const BgzfShard &B, uint64_t h, uint64_t lo, uint64_t hi, const std::string &who);
    // mapped inputs of 64 MiB and more: page-table population running on helper threads
    mutable std::vector<std::thread> populating;
    void populate(void *m, size_t len);
    void join_populate() const;
};

// ---- one rank of an in-process multi-GPU run (tool_shard_main.cpp, VCFX_NGPU) -------------------
// A BGZF input split across the ranks by output offset (the planner's, shared by the ranks): the
// member chain of the mapped file and each member's first output byte (off[nm] = the total)
struct BgzfShard {
    const char *comp = nullptr;
    size_t comp_n = 0;
    std::vector<BgzfSpan> ms;
    std::vector<uint64_t> off;
};
// The driver runs the tool once per rank, each on its own host thread with its own device
// context and its own view of the input file; these thread-local settings replace the
// process-wide ones (gpu(), VCFX_INPUT_VIEW, VCFX_VIEW_SKIP_HEADER) on that thread.
struct ShardRank {
    int rank = 0, world = 1;
    vcfxg_ctx *g = nullptr;                          // this rank's context
    int device = 0, open_rc = 0;                     // its device and vcfxg_open's status
    unsigned long long h = 0, lo = 0, hi = 0;        // view: header [0, h) + records [lo, hi)
    const BgzfShard *bgz = nullptr;                  // a BGZF file: the view is of its inflated bytes
    size_t whole_bytes = 0;                          // the whole input file's size
    int err_fd = -1;                                 // this rank's stderr (a memfd)
    long long err_mark = -1;                         // its bytes before the record phase
    // counters the driver sums over the ranks after the run (RCCL on distinct devices), and
    // on rank 0 the summary lines made from the sums (written after every rank's stderr)
    uint64_t cnt[8] = {};
    std::function<std::string(const uint64_t *)> summary;
};
extern thread_local ShardRank *t_shard;
// the stderr written so far is the argument / header phase, which every rank repeats: ranks
// > 0 drop it (the driver copies their stderr from here on)
void shard_records_begin(Out &err);
// the input's size as the tools report it ("Processing F (X MB)"): the whole file for a rank
size_t reported_size(const Input &in);

// sizes of the input paths (VCFX_PREFETCH_BYTES, VCFX_STREAM_CHUNK, VCFX_RING_SLOT,
// VCFX_WINDOW_BYTES override them; tests use tiny values)
size_t prefetch_bytes();
size_t stream_chunk();
size_t ring_slot();
size_t window_bytes();

// VCFX_TIMING=1 in the environment: "[vcfx-timing] <what> <ms since process start>" on
// stderr (fd 2) at each phase of a tool run -- e2e breakdowns; silent otherwise.
void phase(const char *what);
// set by the drop-in executables (binary_main.cpp): the process exits right after the tool
// returns, so inputs skip unmapping (the kernel drops the mappings at exit anyway)
extern bool g_process_exit_fast;
// VCFX_VIEW_SKIP_HEADER=1: a shard rank other than the first (its header output is rank 0's)
bool view_skip_header();
// VCFX_GZIP=0 turns compressed-input support off (the reference's tools read .gz bytes as text)
bool gzip_enabled();

void write_all(int fd, const char *p, size_t n);
inline void write_str(int fd, const std::string &s) { write_all(fd, s.data(), s.size()); }

// buffered writer over an fd
struct Out {
    int fd;
    std::string buf;
    explicit Out(int f) : fd(f) { buf.reserve(1 << 20); }
    ~Out() { flush(); }
    void put(const char *p, size_t n) {
        if (buf.size() + n > (4u << 20)) flush();
        if (n > (4u << 20)) write_all(fd, p, n);
        else buf.append(p, n);
    }
    void put(const std::string &s) { put(s.data(), s.size()); }
    void putc(char c) { put(&c, 1); }
    void flush() {
        if (!buf.empty()) write_all(fd, buf.data(), buf.size());
        buf.clear();
    }
};

// The process-wide device context (device 0, or $VCFX_DEVICE).  On failure prints
// "Error: vcfx_amd: ..." to err_fd and returns nullptr -- there is no CPU fallback.
vcfxg_ctx *gpu(int err_fd);
// start opening that context on a background thread (the HIP runtime start then overlaps
// the caller's input reading); gpu() / gpu_quiet() wait for it
void gpu_prefetch();
// wait for a background open started by gpu_prefetch (before the process ends)
void gpu_join();
// the same context, opened without a diagnostic (nullptr when there is no device)
vcfxg_ctx *gpu_quiet();
// run a vcfxg_* call; on failure prints the context error and returns false
bool gpu_ok(vcfxg_ctx *c, int rc, const char *what, int err_fd);
// make in's bytes the device-resident input of g: completes the ingest started while stdin
// was read, or copies the whole input (vcfxg_load_host)
bool load_input(vcfxg_ctx *g, const Input &in, int err_fd);

// the device-formatted text of the last call (bytes of it) written to out's fd after out's
// buffer: through the context's pinned file ring when it has one, else one host copy
bool write_device_text(vcfxg_ctx *g, uint64_t bytes, Out &out, int err_fd);

const void *memchr_(const char *p, const char *end);

// iterate lines of [p, end): returns false at end; [ls, le) excludes '\n'
inline bool next_line(const char *&p, const char *end, const char *&ls, const char *&le) {
    if (p >= end) return false;
    const void *nl = memchr_(p, end);
    ls = p;
    le = nl ? (const char *)nl : end;
    p = nl ? le + 1 : end;
    return true;
}

inline bool is_chrom_line(const char *s, size_t n) {
    return n >= 6 && s[0] == '#' && s[1] == 'C' && s[2] == 'H' && s[3] == 'R' && s[4] == 'O' && s[5] == 'M';
}

}  // namespace vcfxh

#define VCFX_VERSION_STR "1.1.4"  // VCFX_VERSION of the reference build (CMakeLists.txt:4-9)

namespace vcfxh {
// vcfx::flag_present (vcfx_core.cpp:31-38)
inline bool flag_present(int argc, char **argv, const char *l, const char *s) {
    for (int i = 1; i < argc; ++i)
        if (strcmp(argv[i], l) == 0 || (s && strcmp(argv[i], s) == 0)) return true;
    return false;
}
}  // namespace vcfxh
