// hostio.cpp -- see hostio.h
#include "hostio.h"

#include "gz.h"

#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <memory>
#include <mutex>
#include <thread>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22  // Linux 5.14
#endif
static constexpr int kMadvPopulateWrite = MADV_POPULATE_WRITE;
static constexpr int kMadvPopulateRead = MADV_POPULATE_READ;

namespace vcfxh {

const void *memchr_(const char *p, const char *end) { return memchr(p, '\n', (size_t)(end - p)); }

bool g_process_exit_fast = false;

namespace {
const std::chrono::steady_clock::time_point t_start = std::chrono::steady_clock::now();
const bool timing_on = getenv("VCFX_TIMING") && atoi(getenv("VCFX_TIMING")) > 0;

size_t env_bytes(const char *name, size_t def) {
    const char *e = getenv(name);
    if (!e || !*e) return def;
    const unsigned long long v = strtoull(e, nullptr, 10);
    return v ? (size_t)v : def;
}
}  // namespace

// Sizes of the input paths.  The environment overrides exist for tests (tiny values push
// small inputs through the streaming and windowed paths).
// inputs from prefetch_bytes() on open the GPU context on a background thread as soon as
// they are seen, so the HIP runtime start (~0.2 s on MI355X) overlaps reading the input
size_t prefetch_bytes() { return env_bytes("VCFX_PREFETCH_BYTES", (size_t)1 << 20); }
// the pipe path streams to the device in chunks of this size
size_t stream_chunk() { return env_bytes("VCFX_STREAM_CHUNK", (size_t)64 << 20); }
// pinned staging slots of a device-only stream (4 of them)
// the pipe ring: 16 slots of 1 MiB (r04 e2e probe, 4.30 GB through `cat F |`: ring read rate 9.0
// GB/s at 1 MiB x 16, 8.2 at 2 MiB x 8, 7.1 at 4 MiB x 8, 6.3 at 32 MiB x 4 -- slots that stay in
// the host's caches between the reader's write and the DMA's read)
size_t ring_slot() { return env_bytes("VCFX_RING_SLOT", (size_t)1 << 20); }
// the host window through which pass-through tools read a device-only input back
size_t window_bytes() { return env_bytes("VCFX_WINDOW_BYTES", (size_t)64 << 20); }

void phase(const char *what) {
    if (!timing_on) return;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    char b[160];
    int k = snprintf(b, sizeof b, "[vcfx-timing] %s %.2f ms\n", what, ms);
    if (k > 0) write_all(2, b, (size_t)std::min<int>(k, (int)sizeof b - 1));
}

// ---- the process-wide device context --------------------------------------------------
namespace {
std::mutex g_mu;
vcfxg_ctx *g_ctx = nullptr;
bool g_tried = false;
std::atomic<bool> g_open_done{false};  // the open (successful or not) has finished
int g_rc = 0;
int g_dev = 0;
struct Opener {
    std::thread t;
    ~Opener() {
        if (t.joinable()) t.join();
    }
} g_opener;

void open_locked() {
    if (g_tried) return;
    g_tried = true;
    g_dev = 0;
    if (const char *e = getenv("VCFX_DEVICE")) g_dev = atoi(e);
    phase("gpu open begin");
    g_rc = vcfxg_open(g_dev, &g_ctx);
    phase("gpu open end");
    if (g_rc != VCFXG_OK) g_ctx = nullptr;
    g_open_done.store(true, std::memory_order_release);
}

void join_opener() {
    std::thread t;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_opener.t.joinable() || g_opener.t.get_id() == std::this_thread::get_id()) return;
        t = std::move(g_opener.t);
    }
    t.join();
}
}  // namespace

void gpu_join() { join_opener(); }

void gpu_prefetch() {
    if (t_shard) return;
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_tried || g_opener.t.joinable()) return;
    g_opener.t = std::thread([] {
        std::lock_guard<std::mutex> l2(g_mu);
        open_locked();
    });
}

vcfxg_ctx *gpu_quiet() {
    if (t_shard) return t_shard->g;  // a rank of an in-process multi-GPU run: its own context
    join_opener();
    std::lock_guard<std::mutex> lk(g_mu);
    open_locked();
    return g_ctx;
}

vcfxg_ctx *gpu(int err_fd) {
    vcfxg_ctx *c = gpu_quiet();
    if (!c && t_shard)
        write_str(err_fd, std::string("Error: vcfx_amd: rank ") + std::to_string(t_shard->rank) + " of " +
                              std::to_string(t_shard->world) + ": no usable MI355X (gfx950) device " +
                              std::to_string(t_shard->device) + " (vcfxg_open rc=" + std::to_string(t_shard->open_rc) +
                              "); this build has no CPU path.\n");
    else if (!c)
        write_str(err_fd, std::string("Error: vcfx_amd: no usable MI355X (gfx950) device ") + std::to_string(g_dev) +
                              " (vcfxg_open rc=" + std::to_string(g_rc) + "); this build has no CPU path.\n");
    return c;
}

bool gpu_ok(vcfxg_ctx *c, int rc, const char *what, int err_fd) {
    if (rc == VCFXG_OK) return true;
    write_str(err_fd, std::string("Error: vcfx_amd: ") + what + " failed (rc=" + std::to_string(rc) + "): " +
                          vcfxg_last_error(c) + "\n");
    return false;
}

// ---- input ----------------------------------------------------------------------------
void Input::join_populate() const {
    for (auto &t : populating) t.join();
    populating.clear();
}

Input::~Input() {
    join_populate();
    if (g_process_exit_fast) return;  // the process ends next: let exit() drop the mappings
    if (ring_ctx)
        for (void *r : ring) vcfxg_host_free(ring_ctx, r);
    if (map_base && map_len) munmap(map_base, map_len);
    phase("input released");
}

bool Input::open_file(const char *path) {
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) < 0) {
        ::close(fd);
        return false;
    }
    n = host_n = (size_t)st.st_size;
    if (n == 0) {
        ::close(fd);
        p = "";
        return true;
    }
    if (n >= prefetch_bytes()) gpu_prefetch();
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) {
        n = host_n = 0;
        return false;
    }
    // the reference's advice (MappedFile, VCFX_allele_freq_calc.cpp:52-63); a large input is
    // populated by helper threads instead of read-ahead (WILLNEED walks every cached page
    // on this thread first: ~30 ms at 4 GB)
    madvise(m, n, n < ((size_t)64 << 20) ? (MADV_SEQUENTIAL | MADV_WILLNEED) : MADV_SEQUENTIAL);
    phase("file mapped");
    p = (const char *)m;
    mapped = true;
    map_base = m;
    map_len = n;
    source_n = n;
    if (gzip_ok && is_gzip(p, n) && gzip_enabled()) return true;  // decompress() takes it from here
    apply_view();
    return true;
}

namespace {
// the pinned staging ring of device-only file reads: allocated once per context and kept for
// the process (a warm in-process context reuses it; hipHostMalloc of 192 MiB costs ~20 ms)
struct FileRing {
    vcfxg_ctx *ctx = nullptr;
    size_t slot = 0;
    std::vector<void *> slots;
    bool busy = false;  // a caller is reading into / copying out of the slots (under g_ring_mu)
};
std::mutex g_ring_mu;
FileRing g_file_ring;

size_t file_slot() { return env_bytes("VCFX_FILE_SLOT", (size_t)16 << 20); }
size_t file_slots() { return std::max<size_t>(2, env_bytes("VCFX_FILE_SLOTS", 12)); }

// pread of [off, off + len) into dst, whole (short reads continued); false on an error
bool pread_full(int fd, char *dst, size_t len, size_t off, int *err) {
    size_t got = 0;
    while (got < len) {
        ssize_t k = ::pread(fd, dst + got, len - got, (off_t)(off + got));
        if (k < 0 && errno == EINTR) continue;
        if (k < 0) *err = errno;
        if (k <= 0) return false;
        got += (size_t)k;
    }
    return true;
}
}  // namespace

// A BGZF file (open_file_device's gzip branch; the tools that take device BGZF, bgzf_device):
// the compressed bytes go through the pinned file ring to the device as they are read
// (vcfxg_bgzf_stage, DMA overlapping the reads), the member chain is parsed from the ring's
// slots in order (BgzfStream), the head -- members inflated here until the output holds the
// '#CHROM' line and 64 KiB after it -- comes from the first bytes read (first[0, fn)), then every
// member is inflated on the device (vcfxg_ingest_bgzf).  No mapping of the file, no page
// population, no pageable copy.  false (nothing changed): the caller maps the file instead
// (decompress() then takes the host inflate, or device_bgzf on the mapping).
bool Input::stream_bgzf_device(int fd, size_t total, const char *first, size_t fn) {
    const char *e = getenv("VCFX_BGZF_DEVICE");
    if ((e && e[0] == '0') || t_shard || !bgzf_device || !gzip_ok || !gzip_enabled()) return false;
    // the head
    const size_t kHeadMax = ((size_t)64 << 20) + 65536;
    void *hm = mmap(nullptr, kHeadMax, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (hm == MAP_FAILED) return false;
    char *head = (char *)hm;
    size_t hn = 0, scanned = 0, at = 0;
    bool chrom = false;
    size_t chrom_end = 0;
    {
        BgzfStream hs;  // (members wholly inside first[0, fn))
        hs.feed(first, fn);
        for (const BgzfSpan &m : hs.members) {
            if (chrom && hn - chrom_end >= 65536) break;
            if (hn + m.olen > kHeadMax) break;
            size_t got = 0;
            if (!gz_inflate_member(first + m.off, m.len, head + hn, m.olen, &got) || got != m.olen) break;
            hn += got;
            at = m.off + m.len;
            while (!chrom && scanned < hn) {
                const char *s0 = head + scanned;
                const char *nl = (const char *)memchr(s0, '\n', hn - scanned);
                if (!nl) break;
                chrom = is_chrom_line(s0, (size_t)(nl - s0));
                scanned = (size_t)(nl - head) + 1;
                if (chrom) chrom_end = scanned;
            }
        }
    }
    (void)at;
    vcfxg_ctx *g = chrom ? gpu_quiet() : nullptr;
    if (!g) {
        munmap(hm, kHeadMax);
        return false;
    }
    phase("bgzf head inflated");
    bool batching = !(getenv("VCFX_BGZF_BATCH") && getenv("VCFX_BGZF_BATCH")[0] == '0');
    const size_t batch_min = env_bytes("VCFX_BGZF_BATCH_MIN", 32768);  // (~128 MB compressed; tests: 1)
    // (a ring of 8 x 8 MiB, a third of the text path's 12 x 16 MiB: pinning costs ~0.2 ms per MiB in
    // a fresh process, and the compressed bytes are 17x fewer; VCFX_FILE_SLOT / _SLOTS override)
    const size_t kSlot = env_bytes("VCFX_FILE_SLOT", (size_t)8 << 20);
    const size_t kSlots = std::max<size_t>(2, env_bytes("VCFX_FILE_SLOTS", 8));
    std::vector<void *> ring_;
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        if (g_file_ring.busy) {
            munmap(hm, kHeadMax);
            return false;
        }
        if (g_file_ring.ctx != g || g_file_ring.slot != kSlot || g_file_ring.slots.size() != kSlots) {
            if (g_file_ring.ctx)
                for (void *r : g_file_ring.slots) vcfxg_host_free(g_file_ring.ctx, r);
            g_file_ring = FileRing{};
            bool ok = true;
            for (size_t i = 0; i < kSlots && ok; i++) {
                void *r = nullptr;
                ok = vcfxg_host_alloc(g, kSlot, &r) == VCFXG_OK;
                if (ok) g_file_ring.slots.push_back(r);
            }
            if (ok) {
                g_file_ring.ctx = g;
                g_file_ring.slot = kSlot;
            } else {
                for (void *r : g_file_ring.slots) vcfxg_host_free(g, r);
                g_file_ring.slots.clear();
            }
        }
        ring_ = g_file_ring.slots;
        g_file_ring.busy = !ring_.empty();
    }
    struct RingRelease {
        bool on;
        ~RingRelease() {
            if (!on) return;
            std::lock_guard<std::mutex> lk(g_ring_mu);
            g_file_ring.busy = false;
        }
    } ring_release{!ring_.empty()};
    // (the input buffer sized for ~24x the compressed bytes, a genotype VCF's BGZF ratio, so the
    // inflate batches launched during the stream have their room; more grows it at the end.
    // vcfxg_ingest_begin cuts a hint past half the device's free memory; when even the cut one
    // cannot be had, 6x: the batches that do not fit wait for the end, E_CAP)
    phase("bgzf ring ready");
    if (ring_.empty() || (vcfxg_ingest_begin(g, 24 * total) != VCFXG_OK && vcfxg_ingest_begin(g, 6 * total) != VCFXG_OK)) {
        munmap(hm, kHeadMax);
        return false;
    }
    phase("bgzf input buffer ready");
    // chunk i = [i*slot, ...) into slot i % S, read by T reader threads, staged in order by this
    // thread (which parses the member chain from the slot before its DMA is waited for)
    // (a quarter of the slots in DMA flight, the rest being read: a slot's 8 MiB copy takes
    // ~0.15 ms, the page-cache reads are the slower side)
    const size_t S = ring_.size(), inflight = std::max<size_t>(1, S / 4);
    const size_t nchunks = (total + kSlot - 1) / kSlot;
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t T = std::max<size_t>(1, std::min<size_t>({S - inflight, env_bytes("VCFX_FILE_THREADS", 8),
                                                           hw ? (size_t)hw : 1}));
    std::mutex mu;
    std::condition_variable cv;
    std::vector<long long> filled(S, -1), freed(S, -1);
    bool stop = false, ok = true;
    std::atomic<int> rerr{0};
    std::vector<std::thread> readers;
    // (each reader walks the member chain of the chunk it just read, from the first header that
    // validates -- the bytes still in its core's caches; the loop below takes that chain when its
    // own walk arrives there: the walk was a dependent miss per member, 14-17 ms on the bench shard)
    std::vector<BgzfChunk> scans(S);
    for (size_t t = 0; t < T; t++)
        readers.emplace_back([&, t] {
            for (size_t i = t; i < nchunks; i += T) {
                const size_t s = i % S;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || i < S || freed[s] >= (long long)(i - S); });
                    if (stop) return;
                }
                const size_t off = i * kSlot, len = std::min(kSlot, total - off);
                int er = 0;
                const bool r = pread_full(fd, (char *)ring_[s], len, off, &er);
                if (r) scans[s].scan((const char *)ring_[s], len, off);
                std::lock_guard<std::mutex> lk(mu);
                if (!r) {
                    rerr = er ? er : EIO;
                    stop = true;
                } else {
                    filled[s] = (long long)i;
                }
                cv.notify_all();
                if (!r) return;
            }
        });
    BgzfStream chain;
    size_t launched = 0;
    std::vector<size_t> ends(nchunks);
    // (VCFX_TIMING: where the loop's time goes -- waiting for the readers, the H2D stage call, the
    // chain walk, the batch launches, waiting for a slot's DMA)
    double t_fill = 0, t_stage = 0, t_stage0 = 0, t_feed = 0, t_batch = 0, t_dma = 0;
    auto clk = [] { return std::chrono::steady_clock::now(); };
    auto dms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    for (size_t i = 0; i < nchunks && ok; i++) {
        const size_t s = i % S, off = i * kSlot, len = std::min(kSlot, total - off);
        auto t0 = clk();
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || filled[s] == (long long)i; });
            if (stop) {
                ok = false;
                break;
            }
        }
        auto t1 = clk();
        ok = vcfxg_bgzf_stage(g, ring_[s], len, off, total) == VCFXG_OK;
        auto t2 = clk();
        chain.adopt((const char *)ring_[s], len, scans[s]);
        ok = ok && !chain.bad;
        auto t3 = clk();
        t_fill += dms(t0, t1), t_stage += dms(t1, t2), t_feed += dms(t2, t3);
        if (i == 0) t_stage0 = dms(t1, t2);
        // the members complete so far inflate on the device while the next chunks are read and
        // copied (batches of >= 32,768 members, about 128 MB compressed, round robin on two
        // streams, each checking its own CRCs; the rest at the end.  r06, the bench shard with the
        // context open: 21-25 ms against 24-36 at 16,384, 25 at 24,576 and 22-50 unbatched)
        if (ok && batching && chain.members.size() - launched >= batch_min) {
            const int br = vcfxg_bgzf_inflate(g, reinterpret_cast<const vcfxg_bgzf_member *>(chain.members.data()) +
                                                     launched,
                                              chain.members.size() - launched);
            if (br == VCFXG_OK) launched = chain.members.size();
            else batching = false;  // (E_CAP: the output outgrew the hint; the rest at the end)
        }
        auto t4 = clk();
        t_batch += dms(t3, t4);
        ends[i] = off + len;
        if (ok && i >= inflight) {
            const size_t j = i - inflight;
            ok = vcfxg_ingest_wait(g, ends[j]) == VCFXG_OK;
            std::lock_guard<std::mutex> lk(mu);
            freed[j % S] = (long long)j;
            cv.notify_all();
        }
        t_dma += dms(t4, clk());
    }
    if (timing_on) {
        char b[200];
        snprintf(b, sizeof b,
                 "bgzf stream loop: readers %.2f, stage %.2f (first %.2f), chain %.2f, batches %.2f, slot DMA %.2f ms",
                 t_fill, t_stage, t_stage0, t_feed, t_batch, t_dma);
        phase(b);
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!ok) stop = true;
        cv.notify_all();
    }
    for (auto &t : readers) t.join();
    // every DMA from the ring finished before the slots are reused, on the failure path too
    if (vcfxg_ingest_wait(g, ok ? total : ~(size_t)0) != VCFXG_OK) ok = false;
    phase("bgzf streamed to the device");
    ok = ok && !rerr && chain.ok(total) && chain.out >= hn;
    uint64_t bad = ~0ull;
    static_assert(sizeof(BgzfSpan) == sizeof(vcfxg_bgzf_member), "member layout");
    if (!ok || vcfxg_ingest_bgzf(g, nullptr, total, reinterpret_cast<const vcfxg_bgzf_member *>(chain.members.data()),
                                 chain.members.size(), head, hn, &bad) != VCFXG_OK) {
        // (a read error, not a BGZF chain, or a member the device refused: the mapped path decides,
        // the host inflate reporting damage as the reference does)
        munmap(hm, kHeadMax);
        phase("bgzf stream not taken");
        return false;
    }
    phase("bgzf inflated on the device");
    p = head;
    host_n = hn;
    n = (size_t)chain.out;
    source_n = total;
    map_base = hm;
    map_len = kHeadMax;
    mapped = false;
    gz = true;
    tail = nullptr;
    stream_ctx = g;
    streamed = n;
    return true;
}

bool Input::open_file_device(const char *path) {
    // where the mapped path stays: views (a shard rank, VCFX_INPUT_VIEW), VCFX_FILE_STREAM=0
    const char *fs = getenv("VCFX_FILE_STREAM");
    if (t_shard || getenv("VCFX_INPUT_VIEW") || (fs && fs[0] == '0')) return open_file(path);
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) < 0 || !S_ISREG(st.st_mode)) {
        ::close(fd);
        return open_file(path);
    }
    const size_t total = (size_t)st.st_size;
    if (total < env_bytes("VCFX_FILE_STREAM_MIN", (size_t)256 << 20)) {
        // (BGZF input streams from VCFX_BGZF_STREAM_MIN compressed bytes, 16 MiB by default)
        unsigned char mg[2] = {0, 0};
        int e = 0;
        const bool gzf = total >= env_bytes("VCFX_BGZF_STREAM_MIN", (size_t)16 << 20) && total >= 2 &&
                         pread_full(fd, (char *)mg, 2, 0, &e) && mg[0] == 0x1f && mg[1] == 0x8b;
        if (!gzf) {
            ::close(fd);
            return open_file(path);
        }
    }
    gpu_prefetch();  // (a fresh process: the HIP runtime starts while the head is read)
    // the head (until it holds the '#CHROM' line: the host's gate runs on it) into host memory
    const size_t kSlot = file_slot(), kHeadMax = std::min(total, (size_t)256 << 20);
    void *hm = mmap(nullptr, kHeadMax, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (hm == MAP_FAILED) {
        ::close(fd);
        return open_file(path);
    }
    char *head = (char *)hm;
    size_t hn = 0;
    bool chrom = false;
    size_t scanned = 0;
    while (!chrom && hn < kHeadMax) {
        const size_t want = std::min(kHeadMax - hn, hn ? hn : env_bytes("VCFX_FILE_HEAD", (size_t)1 << 20));
        if (!pread_full(fd, head + hn, want, hn, &read_errno)) break;
        hn += want;
        if (hn >= 2 && (unsigned char)head[0] == 0x1f && (unsigned char)head[1] == 0x8b) break;  // gzip
        while (!chrom && scanned < hn) {
            const char *s0 = head + scanned;
            const char *nl = (const char *)memchr(s0, '\n', hn - scanned);
            if (!nl) break;
            chrom = is_chrom_line(s0, (size_t)(nl - s0));
            scanned = (size_t)(nl - head) + 1;
        }
    }
    if (!chrom && hn >= 2 && is_gzip(head, hn) && stream_bgzf_device(fd, total, head, hn)) {
        munmap(hm, kHeadMax);
        ::close(fd);
        return true;
    }
    vcfxg_ctx *g = chrom ? gpu_quiet() : nullptr;
    if (!g) {  // gzip, no '#CHROM' in the first 256 MiB, a read error, or no device: the mapping
        munmap(hm, kHeadMax);
        ::close(fd);
        read_errno = 0;
        return open_file(path);
    }
    phase("file head read");
    // the ring (this context's, kept for the process)
    std::vector<void *> ring_;
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        if (g_file_ring.busy) {  // another caller holds the slots: this one maps the file
            munmap(hm, kHeadMax);
            ::close(fd);
            return open_file(path);
        }
        if (g_file_ring.ctx != g || g_file_ring.slot != kSlot || g_file_ring.slots.size() != file_slots()) {
            if (g_file_ring.ctx)
                for (void *r : g_file_ring.slots) vcfxg_host_free(g_file_ring.ctx, r);
            g_file_ring = FileRing{};
            bool ok = true;
            for (size_t i = 0; i < file_slots() && ok; i++) {
                void *r = nullptr;
                ok = vcfxg_host_alloc(g, kSlot, &r) == VCFXG_OK;
                if (ok) g_file_ring.slots.push_back(r);
            }
            if (ok) {
                g_file_ring.ctx = g;
                g_file_ring.slot = kSlot;
            } else {
                for (void *r : g_file_ring.slots) vcfxg_host_free(g, r);
                g_file_ring.slots.clear();
            }
        }
        ring_ = g_file_ring.slots;
        g_file_ring.busy = !ring_.empty();
    }
    struct RingRelease {  // the slots are free again once every DMA from them has finished
        bool on;
        ~RingRelease() {
            if (!on) return;
            std::lock_guard<std::mutex> lk(g_ring_mu);
            g_file_ring.busy = false;
        }
    } ring_release{!ring_.empty()};
    if (ring_.empty() || vcfxg_ingest_begin(g, total) != VCFXG_OK || vcfxg_ingest(g, head, hn, 0) != VCFXG_OK) {
        munmap(hm, kHeadMax);
        ::close(fd);
        return open_file(path);
    }
    phase("file ring ready");
    // the rest: chunk i = [hn + i*slot, ...) into slot i % S, read by T reader threads (reader
    // t takes chunks t, t + T, ...), handed to the device in order by this thread; at most S/2
    // chunks are in DMA flight, the other slots are being filled
    const size_t S = ring_.size(), inflight = std::max<size_t>(1, S / 2);
    const size_t nchunks = (total - hn + kSlot - 1) / kSlot;
    const unsigned hw = std::thread::hardware_concurrency();
    const size_t T = std::max<size_t>(1, std::min<size_t>({S - inflight, env_bytes("VCFX_FILE_THREADS", 8),
                                                           hw ? (size_t)hw : 1}));
    std::mutex mu;
    std::condition_variable cv;
    std::vector<long long> filled(S, -1), freed(S, -1);  // chunk index held / released per slot
    bool stop = false, ok = true;
    std::atomic<int> rerr{0};
    std::vector<std::thread> readers;
    for (size_t t = 0; t < T; t++)
        readers.emplace_back([&, t] {
            for (size_t i = t; i < nchunks; i += T) {
                const size_t s = i % S;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop || i < S || freed[s] >= (long long)(i - S); });
                    if (stop) return;
                }
                const size_t off = hn + i * kSlot, len = std::min(kSlot, total - off);
                int e = 0;
                const bool r = pread_full(fd, (char *)ring_[s], len, off, &e);
                std::lock_guard<std::mutex> lk(mu);
                if (!r) {
                    rerr = e ? e : EIO;
                    stop = true;
                } else {
                    filled[s] = (long long)i;
                }
                cv.notify_all();
                if (!r) return;
            }
        });
    std::vector<size_t> ends(nchunks);
    for (size_t i = 0; i < nchunks && ok; i++) {
        const size_t s = i % S, off = hn + i * kSlot, len = std::min(kSlot, total - off);
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || filled[s] == (long long)i; });
            if (stop) {
                ok = false;
                break;
            }
        }
        ok = vcfxg_ingest(g, (const char *)ring_[s], len, 0) == VCFXG_OK;
        ends[i] = off + len;
        if (ok && i >= inflight) {  // the chunk inflight places back: its DMA done, its slot free
            const size_t j = i - inflight;
            ok = vcfxg_ingest_wait(g, ends[j]) == VCFXG_OK;
            std::lock_guard<std::mutex> lk(mu);
            freed[j % S] = (long long)j;
            cv.notify_all();
        }
    }
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!ok) stop = true;
        cv.notify_all();
    }
    for (auto &t : readers) t.join();
    ::close(fd);
    // every DMA from the ring finished before the slots are reused (the next call's readers),
    // on the failure path too (the chunks queued before it may still be reading their slots)
    if (vcfxg_ingest_wait(g, ok ? total : ~(size_t)0) != VCFXG_OK) ok = false;
    if (rerr) read_errno = rerr;
    phase("file streamed to the device");
    p = head;
    host_n = hn;
    n = total;
    source_n = total;
    map_base = hm;
    map_len = kHeadMax;
    mapped = false;
    stream_ctx = g;
    streamed = ok ? total : 0;  // a failure is reported when the input is used (load_input)
    return true;
}

bool gzip_enabled() {
    const char *e = getenv("VCFX_GZIP");
    return !(e && e[0] == '0');
}

namespace {
// log2 of the largest address-space reservation tried first (1 TiB; VCFX_RESERVE_LOG2 lowers it
// for hosts where faults in a huge reservation fail, e.g. under ThreadSanitizer's shadow map)
int reserve_log2() {
    const char *e = getenv("VCFX_RESERVE_LOG2");
    const int v = e ? atoi(e) : 40;
    return v >= 30 && v <= 40 ? v : 40;
}

// an anonymous region of reserved address space (not memory), transparent huge pages
void *reserve_region(size_t *cap) {
    for (int sh : {40, 36, 32, 30}) {
        if (sh > reserve_log2()) continue;
        *cap = (size_t)1 << sh;
        void *m = mmap(nullptr, *cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (m != MAP_FAILED) {
            madvise(m, *cap, MADV_HUGEPAGE);
            return m;
        }
    }
    *cap = 0;
    return nullptr;
}
}  // namespace

bool Input::decompress(int err_fd) {
    if (read_errno) {  // a failed read(2) is not the end of the input
        write_str(err_fd, std::string("Error: vcfx_amd: reading the input failed: ") + strerror(read_errno) + "\n");
        return false;
    }
    if (!gzip_ok || gz || host_n != n || !is_gzip(p, n) || !gzip_enabled()) return true;
    join_populate();
    if (t_shard && t_shard->bgz)
        return bgzf_view(err_fd, *t_shard->bgz, t_shard->h, t_shard->lo, t_shard->hi,
                         "rank " + std::to_string(t_shard->rank));
    unsigned long long vh = 0, vlo = 0, vhi = 0;
    const char *v = t_shard ? nullptr : getenv("VCFX_INPUT_VIEW");
    if (v && sscanf(v, "bgzf:%llu:%llu:%llu", &vh, &vlo, &vhi) == 3) {
        BgzfShard B;
        uint64_t tot = 0;
        if (!bgzf_chain(p, n, B.ms, &tot)) {
            write_str(err_fd, "Error: vcfx_amd: VCFX_INPUT_VIEW=bgzf:...: the input is not a BGZF member chain\n");
            return false;
        }
        B.comp = p;
        B.comp_n = n;
        B.off.assign(B.ms.size() + 1, 0);
        for (size_t i = 0; i < B.ms.size(); i++) B.off[i + 1] = B.off[i] + B.ms[i].olen;
        return bgzf_view(err_fd, B, vh, vlo, vhi, "view");
    }
    if (bgzf_device && device_bgzf()) return true;
    size_t cap = 0;
    void *m = reserve_region(&cap);
    if (!m) {
        write_str(err_fd, "Error: vcfx_amd: no address space for the decompressed input\n");
        return false;
    }
    unsigned hw = std::thread::hardware_concurrency();
    int threads = (int)std::max(1u, std::min(16u, hw ? hw : 1u));
    if (const char *e = getenv("VCFX_THREADS")) threads = std::max(1, atoi(e));
    phase("gzip inflate begin");
    const GzResult r = gz_inflate(p, n, (char *)m, cap, threads);
    phase(r.bgzf ? "gzip inflate end (BGZF, parallel)" : "gzip inflate end (sequential)");
    if (!r.ok) {
        write_str(err_fd, "Error: vcfx_amd: the gzip input is truncated or corrupt (" + std::to_string(r.n) +
                              " bytes inflated)\n");
        munmap(m, cap);
        return false;
    }
    if (map_base && map_len) munmap(map_base, map_len);  // the compressed bytes
    map_base = m;
    map_len = cap;
    p = (const char *)m;
    n = host_n = r.n;
    mapped = false;
    gz = true;
    tail = nullptr;
    if (n >= prefetch_bytes()) gpu_prefetch();
    return true;
}

bool Input::device_bgzf() {
    const char *e = getenv("VCFX_BGZF_DEVICE");
    // (a rank of a multi-GPU run: only one that takes the whole file, VCFX_ld_calculator's rows)
    const bool view = t_shard && !(t_shard->h == 0 && t_shard->lo == 0 && t_shard->hi == n);
    if ((e && e[0] == '0') || view) return false;
    const char *em = getenv("VCFX_BGZF_DEVICE_MIN");
    const uint64_t min_out = em && *em ? strtoull(em, nullptr, 10) : (uint64_t)64 << 20;
    // the member chain (its headers touch every page of the mapping: fault them in first)
    if (mapped && map_base) {
        populate(map_base, map_len);
        join_populate();
    }
    std::vector<BgzfSpan> ms;
    uint64_t total = 0;
    if (!bgzf_chain(p, n, ms, &total) || total < min_out) return false;
    phase("bgzf chain");
    // the head: members inflated here, in order, until the output holds the complete '#CHROM'
    // line and 64 KiB after it (the host's gate and the tools' header scans run on it: a scan
    // that ends in the head sees the first record line start); at most 64 MiB
    const size_t kHeadMax = std::min<uint64_t>(total, (uint64_t)64 << 20) + 3 * 65536;
    void *hm = mmap(nullptr, kHeadMax, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (hm == MAP_FAILED) return false;
    char *head = (char *)hm;
    size_t hn = 0, scanned = 0, chrom_end = 0;
    bool chrom = false;
    for (size_t i = 0; i < ms.size() && !(chrom && hn - chrom_end >= 65536); i++) {
        if (hn + ms[i].olen > kHeadMax) break;
        size_t got = 0;
        if (!gz_inflate_member(p + ms[i].off, ms[i].len, head + hn, ms[i].olen, &got) || got != ms[i].olen) break;
        hn += got;
        while (!chrom && scanned < hn) {
            const char *s0 = head + scanned;
            const char *nl = (const char *)memchr(s0, '\n', hn - scanned);
            if (!nl) break;
            chrom = is_chrom_line(s0, (size_t)(nl - s0));
            scanned = (size_t)(nl - head) + 1;
            if (chrom) chrom_end = scanned;
        }
    }
    vcfxg_ctx *g = chrom ? gpu_quiet() : nullptr;
    uint64_t bad = ~0ull;
    static_assert(sizeof(BgzfSpan) == sizeof(vcfxg_bgzf_member), "member layout");
    if (!g || vcfxg_ingest_begin(g, total) != VCFXG_OK ||
        vcfxg_ingest_bgzf(g, p, n, reinterpret_cast<const vcfxg_bgzf_member *>(ms.data()), ms.size(), head, hn, &bad) !=
            VCFXG_OK) {
        munmap(hm, kHeadMax);
        phase(bad != ~0ull ? "bgzf device inflate refused a member: host inflate" : "bgzf device path not taken");
        return false;
    }
    phase("bgzf inflated on the device");
    if (map_base && map_len) munmap(map_base, map_len);  // the compressed bytes
    map_base = hm;
    map_len = kHeadMax;
    p = head;
    host_n = hn;
    n = (size_t)total;
    stream_ctx = g;
    streamed = (size_t)total;
    mapped = false;
    gz = true;
    tail = nullptr;
    return true;
}

thread_local ShardRank *t_shard = nullptr;

bool Input::bgzf_view(int err_fd, const BgzfShard &B, uint64_t H, uint64_t lo, uint64_t hi, const std::string &who) {
    const size_t nm = B.ms.size();
    vcfxg_ctx *g = gpu(err_fd);
    if (!g) return false;
    auto fail = [&](const std::string &what) {
        write_str(err_fd, "Error: vcfx_amd: " + who + ": the BGZF input: " + what + "\n");
        return false;
    };
    if (H > lo || lo >= hi || hi > B.off[nm]) return fail("bad view");
    // host memory: the head members' output (the header, then up to a member past it), and the two
    // cut members' output
    const size_t kM = 65536;
    size_t hm_n = 0;
    while (hm_n < nm && B.off[hm_n] < H) hm_n++;  // members [0, hm_n) hold the header
    const size_t head_cap = (size_t)B.off[hm_n] + kM, len = head_cap + 2 * kM;
    void *m = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) return fail("no host memory");
    char *head = (char *)m, *fa = head + head_cap, *fb = fa + kM;
    auto inflate = [&](size_t i, char *dst) {
        size_t got = 0;
        return gz_inflate_member(B.comp + B.ms[i].off, B.ms[i].len, dst, kM, &got) && got == B.ms[i].olen;
    };
    bool ok = true;
    for (size_t i = 0; i < hm_n && ok; i++) ok = inflate(i, head + B.off[i]);
    // the members holding lo and hi - 1
    const size_t mb = (size_t)(std::upper_bound(B.off.begin(), B.off.end(), lo) - B.off.begin()) - 1;
    const size_t me = (size_t)(std::upper_bound(B.off.begin(), B.off.end(), hi - 1) - B.off.begin()) - 1;
    ok = ok && inflate(mb, fa) && (me == mb || inflate(me, fb));
    if (!ok) {
        munmap(m, len);
        return fail("a member does not inflate");
    }
    phase("bgzf shard: head and cut members inflated");
    const uint64_t a0 = lo - B.off[mb], a1 = std::min<uint64_t>(hi, B.off[mb + 1]) - B.off[mb];
    int rc = vcfxg_ingest_begin(g, (size_t)(H + (hi - lo)));
    if (!rc) rc = vcfxg_ingest(g, head, (size_t)H, 0);
    if (!rc) rc = vcfxg_ingest(g, fa + a0, (size_t)(a1 - a0), 0);
    if (!rc && me > mb + 1) {  // the members between: inflated on the device
        const uint64_t c0 = B.ms[mb + 1].off, c1 = B.ms[me - 1].off + B.ms[me - 1].len;
        std::vector<vcfxg_bgzf_member> mm(me - mb - 1);
        for (size_t i = mb + 1; i < me; i++) mm[i - mb - 1] = {B.ms[i].off - c0, B.ms[i].len, B.ms[i].olen};
        uint64_t bad = ~0ull;
        rc = vcfxg_ingest_bgzf(g, B.comp + c0, (size_t)(c1 - c0), mm.data(), mm.size(), head, (size_t)H, &bad);
    }
    if (!rc && me > mb) rc = vcfxg_ingest(g, fb, (size_t)(hi - B.off[me]), 0);
    if (rc) {
        munmap(m, len);
        return gpu_ok(g, rc, "bgzf shard ingest", err_fd);
    }
    phase("bgzf shard on the device");
    if (map_base && map_len) munmap(map_base, map_len);  // the compressed bytes (the planner maps them too)
    map_base = m;
    map_len = len;
    p = head;
    host_n = (size_t)H;
    n = (size_t)(H + (hi - lo));
    stream_ctx = g;
    streamed = n;
    mapped = false;
    gz = true;
    tail = nullptr;
    return true;
}

void shard_records_begin(Out &err) {
    if (!t_shard) return;
    err.flush();
    const off_t at = lseek(t_shard->err_fd, 0, SEEK_CUR);
    t_shard->err_mark = at < 0 ? 0 : (long long)at;
}

size_t reported_size(const Input &in) { return t_shard ? t_shard->whole_bytes : in.source_n; }

bool view_skip_header() {
    if (t_shard) return t_shard->rank > 0;
    const char *e = getenv("VCFX_VIEW_SKIP_HEADER");
    return e && atoi(e) > 0;
}

void Input::apply_view() {
    const char *v = t_shard ? nullptr : getenv("VCFX_INPUT_VIEW");
    unsigned long long h = 0, lo = 0, hi = 0;
    bool have = v && sscanf(v, "%llu:%llu:%llu", &h, &lo, &hi) == 3;
    if (t_shard) {
        h = t_shard->h, lo = t_shard->lo, hi = t_shard->hi;
        have = true;
    }
    if (!have || h > lo || lo > hi || hi > n) {
        populate(map_base, map_len);
        return;
    }
    if (h == 0) {  // no header part: the view is one contiguous range
        p += lo;
        n = host_n = (size_t)(hi - lo);
        populate((void *)p, n);
        return;
    }
    tail = p + lo;
    host_n = (size_t)h;
    n = (size_t)(h + (hi - lo));
    populate((void *)tail, (size_t)(hi - lo));
}

// map a large input's page-cache pages into the page table on a few threads, while the
// context opens: the H2D copy then runs without page faults (load_input joins them)
void Input::populate(void *m, size_t len) {
    if (!m || len < ((size_t)64 << 20)) return;
    const unsigned hw = std::thread::hardware_concurrency();
    const int T = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
    const size_t kStripe = (size_t)32 << 20;
    for (int t = 0; t < T; t++)
        populating.emplace_back([=] {
            for (size_t o = (size_t)t * kStripe; o < len; o += (size_t)T * kStripe)
                if (madvise((char *)m + o, std::min(kStripe, len - o), kMadvPopulateRead) != 0) return;
        });
}

namespace {
// want bytes (fewer at EOF); a read error stops it and leaves its errno in *err
ssize_t read_full(int fd, char *dst, size_t want, int *err) {
    size_t got = 0;
    while (got < want) {
        ssize_t k = ::read(fd, dst + got, want - got);
        if (k < 0 && errno == EINTR) continue;
        if (k < 0) {
            *err = errno;
            return got ? (ssize_t)got : -1;
        }
        if (k == 0) break;
        got += (size_t)k;
    }
    return (ssize_t)got;
}
}  // namespace

// The device-only pipe path's head copy: the head (read into host memory while the context
// opened, often 0.5-2 GB) is copied to the device from pageable memory on a helper thread (~22
// GB/s) while this thread keeps reading the pipe into the region behind it; repeated until the
// bytes left are few, so the pipe never waits for the copy.  eof: the stream ended meanwhile
// (everything then is on the device except the final-chunk marker).  false: a copy failed.
// Faults a reserved region in ahead of a reader (on another core), so read() lands on
// populated pages: 32 MiB steps up to 256 MiB ahead of the reader's position.  Without
// MADV_POPULATE_WRITE (Linux < 5.14) it just stops.
struct Prefaulter {
    std::atomic<size_t> rd;
    std::atomic<bool> done{false};
    std::thread th;
    Prefaulter(char *base, size_t cap, size_t from) : rd(from) {
        const size_t kStep = (size_t)32 << 20, kAhead = (size_t)256 << 20;
        th = std::thread([this, base, cap, from, kStep, kAhead] {
            size_t pop = from & ~(((size_t)2 << 20) - 1);  // (madvise wants page-aligned ranges)
            while (!done.load(std::memory_order_acquire)) {
                if (pop < rd.load(std::memory_order_acquire) + kAhead && pop + kStep <= cap) {
                    if (madvise(base + pop, kStep, kMadvPopulateWrite) != 0) return;
                    pop += kStep;
                } else {
                    std::this_thread::sleep_for(std::chrono::microseconds(50));
                }
            }
        });
    }
    void at(size_t got) { rd.store(got, std::memory_order_release); }
    ~Prefaulter() {
        done.store(true, std::memory_order_release);
        th.join();
    }
};

static bool catch_up(vcfxg_ctx *g, int fd, char *base, size_t cap, size_t &got, bool &eof, int *read_errno,
                     Prefaulter *pf) {
    const size_t kRest = (size_t)8 << 20;
    size_t at = 0;
    for (;;) {
        const size_t upto = got;
        if (upto - at <= kRest || eof) {
            if (upto > at && vcfxg_ingest(g, base + at, upto - at, 0) != VCFXG_OK) return false;
            return true;
        }
        std::atomic<bool> fin{false};
        bool ok = true;
        std::thread t([&] {
            ok = vcfxg_ingest(g, base + at, upto - at, 0) == VCFXG_OK;
            fin.store(true, std::memory_order_release);
        });
        while (!fin.load(std::memory_order_acquire)) {
            if (cap - got < ((size_t)8 << 20)) {
                eof = true;  // the reservation is exhausted: treated as the end (as read_fd does)
                break;
            }
            ssize_t k = ::read(fd, base + got, (size_t)8 << 20);
            if (k < 0 && errno == EINTR) continue;
            if (k < 0) *read_errno = errno;
            if (k <= 0) {
                eof = true;
                break;
            }
            got += (size_t)k;
            if (pf) pf->at(got);
        }
        t.join();
        if (!ok) return false;
        at = upto;
    }
}

void Input::read_fd(int fd, bool host_copy) {
    p = "";
    n = host_n = 0;
    struct stat st;
    if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
        // `< file`: map the rest of the file (the bytes a read loop would return)
        off_t pos = lseek(fd, 0, SEEK_CUR);
        if (pos >= 0 && (off_t)st.st_size > pos) {
            const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
            const size_t lo = (size_t)pos & ~(pg - 1);
            const size_t len = (size_t)st.st_size - lo;
            if ((size_t)st.st_size - (size_t)pos >= prefetch_bytes()) gpu_prefetch();
            void *m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, (off_t)lo);
            if (m != MAP_FAILED) {
                madvise(m, len, len < ((size_t)64 << 20) ? (MADV_SEQUENTIAL | MADV_WILLNEED) : MADV_SEQUENTIAL);
                populate(m, len);
                map_base = m;
                map_len = len;
                p = (const char *)m + ((size_t)pos - lo);
                n = host_n = source_n = (size_t)st.st_size - (size_t)pos;
                lseek(fd, st.st_size, SEEK_SET);  // consumed, as by a read loop
                return;
            }
        } else if (pos >= 0) {
            return;  // at EOF
        }
    }
#ifdef F_SETPIPE_SZ
    if (fcntl(fd, F_GETPIPE_SZ) > 0) (void)fcntl(fd, F_SETPIPE_SZ, 1 << 20);  // fewer, larger reads
#endif
    // reserved address space (not memory): the bytes never move, so chunks already handed
    // to the device copy stay valid while the read continues
    size_t cap = 0;
    void *m = MAP_FAILED;
    for (int sh : {40, 36, 32, 30}) {
        if (sh > reserve_log2()) continue;
        cap = (size_t)1 << sh;
        m = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (m != MAP_FAILED) break;
    }
    if (m == MAP_FAILED) return;
    madvise(m, cap, MADV_HUGEPAGE);
    char *const base = (char *)m;
    map_base = m;
    map_len = cap;
    p = base;

    // the head of the stream (up to 2 chunks) always lands in host memory: the '#CHROM' gate
    // runs on it, and small inputs never reach the device
    const size_t kPre = std::min(prefetch_bytes(), cap / 4), kChunk = stream_chunk();  // reads stay inside the region
    ssize_t k0 = read_full(fd, base, kPre, &read_errno);
    size_t got = k0 > 0 ? (size_t)k0 : 0;
    if (gzip_ok && is_gzip(base, got) && gzip_enabled()) {
        // compressed: all of it to the host (decompress() inflates it)
        for (;;) {
            if (cap - got < ((size_t)8 << 20)) break;
            ssize_t k = ::read(fd, base + got, (size_t)8 << 20);
            if (k < 0 && errno == EINTR) continue;
            if (k < 0) read_errno = errno;
            if (k <= 0) break;
            got += (size_t)k;
        }
        n = host_n = source_n = got;
        return;
    }
    std::unique_ptr<Prefaulter> head_pf;  // the device-only path's head reader's helper
    bool chrom = false;  // the head holds the complete '#CHROM' line
    size_t scanned = 0;
    auto scan = [&] {
        while (!chrom && scanned < got) {
            const char *s0 = base + scanned;
            const char *nl = (const char *)memchr(s0, '\n', got - scanned);
            if (!nl) break;
            chrom = is_chrom_line(s0, (size_t)(nl - s0));
            scanned = (size_t)(nl - base) + 1;
        }
    };
    if (got == kPre) {
        gpu_prefetch();  // a large input: the HIP runtime starts while the rest arrives
        // the head keeps arriving into host memory while the context opens (a read that
        // waited for the open would stall the writer for ~0.2 s); a device-only stream also
        // needs the whole header in it
        const size_t head_cap = std::max<size_t>(2 * kChunk, (size_t)256 << 20);
        // (the pages ahead of the reader faulted in on another core: the head arrives at the
        // pipe's rate, not the page-fault rate)
        if (!host_copy) head_pf.reset(new Prefaulter(base, cap, got));
        for (;;) {
            if (!host_copy) scan();
            const bool enough = got >= 2 * kChunk &&
                                (host_copy || ((chrom || got >= head_cap) && g_open_done.load(std::memory_order_acquire)));
            if (enough) break;
            if (got >= ((size_t)8 << 30) || cap - got < ((size_t)8 << 20)) break;
            ssize_t k = ::read(fd, base + got, std::min<size_t>((size_t)8 << 20, std::max(kChunk, kPre)));
            if (k < 0 && errno == EINTR) continue;
            if (k < 0) read_errno = errno;
            if (k <= 0) {
                n = host_n = got;
                return;  // EOF: everything is on the host
            }
            got += (size_t)k;
            if (head_pf) head_pf->at(got);
        }
    }
    if (got < 2 * kChunk) {
        n = host_n = got;
        return;
    }
    if (!host_copy && chrom) {
        // the caller needs only the header on the host (VCFX_allele_freq_calc): the rest goes
        // straight to the device through a pinned staging ring -- no host copy, no page faults
        vcfxg_ctx *g = gpu_quiet();
        bool eof = false;
        if (g && vcfxg_ingest_begin(g, (size_t)1 << 30) == VCFXG_OK && catch_up(g, fd, base, cap, got, eof, &read_errno, head_pf.get())) {
            head_pf.reset();
            // the host keeps the header only (the records are on the device)
            host_n = scanned;
            stream_ctx = g;
            ring_ctx = g;
            if (eof) {  // all of it arrived while the head was copied
                n = streamed = got;
                phase("stdin streamed to the device (during the head copy)");
                return;
            }
            const int kSlots = (int)std::min<size_t>(64, std::max<size_t>(2, env_bytes("VCFX_RING_SLOTS", 16)));
            const size_t kSlot = ring_slot();
            bool ok = true;
            for (int i = 0; i < kSlots && ok; i++) {
                void *r = nullptr;
                ok = vcfxg_host_alloc(g, kSlot, &r) == VCFXG_OK;
                if (ok) ring.push_back(r);
            }
            size_t total = got;
            std::vector<size_t> slot_end(kSlots, 0);  // input offset where the slot's last chunk ended
            phase("stdin head ingested");
            using clk = std::chrono::steady_clock;
            double t_wait = 0, t_read = 0, t_ing = 0;
            for (int k = 0; ok; k = (k + 1) % kSlots) {
                const auto a0 = clk::now();
                ok = vcfxg_ingest_wait(g, slot_end[k]) == VCFXG_OK;
                if (!ok) break;
                const auto a1 = clk::now();
                ssize_t r = read_full(fd, (char *)ring[k], kSlot, &read_errno);
                const auto a2 = clk::now();
                if (r <= 0) break;
                ok = vcfxg_ingest(g, (const char *)ring[k], (size_t)r, 0) == VCFXG_OK;
                const auto a3 = clk::now();
                t_wait += std::chrono::duration<double, std::milli>(a1 - a0).count();
                t_read += std::chrono::duration<double, std::milli>(a2 - a1).count();
                t_ing += std::chrono::duration<double, std::milli>(a3 - a2).count();
                total += (size_t)r;
                slot_end[k] = total;
                if ((size_t)r < kSlot) break;
            }
            n = total;
            streamed = ok ? total : 0;  // a failure is reported when the input is used
            // (the head's record pages stay mapped until exit: freeing them early with
            // MADV_DONTNEED on a helper thread -- 1-2 GB, ~40 ms/GB -- slowed the ring's DMA when
            // it overlapped the stream and the device work when it came after, more than the
            // exit saves: r04 e2e probes)
            if (timing_on) {
                char b[160];
                snprintf(b, sizeof b, "stdin streamed to the device (head %zu MB; ring: wait %.1f, read %.1f, ingest %.1f ms)",
                         got >> 20, t_wait, t_read, t_ing);
                phase(b);
            } else {
                phase("stdin streamed to the device");
            }
            return;
        }
    }
    n = host_n = got;

    head_pf.reset();
    std::unique_ptr<Prefaulter> pre(new Prefaulter(base, cap, got));
    // device ingest of complete chunks on its own thread, overlapping the pipe read (the
    // context comes from the background open; a failed open here is silent)
    std::mutex mu;
    std::condition_variable cv;
    size_t avail = got;  // bytes read so far, published to the ingest thread
    bool eof = false;
    std::thread ing([&] {
        vcfxg_ctx *g = gpu_quiet();
        if (!g) return;
        size_t at = 0;
        bool ok = vcfxg_ingest_begin(g, (size_t)1 << 30) == VCFXG_OK;
        for (;;) {
            size_t upto;
            bool fin;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return eof || avail - at >= kChunk; });
                fin = eof;
                upto = fin ? avail : at + (avail - at) / kChunk * kChunk;
            }
            if (ok && upto > at) ok = vcfxg_ingest(g, base + at, upto - at, 0) == VCFXG_OK;
            at = upto;
            if (fin) break;
        }
        stream_ctx = g;
        streamed = ok ? at : 0;
    });
    for (;;) {
        if (cap - got < ((size_t)8 << 20)) break;  // reservation exhausted (> 1 TiB of stdin)
        ssize_t k = ::read(fd, base + got, (size_t)8 << 20);
        if (k < 0 && errno == EINTR) continue;
        if (k < 0) read_errno = errno;
        if (k <= 0) break;
        got += (size_t)k;
        pre->at(got);
        std::lock_guard<std::mutex> lk(mu);
        avail = got;
        cv.notify_one();
    }
    pre.reset();
    {
        std::lock_guard<std::mutex> lk(mu);
        avail = got;
        eof = true;
        cv.notify_one();
    }
    ing.join();
    n = host_n = got;
}

bool write_device_text(vcfxg_ctx *g, uint64_t bytes, Out &out, int err_fd) {
    out.flush();
    if (!bytes) return true;
    std::vector<void *> slots;
    size_t slot = 0;
    {
        std::lock_guard<std::mutex> lk(g_ring_mu);
        if (g_file_ring.ctx == g && !g_file_ring.busy) {
            slots = g_file_ring.slots;
            slot = g_file_ring.slot;
            g_file_ring.busy = !slots.empty();
        }
    }
    struct RingRelease {
        bool on;
        ~RingRelease() {
            if (!on) return;
            std::lock_guard<std::mutex> lk(g_ring_mu);
            g_file_ring.busy = false;
        }
    } ring_release{!slots.empty()};
    if (slots.empty()) {  // no pinned ring on this context (or it is in use): one pageable copy
        std::string text(bytes, '\0');
        if (!gpu_ok(g, vcfxg_fetch_text(g, &text[0], text.size()), "fetch", err_fd)) return false;
        write_all(out.fd, text.data(), text.size());
        return true;
    }
    // through the pinned staging slots (the input's DMAs are complete): no page faults on a
    // fresh host buffer, DMA-rate copies
    for (uint64_t o = 0, k = 0; o < bytes; o += slot, k++) {
        const size_t n = (size_t)std::min<uint64_t>(slot, bytes - o);
        void *b = slots[k % slots.size()];
        if (!gpu_ok(g, vcfxg_fetch_text_range(g, o, n, b), "fetch", err_fd)) return false;
        write_all(out.fd, (const char *)b, n);
    }
    return true;
}

bool load_input(vcfxg_ctx *g, const Input &in, int err_fd) {
    in.join_populate();
    if (in.read_errno) {  // a read(2) error is not the end of the input (nor is a full reservation)
        write_str(err_fd, std::string("Error: vcfx_amd: reading the input failed: ") + strerror(in.read_errno) + "\n");
        return false;
    }
    phase("page population joined");
    if (in.tail) {  // a shard view: header + record range, straight from the mapping
        int rc = vcfxg_ingest_begin(g, in.n);
        if (!rc) rc = vcfxg_ingest(g, in.p, in.host_n, 0);
        if (!rc) rc = vcfxg_ingest(g, in.tail, in.n - in.host_n, 1);
        return gpu_ok(g, rc, "load view", err_fd);
    }
    if (in.stream_ctx == g && in.streamed == in.n) {
        // the bytes are on the device already (streamed while stdin was read); complete it
        phase("completing the device input");
        return gpu_ok(g, vcfxg_ingest(g, nullptr, 0, 1), "ingest", err_fd);
    }
    if (in.host_n != in.n) {  // a device-only stream whose ingest failed: nothing to redo
        write_str(err_fd, "Error: vcfx_amd: streaming stdin to the device failed: " +
                              std::string(vcfxg_last_error(in.stream_ctx ? in.stream_ctx : g)) + "\n");
        return false;
    }
    return gpu_ok(g, vcfxg_load_host(g, in.p, in.n), "load", err_fd);
}

void write_all(int fd, const char *p, size_t n) {
    while (n) {
        ssize_t k = ::write(fd, p, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return;
        p += k;
        n -= (size_t)k;
    }
}

}  // namespace vcfxh
