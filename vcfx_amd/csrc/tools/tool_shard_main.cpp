// tool_shard_main.cpp -- the in-process multi-GPU drop-in: VCFX_NGPU=N VCFX_<tool> [args] FILE.
//
// One process, one host thread and one device context per rank (SURVEY §8(b) vcfxg_shard_run,
// §8(e)); no launcher, so argv stays the reference's.  The input file is mapped once to plan
// the cuts; each rank thread runs the tool itself on its VIEW of the file -- the header bytes
// [0, H) (through the '#CHROM' line) and its records [cut_r, cut_r+1) -- cut at i*size/N and
// advanced past the next '\n', the reference's own split (VCFX_allele_counter.cpp:889-901,
// computed by vcfxg_shard_cuts).  Rank 0 writes its stdout straight to the output; ranks > 0
// write per-rank memory files that follow in rank order (on a pipe each as soon as it and the
// ranks before it are done; on a regular file in parallel at exclusive-scan offsets);
// their stderr too, ranks > 0 from the point where their record phase began (the argument and
// header messages are rank 0's).  Each rank leaves its counters (AF's "Processed V variants
// from L data lines", missing_detector's totals) in its ShardRank; they are all-reduced over
// the rank clique (vcfxg_comm: RCCL / xGMI when the ranks sit on distinct devices) and rank 0
// writes the summary after every rank's stderr.
//
//   record tools (a view per rank): VCFX_allele_freq_calc, VCFX_record_filter,
//     VCFX_genotype_query, VCFX_nonref_filter, VCFX_dosage_calculator, VCFX_hwe_tester,
//     VCFX_missing_detector, VCFX_allele_counter (not -z)
//   VCFX_ld_calculator (streaming): every rank parses the file and writes the pair rows of its
//     `--shard r/N` share (equal window-pair counts)
// A BGZF file (.vcf.gz as bgzip writes it) is cut the same way in the coordinates of its inflated
// bytes: the planner parses the member chain, inflates on the host the members up to the '#CHROM'
// line and the W - 1 members that hold the cuts (the cut advanced past the next '\n' there), and
// each rank inflates the members wholly inside its records on its own device (Input::bgzf_view);
// for VCFX_ld_calculator every rank inflates the whole file on its device.
// Anything else -- stdin input, a gzip file that is not such a chain, data lines before '#CHROM',
// help / version, LD matrix mode, other tools -- runs as the plain single-context tool.  VCFX_NGPU larger than
// the device count puts several ranks on a device (round robin): the one-GPU rehearsal.
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/sendfile.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "hostio.h"
#include "tools.h"

using namespace vcfxh;

namespace {

enum Kind { kUnsharded = 0, kView = 1, kRows = 2 };

// value-taking options of each drop-in (their getopt tables / argument loops)
struct ToolOpts {
    const char *tool;
    std::set<std::string> shortv, longv;
    Kind kind;
};
const std::vector<ToolOpts> &tool_opts() {
    static const std::vector<ToolOpts> t = {
        {"VCFX_allele_freq_calc", {"-i"}, {"--input"}, kView},
        {"VCFX_record_filter", {"-f", "-l", "-i"}, {"--filter", "--logic", "--input"}, kView},
        {"VCFX_genotype_query", {"-g", "-i"}, {"--genotype-query", "--input"}, kView},
        {"VCFX_nonref_filter", {"-i"}, {"--input"}, kView},
        {"VCFX_dosage_calculator", {"-i"}, {"--input"}, kView},
        {"VCFX_hwe_tester", {"-i"}, {"--input"}, kView},
        {"VCFX_missing_detector", {"-i"}, {"--input"}, kView},
        {"VCFX_allele_counter", {"-s", "-i", "-t", "-l"}, {"--samples", "--input", "--threads", "--limit-samples"}, kView},
        {"VCFX_ld_calculator", {"-i", "-r", "-w", "-t", "-n", "-d"},
         {"--input", "--region", "--window", "--threshold", "--threads", "--max-distance", "--shard"}, kRows},
    };
    return t;
}

struct Parsed {
    std::vector<std::pair<std::string, std::string>> opts;  // (name, value or "")
    std::vector<std::string> operands;
    bool has(std::initializer_list<const char *> names) const {
        for (auto &o : opts)
            for (const char *n : names)
                if (o.first == n) return true;
        return false;
    }
};

// argv[1:] the GNU getopt_long way: options may follow operands, "--" ends them, a value-taking
// option consumes its attached / '='-joined value or the next argument (vcfx_amd/shard.py
// parse_args is the same rule)
Parsed parse(const ToolOpts &T, int argc, char **argv) {
    Parsed P;
    for (int i = 1; i < argc; i++) {
        const std::string a = argv[i];
        if (a == "--") {
            for (int k = i + 1; k < argc; k++) P.operands.push_back(argv[k]);
            break;
        }
        if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
            const size_t eq = a.find('=');
            const std::string name = a.substr(0, eq);
            if (eq != std::string::npos) P.opts.push_back({name, a.substr(eq + 1)});
            else if (T.longv.count(name)) {
                P.opts.push_back({name, i + 1 < argc ? argv[i + 1] : ""});
                i++;
            } else P.opts.push_back({name, ""});
        } else if (a.size() > 1 && a[0] == '-') {
            for (size_t k = 1; k < a.size(); k++) {
                const std::string o = std::string("-") + a[k];
                if (T.shortv.count(o)) {
                    if (k + 1 < a.size()) P.opts.push_back({o, a.substr(k + 1)});
                    else {
                        P.opts.push_back({o, i + 1 < argc ? argv[i + 1] : ""});
                        i++;
                    }
                    break;
                }
                P.opts.push_back({o, ""});
            }
        } else P.operands.push_back(a);
    }
    return P;
}

const char *base_name(const char *tool) {
    const char *t = strrchr(tool, '/');
    return t ? t + 1 : tool;
}

struct Mapping {
    const char *p = nullptr;
    size_t n = 0;
    ~Mapping() {
        if (p && n) munmap((void *)p, n);
    }
};

// the byte after the first '#CHROM' line (a trailing '\r' dropped first, as the file paths
// do), n if none (*found: whether there is one); pre = a data line (not empty, not '#') comes before it
size_t header_end(const char *p, size_t n, bool *pre, bool *found = nullptr) {
    *pre = false;
    if (found) *found = false;
    size_t at = 0;
    while (at < n) {
        const char *nl = (const char *)memchr(p + at, '\n', n - at);
        const size_t e = nl ? (size_t)(nl - p) : n;
        size_t le = e;
        if (le > at && p[le - 1] == '\r') le--;
        if (le > at) {
            if (p[at] != '#') *pre = true;
            else if (is_chrom_line(p + at, le - at)) {
                if (found) *found = e < n;  // (a '#CHROM' line cut by the end of p is not complete)
                return e < n ? e + 1 : n;
            }
        }
        at = e + 1;
    }
    return n;
}

// the plan: kind, input path, the world actually used and world + 1 cuts (view kind); a BGZF
// file: its member chain, h and the cuts in the inflated bytes' coordinates
struct Plan {
    Kind kind = kUnsharded;
    std::string path;
    size_t whole = 0, h = 0;
    std::vector<uint64_t> cuts;
    int world = 1;
    std::shared_ptr<BgzfShard> bgz;
};

// the cuts of a BGZF file (map): false when it is not a chain the device inflates, has a data line
// before '#CHROM' or no record after it.  The header end H is found in the inflated head; the cut
// r is the byte after the first '\n' at or past H + r (total - H) / W (vcfxg_shard_cuts' rule on the
// inflated bytes), found by inflating the member that holds it (and the next ones, for a line
// longer than the member's rest).
bool plan_bgzf(const Mapping &map, int ngpu, Plan &pl) {
    const char *e = getenv("VCFX_BGZF_DEVICE");
    if ((e && e[0] == '0') || !gzip_enabled()) return false;
    auto B = std::make_shared<BgzfShard>();
    uint64_t total = 0;
    if (!bgzf_chain(map.p, map.n, B->ms, &total) || B->ms.empty()) return false;
    const size_t nm = B->ms.size();
    B->comp = map.p;
    B->comp_n = map.n;
    B->off.resize(nm + 1);
    for (size_t i = 0; i < nm; i++) B->off[i + 1] = B->off[i] + B->ms[i].olen;
    std::vector<char> buf;
    auto inflate = [&](size_t i, std::vector<char> &dst) {  // member i appended to dst
        const size_t at = dst.size();
        dst.resize(at + B->ms[i].olen);
        size_t got = 0;
        return gz_inflate_member(map.p + B->ms[i].off, B->ms[i].len, dst.data() + at, B->ms[i].olen, &got) &&
               got == B->ms[i].olen;
    };
    // the header end
    bool pre = false;
    size_t H = 0;
    for (size_t i = 0;; i++) {
        if (i == nm || buf.size() > ((size_t)64 << 20) || !inflate(i, buf)) return false;
        bool found = false;
        H = header_end(buf.data(), buf.size(), &pre, &found);
        if (pre) return false;
        if (found) break;
    }
    if (H >= total) return false;
    std::vector<uint64_t> cuts((size_t)ngpu + 1);
    cuts[0] = H;
    cuts[(size_t)ngpu] = total;
    for (int r = 1; r < ngpu; r++) {
        // (t > H: a line starts at t when byte t - 1 is a '\n'; else the cut is past the next one)
        const uint64_t t = H + (total - H) * (uint64_t)r / (uint64_t)ngpu;
        if (t <= H || t <= cuts[(size_t)r - 1]) {
            cuts[(size_t)r] = std::max<uint64_t>(t, cuts[(size_t)r - 1]);
            continue;
        }
        size_t k = (size_t)(std::upper_bound(B->off.begin(), B->off.end(), t - 1) - B->off.begin()) - 1;
        uint64_t cut = total, from = t - 1 - B->off[k];
        for (; k < nm; k++, from = 0) {
            std::vector<char> mb;
            if (!inflate(k, mb)) return false;
            const char *nl = from < mb.size() ? (const char *)memchr(mb.data() + from, '\n', mb.size() - from) : nullptr;
            if (nl) {
                cut = B->off[k] + (uint64_t)(nl - mb.data()) + 1;
                break;
            }
        }
        cuts[(size_t)r] = std::max(cut, cuts[(size_t)r - 1]);
    }
    std::vector<uint64_t> keep{cuts[0]};
    for (int r = 1; r <= ngpu; r++)
        if (cuts[(size_t)r] > keep.back() || r == ngpu) keep.push_back(cuts[(size_t)r]);
    if (keep.size() > 2 && keep[keep.size() - 1] == keep[keep.size() - 2]) keep.pop_back();
    if (keep.size() < 3) return false;
    pl.h = H;
    pl.cuts = keep;
    pl.world = (int)keep.size() - 1;
    pl.bgz = B;
    pl.kind = kView;
    return true;
}

Plan make_plan(const char *tool, int argc, char **argv, int ngpu, Mapping &map) {
    Plan pl;
    if (ngpu < 2) return pl;
    const char *t = base_name(tool);
    const ToolOpts *T = nullptr;
    for (auto &x : tool_opts())
        if (!strcmp(x.tool, t)) T = &x;
    if (!T) return pl;
    const Parsed P = parse(*T, argc, argv);
    if (P.has({"-h", "--help", "-v", "--version"})) return pl;
    std::string path;
    bool have = false;
    for (auto &o : P.opts)
        if (o.first == "-i" || o.first == "--input") {
            path = o.second;
            have = true;
        }
    if (!have && T->kind == kView && !P.operands.empty()) {
        path = P.operands[0];
        have = true;
    }
    if (!have || path.empty() || path == "-") return pl;
    if (T->kind == kRows) {
        if (P.has({"-m", "--matrix", "--shard"})) return pl;
    } else if (!strcmp(t, "VCFX_allele_counter") && P.has({"-z", "--gzip"})) {
        return pl;
    }
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return pl;
    struct stat st;
    if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode) || st.st_size < 2) {
        ::close(fd);
        return pl;
    }
    const size_t n = (size_t)st.st_size;
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) return pl;
    map.p = (const char *)m;
    map.n = n;
    pl.path = path;
    pl.whole = n;
    if ((unsigned char)map.p[0] == 0x1f && (unsigned char)map.p[1] == 0x8b) {  // gzip / BGZF
        Plan g = pl;
        if (T->kind == kRows) {  // (every rank inflates the whole file on its device)
            if (gzip_enabled()) {
                g.kind = kRows;
                g.world = ngpu;
                return g;
            }
        } else if (plan_bgzf(map, ngpu, g)) {
            return g;
        }
        return Plan{};
    }
    if (T->kind == kRows) {
        pl.kind = kRows;
        pl.world = ngpu;
        return pl;
    }
    bool pre = false;
    pl.h = header_end(map.p, n, &pre);
    if (pre || pl.h >= n) return pl;  // data before '#CHROM', or no record region
    std::vector<uint64_t> cuts((size_t)ngpu + 1);
    if (vcfxg_shard_cuts(map.p, n, pl.h, ngpu, cuts.data()) != VCFXG_OK) return pl;
    // ranks whose record range came out empty (more ranks than records) are dropped
    std::vector<uint64_t> keep{cuts[0]};
    for (int r = 1; r <= ngpu; r++)
        if (cuts[r] > keep.back() || r == ngpu) keep.push_back(cuts[r]);
    if (keep.size() > 2 && keep[keep.size() - 1] == keep[keep.size() - 2]) keep.pop_back();
    pl.cuts = keep;
    pl.world = (int)keep.size() - 1;
    if (pl.world < 2) return pl;
    pl.kind = kView;
    return pl;
}

size_t fd_size(int fd) {
    struct stat st;
    return fstat(fd, &st) == 0 ? (size_t)st.st_size : 0;
}

// bytes [off, off + n) of src to dst (sendfile, else read / write)
bool copy_range(int src, size_t off, size_t n, int dst) {
    off_t o = (off_t)off;
    size_t left = n;
    while (left) {
        ssize_t k = sendfile(dst, src, &o, std::min<size_t>(left, (size_t)1 << 30));
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) break;
        left -= (size_t)k;
    }
    if (!left) return true;
    std::vector<char> b((size_t)4 << 20);
    while (left) {
        ssize_t k = pread(src, b.data(), std::min(left, b.size()), o);
        if (k <= 0) return false;
        write_all(dst, b.data(), (size_t)k);
        o += k;
        left -= (size_t)k;
    }
    return true;
}

int memfd(const char *name) {
    int fd = memfd_create(name, MFD_CLOEXEC);
    if (fd < 0) {  // (no memfd: an unlinked temporary file)
        char tmpl[] = "/tmp/vcfx_rankXXXXXX";
        fd = mkstemp(tmpl);
        if (fd >= 0) unlink(tmpl);
    }
    return fd;
}

}  // namespace

extern "C" int vcfx_shard_plan(const char *tool, int argc, char **argv, int ngpu, uint64_t *cuts, int *kind) {
    Mapping map;
    const Plan pl = make_plan(tool, argc, argv, ngpu, map);
    if (kind) *kind = pl.bgz ? 3 : (int)pl.kind;
    if (pl.kind == kUnsharded) return 1;
    if (cuts && pl.kind == kView)
        for (int r = 0; r <= pl.world; r++) cuts[r] = pl.cuts[(size_t)r];
    return pl.world;
}

extern "C" int vcfx_tool_main_sharded(const char *tool, int argc, char **argv, int in_fd, int out_fd, int err_fd,
                                      int ngpu) {
    int ndev = 0;
    if (ngpu < 2 || vcfxg_device_count(&ndev) != VCFXG_OK || ndev < 1)
        return vcfx_tool_main(tool, argc, argv, in_fd, out_fd, err_fd);
    Mapping map;
    const Plan pl = make_plan(tool, argc, argv, ngpu, map);
    if (pl.kind == kUnsharded) return vcfx_tool_main(tool, argc, argv, in_fd, out_fd, err_fd);
    const int W = pl.world;
    phase("shard plan");
    std::vector<ShardRank> sr((size_t)W);
    std::vector<int> outs((size_t)W, -1), rc((size_t)W, 0), open_rc((size_t)W, 0);
    std::vector<vcfxg_ctx *> ctx((size_t)W, nullptr);
    std::vector<std::string> shard_arg((size_t)W);
    for (int r = 0; r < W; r++) {
        ShardRank &s = sr[(size_t)r];
        s.rank = r;
        s.world = W;
        s.whole_bytes = pl.whole;
        if (pl.kind == kView) {
            s.h = pl.h;
            s.lo = pl.cuts[(size_t)r];
            s.hi = pl.cuts[(size_t)r + 1];
            s.bgz = pl.bgz.get();
        } else {
            s.h = 0, s.lo = 0, s.hi = pl.whole;
            shard_arg[(size_t)r] = std::to_string(r) + "/" + std::to_string(W);
        }
        outs[(size_t)r] = memfd("vcfx_rank_out");
        s.err_fd = memfd("vcfx_rank_err");
        if (outs[(size_t)r] < 0 || s.err_fd < 0) {
            write_str(err_fd, "Error: vcfx_amd: no memory file for a rank's output\n");
            return 1;
        }
    }
    // rank 0 writes its stdout straight to out_fd (its bytes come first whatever the other ranks
    // do); ranks > 0 write memory files that follow it in rank order
    struct stat ost;
    const int ofl = fcntl(out_fd, F_GETFL);
    const off_t start = lseek(out_fd, 0, SEEK_CUR);
    const bool regular = fstat(out_fd, &ost) == 0 && S_ISREG(ost.st_mode) && start >= 0 && ofl >= 0 &&
                         !(ofl & O_APPEND);
    ::close(outs[0]);
    outs[0] = -1;
    // ranks: open the context (in parallel), wait for the clique, run the tool, reduce
    std::mutex mu;
    std::condition_variable cv;
    int opened = 0;
    bool go = false;
    std::vector<char> done((size_t)W, 0);
    std::vector<int> red_rc((size_t)W, VCFXG_OK);
    vcfxg_comm *comm = nullptr;
    std::vector<std::thread> th;
    for (int r = 0; r < W; r++)
        th.emplace_back([&, r] {
            ShardRank &s = sr[(size_t)r];
            s.device = r % ndev;
            open_rc[(size_t)r] = vcfxg_open(s.device, &ctx[(size_t)r]);
            s.open_rc = open_rc[(size_t)r];
            {
                std::unique_lock<std::mutex> lk(mu);
                opened++;
                cv.notify_all();
                cv.wait(lk, [&] { return go; });
            }
            s.g = open_rc[(size_t)r] == VCFXG_OK ? ctx[(size_t)r] : nullptr;
            std::vector<char *> av(argv, argv + argc);
            std::string shard_opt = "--shard";
            if (pl.kind == kRows) {
                av.push_back(&shard_opt[0]);
                av.push_back(&shard_arg[(size_t)r][0]);
            }
            av.push_back(nullptr);
            t_shard = &s;
            rc[(size_t)r] = vcfx_tool_main(tool, (int)av.size() - 1, av.data(), in_fd, r ? outs[(size_t)r] : out_fd,
                                           s.err_fd);
            t_shard = nullptr;
            {
                std::lock_guard<std::mutex> lk(mu);
                done[(size_t)r] = 1;
                cv.notify_all();
            }
            // every rank takes part, whatever its run did (no rank can be left waiting: the clique
            // votes on the host before any rank enters the collective)
            if (comm) red_rc[(size_t)r] = vcfxg_comm_allreduce_u64(comm, r, s.cnt, 8);
        });
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return opened == W; });
        bool all = true;
        for (int r = 0; r < W; r++) all = all && open_rc[(size_t)r] == VCFXG_OK;
        if (all && vcfxg_comm_init(ctx.data(), W, &comm) != VCFXG_OK) comm = nullptr;
        go = true;
        cv.notify_all();
    }
    // a pipe / terminal: each rank's bytes as soon as it and every rank before it are done
    bool streamed_ok = true;
    int streamed = 0;
    if (!regular) {
        for (int r = 1; r < W; r++) {
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return done[0] && done[(size_t)r]; });
            }
            if (sr[0].err_mark < 0) break;  // rank 0 stopped before its records: its streams alone
            streamed_ok = copy_range(outs[(size_t)r], 0, fd_size(outs[(size_t)r]), out_fd) && streamed_ok;
            streamed = r;
        }
    }
    for (auto &t : th) t.join();
    phase("ranks done");
    uint64_t sum[8] = {};
    bool red_ok = true;
    if (comm) {
        for (int k = 0; k < 8; k++) sum[k] = sr[0].cnt[k];  // (every rank holds the sums)
        for (int r = 0; r < W; r++) red_ok = red_ok && red_rc[(size_t)r] == VCFXG_OK;
    } else {
        for (int r = 0; r < W; r++)
            for (int k = 0; k < 8; k++) sum[k] += sr[(size_t)r].cnt[k];
    }
    // outputs in rank order
    const ShardRank &s0 = sr[0];
    int ret = 0;
    if (s0.err_mark < 0) {  // rank 0 stopped before its records (arguments, open): its streams alone
        copy_range(s0.err_fd, 0, fd_size(s0.err_fd), err_fd);
        ret = rc[0];
    } else {
        if (regular && W > 1) {  // ranks > 0: their bytes at their offsets after rank 0's, in parallel
            const off_t end0 = lseek(out_fd, 0, SEEK_CUR);
            std::vector<size_t> osz((size_t)W, 0), ooff((size_t)W + 1, 0);
            ooff[1] = end0 >= start ? (size_t)(end0 - start) : 0;
            for (int r = 1; r < W; r++) {
                osz[(size_t)r] = fd_size(outs[(size_t)r]);
                ooff[(size_t)r + 1] = ooff[(size_t)r] + osz[(size_t)r];
            }
            std::vector<std::thread> wt;
            std::atomic<bool> ok{end0 >= start};
            for (int r = 1; r < W; r++)
                wt.emplace_back([&, r] {
                    const size_t n = osz[(size_t)r];
                    if (!n) return;
                    void *m = mmap(nullptr, n, PROT_READ, MAP_SHARED, outs[(size_t)r], 0);
                    if (m == MAP_FAILED) {
                        ok = false;
                        return;
                    }
                    size_t at = 0;
                    while (at < n) {
                        ssize_t k = pwrite(out_fd, (const char *)m + at, std::min<size_t>(n - at, (size_t)1 << 30),
                                           start + (off_t)(ooff[(size_t)r] + at));
                        if (k < 0 && errno == EINTR) continue;
                        if (k <= 0) {
                            ok = false;
                            break;
                        }
                        at += (size_t)k;
                    }
                    munmap(m, n);
                });
            for (auto &t : wt) t.join();
            lseek(out_fd, start + (off_t)ooff[(size_t)W], SEEK_SET);
            if (!ok) ret = 1;
        } else {
            for (int r = streamed + 1; r < W; r++)
                streamed_ok = copy_range(outs[(size_t)r], 0, fd_size(outs[(size_t)r]), out_fd) && streamed_ok;
            if (!streamed_ok) ret = 1;
        }
        for (int r = 0; r < W; r++) {
            const ShardRank &s = sr[(size_t)r];
            const size_t n = fd_size(s.err_fd);
            if (r > 0 && s.err_mark < 0) {
                // a rank that stopped before its records where rank 0 did not: its argument /
                // header messages are rank 0's already; only its last line (the error) is its own
                std::string e(n, '\0');
                if (n && pread(s.err_fd, &e[0], n, 0) == (ssize_t)n) {
                    size_t end = e.size();
                    while (end && e[end - 1] == '\n') end--;
                    const size_t b = e.rfind('\n', end ? end - 1 : 0);
                    const size_t from = (b == std::string::npos || end == 0) ? 0 : b + 1;
                    if (end > from) write_str(err_fd, e.substr(from, end - from) + "\n");
                }
                continue;
            }
            const size_t from = r == 0 ? 0 : (size_t)s.err_mark;
            if (n > from) copy_range(s.err_fd, from, n - from, err_fd);
        }
        if (!red_ok) {
            // the summary below is the host reduction's (always computed); the RCCL path failed
            std::string e = "Error: vcfx_amd: the ranks' count all-reduce failed";
            for (int r = 0; r < W; r++)
                if (red_rc[(size_t)r] != VCFXG_OK && ctx[(size_t)r]) {
                    e += std::string(": ") + vcfxg_last_error(ctx[(size_t)r]);
                    break;
                }
            write_str(err_fd, e + "\n");
            ret = 1;
        }
        bool all_ok = true;  // (a failed rank's counts are missing: no summary of partial sums)
        for (int r = 0; r < W; r++) all_ok = all_ok && rc[(size_t)r] == 0;
        if (s0.summary && all_ok) write_str(err_fd, s0.summary(sum));
        for (int r = 0; r < W && !ret; r++) ret = rc[(size_t)r];
    }
    for (int r = 0; r < W; r++) {
        if (outs[(size_t)r] >= 0) ::close(outs[(size_t)r]);
        ::close(sr[(size_t)r].err_fd);
    }
    if (!g_process_exit_fast) {  // (an executable ends right after: the runtime drops them)
        vcfxg_comm_destroy(comm);
        for (int r = 0; r < W; r++)
            if (ctx[(size_t)r]) vcfxg_close(ctx[(size_t)r]);
    }
    phase("shard outputs written");
    return ret;
}
