// host_san_test.cpp -- drives the drop-ins' host input layer (vcfx_amd/csrc/host/hostio.cpp,
// gz.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer and ThreadSanitizer builds
// (`make sanitize`; tests/test_sanitize.py).  No device is needed: every path here is host
// work -- the file mapping with its page-population threads, the shard view, BGZF members
// inflated on many threads, plain and multi-member gzip, a truncated stream, and the pipe
// reader with its pre-fault and ingest threads (whose device open fails cleanly on a host
// without a GPU).  Prints one line per case: "<case> <bytes> <checksum>", checksum = the sum
// of (i + 1) * byte_i mod 2^64 over the logical input (header part, then a view's tail).
//
//   host_san_test PLAIN BGZF GZIP MULTI TRUNC
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "hostio.h"

using vcfxh::Input;

namespace {
void report(const char *what, const Input &in) {
    // the whole logical input: header part [0, host_n) then, for a view, the tail
    unsigned long long h = 0;
    for (size_t i = 0; i < in.host_n; i++) h += (unsigned long long)(i + 1) * (unsigned char)in.p[i];
    for (size_t i = 0; in.tail && i < in.n - in.host_n; i++)
        h += (unsigned long long)(in.host_n + i + 1) * (unsigned char)in.tail[i];
    printf("%s %zu %llu\n", what, in.n, h);
}

bool open_and_inflate(const char *what, const char *path, bool gz) {
    Input in;
    in.gzip_ok = gz;
    if (!in.open_file(path)) {
        printf("%s open-failed\n", what);
        return false;
    }
    if (!in.decompress(2)) {
        printf("%s inflate-failed\n", what);
        return false;
    }
    in.join_populate();
    report(what, in);
    return true;
}
}  // namespace

int main(int argc, char **argv) {
    setvbuf(stdout, nullptr, _IOLBF, 0);
    if (argc < 6) {
        fprintf(stderr, "usage: host_san_test PLAIN BGZF GZIP MULTI TRUNC\n");
        return 2;
    }
    // 1. a mapped file of >= 64 MiB: page-table population on helper threads
    open_and_inflate("plain", argv[1], false);
    // 2. the same as a shard view (header bytes + a record range of the mapping)
    {
        Input probe;
        probe.open_file(argv[1]);
        probe.join_populate();
        const size_t n = probe.n, h = 4096, lo = n / 3, hi = 2 * n / 3;
        std::string v = std::to_string(h) + ":" + std::to_string(lo) + ":" + std::to_string(hi);
        setenv("VCFX_INPUT_VIEW", v.c_str(), 1);
        open_and_inflate("view", argv[1], false);
        unsetenv("VCFX_INPUT_VIEW");
    }
    // 3. BGZF members inflated in parallel; 4. one gzip member; 5. several members; 6. truncated
    open_and_inflate("bgzf", argv[2], true);
    open_and_inflate("gzip", argv[3], true);
    open_and_inflate("multi", argv[4], true);
    open_and_inflate("trunc", argv[5], true);
    // 7. the BGZF chain walked piece by piece as the file ring does (BgzfStream::feed), and with
    //    each piece's chain scanned beforehand (BgzfChunk::scan + adopt, the ring's readers): both
    //    equal to bgzf_chain on the whole file, for pieces smaller than a member, about a member,
    //    and larger (odd sizes: headers and trailers cut at every offset)
    {
        FILE *f = fopen(argv[2], "rb");
        std::string z;
        char b[1 << 16];
        size_t k;
        while (f && (k = fread(b, 1, sizeof b, f)) > 0) z.append(b, k);
        if (f) fclose(f);
        std::vector<vcfxh::BgzfSpan> whole;
        uint64_t tot = 0;
        const bool okw = vcfxh::bgzf_chain(z.data(), z.size(), whole, &tot);
        bool same = okw;
        for (size_t piece : {(size_t)1000, (size_t)4099, (size_t)65536, (size_t)70001, (size_t)1 << 20, (size_t)16 << 20}) {
            vcfxh::BgzfStream fw, ad;
            vcfxh::BgzfChunk c;
            for (size_t o = 0; o < z.size(); o += piece) {
                const size_t n = std::min(piece, z.size() - o);
                fw.feed(z.data() + o, n);
                c.scan(z.data() + o, n, o);
                ad.adopt(z.data() + o, n, c);
            }
            auto eq = [&](const vcfxh::BgzfStream &s) {
                if (!s.ok(z.size()) || s.members.size() != whole.size() || s.out != tot) return false;
                for (size_t i = 0; i < whole.size(); i++)
                    if (s.members[i].off != whole[i].off || s.members[i].len != whole[i].len ||
                        s.members[i].olen != whole[i].olen)
                        return false;
                return true;
            };
            same = same && eq(fw) && eq(ad);
        }
        printf("chain %zu %s\n", whole.size(), same ? "same" : "differs");
    }
    // 8. a pipe read whole into the head; 9. the same with a 1 MiB head and 4 MiB chunks: the
    // reader, its pre-fault thread, the background device open and the ingest thread (no
    // device here: the open fails and the ingest thread leaves)
    for (int round = 0; round < 2; round++) {
        if (round == 1) {
            setenv("VCFX_PREFETCH_BYTES", "1048576", 1);
            setenv("VCFX_STREAM_CHUNK", "4194304", 1);
        }
        int fds[2];
        if (pipe(fds) != 0) return 1;
        std::thread writer([&] {
            int f = ::open(argv[1], O_RDONLY);
            static char buf[1 << 20];
            for (;;) {
                ssize_t k = ::read(f, buf, sizeof buf);
                if (k <= 0) break;
                for (ssize_t o = 0; o < k;) {
                    ssize_t w = ::write(fds[1], buf + o, (size_t)(k - o));
                    if (w <= 0) break;
                    o += w;
                }
            }
            ::close(f);
            ::close(fds[1]);
        });
        Input in;
        in.read_fd(fds[0], true);
        if (in.read_errno) fprintf(stderr, "read error: %s\n", strerror(in.read_errno));
        writer.join();
        ::close(fds[0]);
        report(round ? "pipe_threads" : "pipe", in);
    }
    return 0;
}
