// emit.h -- ordered pass-through of input lines to an fd with writev, merging runs of
// consecutive lines that are contiguous in the (mmap'd / buffered) input.  Pass-through
// tools (record_filter, genotype_query, ld matrix) write kept records straight from the
// host copy of the input; only per-line decisions come back from the device.
#pragma once
#include <errno.h>
#include <sys/uio.h>

#include <algorithm>

#include <vector>

#include "hostio.h"

namespace vcfxh {

struct LineEmitter {
    const char *base, *end;
    int fd;
    std::vector<iovec> iov;
    const char *rs = nullptr, *re = nullptr;
    LineEmitter(const char *b, size_t n, int f) : base(b), end(b + n), fd(f) { iov.reserve(1024); }
    ~LineEmitter() { finish(); }
    // [ls, le) followed by "\n"
    void line(const char *ls, const char *le) {
        if (le < end && *le == '\n') extend(ls, le + 1);
        else {
            extend(ls, le);
            close_run();
            push((const char *)"\n", 1);
        }
    }
    void raw(const char *p, size_t n) {
        close_run();
        push(p, n);
    }
    void finish() {
        close_run();
        drain();
    }

   private:
    void extend(const char *s, const char *e) {
        if (rs && re == s) re = e;
        else {
            close_run();
            rs = s;
            re = e;
        }
    }
    void close_run() {
        if (rs && re > rs) push(rs, (size_t)(re - rs));
        rs = re = nullptr;
    }
    void push(const char *p, size_t n) {
        iov.push_back({const_cast<char *>(p), n});
        if (iov.size() >= 512) drain();
    }
    void drain() {
        size_t i = 0;
        while (i < iov.size()) {
            int cnt = (int)std::min<size_t>(iov.size() - i, 512);
            ssize_t k = ::writev(fd, &iov[i], cnt);
            if (k < 0) {
                if (errno == EINTR) continue;
                break;
            }
            size_t left = (size_t)k;
            while (i < iov.size() && left >= iov[i].iov_len) left -= iov[i++].iov_len;
            if (left && i < iov.size()) {
                iov[i].iov_base = (char *)iov[i].iov_base + left;
                iov[i].iov_len -= left;
            }
        }
        iov.clear();
    }
};

}  // namespace vcfxh
