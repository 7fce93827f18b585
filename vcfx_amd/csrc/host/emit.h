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
    // [s, e) as it is (no newline added)
    void bytes(const char *s, const char *e) { extend(s, e); }
    void raw(const char *p, size_t n) {
        close_run();
        push(p, n);
    }
    void finish() {
        close_run();
        drain();
    }
    // write everything pending, then take a new base buffer (a moved input window)
    void rebase(const char *b, size_t n) {
        finish();
        base = b;
        end = b + n;
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

// Host pointers to the lines of an input's data region, in order, for the pass-through tools.
// A host-resident input (file mapping, `< file`, a host-copied pipe) is addressed in place.
// A device-only stdin stream (Input::host_n < n: the bytes past the header were streamed to
// the device without a host copy) is read back through a pinned window of >= 64 MiB
// (vcfxg_input_fetch, ~50 GB/s; window_bytes()); the emitter writes out what it holds before the window
// moves, so every pointer it keeps stays valid.
struct LineSource {
    const Input &in;
    vcfxg_ctx *g;
    LineEmitter &em;
    char *win = nullptr;
    size_t win_cap = 0;
    uint64_t w0 = 0, w1 = 0;  // window = input bytes [w0, w1)
    bool ok = true;
    LineSource(const Input &i, vcfxg_ctx *ctx, LineEmitter &e) : in(i), g(ctx), em(e) {}
    ~LineSource() {
        if (!win) return;
        em.finish();  // the emitter may still point into the window
        vcfxg_host_free(g, win);
    }
    bool device_only() const { return in.host_n < in.n && !in.tail; }
    bool in_tail = false;
    // bytes [a, b) of the input, plus the byte at b when b < n (the line's newline); nullptr
    // (and ok = false) when the pinned window cannot be allocated or filled: the caller stops
    // at that line and reports the error, writing nothing from it
    const char *at(uint64_t a, uint64_t b) {
        if (in.tail && a >= in.host_n) {  // a shard view: the record range elsewhere in the mapping
            if (!in_tail) {
                em.rebase(in.tail, in.n - in.host_n);
                in_tail = true;
            }
            return in.tail + (a - in.host_n);
        }
        if (!device_only()) return in.p + a;
        const uint64_t need = std::min<uint64_t>(b + 1, in.n);
        if (a >= w0 && need <= w1 && win) return win + (a - w0);
        const size_t want = (size_t)std::max<uint64_t>(window_bytes(), need - a);
        em.finish();  // the emitter may point into the old window: write it out first
        if (want > win_cap) {
            if (win) vcfxg_host_free(g, win);
            win = nullptr;
            if (vcfxg_host_alloc(g, want, (void **)&win) != VCFXG_OK) {
                ok = false;
                win = nullptr;
                win_cap = 0;
                w0 = w1 = 0;
                return nullptr;
            }
            win_cap = want;
        }
        const uint64_t e = std::min<uint64_t>(in.n, a + win_cap);
        if (vcfxg_input_fetch(g, a, (size_t)(e - a), win) != VCFXG_OK) {
            ok = false;  // the window's bytes are stale: nothing may be written from them
            w0 = w1 = 0;
            return nullptr;
        }
        w0 = a;
        w1 = e;
        em.rebase(win, (size_t)(e - a));
        return win;
    }
};

}  // namespace vcfxh
