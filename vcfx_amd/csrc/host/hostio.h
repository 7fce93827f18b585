// hostio.h -- host-side plumbing shared by the VCFX_<tool> drop-ins: whole-input staging
// (mmap of a file = the reference's MappedFile; or all of stdin), fd writers, the per-
// process GPU context, and the '#CHROM' gate scan that runs on the host before the
// device takes the record region.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <string>

#include "vcfx_gpu.h"

namespace vcfxh {

struct Input {
    const char *p = nullptr;
    size_t n = 0;
    bool mapped = false;
    std::string heap;  // stdin bytes
    ~Input();
    // MappedFile::open semantics (VCFX_allele_freq_calc.cpp:52-63): false if open/stat
    // fails; a 0-byte file is a successful empty map.
    bool open_file(const char *path);
    void read_fd(int fd);
};

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
// run a vcfxg_* call; on failure prints the context error and returns false
bool gpu_ok(vcfxg_ctx *c, int rc, const char *what, int err_fd);

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
