// hostio.cpp -- see hostio.h
#include "hostio.h"

#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace vcfxh {

const void *memchr_(const char *p, const char *end) { return memchr(p, '\n', (size_t)(end - p)); }

Input::~Input() {
    if (mapped && p && n) munmap(const_cast<char *>(p), n);
}

bool Input::open_file(const char *path) {
    int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) < 0) {
        ::close(fd);
        return false;
    }
    n = (size_t)st.st_size;
    if (n == 0) {
        ::close(fd);
        p = "";
        return true;
    }
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) {
        n = 0;
        return false;
    }
    madvise(m, n, MADV_SEQUENTIAL | MADV_WILLNEED);
    p = (const char *)m;
    mapped = true;
    return true;
}

void Input::read_fd(int fd) {
    heap.clear();
    size_t cap = 1 << 20;
    heap.resize(cap);
    size_t got = 0;
    for (;;) {
        if (got == heap.size()) heap.resize(heap.size() * 2);
        ssize_t k = ::read(fd, &heap[got], heap.size() - got);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) break;
        got += (size_t)k;
    }
    heap.resize(got);
    p = heap.data();
    n = got;
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

static vcfxg_ctx *g_ctx = nullptr;

vcfxg_ctx *gpu(int err_fd) {
    if (g_ctx) return g_ctx;
    int dev = 0;
    if (const char *e = getenv("VCFX_DEVICE")) dev = atoi(e);
    int rc = vcfxg_open(dev, &g_ctx);
    if (rc != VCFXG_OK) {
        write_str(err_fd, std::string("Error: vcfx_amd: no usable MI355X (gfx950) device ") + std::to_string(dev) +
                              " (vcfxg_open rc=" + std::to_string(rc) + "); this build has no CPU path.\n");
        g_ctx = nullptr;
    }
    return g_ctx;
}

bool gpu_ok(vcfxg_ctx *c, int rc, const char *what, int err_fd) {
    if (rc == VCFXG_OK) return true;
    write_str(err_fd, std::string("Error: vcfx_amd: ") + what + " failed (rc=" + std::to_string(rc) + "): " +
                          vcfxg_last_error(c) + "\n");
    return false;
}

}  // namespace vcfxh
