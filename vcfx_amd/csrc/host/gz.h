// gz.h -- gzip / BGZF input (see gz.cpp)
#pragma once
#include <stddef.h>

namespace vcfxh {

struct GzResult {
    bool ok = false;      // every member inflated (false: truncated / corrupt; n = bytes inflated before)
    bool bgzf = false;    // the parallel BGZF path ran
    size_t n = 0;         // output bytes
    size_t members = 0;
};

// gzip magic (0x1f 0x8b) at p
bool is_gzip(const char *p, size_t n);
// inflate the gzip / BGZF stream [src, src+n) into [dst, dst+cap) on up to `threads` threads
GzResult gz_inflate(const char *src, size_t n, char *dst, size_t cap, int threads);

}  // namespace vcfxh
