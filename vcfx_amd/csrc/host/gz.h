// gz.h -- gzip / BGZF input (see gz.cpp)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

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

// The member chain of [src, src+n) when all of it is BGZF in the form the device inflates
// (vcfxg_ingest_bgzf): each member a gzip member with CM 8 and FLG exactly FEXTRA, a 'BC'
// subfield (BSIZE), ISIZE <= 64 KiB, the members ending exactly at n.  members[i] = {offset,
// bytes, ISIZE}; *total = the sum of ISIZE.  false: not such a chain (the host path inflates it).
struct BgzfSpan {
    uint64_t off;
    uint32_t len, olen;
};
bool bgzf_chain(const char *src, size_t n, std::vector<BgzfSpan> &members, uint64_t *total);
// bgzf_chain on a stream fed in order, piece by piece (a staging ring's slots): feed(d, len) takes
// the next len bytes; a member whose bytes span pieces is completed from a carry of at most
// 64 KiB.  ok(total) after the last piece: the same chain bgzf_chain returns on the whole stream.
// The members of one piece of the stream found without the walk before it (a reader thread's,
// on the bytes it just read): the first offset at which a member header validates, the chain of
// complete members from there and the offset past the last; BgzfStream::adopt takes them when the
// stream's own walk arrives at `first`, else walks the piece itself.
struct BgzfChunk {
    std::vector<BgzfSpan> ms;
    uint64_t first = ~0ull, end = ~0ull;
    void scan(const char *d, size_t len, uint64_t off);  // d = stream bytes [off, off + len)
};
struct BgzfStream {
    std::vector<BgzfSpan> members;
    uint64_t out = 0;   // the sum of ISIZE so far
    uint64_t pos = 0;   // the next member's first byte
    uint64_t fed = 0;   // bytes fed so far
    bool bad = false;   // not a BGZF chain
    std::vector<char> carry;  // bytes [pos, fed) of a member not yet complete
    void feed(const char *d, size_t len);
    // feed(d, len) with the piece's members scanned beforehand (the same chain, faster)
    void adopt(const char *d, size_t len, const BgzfChunk &c);
    bool ok(uint64_t total) const { return !bad && carry.empty() && pos == total && fed == total && !members.empty(); }
};
// one gzip member [src, src+n) inflated into [dst, dst+cap) by zlib (CRC and ISIZE checked);
// *got = its bytes; false on any error
bool gz_inflate_member(const char *src, size_t n, char *dst, size_t cap, size_t *got);

}  // namespace vcfxh
