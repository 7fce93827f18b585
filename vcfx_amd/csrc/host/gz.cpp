// gz.cpp -- compressed input for the record tools: gzip and BGZF
// (blocked gzip, the .vcf.gz of 1000 Genomes and every htslib writer) inflated on the host
// into the tool's input region, BGZF blocks on all host threads at once.
//
// Reference anchors: StreamingGzipReader (src/vcfx_core.cpp:144-354: 64 KiB reads, members
// inflated in sequence, inflateReset between BGZF / gzip members) and countVariantsGzip
// (VCFX_variant_counter.cpp:261-328).  A BGZF member is a gzip member whose FEXTRA field
// holds the subfield 'B','C' with BSIZE = member bytes - 1 (SAM/BAM spec §4.1), so the
// member chain is known before any byte is inflated, and ISIZE (the member's last 4 bytes)
// gives every member's output offset: the members then inflate independently.
#include "gz.h"

#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

namespace vcfxh {

namespace {

struct Member {
    size_t off, len;   // compressed bytes of the whole member
    size_t out, olen;  // its output offset and ISIZE
};

inline uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
inline uint16_t le16(const uint8_t *p) { return (uint16_t)(p[0] | p[1] << 8); }

// BSIZE of a BGZF member header at p (n bytes available), or 0 if it is not one
size_t bgzf_bsize(const uint8_t *p, size_t n) {
    if (n < 18 || p[0] != 0x1f || p[1] != 0x8b || p[2] != 8 || !(p[3] & 4)) return 0;
    const size_t xlen = le16(p + 10);
    if (12 + xlen > n) return 0;
    for (size_t k = 12; k + 4 <= 12 + xlen;) {
        const size_t slen = le16(p + k + 2);
        if (p[k] == 'B' && p[k + 1] == 'C' && slen == 2 && k + 6 <= 12 + xlen) return (size_t)le16(p + k + 4) + 1;
        k += 4 + slen;
    }
    return 0;
}

// inflate one gzip member [src, src+n) into [dst, dst+cap): false on any zlib error or size
// mismatch (the CRC and ISIZE are checked by zlib's gzip wrapper)
bool inflate_member(const uint8_t *src, size_t n, char *dst, size_t cap, size_t *got) {
    z_stream z;
    memset(&z, 0, sizeof z);
    if (inflateInit2(&z, 16 + 15) != Z_OK) return false;
    z.next_in = const_cast<Bytef *>(src);
    z.avail_in = (uInt)n;
    z.next_out = (Bytef *)dst;
    z.avail_out = (uInt)cap;
    const int rc = inflate(&z, Z_FINISH);
    *got = cap - z.avail_out;
    inflateEnd(&z);
    return rc == Z_STREAM_END;
}

}  // namespace

bool bgzf_chain(const char *src_c, size_t n, std::vector<BgzfSpan> &ms, uint64_t *total) {
    const uint8_t *src = (const uint8_t *)src_c;
    ms.clear();
    uint64_t out = 0;
    size_t p = 0;
    while (p < n) {
        const uint8_t *h = src + p;
        if (n - p < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4) return false;
        const size_t xlen = le16(h + 10);
        const size_t bs = bgzf_bsize(h, n - p);
        if (!bs || bs > n - p || bs < 12 + xlen + 8 || bs > 65536) return false;
        const uint32_t olen = le32(h + bs - 4);
        if (olen > 65536) return false;
        ms.push_back({(uint64_t)p, (uint32_t)bs, olen});
        out += olen;
        p += bs;
    }
    *total = out;
    return !ms.empty();
}

// one member at h (n bytes available): 1 = a member of *bs bytes (validated as bgzf_chain does),
// 0 = more bytes needed, -1 = not a BGZF member
static int chain_member(const uint8_t *h, size_t n, size_t *bs, uint32_t *olen) {
    if (n < 4) return 0;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || h[3] != 4) return -1;
    if (n < 18) return 0;
    const size_t xlen = le16(h + 10);
    if (n < 12 + xlen) return 0;
    const size_t b = bgzf_bsize(h, n);
    if (!b || b < 12 + xlen + 8 || b > 65536) return -1;
    if (b > n) return 0;
    *bs = b;
    *olen = le32(h + b - 4);
    return *olen > 65536 ? -1 : 1;
}

void BgzfStream::feed(const char *d_c, size_t len) {
    const uint8_t *d = (const uint8_t *)d_c;
    const uint64_t off = fed;
    fed += len;
    if (bad) return;
    size_t r = 0;  // the next unread byte of d
    if (!carry.empty()) {  // complete the member at pos from this piece (a member is <= 64 KiB)
        const size_t had = carry.size(), take = std::min<size_t>(len, 65536 + 64 - had);
        carry.insert(carry.end(), d_c, d_c + take);
        size_t bs = 0;
        uint32_t olen = 0;
        const int k = chain_member((const uint8_t *)carry.data(), carry.size(), &bs, &olen);
        if (k < 0 || (k == 0 && take < len)) {
            bad = true;
            return;
        }
        if (k == 0) return;  // (the whole piece went to the carry: more to come)
        members.push_back({pos, (uint32_t)bs, olen});
        out += olen;
        r = pos + bs - off;  // (bs > had: the member ends inside this piece)
        pos += bs;
        carry.clear();
    }
    while (r < len) {
        size_t bs = 0;
        uint32_t olen = 0;
        const int k = chain_member(d + r, len - r, &bs, &olen);
        if (k < 0) {
            bad = true;
            return;
        }
        if (k == 0) {  // the member continues in the next piece
            carry.assign(d_c + r, d_c + len);
            return;
        }
        members.push_back({pos, (uint32_t)bs, olen});
        out += olen;
        pos += bs;
        r += bs;
    }
}

void BgzfChunk::scan(const char *d_c, size_t len, uint64_t off) {
    const uint8_t *d = (const uint8_t *)d_c;
    ms.clear();
    first = end = ~0ull;
    // the first position at which a member header validates (a guess: adopt() takes the chain
    // only if the stream's own walk arrives exactly there)
    size_t r = 0, bs = 0;
    uint32_t olen = 0;
    for (;;) {
        const void *q = r < len ? memchr(d + r, 0x1f, len - r) : nullptr;
        if (!q) return;
        r = (size_t)((const uint8_t *)q - d);
        if (chain_member(d + r, len - r, &bs, &olen) > 0) break;
        r++;
    }
    first = off + r;
    int k;
    do {
        ms.push_back({off + r, (uint32_t)bs, olen});
        r += bs;
    } while ((k = chain_member(d + r, len - r, &bs, &olen)) > 0);
    end = off + r;  // (the member at end is cut by the chunk's end, or not a member: the walk decides)
}

void BgzfStream::adopt(const char *d_c, size_t len, const BgzfChunk &c) {
    const uint64_t off = fed;
    if (bad) {
        fed += len;
        return;
    }
    size_t r = 0;  // the bytes of d the carried member takes
    if (!carry.empty()) {
        const size_t had = carry.size(), take = std::min<size_t>(len, 65536 + 64 - had);
        carry.insert(carry.end(), d_c, d_c + take);
        size_t bs = 0;
        uint32_t olen = 0;
        const int k = chain_member((const uint8_t *)carry.data(), carry.size(), &bs, &olen);
        if (k < 0 || (k == 0 && take < len)) {
            bad = true;
            fed += len;
            return;
        }
        if (k == 0) {
            fed += len;
            return;
        }
        members.push_back({pos, (uint32_t)bs, olen});
        out += olen;
        r = pos + bs - off;
        pos += bs;
        carry.clear();
    }
    if (c.first != pos || c.end > off + len) {  // (the guess is not where the walk is: walk it here)
        fed = off + r;
        feed(d_c + r, len - r);
        return;
    }
    for (const BgzfSpan &m : c.ms) out += m.olen;
    members.insert(members.end(), c.ms.begin(), c.ms.end());
    pos = c.end;
    fed = c.end;
    feed(d_c + (c.end - off), len - (size_t)(c.end - off));  // (the rest: the member the chunk cuts)
}

bool gz_inflate_member(const char *src, size_t n, char *dst, size_t cap, size_t *got) {
    return inflate_member((const uint8_t *)src, n, dst, cap, got);
}

bool is_gzip(const char *p, size_t n) { return n >= 2 && (unsigned char)p[0] == 0x1f && (unsigned char)p[1] == 0x8b; }

GzResult gz_inflate(const char *src_c, size_t n, char *dst, size_t cap, int threads) {
    const uint8_t *src = (const uint8_t *)src_c;
    GzResult r;
    // the BGZF member chain (stops at the first member that is not BGZF, or at a truncation)
    std::vector<Member> ms;
    size_t p = 0, out = 0;
    while (p < n) {
        const size_t bs = bgzf_bsize(src + p, n - p);
        if (!bs || p + bs > n || bs < 26) break;
        const size_t olen = le32(src + p + bs - 4);
        ms.push_back({p, bs, out, olen});
        out += olen;
        p += bs;
    }
    if (!ms.empty() && p == n && out <= cap) {
        // every member is BGZF: inflate them on all threads straight into place
        r.bgzf = true;
        r.members = ms.size();
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        const int T = std::max(1, std::min<int>(threads, (int)((ms.size() + 63) / 64)));
        std::vector<std::thread> pool;
        for (int t = 0; t < T; t++)
            pool.emplace_back([&] {
                for (;;) {
                    const size_t i0 = next.fetch_add(64);  // 64 members (~4 MiB of output) per grab
                    if (i0 >= ms.size() || bad.load(std::memory_order_relaxed)) return;
                    for (size_t i = i0; i < std::min(ms.size(), i0 + 64); i++) {
                        size_t got = 0;
                        if (!inflate_member(src + ms[i].off, ms[i].len, dst + ms[i].out, ms[i].olen, &got) ||
                            got != ms[i].olen) {
                            bad.store(true);
                            return;
                        }
                    }
                }
            });
        for (auto &th : pool) th.join();
        if (!bad.load()) {
            r.ok = true;
            r.n = out;
            return r;
        }
        r.bgzf = false;  // a corrupt member: the sequential path finds where it fails
    }
    // plain gzip (or a BGZF file with a damaged member): members inflated in sequence, as
    // StreamingGzipReader does; the output keeps what inflated before an error
    z_stream z;
    memset(&z, 0, sizeof z);
    if (inflateInit2(&z, 16 + 15) != Z_OK) return r;
    z.next_in = const_cast<Bytef *>(src);
    size_t in_left = n, o = 0;
    r.members = 0;
    for (;;) {
        const uInt take = (uInt)std::min<size_t>(in_left, (size_t)1 << 30);
        z.avail_in = take;
        const size_t room = std::min<size_t>(cap - o, (size_t)1 << 30);
        z.next_out = (Bytef *)(dst + o);
        z.avail_out = (uInt)room;
        const int rc = inflate(&z, Z_NO_FLUSH);
        o += room - z.avail_out;
        in_left -= take - z.avail_in;
        if (rc == Z_STREAM_END) {
            r.members++;
            if (in_left == 0) {
                r.ok = true;
                break;
            }
            // more input: the next member (StreamingGzipReader resets and reads on; bytes that
            // are no gzip member -- garbage, zero padding -- fail there as here)
            inflateReset(&z);
            continue;
        }
        if (rc != Z_OK && rc != Z_BUF_ERROR) break;
        if (rc == Z_BUF_ERROR && z.avail_out != 0 && in_left == 0) break;  // truncated stream
        if (o >= cap) break;                                                  // out of room
    }
    inflateEnd(&z);
    r.n = o;
    return r;
}

}  // namespace vcfxh
