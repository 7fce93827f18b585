"""BGZF writers and crafted DEFLATE streams for the device-inflate tests (test infrastructure).

bgzf_member(data, ...) wraps one raw deflate stream (zlib.compressobj with wbits -15, any level,
strategy, memLevel, window, and optional mid-stream flushes that put several blocks -- and empty
stored blocks -- in a member) as a BGZF member (SAM/BAM spec §4.1: gzip header with FLG = FEXTRA
and the 'BC' subfield holding BSIZE - 1, then CRC-32 and ISIZE).  BitWriter builds hand-made
deflate streams (RFC 1951) for the cases zlib must refuse or accept at the edges."""
import struct
import zlib


def wrap_member(raw, data, crc=None, isize=None, extra=b""):
    """a BGZF member around the raw deflate bytes `raw` of `data`"""
    xlen = 6 + len(extra)
    bsize = 12 + xlen + len(raw) + 8
    hdr = b"\x1f\x8b\x08\x04\x00\x00\x00\x00\x00\xff" + struct.pack("<H", xlen) + extra + \
        b"BC" + struct.pack("<HH", 2, bsize - 1)
    c = zlib.crc32(data) & 0xFFFFFFFF if crc is None else crc
    n = len(data) & 0xFFFFFFFF if isize is None else isize
    return hdr + raw + struct.pack("<II", c, n)


def deflate_raw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8, wbits=15, flush_at=(), flush=zlib.Z_FULL_FLUSH):
    co = zlib.compressobj(level, zlib.DEFLATED, -wbits, mem, strategy)
    out, prev = [], 0
    for cut in sorted(flush_at) + [len(data)]:
        out.append(co.compress(data[prev:cut]))
        if cut < len(data):
            out.append(co.flush(flush))
        prev = cut
    out.append(co.flush(zlib.Z_FINISH))
    return b"".join(out)


def bgzf_member(data, **kw):
    return wrap_member(deflate_raw(data, **kw), data)


EOF_MEMBER = bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 0xFF, 6, 0, 0x42, 0x43, 2, 0, 0x1B, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0])


def bgzf(data, block=65280, **kw):
    """the whole of data as BGZF (blocks of `block` bytes) + the EOF member"""
    return b"".join(bgzf_member(data[o:o + block], **kw) for o in range(0, len(data), block)) + EOF_MEMBER


def zlib_member(member):
    """what zlib makes of one gzip member on its own: (ok, output); ok only when the stream ends
    exactly at the member's end (no unused bytes)"""
    d = zlib.decompressobj(31)
    try:
        out = d.decompress(member)
        out += d.flush()
    except zlib.error:
        return False, None
    return d.eof and not d.unused_data, out


class BitWriter:
    """LSB-first bit packing (RFC 1951 §3.1.1); Huffman codes are written MSB-first"""

    def __init__(self):
        self.v, self.n, self.out = 0, 0, bytearray()

    def bits(self, val, n):
        self.v |= (val & ((1 << n) - 1)) << self.n
        self.n += n
        while self.n >= 8:
            self.out.append(self.v & 0xFF)
            self.v >>= 8
            self.n -= 8

    def code(self, code, length):
        self.bits(int(format(code, "0%db" % length)[::-1], 2) if length else 0, length)

    def align(self):
        if self.n:
            self.bits(0, 8 - self.n)

    def done(self):
        self.align()
        return bytes(self.out)


def canonical(lengths):
    """RFC 1951 §3.2.2 codes for a list of code lengths (0 = unused)"""
    bl = [0] * 16
    for l in lengths:
        if l:
            bl[l] += 1
    code, nxt = 0, [0] * 16
    for b in range(1, 16):
        code = (code + bl[b - 1]) << 1
        nxt[b] = code
    out = []
    for l in lengths:
        if l:
            out.append((nxt[l], l))
            nxt[l] += 1
        else:
            out.append(None)
    return out


FIXED_LL = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
FIXED_D = [5] * 32
CL_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


def dynamic_header(w, ll_lens, d_lens, cl_lens=None, hlit=None, hdist=None):
    """write a dynamic block's header with the given code lengths (no run-length codes unless
    cl_lens / explicit symbols are used by the caller); returns the CL code used"""
    hlit = len(ll_lens) if hlit is None else hlit
    hdist = len(d_lens) if hdist is None else hdist
    seq = list(ll_lens) + list(d_lens)
    if cl_lens is None:
        # a complete code over the lengths used: a balanced tree
        used = sorted(set(seq))
        cl_lens = [0] * 19
        # a complete code over the used symbols: lengths from a balanced tree
        k = max(1, (len(used) - 1).bit_length())
        extra = (1 << k) - len(used)
        for i, s in enumerate(used):
            cl_lens[s] = k - 1 if i < extra else k
        if len(used) == 1:
            cl_lens[used[0]] = 1
            cl_lens[0 if used[0] else 1] = 1  # (a single code must still be complete)
    ncl = 19
    while ncl > 4 and cl_lens[CL_ORDER[ncl - 1]] == 0:
        ncl -= 1
    w.bits(hlit - 257, 5)
    w.bits(hdist - 1, 5)
    w.bits(ncl - 4, 4)
    for i in range(ncl):
        w.bits(cl_lens[CL_ORDER[i]], 3)
    cl = canonical(cl_lens)
    for l in seq:
        w.code(*cl[l])
    return cl
