"""Device BGZF inflate (vcfxg_ingest_bgzf, vcfxg_inflate.hip) against zlib -- the library the
reference reads .vcf.gz through (StreamingGzipReader, src/vcfx_core.cpp:144-354).

- Streams zlib makes (every level 0-9, the five strategies, memLevel 1/9, windows of 2^9..2^15,
  mid-member full / sync / block flushes, which put several blocks and empty stored blocks in a
  member) of VCF text, random bytes, runs and long-range repeats: the device output is zlib's,
  byte for byte, member by member and concatenated.
- Damaged members (bit flips in the deflate data, the CRC and ISIZE): whenever zlib refuses a
  member the device refuses it too (the caller then inflates on the host, where zlib reports the
  damage as the reference does); whenever the device accepts one, zlib accepts it with the same
  bytes.
- Hand-made streams at the edges of RFC 1951 / zlib: distance 32768, a single-code literal
  table, an empty distance code, over-subscribed and incomplete codes, a missing end-of-block
  code, repeats with nothing before them, literal/length 286-287 and distance 30-31 in fixed
  blocks, a distance past the member start, stored LEN / NLEN mismatch, block type 3, a stream
  ending before / running into its trailer.
- The drop-in tools on BGZF input through the device path (VCFX_BGZF_DEVICE_MIN=0), against the
  oracle on the plain text, with the schedule log showing the device inflate ran."""
import os
import random
import subprocess
import tempfile
import zlib

import numpy as np
import pytest

from tests import _bgzf as B
from tests._golden import Oracle
from vcfx_amd import engine, synth, tool_binary

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = engine.Engine(0)
    yield e
    e.close()


def _device(eng, chain):
    """the device's output of a BGZF chain (bytes), or ("bad", member, text); ("host", 1, why) when
    the host's chain check already refuses it (e.g. an ISIZE over 64 KiB: the host inflates)"""
    try:
        engine.bgzf_members(np.frombuffer(chain, np.uint8))
    except ValueError as e:
        return ("host", 1, str(e))
    r = eng.load_bgzf(chain)
    if r is not None:
        return ("bad",) + tuple(r)
    total = int(engine.bgzf_members(np.frombuffer(chain, np.uint8))["out_len"].sum())
    return eng.input_bytes(0, total)


def _datasets():
    rnd = random.Random(3)
    vcf = synth.generate(300, 157, 91, 1, 0.01, 0, 0.05, 0)
    rb = bytes(rnd.getrandbits(8) for _ in range(70000))
    far = bytes(rnd.getrandbits(8) for _ in range(32000))
    mixed = bytearray()
    while len(mixed) < 65536:
        k = rnd.random()
        if k < 0.4:
            mixed += vcf[rnd.randrange(len(vcf) - 900):][:rnd.randrange(1, 900)]
        elif k < 0.6:
            mixed += bytes([rnd.getrandbits(8)]) * rnd.randrange(1, 600)
        elif k < 0.8:
            mixed += rb[:rnd.randrange(1, 300)]
        else:
            back = rnd.randrange(1, min(len(mixed), 32768) + 1) if mixed else 1
            mixed += mixed[len(mixed) - back:][:rnd.randrange(1, 300)]
    # (a BGZF member holds at most 64 KiB of compressed bytes: 65,280 B of input, as bgzip cuts)
    return {
        "vcf": vcf[:65280], "vcf_tail": vcf[-40000:], "random": rb[:65280], "zeros": bytes(65280),
        "one": b"x", "empty": b"", "runs": b"ab" * 20000 + b"a" * 25280, "far": far + far[:30000],
        "mixed": bytes(mixed[:65280]), "short_text": b"#CHROM\tPOS\n1\t2\n",
    }


PARAMS = [dict(level=l) for l in range(10)] + [
    dict(level=6, strategy=zlib.Z_FILTERED), dict(level=6, strategy=zlib.Z_HUFFMAN_ONLY),
    dict(level=6, strategy=zlib.Z_RLE), dict(level=6, strategy=zlib.Z_FIXED), dict(level=1, strategy=zlib.Z_FIXED),
    dict(level=9, mem=1), dict(level=9, mem=9), dict(level=6, wbits=9), dict(level=9, wbits=12),
    dict(level=6, flush_at=(1000, 1000, 30000)), dict(level=1, flush_at=(7, 4096), flush=zlib.Z_SYNC_FLUSH),
    dict(level=6, flush_at=(20000, 40000), flush=zlib.Z_BLOCK), dict(level=0, flush_at=(10, 20)),
]


@pytest.mark.parametrize("pi", range(len(PARAMS)))
def test_members_match_zlib(eng, pi):
    kw = PARAMS[pi]
    data = _datasets()
    names = sorted(data)
    members, want = [], []
    for k in names:
        if len(B.deflate_raw(data[k], **kw)) + 26 > 65536:  # (random bytes at memLevel 1 expand past
            data[k] = data[k][:32768]                        # a BGZF member's 64 KiB limit)
        m = B.bgzf_member(data[k], **kw)
        members.append(m)
        want.append(data[k])
    got = _device(eng, b"".join(members) + B.EOF_MEMBER)
    assert got == b"".join(want), (kw, got[:3] if isinstance(got, tuple) else len(got))


def test_whole_vcf_as_bgzf(eng):
    """a 3 MB synthetic VCF as a standard BGZF file (65,280-byte blocks, level 6 and level 1)"""
    buf = synth.generate(1500, 500, 92, 0, 0.001, 0, 0.02, 0)
    for lvl in (1, 6):
        assert _device(eng, B.bgzf(buf, level=lvl)) == buf


def _corrupt_cases():
    rnd = random.Random(11)
    data = _datasets()
    base = [B.bgzf_member(data["vcf"], level=6), B.bgzf_member(data["mixed"], level=1),
            B.bgzf_member(data["random"][:3000], level=9), B.bgzf_member(data["runs"], level=6, strategy=zlib.Z_RLE),
            B.bgzf_member(data["short_text"], level=6, strategy=zlib.Z_FIXED)]
    out = []
    for m in base:
        xlen = m[10] | m[11] << 8
        lo, hi = 12 + xlen, len(m)
        for _ in range(40):
            b = bytearray(m)
            k = rnd.randrange(lo, hi)  # the deflate data and the trailer (the header is the host's)
            b[k] ^= 1 << rnd.randrange(8)
            if rnd.random() < 0.3:
                k2 = rnd.randrange(lo, hi)
                b[k2] ^= 1 << rnd.randrange(8)
            out.append(bytes(b))
    return out


def test_damaged_members_refused_like_zlib(eng):
    good = B.bgzf_member(b"#CHROM\n" * 100, level=6)
    n_bad = n_ok = 0
    for m in _corrupt_cases():
        ok, want = B.zlib_member(m)
        got = _device(eng, good + m)
        if not ok:
            assert isinstance(got, tuple) and got[1] == 1, (got if isinstance(got, tuple) else len(got))
            n_bad += 1
        else:
            # zlib accepts it (a flip it cannot see): the device must agree on every byte or refuse
            assert not isinstance(got, tuple), got
            assert got == b"#CHROM\n" * 100 + want
            n_ok += 1
    assert n_bad > 150


# ---- hand-made streams ----------------------------------------------------------------------------
def _fixed_block(w, syms, final=True):
    """syms: ints < 256 literals, ("m", length, dist) matches, ("raw_ll", sym) / ("raw_d", sym)"""
    ll = B.canonical(B.FIXED_LL)
    dd = B.canonical(B.FIXED_D)
    LB = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
          227, 258]
    LE = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
    DB = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
          6145, 8193, 12289, 16385, 24577]
    DE = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
    w.bits(1 if final else 0, 1)
    w.bits(1, 2)
    for s in syms:
        if isinstance(s, int):
            w.code(*ll[s])
        elif s[0] == "raw_ll":
            w.code(*ll[s[1]])
        elif s[0] == "raw_d":
            w.code(*ll[257])
            w.code(*dd[s[1]])
        else:
            _, length, dist = s
            c = max(i for i in range(29) if LB[i] <= length and (i < 28 or length == 258))
            if length == 258:
                c = 28
            w.code(*ll[257 + c])
            w.bits(length - LB[c], LE[c])
            d = max(i for i in range(30) if DB[i] <= dist)
            w.code(*dd[d])
            w.bits(dist - DB[d], DE[d])
    w.code(*ll[256])


def _crafted():
    """(name, raw deflate bytes, the data it claims, zlib must accept)"""
    rnd = random.Random(5)
    cases = []
    # distance 32768 (zlib's deflate never emits it; inflate accepts it)
    lit = [rnd.getrandbits(8) for _ in range(32768)]
    w = B.BitWriter()
    _fixed_block(w, lit + [("m", 258, 32768), ("m", 3, 32768), ("m", 100, 1)])
    data = bytes(lit) + bytes(lit[:258]) + bytes(lit[258:261]) + bytes([lit[260]]) * 100
    cases.append(("dist32768", w.done(), data))
    # every length code and distance code once
    w = B.BitWriter()
    syms = [ord("a") + i % 26 for i in range(300)]
    for length in (3, 4, 10, 11, 12, 18, 34, 35, 66, 130, 131, 257, 258):
        syms.append(("m", length, 7))
    for dist in (1, 2, 3, 4, 5, 6, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257):
        syms.append(("m", 5, dist))
    w2 = B.BitWriter()
    _fixed_block(w2, syms)
    out = bytearray()
    for s in syms:
        if isinstance(s, int):
            out.append(s)
        else:
            for _ in range(s[1]):
                out.append(out[-s[2]])
    cases.append(("all_lengths", w2.done(), bytes(out)))
    # dynamic block: a literal/length code of one symbol (EOB only, length 1: incomplete, allowed)
    w = B.BitWriter()
    w.bits(1, 1)
    w.bits(2, 2)
    ll = [0] * 257
    ll[256] = 1
    B.dynamic_header(w, ll, [0])
    w.code(0, 1)
    cases.append(("single_code_eob", w.done(), b""))
    # dynamic block, literals only, no distance codes at all (HDIST 1 with length 0)
    w = B.BitWriter()
    w.bits(1, 1)
    w.bits(2, 2)
    ll = [0] * 257
    for c in b"ACGT":
        ll[c] = 3
    ll[256] = 1
    B.dynamic_header(w, ll, [0])
    code = B.canonical(ll)
    msg = b"ACGTTTGA" * 40
    for c in msg:
        w.code(*code[c])
    w.code(*code[256])
    cases.append(("no_dist_codes", w.done(), msg))
    # a stored block of 0 bytes then one of 5, then a fixed block
    w = B.BitWriter()
    w.bits(0, 1)
    w.bits(0, 2)
    w.align()
    w.bits(0, 16)
    w.bits(0xFFFF, 16)
    w.bits(0, 1)
    w.bits(0, 2)
    w.align()
    w.bits(5, 16)
    w.bits(0xFFFA, 16)
    for c in b"hello":
        w.bits(c, 8)
    _fixed_block(w, list(b" world"))
    cases.append(("stored_then_fixed", w.done(), b"hello world"))
    return cases


def _crafted_bad():
    """raw streams zlib refuses"""
    out = []
    w = B.BitWriter()  # block type 3
    w.bits(1, 1)
    w.bits(3, 2)
    out.append(("btype3", w.done() + b"\0\0"))
    w = B.BitWriter()  # stored LEN != ~NLEN
    w.bits(1, 1)
    w.bits(0, 2)
    w.align()
    w.bits(3, 16)
    w.bits(0x1234, 16)
    out.append(("stored_nlen", w.done() + b"abc"))
    w = B.BitWriter()  # literal/length 286 in a fixed block
    _fixed_block(w, [65, ("raw_ll", 286)])
    out.append(("ll286", w.done()))
    w = B.BitWriter()  # distance code 30
    _fixed_block(w, [65, ("raw_d", 30)])
    out.append(("d30", w.done()))
    w = B.BitWriter()  # distance past the start
    _fixed_block(w, [65, 66, ("m", 3, 3)])
    out.append(("too_far", w.done()))
    w = B.BitWriter()  # no end-of-block code
    w.bits(1, 1)
    w.bits(2, 2)
    ll = [0] * 257
    ll[65] = 1
    ll[66] = 1
    B.dynamic_header(w, ll, [1, 1])
    out.append(("no_eob", w.done() + b"\0" * 8))
    w = B.BitWriter()  # over-subscribed literal/length code
    w.bits(1, 1)
    w.bits(2, 2)
    ll = [0] * 257
    ll[65], ll[66], ll[67], ll[256] = 1, 1, 1, 1
    B.dynamic_header(w, ll, [1, 1])
    out.append(("oversubscribed", w.done() + b"\0" * 8))
    w = B.BitWriter()  # incomplete literal/length code with codes of length 2
    w.bits(1, 1)
    w.bits(2, 2)
    ll = [0] * 257
    ll[65], ll[256] = 2, 2
    B.dynamic_header(w, ll, [1, 1])
    out.append(("incomplete", w.done() + b"\0" * 8))
    w = B.BitWriter()  # HLIT 287 (more than 286 symbols)
    w.bits(1, 1)
    w.bits(2, 2)
    w.bits(30, 5)
    w.bits(0, 5)
    w.bits(15, 4)
    out.append(("hlit287", w.done() + b"\0" * 16))
    return out


def _member_of_raw(raw, data):
    return B.wrap_member(raw, data)


def test_crafted_streams(eng):
    for name, raw, data in _crafted():
        m = _member_of_raw(raw, data)
        ok, want = B.zlib_member(m)
        assert ok and want == data, name
        assert _device(eng, m) == data, name
    for name, raw in _crafted_bad():
        m = _member_of_raw(raw, b"")
        ok, _ = B.zlib_member(m)
        assert not ok, name
        got = _device(eng, m)
        assert isinstance(got, tuple), name


def test_stream_end_must_meet_trailer(eng):
    data = b"ACGT" * 5000
    raw = B.deflate_raw(data, level=6)
    early = B.wrap_member(raw + b"\0", data)       # a byte between the stream and its trailer
    cut = B.wrap_member(raw[:-3], data)             # the stream runs into its trailer
    for m in (early, cut):
        assert not B.zlib_member(m)[0]
        assert isinstance(_device(eng, m), tuple)
    wrong_isize = B.wrap_member(raw, data, isize=len(data) - 1)
    wrong_crc = B.wrap_member(raw, data, crc=zlib.crc32(data) ^ 4)
    for m in (wrong_isize, wrong_crc):
        assert not B.zlib_member(m)[0]
        assert isinstance(_device(eng, m), tuple)


# ---- the drop-in tools on BGZF input through the device path --------------------------------------
TOOL_CASES = [
    ["VCFX_allele_freq_calc", "-i", "{F}"], ["VCFX_allele_freq_calc"],
    ["VCFX_record_filter", "--filter", "QUAL>=30", "-i", "{F}"], ["VCFX_record_filter", "--filter", "POS>9420000"],
    ["VCFX_genotype_query", "-g", "0|1", "-i", "{F}"], ["VCFX_genotype_query", "-g", "1|1", "--strict"],
    ["VCFX_nonref_filter", "-i", "{F}"], ["VCFX_hwe_tester", "-i", "{F}"], ["VCFX_hwe_tester"],
    ["VCFX_ld_calculator", "-w", "60", "-t", "0.2", "-i", "{F}"], ["VCFX_ld_calculator", "-w", "40", "-t", "0.1"],
    ["VCFX_dosage_calculator", "-i", "{F}"], ["VCFX_dosage_calculator"],
    ["VCFX_missing_detector", "-i", "{F}"], ["VCFX_missing_detector"],
    ["VCFX_missing_detector", "-i", "{F}", "(no missing)"],  # the pre-scan's fast path: the input as it is
    ["VCFX_allele_counter", "-i", "{F}"], ["VCFX_allele_counter", "-q", "-a", "-i", "{F}"], ["VCFX_allele_counter"],
    ["VCFX_haplotype_phaser", "-i", "{F}"], ["VCFX_haplotype_phaser", "--streaming"],
]


@pytest.mark.parametrize("argv", TOOL_CASES)
def test_tools_on_device_bgzf(argv):
    oracle = Oracle()
    if argv[-1] == "(no missing)":
        argv = argv[:-1]
        buf = synth.generate(800, 400, 93, 1, 0.0, 0, 0.0, 0)
    else:
        buf = synth.generate(800, 400, 93, 1, 0.005, 0, 0.05, 1)
    d = tempfile.mkdtemp(prefix="vcfx_bgz_")
    plain, gz, log = os.path.join(d, "in.vcf"), os.path.join(d, "in.vcf.gz"), os.path.join(d, "sched.log")
    try:
        with open(plain, "wb") as f:
            f.write(buf)
        with open(gz, "wb") as f:
            f.write(B.bgzf(buf, level=6))
        want = oracle.run([a.replace("{F}", plain) for a in argv], b"" if "{F}" in " ".join(argv) else buf)
        env = dict(os.environ, VCFX_BGZF_DEVICE_MIN="0", VCFXG_SCHEDULE_LOG=log)
        args = [tool_binary(argv[0])] + [a.replace("{F}", gz) for a in argv[1:]]
        stdin = None if "{F}" in " ".join(argv) else open(gz, "rb")
        try:
            r = subprocess.run(args, stdin=stdin, capture_output=True, env=env, timeout=120)
        finally:
            if stdin:
                stdin.close()
        assert (r.stdout, r.returncode) == (want[0], want[2]), (argv, r.stderr[-500:])
        # (the file modes' "Processing F (size)" line names the .gz file and its own size)
        keep = lambda e: [x.replace(gz.encode(), plain.encode()) for x in e.split(b"\n") if not x.startswith(b"Processing ")]
        assert keep(r.stderr) == keep(want[1]), argv
        assert "bgzf_inflate" in open(log).read(), argv
    finally:
        for x in os.listdir(d):
            os.unlink(os.path.join(d, x))
        os.rmdir(d)


# ---- the streamed form (VCFX_allele_freq_calc -i F.gz): the compressed file through the pinned file
# ring, the member chain parsed from the ring's slots, every member inflated on the device -------------
@pytest.mark.parametrize("slot,batch,table", [("4096", "1", None), ("65536", "1", None), ("65536", "0", None),
                                               ("default", "1024", None), ("65536", "1", "3")])
def test_af_streams_bgzf_through_the_ring(slot, batch, table):
    """Slots far smaller than a member (a member's header and trailer in different slots), about one
    member, and the default 16 MiB; inflate batches launched per slot, or none until the end: the
    same rows as the oracle on the plain text, with the schedule
    log showing the staged inflate ran; a plain (single-member) gzip file, a truncated BGZF file and
    one with a zeroed tail are not a BGZF chain to the stream and take the mapped path (its host
    inflate output, or the reference's "truncated or corrupt" failure)."""
    import gzip
    oracle = Oracle()
    buf = synth.generate(900, 350, 97, 0, 0.004, 1, 0.02, 0)
    d = tempfile.mkdtemp(prefix="vcfx_bgzs_")
    plain, bg, gz, log = (os.path.join(d, x) for x in ("in.vcf", "in.vcf.gz", "in1.vcf.gz", "sched.log"))
    try:
        with open(plain, "wb") as f:
            f.write(buf)
        comp = B.bgzf(buf, level=6)
        with open(bg, "wb") as f:
            f.write(comp)
        with open(gz, "wb") as f:
            f.write(gzip.compress(buf, 6))
        want = oracle.run(["VCFX_allele_freq_calc", "-i", plain], b"")
        env = dict(os.environ, VCFX_BGZF_STREAM_MIN="1", VCFXG_SCHEDULE_LOG=log)  # (0 reads as unset)
        # the members inflate in batches launched while later slots are still copied (batch 1: one
        # launch per slot that completes a member; "0": all at the end)
        if batch == "0":
            env["VCFX_BGZF_BATCH"] = "0"
        else:
            env["VCFX_BGZF_BATCH_MIN"] = batch
        if slot != "default":
            env["VCFX_FILE_SLOT"] = slot
        if table:  # member tables sized for 3 members: the batches stop (E_CAP), the tables grow at the end
            env["VCFXG_BGZF_TABLE"] = table

        def run(path):
            if os.path.exists(log):
                os.unlink(log)
            r = subprocess.run([tool_binary("VCFX_allele_freq_calc"), "-i", path], capture_output=True, env=env,
                               timeout=120)
            return r, (open(log).read() if os.path.exists(log) else "")

        r, sch = run(bg)
        assert (r.stdout, r.returncode) == (want[0], want[2]), r.stderr[-500:]
        assert "bgzf_inflate_staged" in sch, sch
        r, sch = run(gz)  # one gzip member: the mapped path's sequential host inflate
        assert (r.stdout, r.returncode) == (want[0], want[2]), r.stderr[-500:]
        assert "bgzf_inflate_staged" not in sch
        for cut in (comp[:len(comp) // 2], comp[:len(comp) - 3000] + bytes(3000)):
            with open(bg, "wb") as f:
                f.write(cut)
            r, sch = run(bg)
            assert r.returncode == 1 and b"truncated or corrupt" in r.stderr, r.stderr[-300:]
            assert "bgzf_inflate_staged" not in sch
    finally:
        for x in os.listdir(d):
            os.unlink(os.path.join(d, x))
        os.rmdir(d)


def test_af_streams_bgzf_past_the_output_hint():
    """A BGZF file that inflates to far more than the stream's 24x output hint (every genotype
    0|0: deflate ratio ~100): batches launched per slot run until the output outgrows the buffer
    (E_CAP), the rest inflates at the end after the buffer grows -- the grow waits for the
    launched batches before it copies their output.  Same rows as the oracle on the
    plain text, and the schedule log shows the staged inflate."""
    oracle = Oracle()
    names = "\t".join("S%d" % k for k in range(400))
    rows = "".join("1\t%d\t.\tA\tC\t50\tPASS\t.\tGT\t%s\n" % (1000 + 7 * k, "\t".join(["0|0"] * 400)) for k in range(3000))
    buf = ("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + names + "\n" + rows).encode()
    comp = B.bgzf(buf, level=6)
    assert len(buf) > 40 * len(comp), (len(buf), len(comp))
    d = tempfile.mkdtemp(prefix="vcfx_bgzh_")
    plain, bg, log = (os.path.join(d, x) for x in ("in.vcf", "in.vcf.gz", "sched.log"))
    try:
        with open(plain, "wb") as f:
            f.write(buf)
        with open(bg, "wb") as f:
            f.write(comp)
        want = oracle.run(["VCFX_allele_freq_calc", "-i", plain], b"")
        env = dict(os.environ, VCFX_BGZF_STREAM_MIN="1", VCFXG_SCHEDULE_LOG=log, VCFX_BGZF_BATCH_MIN="1",
                   VCFX_FILE_SLOT="4096")
        r = subprocess.run([tool_binary("VCFX_allele_freq_calc"), "-i", bg], capture_output=True, env=env, timeout=120)
        assert (r.stdout, r.returncode) == (want[0], want[2]), r.stderr[-500:]
        assert "bgzf_inflate_staged" in open(log).read()
    finally:
        for x in os.listdir(d):
            os.unlink(os.path.join(d, x))
        os.rmdir(d)


# ---- BGZF input split across ranks in its inflated bytes ------------------------------------------
NGPU_CASES = [
    ["VCFX_allele_freq_calc", "-i", "{F}"], ["VCFX_record_filter", "--filter", "QUAL>=30", "-i", "{F}"],
    ["VCFX_genotype_query", "-g", "0|1", "-i", "{F}"], ["VCFX_nonref_filter", "-i", "{F}"],
    ["VCFX_dosage_calculator", "-i", "{F}"], ["VCFX_hwe_tester", "-i", "{F}"], ["VCFX_missing_detector", "-i", "{F}"],
    ["VCFX_allele_counter", "-q", "-a", "-i", "{F}"], ["VCFX_ld_calculator", "-w", "60", "-t", "0.2", "-i", "{F}"],
]


@pytest.fixture(scope="module")
def bgz_pair():
    buf = synth.generate(1200, 300, 95, 1, 0.005, 0, 0.05, 1)
    d = tempfile.mkdtemp(prefix="vcfx_bgzn_")
    plain, gz = os.path.join(d, "in.vcf"), os.path.join(d, "in.vcf.gz")
    with open(plain, "wb") as f:
        f.write(buf)
    with open(gz, "wb") as f:
        f.write(B.bgzf(buf, level=6))
    yield plain, gz, buf
    for x in os.listdir(d):
        os.unlink(os.path.join(d, x))
    os.rmdir(d)


def _keep(e, gz, plain):
    return [x.replace(gz.encode(), plain.encode()) for x in e.split(b"\n") if not x.startswith(b"Processing ")]


@pytest.mark.parametrize("argv", NGPU_CASES)
def test_ngpu_ranks_on_bgzf(argv, bgz_pair):
    """VCFX_NGPU=3 on a BGZF file (three rank contexts on the one GPU, round robin): the member
    chain cut in the inflated bytes (vcfx_shard_plan kind 3; LD: rows, every rank inflating the
    whole file), each rank inflating its members on its device; the reference's output on the
    plain bytes"""
    from vcfx_amd import tools
    plain, gz, _ = bgz_pair
    w, kind, _ = tools.shard_plan([a.replace("{F}", gz) for a in argv], 3)
    assert w == 3 and kind == (2 if argv[0] == "VCFX_ld_calculator" else 3), (argv, w, kind)
    want = Oracle().run([a.replace("{F}", plain) for a in argv], b"")
    env = dict(os.environ, VCFX_NGPU="3", VCFX_BGZF_DEVICE_MIN="0")
    r = subprocess.run([tool_binary(argv[0])] + [a.replace("{F}", gz) for a in argv[1:]], capture_output=True, env=env,
                       timeout=120)
    assert (r.stdout, r.returncode) == (want[0], want[2]), (argv, r.stderr[-500:])
    assert _keep(r.stderr, gz, plain) == _keep(want[1], gz, plain), argv


@pytest.mark.parametrize("tool", ["VCFX_allele_freq_calc", "VCFX_record_filter"])
def test_env_bgzf_views(tool, bgz_pair):
    """the per-process form vcfx_amd/shard.py uses (VCFX_INPUT_VIEW="bgzf:H:LO:HI" +
    VCFX_VIEW_SKIP_HEADER on ranks > 0): the views' outputs in rank order are the whole run's"""
    from vcfx_amd import shard
    plain, gz, _ = bgz_pair
    argv = [tool] + (["--filter", "QUAL>=30"] if tool == "VCFX_record_filter" else ["-q"]) + ["-i", gz]
    cuts = shard.bgzf_cuts(argv, 4)
    assert cuts is not None
    want = Oracle().run([plain if a == gz else a for a in argv], b"")
    out = b""
    for r in range(4):
        env = dict(os.environ, VCFX_INPUT_VIEW="bgzf:%d:%d:%d" % (cuts[0], cuts[r], cuts[r + 1]))
        if r:
            env["VCFX_VIEW_SKIP_HEADER"] = "1"
        p = subprocess.run([tool_binary(tool)] + argv[1:], capture_output=True, env=env, timeout=120)
        assert p.returncode == 0, p.stderr[-500:]
        out += p.stdout
    assert out == want[0]
