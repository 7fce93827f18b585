"""GPU parity of vcfxg_allele_freq_region -- every device schedule (the walk, the two-sweep
schedule with one host synchronisation, the synchronous two-sweep schedule) -- against the
two-pass path
(vcfxg_index + vcfxg_allele_freq) and the C oracle: every per-line array and the output
text must be identical, including inputs that put many line starts in one 16 KiB chunk
(more than the kernel's per-pass mark list), lines that span several chunks, CRLF, empty
lines, no trailing newline and chunk-boundary newlines."""
import numpy as np
import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["default", "sync", "walk", "walk4k", "walk1k", "walk8m", "twosweep"])
def eng(request):
    """every region schedule: default (the walk for long records, else the two-sweep
    schedule), two-sweep = index + head pass + sweep with one host synchronisation;
    sync: the same kernels with the line count read back after the index; walk (no index
    sweep: predicted record ends validated by the sweep; chunks of 128 KiB, 4 KiB and 1 KiB,
    so lines start in, span and skip over many walkers' chunks; 8 MiB: short records would
    overflow a walker's 16-bit line count, so the forced walk takes the two-sweep schedule)"""
    import os
    env = {"VCFXG_AF_FUSED": {"default": "0", "sync": "3", "walk": "7", "walk4k": "7", "walk1k": "7",
                              "walk8m": "7", "twosweep": "8"}[request.param],
           "VCFXG_WALK_CHUNK": {"walk4k": "4096", "walk1k": "1024",
                                "walk8m": str(8 << 20)}.get(request.param, str(128 * 1024))}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return engine.Engine(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _both(eng, buf, mode):
    ds = engine.data_start_of(buf, strip_cr=(mode == engine.MODE_FILE))
    eng.load(buf)
    nl = eng.index(ds)
    s2 = eng.allele_freq(mode)
    two = (eng.line_ends(nl), eng.lines(nl), eng.text(s2.text_bytes), s2)
    eng.load(buf)
    s1 = eng.allele_freq_region(ds, mode)
    nl1 = s1.n_lines
    one = (eng.line_ends(nl1), eng.lines(nl1), eng.text(s1.text_bytes), s1)
    return ds, two, one


def _same(two, one):
    e2, (a2, t2, st2), x2, s2 = two
    e1, (a1, t1, st1), x1, s1 = one
    assert s1.n_lines == s2.n_lines
    np.testing.assert_array_equal(e1, e2)
    np.testing.assert_array_equal(st1, st2)
    rows = st2 == 1
    np.testing.assert_array_equal(a1[rows], a2[rows])
    np.testing.assert_array_equal(t1[rows], t2[rows])
    assert x1 == x2
    assert (s1.rows, s1.data_lines, s1.warn_lines, s1.general_records) == \
        (s2.rows, s2.data_lines, s2.warn_lines, s2.general_records)


SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (3000, 2504, 11, 0, 0.0, 0, 0.0, 0),   # 10 KB lines spanning chunks
    (2000, 997, 12, 1, 0.01, 0, 0.2, 0),
    (4000, 3, 13, 0, 0.05, 0, 0.3, 1),     # ~60 B lines: > 256 starts per chunk, CRLF
    (30000, 1, 14, 0, 0.0, 0, 0.0, 0),     # ~45 B lines: several mark passes per chunk
    (160, 5000, 16, 0, 0.01, 0, 0.1, 0),   # 20 KB lines: segments over 2-3 chunks
    (120, 9000, 17, 1, 0.0, 0, 0.0, 1),    # 36 KB CRLF lines
    (900, 2504, 18, 0, 0.0, 1, 0.0, 0),
]


@pytest.mark.parametrize("cfg", SYNTH)
@pytest.mark.parametrize("mode", [engine.MODE_FILE, engine.MODE_STDIN])
def test_fused_matches_two_pass(eng, cfg, mode):
    buf = synth.generate(*cfg)
    _, two, one = _both(eng, buf, mode)
    _same(two, one)


def test_fused_edge_layouts(eng, oracle):
    head = b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\tB\n"
    row = b"1\t5\t.\tA\tG\t.\t.\t.\tGT\t0|1\t1|1\n"
    cases = [
        head + row * 3,                       # trailing newline
        head + row * 3 + row[:-1],            # no trailing newline
        head + b"\n\n" + row + b"\n" + row,   # empty lines
        head + b"\n",                         # one empty data line
        head + row[:-1],                      # a single unterminated record
        head + b"#late header\n" + row,
    ]
    # a newline on the last byte of chunk 0, on the first byte of chunk 1, and just before
    # (16 KiB index chunks; 32 KiB one-sweep chunks)
    ds = len(head)
    for last0, shift in [(((ds - 1) & ~15) + 16384 - 1, sh) for sh in (-1, 0, 1)] + \
            [((ds & ~15) + 32768 - 1, sh) for sh in (-1, 0, 1)]:
        # (long fillers on the 32 KiB grid: under the one-sweep kernel's lines-per-chunk cap)
        filler = b"1\t7\t.\tA\tG\t.\t.\t" + (b"I" * 150 if last0 > 20000 else b".") + b"\tGT\t0|0\t0|1\n"
        body = b""
        while ds + len(body) + 2 * len(filler) + 64 < last0:
            body += filler
        tail = b"\tA\tG\t.\t.\t.\tGT\t0|0\t0|1\n"
        k = last0 + shift - (ds + len(body)) - len(b"1\t7\t") - len(tail) + 1
        line = b"1\t7\t" + b"x" * k + tail
        assert ds + len(body) + len(line) - 1 == last0 + shift
        cases.append(head + body + line + row * 5)
    for buf in cases:
        for mode in (engine.MODE_FILE, engine.MODE_STDIN):
            _, two, one = _both(eng, buf, mode)
            _same(two, one)


def test_fused_text_matches_oracle(eng, oracle):
    import tempfile
    buf = synth.generate(1200, 401, 15, 1, 0.02, 0, 0.2, 0)
    ds = engine.data_start_of(buf)
    eng.load(buf)
    s = eng.allele_freq_region(ds, engine.MODE_FILE)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        want, _, _ = oracle.run(["VCFX_allele_freq_calc", "-q", "-i", f.name])
    assert b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes) == want


def _walk_layouts(seed):
    """long GT-only records whose ends the walk path predicts from the previous record:
    heads longer than the head window, varying sample counts, missing alleles, non-fixed-stride samples, CRLF records, '#' and
    empty lines between records, and a short record followed by a line whose '\n' sits
    exactly where the previous record's span predicts this one's end (the sweep must reject
    the prediction and the '\n' search must find the true end)"""
    rng = np.random.default_rng(seed)
    ns = 300
    head = b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + \
        b"\t".join(b"S%d" % i for i in range(ns)) + b"\n"
    toks = [b"0|0", b"0|1", b"1|0", b"1|1", b".|.", b"2|1"]

    def rec(pos, n, bad=False, cr=False, info=b"."):
        g = [toks[int(k)] for k in rng.integers(0, len(toks), n)]
        if bad:
            g[int(rng.integers(0, n))] = [b"0|1:7", b"0/1", b"10|1"][int(rng.integers(0, 3))]
        return b"21\t%d\trs%d\tA\tG\t100\tPASS\t%s\tGT\t" % (pos, pos, info) + b"\t".join(g) + \
            (b"\r\n" if cr else b"\n")

    body = []
    pos = 100
    for i in range(400):
        pos += 1
        r = rng.random()
        if r < 0.05:
            body.append(b"#interleaved header line\n")
        elif r < 0.08:
            body.append(b"\n")
        elif r < 0.12:
            body.append(rec(pos, ns, bad=True))
        elif r < 0.16:
            body.append(rec(pos, ns, cr=True))
        elif r < 0.22:
            body.append(rec(pos, int(rng.integers(200, 400))))
        elif r < 0.24:
            # heads longer than the walk's 256 B window (and than 1 KiB)
            body.append(rec(pos, ns, info=b"AF=0.5;X=" + b"y" * int(rng.integers(150, 1500))))
        elif r < 0.28:
            # a record 50 samples short, then a line whose '\n' is at the predicted end
            body.append(rec(pos, ns))
            short = rec(pos + 1, ns - 50)
            body.append(short)
            gap = 4 * ns - 1 - (4 * (ns - 50) - 1) - 1   # bytes of the next line before its '\n'
            body.append(b"21\t%d\t" % (pos + 2) + b"x" * (gap - len(b"21\t%d\t" % (pos + 2))) + b"\n")
            pos += 2
        else:
            body.append(rec(pos, ns))
    tail = rec(pos + 1, ns)
    return head + b"".join(body), head + b"".join(body) + tail[:-1]


@pytest.mark.parametrize("seed", [1, 2])
def test_walk_predicted_ends(eng, seed):
    for buf in _walk_layouts(seed):
        for mode in (engine.MODE_FILE, engine.MODE_STDIN):
            _, two, one = _both(eng, buf, mode)
            _same(two, one)
