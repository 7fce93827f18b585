"""GPU parity of VCFX_allele_counter beyond the golden cases: seeded
synthetic VCFs (fixed-stride records, missing calls, irregular GT shapes, GT:AD:DP, CRLF) in
every output mode (text, -a, -b, -l, -s, -z) and both input modes, and crafted traps (ragged
samples, trailing tabs, unordered / duplicated selections, counts of two digits and past int8,
'#CHROM' lines among the records on stdin) against the C oracle."""
import pytest

from tests._golden import Oracle
from vcfx_amd import synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    dict(n_records=300, n_samples=2504, seed=101),
    dict(n_records=200, n_samples=997, seed=102, info_mode=1, missing_rate=0.01, irregular_rate=0.2, crlf=1),
    dict(n_records=1500, n_samples=3, seed=103, missing_rate=0.05, irregular_rate=0.3),
    dict(n_records=200, n_samples=301, seed=104, missing_rate=0.002, format_mode=1),
    dict(n_records=150, n_samples=64, seed=105, irregular_rate=0.3, crlf=1, format_mode=1),
]


def _names(buf):
    for line in buf.split(b"\n"):
        if line.startswith(b"#CHROM"):
            return [x.decode() for x in line.rstrip(b"\r").split(b"\t")[9:]]
    return []


def _check(oracle, argv, stdin=b""):
    want = oracle.run(argv, stdin)
    got = tools.run(argv, stdin)
    assert got[2] == want[2] and got[1] == want[1], (argv[1:], got[1][-200:], want[1][-200:])
    assert got[0] == want[0], (argv[1:], len(got[0]), len(want[0]))


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_allele_counter_modes(oracle, cfg, tmp_path):
    buf = synth.generate(**cfg)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    p = str(path)
    nm = _names(buf)
    pick = " ".join([nm[len(nm) // 2], nm[0], nm[-1], nm[len(nm) // 3]])
    T = "VCFX_allele_counter"
    for argv in ([T, "-i", p], [T, "-q", "-a", "-i", p], [T, "-q", "-b", "-i", p], [T, "-q", "-l", "5", "-i", p],
                 [T, "-q", "-s", pick, "-i", p], [T, "-q", "-s", pick, "-a", p], [T, "-q", "-z", "-i", p],
                 [T, "-q", "-a", "-z", p], [T, "-q", "-b", "-l", "3", p]):
        _check(oracle, argv)
    _check(oracle, [T], buf)
    _check(oracle, [T, "-q", "-s", pick], buf)


HEAD = b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\tB\tC\tB\n"
MANY = "/".join(["1"] * 12) + "|" + "/".join(["0"] * 11)
HUGE = "/".join(["2"] * 140)
TRAPS = [
    # ragged records: fewer samples, no samples, short heads, a trailing tab
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\n1\t2\t.\tA\tC\t.\t.\t.\tGT\n1\t3\t.\tA\n"
    b"1\t4\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\t1/1\t\n\n1\t5\t.\tA\tC\t.\t.\t.\tGT\t\t\t\t\n",
    # multi-digit alleles, haploid, dots, 0 written as 00, sub-fields
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT:DP\t10/0:5\t1:3\t./.:1\t00|3\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t.\t0\t1/2/3\t0.5\n",
    # counts of two digits and past int8
    HEAD + ("1\t1\t.\tA\tC\t.\t.\t.\tGT\t%s\t%s\t0/1\t1/1\n" % (MANY, HUGE)).encode(),
    # '#' lines among the records, CRLF
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\t1/1\r\n##x\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\t1/1\n",
]
STREAM_ONLY = [
    # a second '#CHROM' line among the records (countAllelesStream re-selects)
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\t1/1\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tD\tE\n"
    b"1\t2\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\t1/1\t1/0\t0/0\n",
    # no '#CHROM', data before it, header only
    b"##x\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t0/1\n",
    HEAD,
]


@pytest.mark.parametrize("k", range(len(TRAPS)))
def test_allele_counter_traps(oracle, k, tmp_path):
    path = tmp_path / "t.vcf"
    path.write_bytes(TRAPS[k])
    p = str(path)
    T = "VCFX_allele_counter"
    for argv in ([T, "-q", "-i", p], [T, "-q", "-a", "-i", p], [T, "-q", "-b", "-i", p], [T, "-q", "-l", "2", "-i", p],
                 [T, "-q", "-s", "C A B", "-i", p], [T, "-q", "-s", "C A", "-a", p]):
        _check(oracle, argv)
    _check(oracle, [T, "-q"], TRAPS[k])
    _check(oracle, [T, "-q", "-s", "C B A"], TRAPS[k])


@pytest.mark.parametrize("k", range(len(STREAM_ONLY)))
def test_allele_counter_stream_traps(oracle, k):
    T = "VCFX_allele_counter"
    _check(oracle, [T], STREAM_ONLY[k])
    _check(oracle, [T, "-q", "-s", "A"], STREAM_ONLY[k])


def test_allele_counter_selection_in_global_memory(oracle, tmp_path, monkeypatch):
    """the row writer with the selection read from global memory (too large for LDS)"""
    monkeypatch.setenv("VCFXG_AC_SEL_GLOBAL", "1")
    buf = synth.generate(n_records=200, n_samples=700, seed=106)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    T = "VCFX_allele_counter"
    for argv in ([T, "-q", "-i", str(path)], [T, "-q", "-l", "9", "-i", str(path)]):
        _check(oracle, argv)
    _check(oracle, [T, "-q"], buf)


def test_allele_counter_long_rows_and_identity_selection(oracle, tmp_path):
    """Text rows composed in 3 KiB LDS tiles (64 rows of up to 48 bytes) next to records whose
    rows are longer (IDs of 20..200 bytes: written straight out), under the identity selection
    (every sample in order: no index array in LDS) and a reordered one (the index array)."""
    import random
    buf = synth.generate(n_records=160, n_samples=70, seed=106)
    rnd = random.Random(106)
    lines = buf.split(b"\n")
    for k, ln in enumerate(lines):
        if ln and not ln.startswith(b"#") and rnd.random() < 0.4:
            f = ln.split(b"\t")
            f[2] = b"id%d_" % k + b"y" * rnd.randint(20, 200)
            lines[k] = b"\t".join(f)
    buf = b"\n".join(lines)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    p = str(path)
    nm = _names(buf)
    T = "VCFX_allele_counter"
    for argv in ([T, "-q", "-i", p], [T, "-q", "-s", " ".join(nm[::-1]), "-i", p], [T, "-q", "-s", " ".join(nm), "-i", p]):
        _check(oracle, argv)


@pytest.mark.parametrize("L", [1, 6, 11, 12])
def test_allele_counter_direct_rows(oracle, L, tmp_path, monkeypatch):
    """k_ac_rows (text rows written straight from registers: names of one length L <= 11, record
    prefixes of 16..64 bytes) beside k_ac_fmt for the other records: prefixes on both sides of
    16 / 32 / 48 / 64 bytes, records with fewer samples than the selection (all: 0 / 0 past them;
    seq: the rows stop), 130 samples (a partial last tile), the identity selection, a reordered
    one and a limit; and the same calls with k_ac_rows off (VCFXG_AC_DIRECT=0)."""
    import random
    rnd = random.Random(L)
    ns = 130
    names = ["%0*d" % (L, k) if L > 1 else chr(65 + k % 26) for k in range(ns)]
    head = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(names) + "\n"
    rows = []
    for k, P in enumerate([15, 16, 17, 31, 32, 33, 47, 48, 49, 63, 64, 65, 80, 20, 40, 60]):
        rid = ("r%d_" % k + "x" * 80)[:P - 9]
        for n in (ns, 100):
            gts = "\t".join("%d%s%d" % (rnd.randint(0, 1), rnd.choice("|/"), rnd.randint(0, 2)) for _ in range(n))
            rows.append("1\t%d\t%s\tA\tC\t.\t.\t.\tGT\t%s\n" % (k + 1, rid, gts))
    buf = (head + "".join(rows)).encode()
    path = tmp_path / "d.vcf"
    path.write_bytes(buf)
    p = str(path)
    pick = " ".join(names[::-3])
    T = "VCFX_allele_counter"
    for direct in ("1", "0"):
        monkeypatch.setenv("VCFXG_AC_DIRECT", direct)
        for argv in ([T, "-q", "-i", p], [T, "-q", "-s", pick, "-i", p], [T, "-q", "-l", "7", "-i", p],
                     [T, "-q", "-s", " ".join(names), "-a", p]):
            _check(oracle, argv)
        _check(oracle, [T, "-q"], buf)
