"""GPU parity of VCFX_missing_detector beyond the golden cases: seeded
synthetic VCFs (missing calls, irregular GT shapes, GT:AD:DP records, CRLF) and crafted traps
(dots outside GT, INFO forms, '#' lines among the records, an unterminated last record that
the file pre-scan does not read) in both input modes against the C oracle."""
import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    dict(n_records=1200, n_samples=2504, seed=91),
    dict(n_records=1200, n_samples=2504, seed=92, missing_rate=0.0005),
    dict(n_records=800, n_samples=997, seed=93, info_mode=1, missing_rate=0.01, irregular_rate=0.2, crlf=1),
    dict(n_records=3000, n_samples=3, seed=94, missing_rate=0.05, irregular_rate=0.3),
    dict(n_records=600, n_samples=301, seed=95, missing_rate=0.002, format_mode=1),
    dict(n_records=400, n_samples=64, seed=96, irregular_rate=0.3, crlf=1, format_mode=1),
]

HEAD = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tA\tB\tC\n")
TRAPS = [
    # no '.' in samples at all, and '.' only outside GT
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\n1\t2\t.\tA\tC\t.\tPASS\tDP=3\tGT:AD\t0/1:.,3\t0/0:.\t1/1:2,.\n",
    # the GT dot rules: start / end / next to a separator, and dots inside numbers
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t1.5\t0/0\t0/0\n1\t2\t.\tA\tC\t.\t.\tX=1;\tGT\t0/.\t0/0\t0/0\n"
    b"1\t3\t.\tA\tC\t.\t.\t\tGT:DP\t0/0:4\t.:3\t0/0\n1\t4\t.\tA\tC\t.\t.\tAF=0.5\tGT\t0/0\t0/0\t.|1\n"
    b"1\t5\t.\tA\tC\t.\t.\tAF=1\tGT\t0/0\t0/0\t1..2\n",
    # '#' lines among the records (the pre-scan reads them), CRLF, empty lines
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\r\n\n#x\t\t\t\t\t\t\t\t\t.\n\r\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t./.\t1\t0\r\n",
    # the last record has no '\n': the file pre-scan skips it
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/1\t1|1\t0/0\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t./.\t1\t0",
    HEAD + b"1\t1\t.\tA\tC\t.\t.\t.\tGT\t0/.\t1|1\t0/0\n1\t2\t.\tA\tC\t.\t.\t.\tGT\t./.\t1\t0",
    # short records, records with 9 fields, a trailing tab
    HEAD + b"1\t1\t.\tA\n1\t2\t.\tA\tC\t.\t.\t.\tGT\n1\t3\t.\tA\tC\t.\t.\t.\tGT\t\n1\t4\t.\tA\tC\t.\t.\t.\tGT\t.\t\n",
    # data before any header, header only
    b"1\t2\t.\tA\tC\t.\t.\t.\tGT\t./.\n" + HEAD,
    HEAD,
]


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _both_modes(oracle, buf, path):
    path.write_bytes(buf)
    for argv, stdin in ((["VCFX_missing_detector", "-i", str(path)], b""), (["VCFX_missing_detector"], buf),
                        (["VCFX_missing_detector", "-q", str(path)], b"")):
        want = oracle.run(argv, stdin)
        got = tools.run(argv, stdin)
        assert got[2] == want[2] and got[1] == want[1], (argv[1:2], got[1], want[1])
        assert got[0] == want[0], (argv[1:2], len(got[0]), len(want[0]))


@pytest.mark.parametrize("cfg", SYNTH)
def test_missing_tool_matches_oracle(oracle, cfg, tmp_path):
    _both_modes(oracle, synth.generate(**cfg), tmp_path / "in.vcf")


@pytest.mark.parametrize("k", range(len(TRAPS)))
def test_missing_traps(oracle, k, tmp_path):
    _both_modes(oracle, TRAPS[k], tmp_path / "in.vcf")


def test_missing_engine_counts(oracle):
    buf = synth.generate(1500, 2504, 97, 0, 0.001, 0, 0.0, 0)
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    s = eng.missing_region(ds, engine.MODE_FILE)
    st = eng.statuses(s.n_lines)
    assert s.data_lines == 1500 and s.rows == int((st == 6).sum()) and s.general_records >= s.rows > 0
    assert s.rows == oracle.run(["VCFX_missing_detector"], buf)[0].count(b"MISSING_GENOTYPES=1")
    eng.close()


def test_missing_walk_and_index_paths_agree(oracle, monkeypatch):
    """the walk (long GT-only records: VCFXG_FQ_WALK=1) and the index path (-1) give the same
    per-line statuses, INFO spans and counts, and the counts the reference prints"""
    import numpy as np
    for cfg in (dict(n_records=900, n_samples=2504, seed=98, missing_rate=0.0003),
                dict(n_records=700, n_samples=1200, seed=99, missing_rate=0.001, irregular_rate=0.1, crlf=1)):
        buf = synth.generate(**cfg)
        ds = engine.data_start_of(buf)
        got = []
        for walk in ("1", "-1"):
            monkeypatch.setenv("VCFXG_FQ_WALK", walk)
            eng = engine.Engine(0)
            eng.load(buf)
            s = eng.missing_region(ds, engine.MODE_FILE)
            a, t, st = eng.lines(s.n_lines)
            got.append(((s.n_lines, s.data_lines, s.rows, s.general_records), st.copy(), a.copy(), t.copy()))
            eng.close()
        assert got[0][0] == got[1][0]
        for k in (1, 2, 3):
            assert np.array_equal(got[0][k], got[1][k])
        assert got[0][0][2] == oracle.run(["VCFX_missing_detector"], buf)[0].count(b"MISSING_GENOTYPES=1")
