"""GPU parity of VCFX_dosage_calculator beyond the golden cases: seeded
synthetic VCFs -- fixed-stride records, missing calls, irregular GT shapes (GT:DP, DP:GT, mixed
separators, haploid, multi-digit alleles), GT:AD:DP records, CRLF -- in both input modes
against the C oracle, through the drop-in tool and the engine's per-line statuses."""
import numpy as np
import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    dict(n_records=1200, n_samples=2504, seed=81),
    dict(n_records=800, n_samples=997, seed=82, info_mode=1, missing_rate=0.01, irregular_rate=0.2, crlf=1),
    dict(n_records=3000, n_samples=3, seed=83, missing_rate=0.05, irregular_rate=0.3),
    dict(n_records=300, n_samples=3999, seed=84, irregular_rate=0.1),
    dict(n_records=600, n_samples=301, seed=85, missing_rate=0.002, format_mode=1),
    dict(n_records=400, n_samples=64, seed=86, irregular_rate=0.3, crlf=1, format_mode=1),
]


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_dosage_tool_matches_oracle(oracle, cfg, tmp_path):
    buf = synth.generate(**cfg)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    for argv, stdin in ((["VCFX_dosage_calculator", "-i", str(path)], b""), (["VCFX_dosage_calculator"], buf),
                        (["VCFX_dosage_calculator", "-q", str(path)], b"")):
        want = oracle.run(argv, stdin)
        got = tools.run(argv, stdin)
        assert got == want, (argv[1:2], len(got[0]), len(want[0]))


def test_dosage_engine_statuses(oracle):
    buf = synth.generate(1500, 2504, 87, 0, 0.001, 0, 0.0, 0)
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    s = eng.dosage_region(ds, engine.MODE_FILE)
    assert s.rows == 1500 and s.general_records == 0 and s.warn_lines == 0
    st = eng.statuses(s.n_lines)
    assert int((st == 1).sum()) == 1500
    want = oracle.run(["VCFX_dosage_calculator"], buf)[0]
    assert b"CHROM\tPOS\tID\tREF\tALT\tDosages\n" + eng.text(s.text_bytes) == want
    eng.close()


def _mutate(buf, rec, sample, new):
    """replace sample `sample` of data record `rec` (fixed-stride "a|b" units) by `new` bytes"""
    lines = buf.split(b"\n")
    k = next(i for i, l in enumerate(lines) if l.startswith(b"#CHROM")) + 1 + rec
    f = lines[k].split(b"\t")
    f[9 + sample] = new
    lines[k] = b"\t".join(f)
    return b"\n".join(lines)


# the head walk (DoseHeadOp) takes a record on its predicted '\n' alone; k_dose_fmt's check of
# every sample byte must catch each way such a record can differ, and the call must be redone
# with the sweeping walk: an "NA" ('.'), a non-digit allele, another separator, a sample of the
# same width in another shape, and a '\n' inside a record of the predicted length (two lines)
MUTATIONS = [
    (7, 100, b".|0"), (300, 2503, b"0|."), (11, 0, b"x|1"), (12, 5, b"1/0"), (13, 9, b"11|"),
    (14, 1000, b"0\n0"),
]


@pytest.mark.parametrize("rec,sample,new", MUTATIONS)
def test_dosage_head_walk_fallback(oracle, rec, sample, new):
    buf = _mutate(synth.generate(600, 2504, 88, 0, 0.0, 0, 0.0, 0), rec, sample, new)
    want = oracle.run(["VCFX_dosage_calculator"], buf)[0]
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    for _ in range(2):  # the failed head attempt, then the input's remembered sweeping walk
        s = eng.dosage_region(ds, engine.MODE_FILE)
        assert b"CHROM\tPOS\tID\tREF\tALT\tDosages\n" + eng.text(s.text_bytes) == want
    eng.close()


def test_dosage_head_walk_clean(oracle):
    # a clean fixed-stride input: the head walk's rows all pass, every record a fixed-stride row
    buf = synth.generate(900, 2504, 89, 0, 0.0, 0, 0.0, 0)
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    s = eng.dosage_region(ds, engine.MODE_FILE)
    assert s.rows == 900 and s.general_records == 0
    assert b"CHROM\tPOS\tID\tREF\tALT\tDosages\n" + eng.text(s.text_bytes) == \
        oracle.run(["VCFX_dosage_calculator"], buf)[0]
    eng.close()
