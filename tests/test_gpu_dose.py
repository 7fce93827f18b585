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
