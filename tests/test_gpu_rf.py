"""GPU parity for VCFX_record_filter (exact strtod semantics on the device) and for the
fused record_filter | genotype_query pipeline (BASELINE config 3) against the C oracle."""
import os
import tempfile

import pytest

from tests._golden import GOLDEN, Oracle
from vcfx_amd import synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    (1200, 500, 41, 1, 0.0, 0, 0.0, 0),
    (900, 301, 42, 1, 0.02, 0, 0.3, 0),
    (400, 64, 43, 1, 0.01, 0, 0.2, 1),
]
FILTERS = ["FILTER==PASS;AF>=0.01", "AF>=0.01", "AF<0.0005", "DP>2500", "DP<=100;QUAL>=100", "QUAL>99.99999999999999",
           "POS>9411500", "AF==0.0002", "AF!=0.0002", "AF>0.00019999999999999998", "AF>=0.0002000000000000000096",
           "DP>=1e3", "FILTER!=PASS", "AF>1e-400", "POS<=0x8F9B00"]


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_rf_matches_oracle(oracle, cfg):
    buf = synth.generate(*cfg)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for flt in FILTERS:
            for logic in ("and", "or"):
                for argv, stdin in ((["VCFX_record_filter", "--filter", flt, "-l", logic, "-i", f.name], b""),
                                    (["VCFX_record_filter", "-f", flt, "--logic", logic], buf)):
                    got = tools.run(argv, stdin)
                    want = oracle.run(argv, stdin)
                    assert got == want, (argv[1:], cfg)


# values around a threshold's rounding boundaries: the device decides x OP t from the text
EDGE_VALUES = ["0.1", "0.10000000000000000555", "0.1000000000000000055511151231257827",
               "0.10000000000000000555111512312578270211815834045410156250", "0.1000000000000000055511151231257828",
               "0.09999999999999999167", "0.099999999999999998612221219218554", "1e-1", "10e-2", "0x1.999999999999ap-4",
               "0x1.999999999999bp-4", " 0.1", "+.1", "-0.1", "inf", "-Infinity", "nan", "NaN(123)", "0.1x", "",
               "1e", "0x", ".", "-0", "4.9406564584124654e-324", "2.4703282292062328e-324", "2.4703282292062327e-324",
               "1.7976931348623158e308", "1.7976931348623159e308", "1e400", "-1e400", "0.0000000000000000000001e21"]


@pytest.mark.parametrize("thr", ["0.1", "0", "-0.1", "1e-300", "4.9406564584124654e-324", "1.7976931348623157e308",
                                 "inf", "nan", "0x1p-1074"])
def test_rf_numeric_edges(oracle, thr):
    hdr = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
    body = "".join("1\t%d\t.\tA\tC\t%s\tPASS\tX=%s\n" % (i + 1, v if v else ".", v) for i, v in enumerate(EDGE_VALUES))
    buf = (hdr + body).encode()
    for op in (">", ">=", "<", "<=", "==", "!="):
        for field in ("X", "QUAL"):
            argv = ["VCFX_record_filter", "--filter", "%s%s%s" % (field, op, thr)]
            assert tools.run(argv, buf) == oracle.run(argv, buf), (field, op, thr)


def _pipe_oracle(oracle, flt, q, path, logic="and", strict=False):
    a = ["VCFX_record_filter", "--filter", flt, "--logic", logic, path]
    mid, err1, rc1 = oracle.run(a)
    b = ["VCFX_genotype_query", "-g", q] + (["--strict"] if strict else [])
    out, err2, rc2 = oracle.run(b, mid)
    return out, err1 + err2


@pytest.mark.parametrize("cfg", SYNTH + [(300, 2504, 44, 1, 0.0, 0, 0.0, 0)])
def test_pipeline_matches_oracle(oracle, cfg):
    buf = synth.generate(*cfg)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for flt, q, strict in (("FILTER==PASS;AF>=0.01", "0/1", False), ("AF>=0.001", "1|1", True),
                               ("DP>100", "0|1", False), ("QUAL>1000", "0/1", False)):
            out, err, rc = tools.pipeline_filter_query(flt, q, input_path=f.name, strict=strict)
            wout, werr = _pipe_oracle(oracle, flt, q, f.name, strict=strict)
            assert rc == 0 and out == wout and err == werr, (flt, q, cfg)


def test_pipeline_on_golden_fixtures(oracle):
    for name in sorted(os.listdir(os.path.join(GOLDEN, "data"))):
        if not name.endswith(".vcf"):
            continue
        path = os.path.join(GOLDEN, "data", name)
        out, err, rc = tools.pipeline_filter_query("FILTER==PASS;AF>=0.01", "0/1", input_path=path)
        wout, werr = _pipe_oracle(oracle, "FILTER==PASS;AF>=0.01", "0/1", path)
        assert (out, err) == (wout, werr), name
