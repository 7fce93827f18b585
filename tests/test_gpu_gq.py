"""GPU parity for VCFX_genotype_query on synthetic inputs: kept-record decisions are
bit-exact against the C oracle for flexible and strict queries, both input modes."""
import os
import tempfile

import pytest

from tests._golden import Oracle
from vcfx_amd import synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    (1200, 2504, 31, 0, 0.0, 0, 0.0, 0),
    (900, 301, 32, 1, 0.02, 0, 0.3, 0),
    (400, 64, 33, 1, 0.01, 0, 0.2, 1),
    (500, 3, 34, 0, 0.2, 0, 0.5, 0),
]
QUERIES = [["-g", "0/1"], ["-g", "1|1"], ["-g", "1/1", "--strict"], ["-g", "0|1", "--strict"], ["-g", "2/1"],
           ["-g", "0/0"], ["-g", "./.", "--strict"], ["-g", "10/1"], ["-g", "1/x"]]


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_gq_matches_oracle(oracle, cfg):
    buf = synth.generate(*cfg)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for q in QUERIES:
            for argv, stdin in ((["VCFX_genotype_query"] + q + ["-i", f.name], b""),
                                (["VCFX_genotype_query"] + q, buf)):
                got = tools.run(argv, stdin)
                want = oracle.run(argv, stdin)
                assert got == want, (argv[1:], cfg)
