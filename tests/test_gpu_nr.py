"""GPU parity of VCFX_nonref_filter beyond the golden cases: seeded
synthetic VCFs -- fixed-stride records (the sweep with its early exit), irregular and
missing genotypes, CRLF -- with a share of records rewritten to all hom-ref (dropped), in
both input modes, against the C oracle; plus the engine's per-line statuses."""
import re

import numpy as np
import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (1500, 2504, 61, 0, 0.0, 0, 0.0, 0),
    (800, 997, 62, 1, 0.01, 0, 0.2, 1),
    (3000, 3, 63, 1, 0.05, 0, 0.3, 0),
    (200, 5000, 64, 0, 0.0, 0, 0.1, 0),
]


def _homref_share(buf, every, seed):
    """every `every`-th data record's genotypes become 0|0 / 0/0 (same lengths)"""
    rng = np.random.default_rng(seed)
    out, k = [], 0
    for line in buf.split(b"\n"):
        if line and not line.startswith(b"#"):
            k += 1
            if k % every == 0:
                cr = line.endswith(b"\r")
                f = (line[:-1] if cr else line).split(b"\t", 9)
                if len(f) == 10:
                    g = re.sub(rb"[0-9.]([|/])[0-9.]", lambda m: b"0" + m.group(1) + b"0", f[9])
                    if rng.random() < 0.3 and re.fullmatch(rb".*\t0[|/]0", g, re.S):
                        g = g[:-3] + b"1" + g[-2:]  # one late non-ref sample: the sweep must reach it
                    f[9] = g
                    line = b"\t".join(f) + (b"\r" if cr else b"")
        out.append(line)
    return b"\n".join(out)


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_nonref_tool_matches_oracle(oracle, cfg, tmp_path):
    buf = _homref_share(synth.generate(*cfg), 3, cfg[2])
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    for argv, stdin in ((["VCFX_nonref_filter", "-i", str(path)], b""), (["VCFX_nonref_filter"], buf)):
        want = oracle.run(argv, stdin)
        got = tools.run(argv, stdin)
        assert got == want, (argv[1:2], len(got[0]), len(want[0]))


def test_nonref_statuses(oracle):
    buf = _homref_share(synth.generate(2000, 2504, 65, 0, 0.0, 0, 0.0, 0), 2, 65)
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    nl = eng.index(ds)
    s = eng.nonref_filter(engine.MODE_FILE)
    st = eng.statuses(nl)
    assert s.data_lines == 2000 and s.general_records == 0
    assert s.rows == int((st == 1).sum()) and int((st == 2).sum()) > 500
    out, _, _ = oracle.run(["VCFX_nonref_filter"], buf)
    assert s.rows == out.count(b"\n") - buf[:ds].count(b"\n")
    eng.close()
