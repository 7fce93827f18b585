"""GPU parity of the filter / query walk (vcfxg_fq_walk.hip): VCFX_record_filter,
VCFX_genotype_query and the fused record_filter | genotype_query pipeline in one device pass
without a separate line index give the same per-line statuses, line ends and summaries as
vcfxg_index + the per-tool kernels -- on every walk chunk size (lines that start in, span and
skip over walkers' chunks), with the walk forced onto short lines, on layouts where the walk
must reject the record ends it predicts, and when a walker overflows its line slots."""
import numpy as np
import pytest

from tests.test_gpu_af_fused import _walk_layouts
from vcfx_amd import engine, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["default", "walk", "walk4k", "walk1k"])
def eng(request):
    """default: the walk for long records (else index + per-tool kernels); walk: forced, on
    chunks of 128 KiB, 4 KiB and 1 KiB"""
    import os
    env = {"VCFXG_FQ_WALK": "0" if request.param == "default" else "1",
           "VCFXG_WALK_CHUNK": {"walk4k": "4096", "walk1k": "1024"}.get(request.param, str(128 * 1024))}
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


# (target, op, numeric, value, INFO key, string value) as vcfxg_criterion
PASS_QUAL = [(engine.QUAL, engine.GE, 1, 30.0, "", ""), (engine.FILTER, engine.EQ, 0, 0.0, "", "PASS")]
CRITS = [(PASS_QUAL, True),
         ([(engine.INFO, engine.GE, 1, 0.01, "AF", "")], True),
         ([(engine.POS, engine.GT, 1, 9411500.0, "", ""), (engine.FILTER, engine.NE, 0, 0.0, "", "PASS")], False)]
QUERIES = [("0|1", False), ("1/1", False), ("0|1", True), ("1/x", False)]
SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (1500, 2504, 51, 1, 0.0, 0, 0.0, 0),
    (800, 997, 52, 1, 0.01, 0, 0.2, 1),
    (3000, 3, 53, 1, 0.05, 0, 0.3, 1),
    (200, 5000, 54, 0, 0.0, 0, 0.1, 0),
]


def _result(eng, s):
    n = s.n_lines
    return eng.line_ends(n), eng.statuses(n), (s.n_lines, s.rows, s.data_lines, s.warn_lines, s.general_records)


def _check(eng, buf, ds, region, per_tool, what):
    eng.load(buf)
    got = _result(eng, region())
    eng.load(buf)
    eng.index(ds)
    want = _result(eng, per_tool())
    np.testing.assert_array_equal(got[0], want[0], err_msg=what)
    np.testing.assert_array_equal(got[1], want[1], err_msg=what)
    assert got[2] == want[2], what


def _all(eng, buf):
    ds = engine.data_start_of(buf)
    dsq = engine.data_start_of(buf, strip_cr=False)
    for crits, logic in CRITS:
        _check(eng, buf, ds, lambda: eng.record_filter_region(ds, crits, logic),
               lambda: eng.record_filter(crits, logic), ("rf", crits, logic))
    for q, strict in QUERIES:
        for strip in (False, True):
            _check(eng, buf, dsq, lambda: eng.genotype_query_region(dsq, q, strict, strip),
                   lambda: eng.genotype_query(q, strict, strip), ("gq", q, strict, strip))
        for crits, logic in CRITS[:2]:
            _check(eng, buf, ds, lambda: eng.filter_query_region(ds, crits, q, logic, strict),
                   lambda: eng.filter_query(crits, q, logic, strict), ("pipe", crits, q, strict))


@pytest.mark.parametrize("cfg", SYNTH)
def test_walk_matches_per_tool(eng, cfg):
    _all(eng, synth.generate(*cfg))


@pytest.mark.parametrize("seed", [1, 2])
def test_walk_predicted_ends(eng, seed):
    for buf in _walk_layouts(seed):
        _all(eng, buf)


def test_walk_overflow_falls_back(eng):
    """long first records (the line-slot estimate) followed by thousands of short lines: a
    walker runs out of slots and the call is redone on index + per-tool kernels"""
    long_part = synth.generate(300, 2504, 55, 1, 0.0, 0, 0.0, 0)
    short = b"".join(b"21\t%d\t.\tA\tG\t%d\tPASS\tAF=0.5\tGT\t0|1\n" % (10 ** 8 + i, i % 60) for i in range(40000))
    _all(eng, long_part + short)
