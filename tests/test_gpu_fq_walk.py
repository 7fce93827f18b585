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
    # VCFX_nonref_filter on the same walk (its own reducer), both input modes
    for mode, d in ((engine.MODE_FILE, ds), (engine.MODE_STDIN, dsq)):
        _check(eng, buf, d, lambda: eng.nonref_filter_region(d, mode), lambda: eng.nonref_filter(mode), ("nr", mode))


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


def _rf_edge_vcf(seed):
    """record heads the filter must read exactly from the tab offsets the walk stores: lines
    with under 8 fields, empty fields, QUAL '.', a leading space, hex / inf / long decimal
    values, INFO flags and keys that are prefixes of other keys, non-ASCII FILTER bytes, CRLF,
    empty and '#' lines, and INFO fields long enough to push the first 8 tabs out of the
    walk's window (those lines take k_fq_finish's own tab scan)"""
    rng = np.random.default_rng(seed)
    ns = 40
    head = b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + \
        b"\t".join(b"S%d" % i for i in range(ns)) + b"\n"
    toks = [b"0|0", b"0|1", b"1|0", b"1|1"]

    def gts():
        return b"\t".join(toks[int(k)] for k in rng.integers(0, 4, ns))

    quals = [b"30", b"29.9999999999999999", b"30.0000000000000001", b".", b"", b" 31", b"0x1F", b"inf",
             b"-inf", b"nan", b"1e2", b"3e1", b"29", b"abc", b"+30", b"00030"]
    filters = [b"PASS", b"LowQual", b"", b".", b"P\xc3\xa9SS", b"PASS;q10", b"pass"]
    infos = [b".", b"AF=0.5", b"AF=0.01;DP=3", b"DB;AF=0.009", b"AFX=0.5;AF=0.02", b"AF", b"AF=", b"AF=0x1p-6",
             b"DP=7;AF=1e-2", b"AF=0.2;" + b"X=" + b"y" * 1500]
    body = []
    for i in range(2500):
        pos = 9411239 + i
        r = rng.random()
        q, f, inf = (quals[int(rng.integers(0, len(quals)))], filters[int(rng.integers(0, len(filters)))],
                     infos[int(rng.integers(0, len(infos)))])
        if r < 0.03:
            body.append(b"\n")
        elif r < 0.05:
            body.append(b"#interleaved\n")
        elif r < 0.10:  # under 8 fields
            k = int(rng.integers(1, 8))
            body.append(b"\t".join([b"21", b"%d" % pos, b"rs", b"A", b"C", q, f][:k]) + b"\n")
        elif r < 0.13:
            body.append(b"\t" * int(rng.integers(1, 12)) + b"\n")
        else:
            line = b"21\t%d\trs%d\tA\tC\t%s\t%s\t%s\tGT\t%s" % (pos, i, q, f, inf, gts())
            body.append(line + (b"\r\n" if rng.random() < 0.1 else b"\n"))
    return head + b"".join(body)


EDGE_CRITS = [
    ([(engine.QUAL, engine.GE, 1, 30.0, "", "")], True),
    ([(engine.QUAL, engine.LT, 1, 30.0, "", ""), (engine.FILTER, engine.NE, 0, 0.0, "", "PASS")], False),
    ([(engine.FILTER, engine.EQ, 0, 0.0, "", b"P\xc3\xa9SS")], True),
    ([(engine.INFO, engine.GE, 1, 0.01, "AF", "")], True),
    ([(engine.INFO, engine.EQ, 0, 0.0, "DB", "DB"), (engine.POS, engine.LE, 1, 9412000.0, "", "")], True),
    ([(engine.INFO, engine.NE, 0, 0.0, "AF", "0.5"), (engine.QUAL, engine.GT, 1, 29.5, "", "")], False),
]


@pytest.mark.parametrize("seed", [3, 4])
def test_walk_filter_edge_heads(eng, seed):
    buf = _rf_edge_vcf(seed)
    ds = engine.data_start_of(buf)
    for crits, logic in EDGE_CRITS:
        _check(eng, buf, ds, lambda: eng.record_filter_region(ds, crits, logic),
               lambda: eng.record_filter(crits, logic), ("rf-edge", crits, logic))
        _check(eng, buf, ds, lambda: eng.filter_query_region(ds, crits, "0|1", logic, False),
               lambda: eng.filter_query(crits, "0|1", logic, False), ("pipe-edge", crits, logic))
