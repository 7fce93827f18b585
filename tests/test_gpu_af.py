"""GPU parity for VCFX_allele_freq_calc: the HIP path against the C-restatement oracle and
the reference goldens.  Bit-exact: integer counts, and the formatted 4-dp text (which
pins the fp64 frequency and both rounding rules)."""
import os

import numpy as np
import pytest

from tests._golden import GOLDEN, Oracle, case_stdin, load_cases, matches
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu



@pytest.fixture(scope="module")
def eng():
    return engine.Engine(0)


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (2000, 2504, 1, 0, 0.0, 0, 0.0, 0),
    (1500, 997, 2, 1, 0.01, 0, 0.0, 0),
    (1500, 301, 3, 1, 0.02, 0, 0.3, 0),
    (800, 64, 4, 1, 0.01, 0, 0.2, 1),
    (600, 5, 5, 0, 0.1, 0, 0.5, 0),
    (300, 1, 6, 0, 0.0, 0, 0.0, 0),
]


@pytest.mark.parametrize("cfg", SYNTH)
@pytest.mark.parametrize("mode", [engine.MODE_FILE, engine.MODE_STDIN])
def test_af_counts_match_oracle(eng, oracle, cfg, mode):
    buf = synth.generate(*cfg)
    ds = engine.data_start_of(buf, strip_cr=(mode == engine.MODE_FILE))
    eng.load(buf)
    nl = eng.index(ds)
    s = eng.allele_freq(mode)
    alt, tot, st = eng.lines(nl)
    ralt, rtot = oracle.af_counts(buf, stdin_mode=(mode == engine.MODE_STDIN))
    rows = st == 1
    assert rows.sum() == len(ralt) == s.rows
    np.testing.assert_array_equal(alt[rows], ralt)
    np.testing.assert_array_equal(tot[rows], rtot)
    # full output text vs the restated tool
    text = eng.text(s.text_bytes)
    argv = ["VCFX_allele_freq_calc", "-q"]
    if mode == engine.MODE_FILE:
        import tempfile
        with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
            f.write(buf)
            f.flush()
            want, _, _ = oracle.run(argv + ["-i", f.name])
    else:
        want, _, _ = oracle.run(argv, buf)
    assert b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + text == want


def test_af_fast_path_taken_on_regular_records(eng):
    buf = synth.generate(1000, 2504, 9, 0, 0.0, 0, 0.0, 0)
    eng.load(buf)
    eng.index(engine.data_start_of(buf))
    s = eng.allele_freq(engine.MODE_FILE)
    assert s.rows == 1000 and s.general_records == 0


def test_af_cli_binary_end_to_end(tmp_path):
    import subprocess
    from vcfx_amd import tool_binary
    buf = synth.generate(3000, 2504, 21, 0, 0.001, 0, 0.01, 0)
    p = tmp_path / "in.vcf"
    p.write_bytes(buf)
    o = Oracle()
    for args in (["-i", str(p)], [str(p)]):
        r = subprocess.run([tool_binary("VCFX_allele_freq_calc")] + args, capture_output=True, timeout=300)
        want, werr, wrc = o.run(["VCFX_allele_freq_calc"] + args)
        assert (r.stdout, r.stderr, r.returncode) == (want, werr, wrc)
    r = subprocess.run([tool_binary("VCFX_allele_freq_calc")], input=buf, capture_output=True, timeout=300)
    want, werr, wrc = o.run(["VCFX_allele_freq_calc"], buf)
    assert (r.stdout, r.stderr, r.returncode) == (want, werr, wrc)


@pytest.mark.parametrize("cfg", [dict(n_records=1200, n_samples=2504, seed=31, missing_rate=0.001, format_mode=1),
                                 dict(n_records=700, n_samples=301, seed=32, missing_rate=0.05, irregular_rate=0.2,
                                      crlf=1, format_mode=1)])
def test_af_gt_ad_dp_region_matches_oracle(eng, oracle, cfg, tmp_path):
    """FORMAT=GT:AD:DP (variable-width samples: every record off the fixed-stride sweep) through
    the region path (walk + leftover lines) and the drop-in tool, both modes"""
    buf = synth.generate(**cfg)
    for mode in (engine.MODE_FILE, engine.MODE_STDIN):
        ds = engine.data_start_of(buf, strip_cr=(mode == engine.MODE_FILE))
        eng.load(buf)
        s = eng.allele_freq_region(ds, mode)
        assert s.general_records == cfg["n_records"]
        p = tmp_path / "in.vcf"
        p.write_bytes(buf)
        argv = ["VCFX_allele_freq_calc", "-q"] + (["-i", str(p)] if mode == engine.MODE_FILE else [])
        stdin = b"" if mode == engine.MODE_FILE else buf
        want = oracle.run(argv, stdin)
        assert b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes) == want[0]
        assert tools.run(argv, stdin) == want


def _mutate_gtadp(buf, edits):
    """replace sample k of data record r (0-based) with the given bytes; (r, None, tail) appends
    tail bytes to the record's end instead (before its newline)"""
    lines = buf.split(b"\n")
    first = next(i for i, l in enumerate(lines) if l.startswith(b"#CHROM")) + 1
    for r, k, new in edits:
        f = lines[first + r].split(b"\t")
        if k is None:
            lines[first + r] = lines[first + r] + new
            continue
        f[9 + k] = new
        lines[first + r] = b"\t".join(f)
    return b"\n".join(lines)


def test_af_gt_first_flag_sweep_edge_samples(eng, oracle, tmp_path):
    """the GT-first walk's per-byte-flag sweep (gt_first_af) against the oracle on GT:AD:DP
    records holding every sample shape it must either count as a quick 'c0 s c2' GT or hand to
    the exact path: letters, haploid and multi-digit GTs, spaces, empty samples, a non-ASCII
    byte (also right before the line end), a CRLF line end, a bare last GT ('0|1' then the line
    end), a sample cut to 1-2 bytes at the line end, a GT at a lane / step boundary"""
    buf = synth.generate(n_records=400, n_samples=600, seed=41, missing_rate=0.01, format_mode=1)
    edits = [
        (3, 5, b"A|1:3,4:7"), (7, 0, b"0:3,4:7"), (11, 599, b"10|1:2,2:4"), (13, 100, b"0 |1:2,2:4"),
        (17, 200, b""), (19, 300, b"0|1:\xc3\xa9,4:7"), (23, 599, b"0|1"), (29, 599, b"0"), (31, 599, b"0|"),
        (37, 42, b"0|1:1,2:3:4:5"), (41, 63, b".|1:1,1:2"), (43, 64, b"1/.:1,1:2"), (47, 1, b"|0:1,1:2"),
        (53, 2, b"0||:1,1:2"), (59, 77, b"0|1\t"), (61, 599, b"1|1:"), (67, 5, b"0/1:"), (71, 9, b"-|1:1,1:2"),
        # a non-ASCII byte right before the line end, at each offset in a dword (its SWAR carry
        # must not hide the '\n' from the end search)
        (83, 599, b"0|1:3,4:\xc3\xa9"), (85, 599, b"0|1:3,4:7\xc3\xa9"), (87, 599, b"0|1:3,4:77\xc3\xa9"),
        (89, 599, b"0|1:3,4:777\xc3\xa9"),
    ]
    buf = _mutate_gtadp(buf, edits)
    # one CRLF record
    lines = buf.split(b"\n")
    first = next(i for i, l in enumerate(lines) if l.startswith(b"#CHROM")) + 1
    lines[first + 79] += b"\r"
    buf = b"\n".join(lines)
    for mode in (engine.MODE_FILE, engine.MODE_STDIN):
        ds = engine.data_start_of(buf, strip_cr=(mode == engine.MODE_FILE))
        eng.load(buf)
        s = eng.allele_freq_region(ds, mode)
        p = tmp_path / "in.vcf"
        p.write_bytes(buf)
        argv = ["VCFX_allele_freq_calc", "-q"] + (["-i", str(p)] if mode == engine.MODE_FILE else [])
        stdin = b"" if mode == engine.MODE_FILE else buf
        want = oracle.run(argv, stdin)
        assert b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes) == want[0]
        assert tools.run(argv, stdin) == want
