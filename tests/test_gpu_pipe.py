"""vcfx_pipe (tool_pipe.cpp): a chain of drop-ins in one process, stdout byte-identical to the
shell pipeline.  The expected bytes come from the C oracle run stage by stage (each stage's
stdout the next one's stdin, as the shell pipes them: VCFX_record_filter.cpp:498-549,
VCFX_genotype_query.cpp:527-617, VCFX_nonref_filter.cpp:553-636, VCFX_allele_freq_calc.cpp:
477-557).  Both schedules: fused (the input in HBM once, one walk per filter stage, the
decisions AND-ed, AF rows gathered) where it applies, the stage-by-stage chain (VCFX_PIPE_FUSED=0,
and every input the fused schedule hands to it: CRLF, data before '#CHROM', no survivors,
empty / header-only input, ragged records, gzip, abbreviated options)."""
import os
import subprocess
import tempfile

import pytest

from tests._golden import GOLDEN, Oracle
from vcfx_amd import BUILD, synth

pytestmark = pytest.mark.gpu
PIPE = os.path.join(BUILD, "bin", "vcfx_pipe")


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def oracle_chain(oracle, stages, stdin=b""):
    data, err, rc = stdin, b"", 0
    for st in stages:
        out, e, rc = oracle.run(st, data if not any(a in ("-i", "--input") for a in st) else b"")
        err += e
        data = out
    return data, rc


def run_pipe(chain, stdin=b"", env=None):
    r = subprocess.run([PIPE, chain], input=stdin, capture_output=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    return r.stdout, r.stderr, r.returncode


def _q(a):
    return "'" + a.replace("'", "'\\''") + "'"


def chain_str(stages):
    return " | ".join(" ".join(_q(a) for a in st) for st in stages)


RF, GQ, NR, AF = "VCFX_record_filter", "VCFX_genotype_query", "VCFX_nonref_filter", "VCFX_allele_freq_calc"
CHAINS = [
    [[RF, "--filter", "FILTER==PASS;AF>=0.01", "-i", "{F}"], [GQ, "-g", "0/1"], [AF]],
    [[RF, "--filter", "QUAL>=30", "--logic", "or", "{F}"], [AF, "-q"]],
    [[GQ, "-g", "0|1", "-i", "{F}"], [NR], [AF]],
    [[NR, "{F}"], [RF, "-f", "DP>10"], [GQ, "--genotype-query", "1/1", "--strict"]],
    [[GQ, "-g", "0/1", "--strict", "-i", "{F}"], [RF, "--filter=QUAL>=20"]],
    [[RF, "--filter", "FILTER==PASS"], [GQ, "-g", "0/1"], [AF]],           # stdin input
    [[NR], [AF]],
    [[RF, "--filt", "QUAL>=30", "-i", "{F}"], [AF]],                        # abbreviated: the chain parses it
    [[RF, "--filter", "QUAL>=30", "-i", "{F}"], ["VCFX_hwe_tester"]],       # not fusable: the chain
    [[RF, "--filter", "QUAL>=1e9", "-i", "{F}"], [GQ, "-g", "0/1"], [AF]],  # no survivors
]
FILES = ["synth_annot.vcf", "synth_regular.vcf", "synth_missing.vcf", "synth_irregular.vcf", "synth_crlf.vcf",
         "data_before_header.vcf", "edge_zoo.vcf", "empty.vcf", "header_only.vcf", "ragged_samples.vcf",
         "no_trailing_newline.vcf", "no_chrom.vcf"]


@pytest.mark.parametrize("fname", FILES)
def test_pipe_chains_match_oracle_pipeline(oracle, fname):
    path = os.path.join(GOLDEN, "data", fname)
    buf = open(path, "rb").read()
    bad = []
    for ch in CHAINS:
        stages = [[a.replace("{F}", path) for a in st] for st in ch]
        stdin = b"" if any("{F}" in " ".join(st) for st in ch) else buf
        want_out, want_rc = oracle_chain(oracle, stages, stdin)
        for env in ({}, {"VCFX_PIPE_FUSED": "0"}, {"VCFX_PIPE_FUSED": "1", "VCFX_FILE_STREAM_MIN": "1",
                                                    "VCFX_FILE_HEAD": "64", "VCFX_FILE_SLOT": "4096",
                                                    "VCFX_FILE_SLOTS": "4"}):
            out, err, rc = run_pipe(chain_str(stages), stdin, env)
            if out != want_out or rc != want_rc:
                bad.append((chain_str(ch), env, rc, want_rc, len(out), len(want_out), err[-300:]))
    assert not bad, bad[:4]


def test_pipe_fused_larger_synthetic(oracle):
    """a 6,000-record annotated input (fused: RF file mode -> GQ -> AF; and a filter last) against
    the oracle pipeline, the input streamed through the pinned file ring"""
    buf = synth.generate(6000, 300, 95, 1, 0.0005, 0, 0.0, 0)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for ch in CHAINS[:5]:
            stages = [[a.replace("{F}", f.name) for a in st] for st in ch]
            want = oracle_chain(oracle, stages)
            got = run_pipe(chain_str(stages), b"", {"VCFX_FILE_STREAM_MIN": "1", "VCFX_FILE_SLOT": "65536"})
            assert (got[0], got[2]) == want, (ch, got[1][-500:])
            assert got[1] == b""


def test_pipe_argv_form_and_errors():
    r = subprocess.run([PIPE], capture_output=True, timeout=60)
    assert r.returncode == 2 and b"Usage" in r.stderr
    r = subprocess.run([PIPE, "VCFX_record_filter --filter 'QUAL>=1"], capture_output=True, timeout=60)
    assert r.returncode == 2 and b"unterminated quote" in r.stderr
    r = subprocess.run([PIPE, "VCFX_nope | VCFX_allele_freq_calc"], capture_output=True, timeout=60)
    assert b"unknown tool 'VCFX_nope'" in r.stderr
    path = os.path.join(GOLDEN, "data", "synth_annot.vcf")
    a = subprocess.run([PIPE, "VCFX_record_filter", "--filter", "QUAL>=30", "-i", path, "|", "VCFX_allele_freq_calc"],
                       capture_output=True, timeout=120)
    b = subprocess.run([PIPE, "VCFX_record_filter --filter QUAL>=30 -i %s | VCFX_allele_freq_calc" % path],
                       capture_output=True, timeout=120)
    assert a.returncode == 0 and (a.stdout, a.stderr) == (b.stdout, b.stderr)
