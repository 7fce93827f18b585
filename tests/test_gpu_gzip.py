"""Compressed input for the record tools: gzip, multi-member gzip and
BGZF (build/bin/vcfx_bgzf) forms of the golden fixtures through AF, RF, GQ, NR and LD -- file
path, `< file` and a pipe -- must give exactly the output the same tool gives on the
uncompressed bytes (itself pinned to the reference by the golden cases).  Truncated streams
fail loudly; VCFX_GZIP=0 restores the reference's own behaviour on .gz bytes (read as text),
checked against the C oracle on the same bytes."""
import gzip
import os
import subprocess

import pytest

from tests._golden import GOLDEN, Oracle
from vcfx_amd import BUILD, tools

pytestmark = pytest.mark.gpu

FIXTURES = ["synth_regular.vcf", "synth_annot.vcf", "synth_irregular.vcf", "synth_missing.vcf", "crlf.vcf",
            "edge_zoo.vcf", "no_trailing_newline.vcf"]
COMMANDS = [["VCFX_allele_freq_calc", "-q", "-i", "{F}"], ["VCFX_allele_freq_calc", "-q"],
            ["VCFX_record_filter", "--filter", "QUAL>=30;FILTER==PASS", "-i", "{F}"],
            ["VCFX_record_filter", "--filter", "AF>0.1", "--logic", "or"],
            ["VCFX_genotype_query", "-g", "0/1", "-i", "{F}"], ["VCFX_genotype_query", "-g", "1|1", "--strict"],
            ["VCFX_nonref_filter", "-i", "{F}"], ["VCFX_nonref_filter"]]


def _forms(tmp, name):
    raw = open(os.path.join(GOLDEN, "data", name), "rb").read()
    src = os.path.join(tmp, name)
    open(src, "wb").write(raw)
    out = {"plain": src}
    subprocess.check_call([os.path.join(BUILD, "bin", "vcfx_bgzf"), src, src + ".bgz", "4", "1"])
    out["bgzf"] = src + ".bgz"
    open(src + ".gz", "wb").write(gzip.compress(raw, 6, mtime=0))
    out["gzip"] = src + ".gz"
    h = len(raw) // 3
    open(src + ".mm.gz", "wb").write(gzip.compress(raw[:h], 1, mtime=0) + gzip.compress(raw[h:], 9, mtime=0))
    out["members"] = src + ".mm.gz"
    return raw, out


def _run(argv, path, how):
    a = [x.replace("{F}", path) for x in argv]
    if "{F}" in " ".join(argv):
        return tools.run(a)
    data = open(path, "rb").read()
    return tools.run_pipe(a, data) if how == "pipe" else tools.run(a, data)


@pytest.mark.parametrize("name", FIXTURES)
def test_compressed_forms_match_plain(tmp_path, name):
    _, forms = _forms(str(tmp_path), name)
    for argv in COMMANDS:
        want = _run(argv, forms["plain"], "file")
        for kind in ("bgzf", "gzip", "members"):
            for how in ("file", "pipe"):
                got = _run(argv, forms[kind], how)
                assert got == want, (name, argv, kind, how, got[1][-300:])


def test_ld_on_bgzf(tmp_path):
    _, forms = _forms(str(tmp_path), "synth_ld.vcf")
    for argv in (["VCFX_ld_calculator", "-q", "-w", "60", "-t", "0.2", "-i", "{F}"],
                 ["VCFX_ld_calculator", "-q", "-w", "40", "-t", "0.1"]):
        want = _run(argv, forms["plain"], "file")
        assert want[2] == 0 and want[0]
        for kind in ("bgzf", "gzip"):
            assert _run(argv, forms[kind], "file") == want, (argv, kind)


def test_truncated_and_corrupt_streams_fail(tmp_path):
    _, forms = _forms(str(tmp_path), "synth_annot.vcf")
    for kind in ("bgzf", "gzip"):
        b = open(forms[kind], "rb").read()
        for cut, label in ((b[:len(b) // 2], "trunc"), (b[:5000] + bytes(len(b) - 5000), "zeroed")):
            p = str(tmp_path / ("bad_%s_%s.gz" % (kind, label)))
            open(p, "wb").write(cut)
            out, err, rc = tools.run(["VCFX_allele_freq_calc", "-q", "-i", p])
            assert rc == 1 and b"truncated or corrupt" in err, (kind, label, err)


def test_gzip_off_reads_bytes_as_text_like_the_reference(tmp_path, monkeypatch):
    _, forms = _forms(str(tmp_path), "synth_annot.vcf")
    monkeypatch.setenv("VCFX_GZIP", "0")
    o = Oracle()
    for argv in (["VCFX_allele_freq_calc", "-q", "-i", forms["gzip"]],
                 ["VCFX_record_filter", "--filter", "QUAL>=30", "-i", forms["bgzf"]],
                 ["VCFX_nonref_filter", "-i", forms["gzip"]]):
        assert tools.run(argv) == o.run(argv), argv
