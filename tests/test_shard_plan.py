"""CPU coverage of the in-process multi-GPU drop-in's planning (vcfx_shard_plan in
libvcfx_tools, tool_shard_main.cpp; no device): which invocations shard, and the record cuts
against the Python runner's rule (vcfx_amd/shard.py record_cuts_py: the reference's split at
i*size/N advanced past the next '\\n', VCFX_allele_counter.cpp:889-901)."""
import gzip
import os

import pytest

from tests import _bgzf as B
from vcfx_amd import shard, synth, tools


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("plan"))
    buf = synth.generate(500, 17, 71, 1, 0.02, 0, 0.2, 0)
    out = {}
    big = synth.generate(1500, 40, 73, 1, 0.02, 0, 0.2, 0)  # (several 64 KiB BGZF members)
    for name, b in (("synth.vcf", buf), ("synth.vcf.gz", gzip.compress(buf, mtime=0)),
                    ("big.vcf", big), ("big.vcf.bgz", B.bgzf(big, level=6)),
                    ("pre.vcf.bgz", B.bgzf(b"1\t5\t.\tA\tG\t.\t.\t.\tGT\t0|1\n" + big, level=6)),
                    ("pre.vcf", b"1\t5\t.\tA\tG\t.\t.\t.\tGT\t0|1\n" + buf),
                    ("head.vcf", buf[:buf.index(b"\n#CHROM") + 1] + buf[buf.index(b"\n#CHROM") + 1:].split(b"\n")[0] +
                     b"\n"),
                    ("crlf.vcf", synth.generate(60, 5, 72, 0, 0.0, 0, 0.0, 1))):
        p = os.path.join(d, name)
        open(p, "wb").write(b)
        out[name] = p
    return out


RECORD_TOOLS = [["VCFX_allele_freq_calc", "-q", "-i"], ["VCFX_allele_freq_calc"], ["VCFX_record_filter", "-f", "QUAL>1",
                                                                                      "-i"],
                ["VCFX_genotype_query", "-g", "0|1", "--strict"], ["VCFX_nonref_filter"], ["VCFX_dosage_calculator", "-i"],
                ["VCFX_hwe_tester", "-i"], ["VCFX_missing_detector", "-i"], ["VCFX_allele_counter", "-s", "S1 S2", "-i"]]


@pytest.mark.parametrize("head", RECORD_TOOLS)
@pytest.mark.parametrize("world", [2, 3, 8])
def test_record_cuts_match_the_reference_split(files, head, world):
    p = files["synth.vcf"]
    buf = open(p, "rb").read()
    w, kind, cuts = tools.shard_plan(head + [p], world)
    assert kind == 1 and w == world
    assert cuts == shard.record_cuts_py(buf, shard.header_end(buf), world)


def test_crlf_header_gate(files):
    p = files["crlf.vcf"]
    buf = open(p, "rb").read()
    w, kind, cuts = tools.shard_plan(["VCFX_allele_freq_calc", "-i", p], 4)
    assert kind == 1 and cuts == shard.record_cuts_py(buf, shard.header_end(buf), 4)


def test_unsharded_invocations(files):
    p = files["synth.vcf"]
    for argv in (["VCFX_allele_freq_calc", "-i", files["synth.vcf.gz"]],      # gzip: no byte cuts
                 ["VCFX_allele_freq_calc", "-i", files["pre.vcf"]],           # data before '#CHROM'
                 ["VCFX_allele_freq_calc", "-h", "-i", p],                    # help
                 ["VCFX_allele_freq_calc"],                                    # stdin
                 ["VCFX_allele_counter", "-z", "-i", p],                      # gzip output
                 ["VCFX_ld_calculator", "-m", "-i", p],                       # LD matrix
                 ["VCFX_ld_calculator", "-w", "5", p],                        # LD takes -i only
                 ["VCFX_haplotype_phaser", "-i", p],                          # not a sharded tool
                 ["VCFX_variant_counter", p],
                 ["VCFX_genotype_query", "-g", p]):                           # p is the query
        assert tools.shard_plan(argv, 4)[:2] == (1, 0), argv
    assert tools.shard_plan(["VCFX_allele_freq_calc", "-i", p], 1)[:2] == (1, 0)


def test_ld_rows_and_dropped_empty_ranks(files):
    p = files["synth.vcf"]
    assert tools.shard_plan(["VCFX_ld_calculator", "-w", "10", "-i", p], 5)[:2] == (5, 2)
    # one record: more ranks than records -> the ranks with an empty range are dropped
    w, kind, cuts = tools.shard_plan(["VCFX_allele_freq_calc", "-i", files["head.vcf"]], 8)
    assert (w, kind) == (1, 0) or (kind == 1 and all(a < b for a, b in zip(cuts, cuts[1:])))


@pytest.mark.parametrize("head", RECORD_TOOLS)
@pytest.mark.parametrize("world", [2, 3, 8])
def test_bgzf_cuts_in_the_inflated_bytes(files, head, world):
    """a BGZF member chain: kind 3, the same cuts as the reference split on the inflated bytes"""
    buf = open(files["big.vcf"], "rb").read()
    w, kind, cuts = tools.shard_plan(head + [files["big.vcf.bgz"]], world)
    assert kind == 3 and w == world
    assert cuts == shard.record_cuts_py(buf, shard.header_end(buf), world)


def test_bgzf_unsharded_and_ld_rows(files):
    # data before '#CHROM' in the inflated bytes; variant_counter (its own gzip handling); one
    # plain gzip member (not a BGZF chain); allele_counter -z
    for argv in (["VCFX_allele_freq_calc", "-i", files["pre.vcf.bgz"]], ["VCFX_variant_counter", files["big.vcf.bgz"]],
                 ["VCFX_allele_counter", "-z", "-i", files["big.vcf.bgz"]]):
        assert tools.shard_plan(argv, 4)[:2] == (1, 0), argv
    # LD rows: every rank inflates the whole file
    assert tools.shard_plan(["VCFX_ld_calculator", "-w", "10", "-i", files["big.vcf.bgz"]], 4)[:2] == (4, 2)
