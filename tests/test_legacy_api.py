"""The reference's per-tool library interfaces: VCFX_record_filter's
legacy free functions (VCFX_record_filter.h:99-102) and VCFX_genotype_query's stream API
(VCFX_genotype_query.h:9-24), as build/libvcfx_record_filter.so and
build/libvcfx_genotype_query.so serve them.

tests/legacy_rf_test.cpp is built against our library and -- where /root/reference exists --
against the reference's own VCFX_record_filter.cpp (oracle/_ref/record_filter_lib_ref.o, main
renamed); both outputs must equal the committed goldens the reference build produced
(regenerate with VCFX_REGEN_LEGACY_GOLDEN=1).  parseCriteria / recordPasses run on the host
(CPU tests); processVCF evaluates the records on the GPU (gpu tests), including the lines the
device hands back for strtod's prefix value (OR-mode QUAL) and '\\r'-terminated lines."""
import os
import subprocess

import pytest

from tests._golden import GOLDEN
from vcfx_amd import BUILD, REPO

HARNESS = os.path.join(REPO, "tests", "legacy_rf_test.cpp")
CRITS = os.path.join(REPO, "tests", "legacy_rf_criteria.txt")
RECORDS = os.path.join(REPO, "tests", "legacy_rf_records.txt")
REF = "/root/reference"
REF_CORE = os.path.join(REPO, "oracle", "_ref", "vcfx_core_ref.o")
REF_RF = os.path.join(REPO, "oracle", "_ref", "record_filter_lib_ref.o")
GOLD_REC = os.path.join(GOLDEN, "legacy_rf_records_expected.txt")
GOLD_PROC = os.path.join(GOLDEN, "legacy_rf_process_expected.txt")
PROC_VCFS = [os.path.join(REPO, "tests", "legacy_rf_process.vcf"), "data/crlf.vcf", "data/edge_zoo.vcf",
             "data/data_before_header.vcf", "data/no_trailing_newline.vcf", "data/ties.vcf", "data/ragged_samples.vcf"]


def _build_ours(out):
    lib = os.path.join(BUILD, "libvcfx_record_filter.so")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-DVCFX_OURS", "-o", out, HARNESS,
                           "-I" + os.path.join(REPO, "include"), lib, "-Wl,-rpath," + BUILD])


def _build_ref(out):
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "Makefile.ref"), REF_RF, REF_CORE])
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-o", out, HARNESS,
                           "-I" + os.path.join(REF, "src", "VCFX_record_filter"), "-I" + os.path.join(REF, "include"),
                           REF_RF, REF_CORE, "-lz"])


def _run(exe, *args):
    r = subprocess.run([exe] + list(args), capture_output=True, timeout=300, cwd=GOLDEN)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout + b"\n--stderr--\n" + r.stderr


@pytest.fixture(scope="module")
def ours(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("legacy") / "legacy_rf_ours")
    _build_ours(exe)
    return exe


@pytest.fixture(scope="module")
def ref(tmp_path_factory):
    if not os.path.isdir(REF):
        pytest.skip("reference sources absent (GPU box)")
    exe = str(tmp_path_factory.mktemp("legacy") / "legacy_rf_ref")
    _build_ref(exe)
    return exe


def test_record_passes_matches_reference_golden(ours):
    got = _run(ours, "records", CRITS, RECORDS)
    if os.environ.get("VCFX_REGEN_LEGACY_GOLDEN"):
        pytest.skip("regenerating")
    assert got == open(GOLD_REC, "rb").read()


def test_record_passes_matches_reference_build(ours, ref):
    want = _run(ref, "records", CRITS, RECORDS)
    if os.environ.get("VCFX_REGEN_LEGACY_GOLDEN"):
        open(GOLD_REC, "wb").write(want)
    assert _run(ours, "records", CRITS, RECORDS) == want


def test_process_golden_from_reference(ref):
    """(CPU) the processVCF golden is the reference build's output"""
    want = b"".join(b"== %s\n" % os.path.basename(v).encode() + _run(ref, "process", CRITS, v) for v in PROC_VCFS)
    if os.environ.get("VCFX_REGEN_LEGACY_GOLDEN"):
        open(GOLD_PROC, "wb").write(want)
    assert want == open(GOLD_PROC, "rb").read()


@pytest.mark.gpu
def test_process_vcf_on_gpu_matches_reference(ours):
    got = b"".join(b"== %s\n" % os.path.basename(v).encode() + _run(ours, "process", CRITS, v) for v in PROC_VCFS)
    assert got == open(GOLD_PROC, "rb").read()


@pytest.mark.gpu
def test_genotype_query_stream_api(tmp_path):
    """genotypeQueryStream / genotypeQuery through build/libvcfx_genotype_query.so against the
    drop-in's own stdin path (pinned to the reference by the golden cases)"""
    from vcfx_amd import tools
    src = tmp_path / "gq.cpp"
    src.write_text(r'''
#include <fstream>
#include <iostream>
#include "vcfx_genotype_query.h"
int main(int argc, char **argv) {
    std::ifstream in(argv[1], std::ios::binary);
    if (argc > 3) genotypeQueryStream(in, std::cout, argv[2], argv[3][0] == 's', argv[3][1] == 'q');
    else genotypeQuery(in, std::cout, argv[2], false);
    return 0;
}''')
    exe = str(tmp_path / "gq")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-o", exe, str(src), "-I" + os.path.join(REPO, "include"),
                           os.path.join(BUILD, "libvcfx_genotype_query.so"), "-Wl,-rpath," + BUILD])
    for vcf in ("data/synth_annot.vcf", "data/crlf.vcf", "data/edge_zoo.vcf", "data/no_chrom.vcf"):
        data = open(os.path.join(GOLDEN, vcf), "rb").read()
        for q, flags in (("0/1", None), ("1|1", "s-"), ("0|1", "sq"), ("1/0", "-q")):
            argv = ["VCFX_genotype_query", "-g", q] + (["--strict"] if flags and flags[0] == "s" else []) + \
                (["-q"] if flags and flags[1] == "q" else [])
            want = tools.run(argv, data)
            r = subprocess.run([exe, os.path.join(GOLDEN, vcf), q] + ([flags] if flags else []), capture_output=True,
                               timeout=120)
            assert (r.stdout, r.stderr) == (want[0], want[1]), (vcf, q, flags)
