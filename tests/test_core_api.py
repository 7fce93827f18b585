"""CPU parity of the host core API (include/vcfx_core.h, include/vcfx_io.h; SURVEY §8(a)
rows a1-a4): tests/core_api_test.cpp is compiled against libvcfx_core and, when the
reference sources are present in this container, against the reference's own
src/vcfx_core.cpp (oracle/_ref/vcfx_core_ref.o, built by oracle/Makefile.ref); both outputs
must equal tests/golden/core_api_expected.txt, which was produced by the reference build
(regenerate with VCFX_REGEN_CORE_GOLDEN=1)."""
import gzip
import os
import shutil
import subprocess

import pytest

from vcfx_amd import BUILD, REPO

SRC = os.path.join(REPO, "tests", "core_api_test.cpp")
GOLD = os.path.join(REPO, "tests", "golden", "core_api_expected.txt")
REF = "/root/reference"
REF_OBJ = os.path.join(REPO, "oracle", "_ref", "vcfx_core_ref.o")


def _data(d):
    vcf = "".join("##h%d\n" % i for i in range(3)) + "#CHROM\tPOS\n" + "".join(
        "1\t%d\tx\n" % i for i in range(20000))
    w = lambda n, b: open(os.path.join(d, n), "wb").write(b)  # noqa: E731
    w("plain.vcf", vcf.encode())
    w("one.vcf.gz", gzip.compress(vcf.encode(), mtime=0))
    half = len(vcf) // 2
    w("multi.vcf.bgz", gzip.compress(vcf[:half].encode(), mtime=0) + gzip.compress(vcf[half:].encode(), mtime=0))
    w("trunc.gz", gzip.compress(vcf.encode(), mtime=0)[:5000])
    w("empty.vcf", b"")
    w("fake.gz", b"not gzip at all\n")
    w("crlf.vcf", b"a\r\nb\r\n\r\nc\r\n")
    w("one_byte.txt", b"x")
    w("magic_named.txt", gzip.compress(b"hello\nworld\n", mtime=0))
    w("noeol.vcf", b"l1\nl2\r")


def _build(out, objs, incs):
    cmd = ["g++", "-std=c++17", "-O1", "-o", out, SRC] + ["-I" + i for i in incs] + objs + ["-lz"]
    subprocess.check_call(cmd)


def _run(exe, d):
    return subprocess.run([exe, d], check=True, capture_output=True, timeout=120).stdout.decode()


@pytest.fixture(scope="module")
def datadir(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("coredata"))
    _data(d)
    return d


@pytest.fixture(scope="module")
def ours(tmp_path_factory, datadir):
    lib = os.path.join(BUILD, "libvcfx_core.a")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", REPO, lib])
    exe = str(tmp_path_factory.mktemp("core") / "core_api_ours")
    _build(exe, [lib], [os.path.join(REPO, "include")])
    return _run(exe, datadir)


def test_core_api_matches_golden(ours):
    if os.environ.get("VCFX_REGEN_CORE_GOLDEN"):
        pytest.skip("regenerating")
    assert ours == open(GOLD).read()


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent (GPU box)")
def test_core_api_matches_reference_build(ours, datadir, tmp_path):
    subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "Makefile.ref"), REF_OBJ])
    exe = str(tmp_path / "core_api_ref")
    _build(exe, [REF_OBJ], [os.path.join(REF, "include")])
    ref = _run(exe, datadir)
    if os.environ.get("VCFX_REGEN_CORE_GOLDEN"):
        open(GOLD, "w").write(ref)
    assert ours == ref


def test_split_semantics_spot_checks(ours):
    # vcfx::split drops a trailing empty field; split_tabs keeps it
    assert "split, <a,> n=1 size=1: <a>" in ours
    assert "split_tabs <a\\t> n=2 size=2: <a> <>" in ours
    assert "split, <> n=0 size=0:" in ours
    assert shutil.which("g++")
