"""Host sanitizer runs (race detection; VERDICT r02 hygiene): `make sanitize` builds
the drop-ins' input layer (hostio.cpp + gz.cpp, driven by tests/host_san_test.cpp) under
AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer, and the vcfx:: core
API (tests/core_api_test.cpp + vcfx_core.cpp) under ASan + UBSan.  Each run must finish with
exit code 0, no sanitizer report, and the same bytes as the plain inputs: a > 64 MiB mapped
file (page-population threads), a shard view, BGZF members inflated on 8 threads, one and
several gzip members, a truncated stream (must fail), and a pipe (read whole; and in 4 MiB chunks
with the pre-fault, background device-open and ingest threads).  No device: the device open
fails cleanly on this host.  (The first TSan runs found a head read sized past the pipe
reader's address reservation -- EFAULT taken for end of input -- fixed in hostio.cpp.)"""
import gzip
import os
import subprocess

import numpy as np
import pytest

from vcfx_amd import BUILD, REPO, synth

from tests.test_core_api import GOLD, _data

SAN = os.path.join(BUILD, "san")


def _sum(b):
    a = np.frombuffer(b, np.uint8).astype(np.uint64)
    w = np.arange(1, a.size + 1, dtype=np.uint64)
    return int(np.sum(a * w, dtype=np.uint64))


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-j8", "-C", REPO, "sanitize"])
    return SAN


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("san"))
    one = synth.generate(4000, 1000, 5, 0, 0.002, 0, 0.05, 0)
    b = one
    while len(b) < (66 << 20):
        b += one[one.index(b"\n#CHROM") + 1:].split(b"\n", 1)[1]  # more records, no second header
    paths = {k: os.path.join(d, k) for k in ("plain.vcf", "plain.bgz", "one.gz", "multi.gz", "trunc.gz")}
    open(paths["plain.vcf"], "wb").write(b)
    subprocess.check_call([os.path.join(BUILD, "bin", "vcfx_bgzf"), paths["plain.vcf"], paths["plain.bgz"], "8", "1"])
    open(paths["one.gz"], "wb").write(gzip.compress(b[:9 << 20], mtime=0))
    open(paths["multi.gz"], "wb").write(gzip.compress(b[:3 << 20], mtime=0) + gzip.compress(b[3 << 20:5 << 20], mtime=0))
    open(paths["trunc.gz"], "wb").write(gzip.compress(b[:3 << 20], mtime=0)[:100000])
    n = len(b)
    lo, hi = n // 3, 2 * n // 3
    want = {"plain": (n, _sum(b)), "view": (4096 + hi - lo, _sum(b[:4096] + b[lo:hi])), "bgzf": (n, _sum(b)),
            "gzip": (9 << 20, _sum(b[:9 << 20])), "multi": (5 << 20, _sum(b[:5 << 20])), "pipe": (n, _sum(b)),
            "pipe_threads": (n, _sum(b))}
    return paths, want


def _env(extra):
    env = dict(os.environ, VCFX_PREFETCH_BYTES=str(1 << 40), VCFX_THREADS="8")
    env.update(extra)
    return env


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_input_layer_under_sanitizer(built, inputs, kind):
    paths, want = inputs
    env = _env({"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1",
                "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"})
    r = subprocess.run([os.path.join(built, "host_san_" + kind), paths["plain.vcf"], paths["plain.bgz"], paths["one.gz"],
                        paths["multi.gz"], paths["trunc.gz"]], capture_output=True, env=env, timeout=600)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-3000:]
    assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
    got = {}
    for line in r.stdout.decode().splitlines():
        f = line.split()
        got[f[0]] = (f[1], f[2]) if f[0] == "chain" else tuple(int(x) for x in f[1:]) if len(f) == 3 else f[1]
    assert got.pop("trunc") == "inflate-failed"
    assert got.pop("chain")[1] == "same"  # (BgzfStream: the walk, and the pieces' scans adopted)
    assert got == want


def test_core_api_under_asan_ubsan(built, tmp_path):
    d = str(tmp_path)
    _data(d)
    r = subprocess.run([os.path.join(built, "core_api_asan"), d], capture_output=True, timeout=300,
                       env=_env({"ASAN_OPTIONS": "detect_leaks=1"}))
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0, err[-3000:]
    assert "Sanitizer" not in err and "runtime error" not in err, err[-3000:]
    assert r.stdout.decode() == open(GOLD).read()


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_shard_runner_under_sanitizer(built, tmp_path, kind):
    """The in-process multi-GPU runner's host side (tool_shard_main.cpp: rank threads, the getopt
    lock, the thread-local ShardRank overrides, rank 0 writing straight to stdout and the ordered
    writer of the other ranks, the clique's reduction) with the real AF tool and input layer and
    vcfxg_* replaced by a host stand-in (tests/shard_tsan_stub.cpp): VCFX_NGPU = 2..8 ranks over
    2 stub devices, stdout a regular file and a pipe, equal to the one-context run; a rank whose
    context fails to open reports its rank and device, exits 1 and prints no partial summary."""
    p = str(tmp_path / "a.vcf")
    open(p, "wb").write(synth.generate(3000, 50, 7, 0, 0.01, 0, 0.1, 0))
    exe = os.path.join(built, "shard_" + kind)
    env = _env({"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1",
                "ASAN_OPTIONS": "detect_leaks=0", "UBSAN_OPTIONS": "print_stacktrace=1"})

    def run(ngpu, pipe=False, **extra):
        e = dict(env, VCFX_NGPU=str(ngpu), **extra)
        if pipe:
            r = subprocess.run([exe, "VCFX_allele_freq_calc", "-i", p], capture_output=True, env=e, timeout=300)
            return r.stdout, r.stderr, r.returncode
        out = str(tmp_path / ("o%d" % ngpu))
        with open(out, "wb") as fo:
            r = subprocess.run([exe, "VCFX_allele_freq_calc", "-i", p], stdout=fo, stderr=subprocess.PIPE, env=e,
                               timeout=300)
        return open(out, "rb").read(), r.stderr, r.returncode

    want = run(1)
    assert want[2] == 0 and want[1].endswith(b"Processed 3000 variants from 3000 data lines\n"), want[1][-2000:]
    for n in (2, 3, 8):
        for pipe in (False, True):
            got = run(n, pipe)
            assert b"Sanitizer" not in got[1] and b"runtime error" not in got[1], got[1][-3000:]
            assert got == want, (n, pipe, got[1][-500:])
    got = run(4, True, VCFX_STUB_DEVICES="4", VCFX_STUB_FAIL_RANK="2")
    assert b"Sanitizer" not in got[1], got[1][-3000:]
    assert got[2] == 1
    assert b"rank 2 of 4: no usable MI355X (gfx950) device 2" in got[1]
    assert b"Processed" not in got[1].split(b"\n", 1)[1]
