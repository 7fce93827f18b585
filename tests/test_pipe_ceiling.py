"""build/bin/vcfx_pipe_ceiling -- the e2e leg's stdin-pipe ceiling (bench.py): the drop-in's own
reader (Input::read_fd with host_copy = false) with the device stage stubbed
(tests/shard_tsan_stub.cpp, -DVCFX_STUB_DISCARD).  It must read a pipe to its end and exit 0 on
inputs that take each branch of the reader: all on the host (short), a head then the pinned ring
(small VCFX_STREAM_CHUNK / VCFX_PREFETCH_BYTES), no '#CHROM' line, and an empty pipe."""
import os
import subprocess

import pytest

from vcfx_amd import synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "bin", "vcfx_pipe_ceiling")


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", REPO, "build/bin/vcfx_pipe_ceiling"])
    return EXE


@pytest.mark.parametrize("case", ["short", "ring", "no_chrom", "empty"])
def test_pipe_ceiling_reads_to_the_end(built, case):
    env = dict(os.environ)
    if case == "short":
        data = synth.generate(50, 20, 3, 0, 0.0, 1, 0.0, 0)
    elif case == "ring":
        data = synth.generate(3000, 300, 4, 0, 0.0, 1, 0.0, 0)
        env.update(VCFX_STREAM_CHUNK="65536", VCFX_PREFETCH_BYTES="4096")
    elif case == "no_chrom":
        data = b"".join(b"21\t%d\t.\tA\tG\t.\tPASS\t.\tGT\t0|1\n" % k for k in range(200000))
        env.update(VCFX_STREAM_CHUNK="65536", VCFX_PREFETCH_BYTES="4096")
    else:
        data = b""
    assert len(data) > 1 << 20 or case in ("short", "empty")
    r = subprocess.run([built], input=data, capture_output=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-500:]
