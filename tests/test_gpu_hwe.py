"""GPU parity of VCFX_hwe_tester beyond the 173 golden cases
(tests/test_gpu_cli.py): seeded synthetic VCFs -- fixed-stride records on the walk, irregular
and missing genotypes, multi-allelic sites, CRLF, tiny and large sample counts -- in both
input modes against the C oracle; the walk against the two-sweep schedule; and the host
recheck path (every exp()-derived p-value sent to the host) through the engine and the
drop-in binary."""
import os
import subprocess

import pytest

from tests._golden import Oracle, REPO
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (1500, 2504, 71, 0, 0.0, 0, 0.0, 0),
    (800, 997, 72, 1, 0.01, 0, 0.2, 1),
    (3000, 3, 73, 1, 0.05, 0, 0.3, 0),
    (200, 5000, 74, 0, 0.0, 40, 0.1, 0),
    (2000, 64, 75, 0, 0.002, 0, 0.0, 1),
]
BIN = os.path.join(REPO, "build", "src", "VCFX_hwe_tester", "VCFX_hwe_tester")


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_hwe_tool_matches_oracle(oracle, cfg, tmp_path):
    buf = synth.generate(*cfg)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    for argv, stdin in ((["VCFX_hwe_tester", "-i", str(path)], b""), (["VCFX_hwe_tester"], buf),
                        (["VCFX_hwe_tester", "-q", str(path)], b"")):
        want = oracle.run(argv, stdin)
        got = tools.run(argv, stdin)
        assert got == want, (argv[1:2], len(got[0]), len(want[0]))


def _engine_text(buf, mode, env=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        eng = engine.Engine(0)  # the context reads the VCFXG_* knobs when it opens
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    eng.load(buf)
    ds = 0
    while ds < len(buf) and buf[ds:ds + 1] == b"#":
        ds = buf.index(b"\n", ds) + 1
    s = eng.hwe_region(ds, mode)
    text = eng.text(s.text_bytes)
    rc = eng.hwe_rechecks()
    eng.close()
    return s, text, rc


@pytest.mark.parametrize("mode", [engine.MODE_FILE, engine.MODE_STDIN])
def test_hwe_walk_vs_two_sweep(oracle, mode):
    """walk (several chunk sizes) and the index + per-line schedule give the same rows"""
    buf = synth.generate(2500, 2504, 76, 0, 0.001, 0, 0.05, 0)
    s0, t0, _ = _engine_text(buf, mode, {"VCFXG_AF_FUSED": "8"})
    assert s0.rows > 2000
    for chunk in ("131072", "20000", "4096"):
        s, t, _ = _engine_text(buf, mode, {"VCFXG_AF_FUSED": "7", "VCFXG_WALK_CHUNK": chunk})
        assert (s.rows, s.n_lines, s.general_records) == (s0.rows, s0.n_lines, s0.general_records), chunk
        assert t == t0, chunk
    if mode == engine.MODE_STDIN:
        want = oracle.run(["VCFX_hwe_tester"], buf)[0]
        assert b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n" + t0 == want


@pytest.mark.parametrize("mode", [engine.MODE_FILE, engine.MODE_STDIN])
def test_hwe_recheck_path(oracle, mode, tmp_path):
    """a huge ulp margin lists every exp()-derived row for the host; the rows patched with the
    host libm's p-value (the oracle's restatement here) equal the reference output"""
    import ctypes
    buf = synth.generate(1200, 301, 77, 0, 0.01, 0, 0.1, 0)
    s, text, rc = _engine_text(buf, mode, {"VCFXG_HWE_ULPS": str(1 << 50)})
    assert len(rc) > 200  # the rows whose p-value went through exp()
    lib = oracle.lib
    lib.oracle_hwe_pvalue.restype = ctypes.c_double
    lib.oracle_hwe_pvalue.argtypes = [ctypes.c_int] * 3
    lib.oracle_hwe_fmt_mmap.restype = ctypes.c_size_t
    lib.oracle_hwe_fmt_mmap.argtypes = [ctypes.c_double, ctypes.c_char_p]
    t = bytearray(text)
    seen = set()
    for off, a, b, c in rc:
        assert off not in seen and t[off + 8:off + 9] == b"\n" and t[off - 1:off] == b"\t"
        seen.add(off)
        v = lib.oracle_hwe_pvalue(a, b, c)
        if mode == engine.MODE_FILE:
            dig = ctypes.create_string_buffer(40)
            n = lib.oracle_hwe_fmt_mmap(v, dig)
            d = dig.raw[:n]
        else:
            d = b"%.6f" % v
        assert len(d) == 8
        t[off:off + 8] = d
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    argv = ["VCFX_hwe_tester", "-q", str(path)] if mode == engine.MODE_FILE else ["VCFX_hwe_tester"]
    want = oracle.run(argv, b"" if mode == engine.MODE_FILE else buf)[0]
    assert b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n" + bytes(t) == want
    # the drop-in binary's own patching (fresh process: the knob applies to its context)
    env = dict(os.environ, VCFXG_HWE_ULPS=str(1 << 50))
    if mode == engine.MODE_FILE:
        got = subprocess.run([BIN, "-q", str(path)], capture_output=True, env=env, timeout=120)
    else:
        got = subprocess.run([BIN], input=buf, capture_output=True, env=env, timeout=120)
    assert got.returncode == 0 and got.stdout == want


@pytest.mark.parametrize("cfg", [dict(n_records=900, n_samples=2504, seed=78, missing_rate=0.002, format_mode=1),
                                 dict(n_records=600, n_samples=97, seed=79, irregular_rate=0.3, crlf=1,
                                      format_mode=1)])
def test_hwe_gt_ad_dp_matches_oracle(oracle, cfg, tmp_path):
    """FORMAT=GT:AD:DP records (the per-line path) in both modes"""
    buf = synth.generate(**cfg)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    for argv, stdin in ((["VCFX_hwe_tester", "-i", str(path)], b""), (["VCFX_hwe_tester"], buf)):
        assert tools.run(argv, stdin) == oracle.run(argv, stdin), argv[1:2]
