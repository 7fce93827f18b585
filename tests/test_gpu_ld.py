"""GPU parity for VCFX_ld_calculator: MFMA pair sums (block-scaled FP4: X.X^T for complete
256-variant groups, the six masked sums for 128-variant tiles with missing calls) + the exact
fp64 epilogue against the C oracle's computeRsqFast / computeRsq, streaming and matrix modes,
both input paths."""
import os
import tempfile

import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu
REF_LD_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                         "libref_ld_rsq.so")


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_mfma_i8_layout():
    e = engine.Engine(0)
    assert e.selftest_mfma_i8() == 0
    assert e.selftest_mfma_fp4() == 0
    e.close()


SYNTH = [
    # records, samples, seed, info, missing, hap, irregular, crlf
    (300, 200, 51, 0, 0.0, 1, 0.0, 0),
    (260, 131, 52, 0, 0.05, 1, 0.0, 0),
    (200, 77, 53, 1, 0.02, 1, 0.3, 0),
    (150, 2504, 54, 0, 0.0, 1, 0.0, 0),
    (130, 33, 55, 0, 0.1, 0, 0.5, 1),
]
ARGS = [["-w", "1000"], ["-w", "1"], ["-w", "7", "-t", "0.3"], ["-w", "100", "-t", "0.8"], ["-d", "300"],
        ["-w", "64", "-d", "2000", "-t", "0.1"], ["-r", "21:9411239-9430000"], ["-w", "65"], ["-w", "129"]]


@pytest.mark.parametrize("cfg", SYNTH)
def test_ld_stream_matches_oracle(oracle, cfg):
    buf = synth.generate(*cfg)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in ARGS:
            for argv, stdin in ((["VCFX_ld_calculator"] + a + ["-i", f.name], b""), (["VCFX_ld_calculator"] + a, buf)):
                got = tools.run(argv, stdin)
                want = oracle.run(argv, stdin)
                assert got == want, (a, cfg, len(got[0]), len(want[0]))


@pytest.mark.parametrize("cfg", SYNTH[:3] + [(90, 40, 56, 0, 0.2, 1, 0.4, 0)])
def test_ld_matrix_matches_oracle(oracle, cfg):
    buf = synth.generate(*cfg)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-m"], ["-m", "-r", "21:9411239-9420000"]):
            for argv, stdin in ((["VCFX_ld_calculator"] + a + ["-i", f.name], b""), (["VCFX_ld_calculator"] + a, buf)):
                got = tools.run(argv, stdin)
                want = oracle.run(argv, stdin)
                assert got == want, (a, cfg)


def _codes(buf, oracle):
    """int8 genotype codes per data line (parseGenotypeRaw on the GT prefix, -1 missing)."""
    import ctypes

    import numpy as np
    f = oracle.lib.oracle_ld_parse_gt_raw
    f.argtypes, f.restype = [ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int
    rows = []
    for ln in buf.split(b"\n"):
        if not ln or ln[:1] == b"#":
            continue
        gts = [s.split(b":", 1)[0] for s in ln.split(b"\t")[9:]]
        rows.append(np.array([f(g, len(g)) if g else -1 for g in gts], np.int8))
    return rows


@pytest.mark.parametrize("cfg,knock", [((200, 300, 57, 0, 0.03, 1, 0.0, 0), None),   # masked tiles only
                                       ((700, 2504, 64, 0, 0.001, 1, 0.0, 0), None),  # sparse-missing tiles (kSp)
                                       ((600, 300, 63, 0, 0.0, 1, 0.0, 0), None),    # complete: FP4 fast blocks
                                       ((600, 300, 63, 0, 0.0, 1, 0.0, 0), 300)])    # fast + masked mix
def test_ld_r2_values_bitexact(oracle, cfg, knock):
    """Every window pair's fp64 r^2 on the device (vcfxg_ld_fetch_pairs: the value each output line
    was formatted from) equals the oracle's computeRsqFast on the same two genotype vectors, bit
    for bit -- north_star's "r^2 within 1e-6" pinned at 0 ulp, not only through the 4-dp text."""
    import ctypes

    import numpy as np
    buf = synth.generate(*cfg)
    if knock is not None:
        buf = _knock_out(buf, knock)
    g = _codes(buf, oracle)
    m, ns = len(g), cfg[1]
    e = engine.Engine(0)
    try:
        e.load(buf)
        e.index(engine.data_start_of(buf, strip_cr=False))
        assert e.ld_prepare(ns) == m
        # threshold 0: every window pair is written (r^2 >= 0 always), in (j, i ascending) order
        np_, _ = e.ld_stream_chunk(0, m, m, 0.0)
        assert np_ == m * (m - 1) // 2
        vi, vj, r2 = e.ld_pairs(0, np_)
    finally:
        e.close()
    want_i = np.concatenate([np.arange(j, dtype=np.uint32) for j in range(1, m)])
    want_j = np.concatenate([np.full(j, j, np.uint32) for j in range(1, m)])
    assert (vi == want_i).all() and (vj == want_j).all()
    ptr = [x.ctypes.data_as(ctypes.c_void_p) for x in g]
    # first the reference's own computeRsqFast (its source compiled into oracle/_ref by
    # oracle/Makefile.ref, shipped with the tree), then the oracle's restatement of it
    # (the shim is part of the tree's build, __graft_entry__.build(): a missing one is a failure,
    # not a quieter test)
    assert os.path.exists(REF_LD_SO), "%s missing: build it (oracle/Makefile.ref via __graft_entry__.build())" % REF_LD_SO
    ref = ctypes.CDLL(REF_LD_SO).ref_rsq_fast
    ref.argtypes, ref.restype = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_double
    checkers = [("reference", ref), ("oracle", oracle.lib.oracle_ld_rsq_fast)]
    for name, rs in checkers:
        want = np.array([rs(ptr[i], ptr[j], ns) for i, j in zip(want_i.tolist(), want_j.tolist())], np.float64)
        bad = np.flatnonzero(r2.view(np.uint64) != want.view(np.uint64))
        assert bad.size == 0, (name, [(int(want_i[k]), int(want_j[k]), r2[k], want[k]) for k in bad[:5]])
        assert (want > 0.0).sum() > np_ // 4  # the values are not all the gate's 0.0


def _knock_out(buf, line_no):
    """Make one genotype of data line `line_no` missing (its 256-group leaves the fast kernel)."""
    lines = buf.split(b"\n")
    data = [k for k, ln in enumerate(lines) if ln and not ln.startswith(b"#")]
    k = data[line_no]
    f = lines[k].split(b"\t")
    f[9] = b".|."
    lines[k] = b"\t".join(f)
    return b"\n".join(lines)


@pytest.mark.parametrize("knock", [None, 600])
def test_ld_fast_blocks_across_groups(oracle, knock):
    """Several 256-variant fast blocks (and, with a knocked-out genotype, a mix of fast and
    general blocks): window edges inside and across blocks, thresholds that exercise the
    fp32 candidate prefilter, threshold 0 (every pair a candidate) and the distance cap."""
    buf = synth.generate(1100, 203, 58, 0, 0.0, 1, 0.0, 0)
    if knock is not None:
        buf = _knock_out(buf, knock)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-w", "1100", "-t", "0.5"], ["-w", "300", "-t", "0.2"], ["-w", "257", "-t", "0.9"],
                  ["-w", "511", "-t", "0.0"], ["-w", "700", "-t", "0.35", "-d", "5000"]):
            argv = ["VCFX_ld_calculator"] + a + ["-i", f.name]
            got = tools.run(argv, b"")
            want = oracle.run(argv, b"")
            assert got == want, (a, knock, len(got[0]), len(want[0]))


def test_ld_staging_overflow_falls_back(oracle):
    """A staging area too small for the count pass's pairs: the emit pass recomputes them
    (same bytes); and a roomy one: the scatter path."""
    import os
    buf = synth.generate(700, 150, 59, 0, 0.0, 1, 0.0, 0)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        argv = ["VCFX_ld_calculator", "-w", "700", "-t", "0.2", "-i", f.name]
        want = oracle.run(argv, b"")
        for cap in ("7", "100000000"):
            os.environ["VCFXG_LD_STAGE_CAP"] = cap
            try:
                got = tools.run(argv, b"")
            finally:
                del os.environ["VCFXG_LD_STAGE_CAP"]
            assert got == want, cap


def test_ld_pair_lines_long_and_short_fields(oracle):
    """The pair-line writer composes 64 lines per wave in an 8 KiB LDS tile and writes it as
    aligned 16 B stores; waves whose lines outgrow the tile write each line straight out.
    IDs of 1..400 bytes (some records long enough to force the straight path, the rest short)
    at threshold 0: every window pair's line, tile edges at every alignment."""
    import random
    buf = synth.generate(300, 60, 61, 0, 0.0, 1, 0.0, 0)
    rnd = random.Random(61)
    lines = buf.split(b"\n")
    for k, ln in enumerate(lines):
        if ln and not ln.startswith(b"#"):
            f = ln.split(b"\t")
            n = rnd.choice([1, 2, 7, 15, 16, 17, 33]) if rnd.random() < 0.8 else rnd.randint(100, 400)
            f[2] = (b"rs%d_" % k + b"x" * n)
            lines[k] = b"\t".join(f)
    buf = b"\n".join(lines)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-w", "300", "-t", "0.0"], ["-w", "40", "-t", "0.1"]):
            argv = ["VCFX_ld_calculator"] + a + ["-i", f.name]
            got = tools.run(argv, b"")
            want = oracle.run(argv, b"")
            assert got == want, (a, len(got[0]), len(want[0]))


@pytest.mark.parametrize("rate", [0.001, 0.08])
def test_ld_mask_tiles_missing_calls(oracle, rate):
    """Missing calls in most variants (per-sample rate 0.1 %: ~8 % of the 2,504-sample variants
    complete; 8 %: none): the 128 x 128 masked FP4 tiles (n, Sx, Sy, Sxx, Syy, Sxy per pair)
    next to complete 256-groups, window edges inside and across tiles, thresholds that exercise
    the fp32 prefilter, threshold 0 (every window pair a candidate) and the distance cap; the
    same bytes through the previous int8 general kernel (VCFXG_LD_MASK=0, a fresh process)."""
    import os
    import subprocess
    buf = synth.generate(1100, 2504 if rate < 0.01 else 517, 62, 0, rate, 1, 0.0, 0)
    if rate < 0.01:  # two complete 256-groups among the incomplete ones
        lines = buf.split(b"\n")
        data = [k for k, ln in enumerate(lines) if ln and not ln.startswith(b"#")]
        for k in data[256:768]:
            f = lines[k].split(b"\t")
            f[9:] = [b"0|0" if x[:1] == b"." or x[2:3] == b"." else x for x in f[9:]]
            lines[k] = b"\t".join(f)
        buf = b"\n".join(lines)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-w", "1100", "-t", "0.5"], ["-w", "300", "-t", "0.2"], ["-w", "129", "-t", "0.0"],
                  ["-w", "700", "-t", "0.35", "-d", "5000"], ["-w", "64", "-t", "0.05"]):
            argv = ["VCFX_ld_calculator"] + a + ["-i", f.name]
            got = tools.run(argv, b"")
            want = oracle.run(argv, b"")
            assert got == want, (a, rate, len(got[0]), len(want[0]))
        argv = ["VCFX_ld_calculator", "-w", "1100", "-t", "0.3", "-i", f.name]
        old = subprocess.run([tools_binary("VCFX_ld_calculator")] + argv[1:], capture_output=True,
                             env=dict(os.environ, VCFXG_LD_MASK="0"), timeout=300)
        assert (old.stdout, old.returncode) == (oracle.run(argv, b"")[0], 0)


def tools_binary(t):
    from vcfx_amd import tool_binary
    return tool_binary(t)


@pytest.mark.parametrize("rate,ns", [(0.001, 2504), (0.004, 1000), (0.0005, 4100)])
def test_ld_sparse_missing_tiles(oracle, rate, ns):
    """The sparse-missing form of the 256 x 256 FP4 kernel (every variant of both groups misses
    <= 15 calls): X.X^T from the MFMA, the other five sums of computeRsqSIMD corrected at the
    missing samples (LDS contribution tables), the k_ld_mask prefilter and fp64 sequence.
    Against the oracle over windows / thresholds / distance caps (threshold 0: every pair a
    candidate), the count pass's staging both roomy and overflowing (the emit pass recomputes),
    and against the dense masked kernel (VCFXG_LD_SPARSE=0, a fresh process)."""
    import os
    import subprocess
    buf = synth.generate(1100, ns, 66, 0, rate, 1, 0.0, 0)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-w", "1100", "-t", "0.5"], ["-w", "300", "-t", "0.2"], ["-w", "129", "-t", "0.0"],
                  ["-w", "700", "-t", "0.35", "-d", "5000"], ["-w", "64", "-t", "0.05"]):
            argv = ["VCFX_ld_calculator"] + a + ["-i", f.name]
            want = oracle.run(argv, b"")
            got = tools.run(argv, b"")
            assert got == want, (a, rate, len(got[0]), len(want[0]))
        argv = ["VCFX_ld_calculator", "-w", "1100", "-t", "0.3", "-i", f.name]
        want = oracle.run(argv, b"")
        os.environ["VCFXG_LD_STAGE_CAP"] = "7"
        try:
            assert tools.run(argv, b"") == want
        finally:
            del os.environ["VCFXG_LD_STAGE_CAP"]
        old = subprocess.run([tools_binary("VCFX_ld_calculator")] + argv[1:], capture_output=True,
                             env=dict(os.environ, VCFXG_LD_SPARSE="0"), timeout=300)
        assert (old.stdout, old.returncode) == (want[0], 0)
        # the sparse planes' allocation failing (test hook): the sparse groups go back to the
        # masked kernel and the call still succeeds with the same bytes
        nomem = subprocess.run([tools_binary("VCFX_ld_calculator")] + argv[1:], capture_output=True,
                               env=dict(os.environ, VCFXG_LD_SPARSE_NOMEM="1"), timeout=300)
        assert (nomem.stdout, nomem.returncode) == (want[0], 0)


def _wide_sparse_vcf(m, ns, seed):
    """m variants x ns samples, dosage 2 (1|1) on ~95 % of the calls (Sxy close to the u16 limit
    4 ns of the sparse epilogue's packed accumulators at ns = 16383), and exactly 15 missing calls
    per variant (the most a sparse group allows): on odd variants the first 15 samples where the
    previous variant's dosage is not 2 (the other variant's informative samples missing), on even
    ones random samples.  Rows share one carrier pattern, so many pairs sit near every threshold."""
    import numpy as np
    rng = np.random.default_rng(seed)
    head = (b"##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" +
            b"\t".join(b"S%d" % i for i in range(ns)) + b"\n")
    codes = np.frombuffer(b"0|0\t0|1\t1|1\t.|.\t", dtype="<u4")
    base = rng.random(ns) < 0.05
    prev = None
    out = [head]
    for v in range(m):
        d = np.full(ns, 2, np.int64)
        alt = np.where(rng.random(ns) < 0.9, base, rng.random(ns) < 0.05)
        d[alt] = rng.integers(0, 2, int(alt.sum()))
        if v % 2 and prev is not None:
            miss = np.flatnonzero(prev != 2)[:15]
            if miss.size < 15:
                miss = np.concatenate([miss, np.setdiff1d(np.arange(ns), miss)[:15 - miss.size]])
        else:
            miss = rng.choice(ns, 15, replace=False)
        d[miss] = 3
        prev = np.where(d == 3, 2, d)
        row = bytearray(codes[d].tobytes())
        row[-1:] = b"\n"
        out.append(b"1\t%d\trs%d\tA\tG\t.\tPASS\t.\tGT\t" % (1000 + v, v) + bytes(row))
    return b"".join(out)


def test_ld_sparse_at_the_sample_limit(oracle):
    """the sparse epilogue's fp32 prefilter and its u16 packed sums where they are
    tightest -- ns = 16,383 (the largest the sparse groups take), 15 missing calls per variant,
    adversarial patterns (a variant missing the other's informative samples) and Sxy near 2^16 --
    against the oracle, with the reference's own r^2 doubles on every pair at threshold 0."""
    import ctypes

    import numpy as np
    ns, m = 16383, 512
    buf = _wide_sparse_vcf(m, ns, 71)
    with tempfile.NamedTemporaryFile(suffix=".vcf") as f:
        f.write(buf)
        f.flush()
        for a in (["-w", "512", "-t", "0.5"], ["-w", "512", "-t", "0.55"], ["-w", "512", "-t", "0.57"],
                  ["-w", "300", "-t", "0.2"]):
            argv = ["VCFX_ld_calculator"] + a + ["-i", f.name]
            got = tools.run(argv, b"")
            want = oracle.run(argv, b"")
            assert got == want, (a, len(got[0]), len(want[0]))
            assert want[0].count(b"\n") > 300, a  # pairs pass: the prefilter decided real cases
    g = _codes(buf, oracle)
    e = engine.Engine(0)
    try:
        e.load(buf)
        e.index(engine.data_start_of(buf, strip_cr=False))
        assert e.ld_prepare(ns) == m
        np_, _ = e.ld_stream_chunk(0, m, m, 0.0)
        vi, vj, r2 = e.ld_pairs(0, np_)
    finally:
        e.close()
    rs = oracle.lib.oracle_ld_rsq_fast
    if os.path.exists(REF_LD_SO):
        rs = ctypes.CDLL(REF_LD_SO).ref_rsq_fast
        rs.argtypes, rs.restype = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_double
    ptr = [x.ctypes.data_as(ctypes.c_void_p) for x in g]
    want = np.array([rs(ptr[i], ptr[j], ns) for i, j in zip(vi.tolist(), vj.tolist())], np.float64)
    assert np_ == m * (m - 1) // 2
    assert (r2.view(np.uint64) == want.view(np.uint64)).all()
