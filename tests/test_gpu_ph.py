"""GPU parity of VCFX_haplotype_phaser (LD reuse in block phasing) beyond
the golden cases: seeded synthetic VCFs with founder-haplotype blocks (so thresholds give long
and short blocks), missing calls, irregular GT shapes and GT:AD:DP records, in the default and
streaming modes (windows 0, 1, 3, 1000) and both input forms, against the C oracle; and the
device's per-pair r^2 against the oracle's calculateLDFast restatement."""
import numpy as np
import pytest

from tests._golden import Oracle
from vcfx_amd import engine, synth, tools

pytestmark = pytest.mark.gpu

SYNTH = [
    dict(n_records=1500, n_samples=2504, seed=111, hap_blocks=1),
    dict(n_records=800, n_samples=997, seed=112, hap_blocks=1, missing_rate=0.01, irregular_rate=0.2, crlf=1),
    dict(n_records=3000, n_samples=7, seed=113, hap_blocks=1, missing_rate=0.05, irregular_rate=0.3),
    dict(n_records=500, n_samples=301, seed=114, hap_blocks=1, format_mode=1, missing_rate=0.002),
]


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


@pytest.mark.parametrize("cfg", SYNTH)
def test_phaser_matches_oracle(oracle, cfg, tmp_path):
    buf = synth.generate(**cfg)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    T = "VCFX_haplotype_phaser"
    for args in ([], ["-l", "0.5"], ["-l", "0.2"], ["-s"], ["-s", "-w", "3", "-l", "0.3"], ["-s", "-w", "0"],
                 ["-q", "-s", "-w", "1", "-l", "0.1"]):
        for argv, stdin in (([T] + args + ["-i", str(path)], b""), ([T] + args, buf)):
            want = oracle.run(argv, stdin)
            got = tools.run(argv, stdin)
            assert got[2] == want[2] and got[1] == want[1], (argv[1:], got[1][-300:], want[1][-300:])
            assert got[0] == want[0], (argv[1:], len(got[0]), len(want[0]))


def test_phaser_pair_r2_matches_oracle(oracle):
    import ctypes
    buf = synth.generate(600, 2504, 115, 0, 0.001, 1, 0.0, 0)
    ds = engine.data_start_of(buf)
    eng = engine.Engine(0)
    eng.load(buf)
    s = eng.haplotype_phaser(ds, engine.MODE_FILE, 0.5, 2504)
    assert s.rows == 600
    flags, r2, _ = eng.phaser_variants(s.rows)
    eng.close()
    # the oracle's calculateLDFast on the same genotype codes (GT-only fixed-stride records)
    lines = [l for l in buf.split(b"\n") if l and not l.startswith(b"#")]

    def codes(line):
        out = []
        for g in line.split(b"\t")[9:]:
            out.append(-1 if b"." in g else int(g[0:1]) + int(g[2:3]))
        return np.array(out, np.int8)

    lib = oracle.lib
    lib.oracle_ph_ld.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_double)]
    prev = codes(lines[0])
    for v in range(1, len(lines)):
        cur = codes(lines[v])
        r, rr = ctypes.c_double(), ctypes.c_double()
        lib.oracle_ph_ld(prev.ctypes.data, cur.ctypes.data, len(cur), ctypes.byref(r), ctypes.byref(rr))
        assert r2[v] == rr.value, (v, r2[v], rr.value)
        assert bool(flags[v] & 1) == (rr.value >= 0.5)
        prev = cur


def _mutate(buf, rec, sample, new):
    lines = buf.split(b"\n")
    k = next(i for i, l in enumerate(lines) if l.startswith(b"#CHROM")) + 1 + rec
    f = lines[k].split(b"\t")
    f[9 + sample] = new
    lines[k] = b"\t".join(f)
    return b"\n".join(lines)


# the phaser's line index from the dosage HEAD walk: records taken on their predicted '\n' alone
# must be validated by k_ph_lines' fixed-stride sweep; each way such a record can differ (a
# missing allele -- valid for the sweep --, a non-digit allele, another separator, a wider
# sample, a '\n' inside a record of the predicted length, a non-digit POS) against the oracle
PH_MUTATIONS = [None, (7, 100, b".|0"), (11, 0, b"x|1"), (12, 5, b"1/0"), (13, 9, b"11|"), (14, 1000, b"0\n0"),
                (300, 2503, b"0|\n")]


@pytest.mark.parametrize("mut", PH_MUTATIONS)
def test_phaser_head_walk_index(oracle, mut, tmp_path):
    import os
    buf = synth.generate(600, 2504, 116, 0, 0.0, 1, 0.0, 0)
    if mut:
        buf = _mutate(buf, *mut)
    path = tmp_path / "in.vcf"
    path.write_bytes(buf)
    T = "VCFX_haplotype_phaser"
    log = str(tmp_path / "sched.log")
    os.environ["VCFXG_SCHEDULE_LOG"] = log
    try:
        for args in (["-l", "0.5"], ["-s", "-w", "3", "-l", "0.3"]):
            for argv, stdin in (([T] + args + ["-i", str(path)], b""), ([T] + args, buf)):
                want = oracle.run(argv, stdin)
                got = tools.run(argv, stdin)
                assert got == want, (mut, argv[1:], got[1][-300:], want[1][-300:])
    finally:
        del os.environ["VCFXG_SCHEDULE_LOG"]
    sched = open(log).read().split()
    assert sched and sched[0] == "ph_head_walk", sched
    if mut is None:
        assert set(sched) == {"ph_head_walk"}, sched
