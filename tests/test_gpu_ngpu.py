"""The in-process multi-GPU drop-in (vcfx_tool_main_sharded, tool_shard_main.cpp; VCFX_NGPU=N
VCFX_<tool> ...) on one MI355X: N rank contexts on device 0 (round robin), each running the
tool on its record range of the file.  stdout, stderr and the exit code must equal the
single-context run byte for byte, for N = 2, 3 and 8 -- including the ranks' count all-reduce
(AF totals, missing_detector's summary), header rows written once, per-line warnings in file
order, and LD's pair rows split by equal pair counts.  The executables are run too (VCFX_NGPU in
the environment), stdout to a regular file (parallel pwrite at offsets) and to a pipe."""
import os
import subprocess
import tempfile

import pytest

from vcfx_amd import synth, tool_binary, tools

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def files():
    d = tempfile.mkdtemp(prefix="vcfx_ngpu_")
    out = {}
    # records, samples, seed, info, missing, hap, irregular, crlf
    for name, cfg in (("gt", (2500, 120, 81, 1, 0.0, 0, 0.0, 0)),
                      ("mixed", (1800, 77, 82, 1, 0.01, 0, 0.25, 0)),
                      ("crlf", (700, 31, 83, 0, 0.02, 0, 0.2, 1)),
                      ("ld", (400, 200, 84, 0, 0.001, 1, 0.0, 0))):
        p = os.path.join(d, name + ".vcf")
        open(p, "wb").write(synth.generate(*cfg))
        out[name] = p
    yield out
    for p in out.values():
        os.unlink(p)
    os.rmdir(d)


CASES = [
    ["VCFX_allele_freq_calc", "-i", "{gt}"], ["VCFX_allele_freq_calc", "{mixed}"],
    ["VCFX_allele_freq_calc", "-q", "-i", "{crlf}"],
    ["VCFX_record_filter", "--filter", "QUAL>=30;AF>=0.05", "-i", "{mixed}"],
    ["VCFX_record_filter", "--filter", "FILTER==PASS", "--logic", "or", "-i", "{crlf}"],
    ["VCFX_genotype_query", "-g", "0/1", "-i", "{mixed}"], ["VCFX_genotype_query", "-g", "1|1", "--strict", "{gt}"],
    ["VCFX_nonref_filter", "-i", "{mixed}"], ["VCFX_nonref_filter", "{crlf}"],
    ["VCFX_dosage_calculator", "-i", "{mixed}"], ["VCFX_dosage_calculator", "-q", "-i", "{gt}"],
    ["VCFX_hwe_tester", "-i", "{mixed}"], ["VCFX_hwe_tester", "-q", "-i", "{crlf}"],
    ["VCFX_missing_detector", "-i", "{mixed}"], ["VCFX_missing_detector", "-i", "{gt}"],
    ["VCFX_missing_detector", "-q", "-i", "{crlf}"],
    ["VCFX_allele_counter", "-i", "{gt}"], ["VCFX_allele_counter", "-a", "-i", "{mixed}"],
    ["VCFX_allele_counter", "-b", "-i", "{gt}"], ["VCFX_allele_counter", "-s", "S00003 S00001", "-i", "{mixed}"],
    ["VCFX_ld_calculator", "-w", "60", "-t", "0.2", "-i", "{ld}"],
    ["VCFX_ld_calculator", "-w", "400", "-t", "0.5", "-q", "-i", "{ld}"],
]


def _argv(case, files):
    return [a.format(**files) for a in case]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "_".join(x.strip("{}-") for x in c)[:60])
def test_sharded_equals_single_context(files, case):
    argv = _argv(case, files)
    want = tools.run(argv)
    assert want[2] == 0, want[1][-500:]
    for n in ((2, 3, 8) if case[0] in ("VCFX_allele_freq_calc", "VCFX_missing_detector") else (3,)):
        got = tools.run(argv, ngpu=n)
        assert got == want, (argv, n, len(got[0]), len(want[0]), got[1][-300:], want[1][-300:])


@pytest.mark.parametrize("case", [CASES[0], CASES[3], CASES[13], CASES[16]],
                         ids=["af", "rf", "md", "ac"])
def test_executable_with_vcfx_ngpu(files, case):
    argv = _argv(case, files)
    exe = tool_binary(argv[0])
    want = subprocess.run([exe] + argv[1:], capture_output=True, timeout=120)
    with tempfile.TemporaryFile() as fo:  # a regular file: the ranks' bytes written at their offsets
        r = subprocess.run([exe] + argv[1:], stdout=fo, stderr=subprocess.PIPE, timeout=120,
                           env=dict(os.environ, VCFX_NGPU="4"))
        fo.seek(0)
        assert (fo.read(), r.stderr, r.returncode) == (want.stdout, want.stderr, want.returncode)
    r = subprocess.run([exe] + argv[1:], capture_output=True, timeout=120, env=dict(os.environ, VCFX_NGPU="3"))
    assert (r.stdout, r.stderr, r.returncode) == (want.stdout, want.stderr, want.returncode)


def test_rccl_one_rank_clique():
    """The RCCL branch of the rank clique on one GPU (VCFX_RCCL=1 forms a one-rank clique):
    librccl's ncclCommInitAll, ncclAllReduce on the rank's stream with the ncclUint64 / ncclSum
    values of rccl.h, the read-back checked against the host reduction, ncclCommDestroy."""
    import ctypes

    from vcfx_amd import engine
    e = engine.Engine(0)
    L = e.L
    os.environ["VCFX_RCCL"] = "1"
    comm = ctypes.c_void_p()
    try:
        arr = (ctypes.c_void_p * 1)(e.h)
        assert L.vcfxg_comm_init(arr, 1, ctypes.byref(comm)) == 0, L.vcfxg_last_error(e.h)
        assert L.vcfxg_comm_uses_rccl(comm) == 1
        for k in range(3):
            vals = (ctypes.c_uint64 * 8)(*[(0x0123456789ABCDEF * (i + 1 + k)) & (2 ** 64 - 1) for i in range(8)])
            want = list(vals)
            assert L.vcfxg_comm_allreduce_u64(comm, 0, vals, 8) == 0, L.vcfxg_last_error(e.h)
            assert list(vals) == want
        calls, bad = ctypes.c_uint64(), ctypes.c_uint64()
        assert L.vcfxg_comm_rccl_stats(comm, ctypes.byref(calls), ctypes.byref(bad)) == 0
        assert (calls.value, bad.value) == (3, 0)
    finally:
        del os.environ["VCFX_RCCL"]
        if comm.value:
            L.vcfxg_comm_destroy(comm)
        e.close()


def test_host_clique_sums_threads():
    """The host reduction (ranks sharing a device): 8 rank threads, three rounds, sums of all."""
    import ctypes
    import threading

    from vcfx_amd import engine
    es = [engine.Engine(0) for _ in range(8)]
    L = es[0].L
    comm = ctypes.c_void_p()
    try:
        arr = (ctypes.c_void_p * 8)(*[e.h for e in es])
        assert L.vcfxg_comm_init(arr, 8, ctypes.byref(comm)) == 0
        assert L.vcfxg_comm_uses_rccl(comm) == 0
        got = [None] * 8

        def rank(r):
            out = []
            for k in range(3):
                v = (ctypes.c_uint64 * 4)(*[r + 10 * k + i for i in range(4)])
                assert L.vcfxg_comm_allreduce_u64(comm, r, v, 4) == 0
                out.append(list(v))
            got[r] = out

        th = [threading.Thread(target=rank, args=(r,)) for r in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        want = [[sum(r + 10 * k + i for r in range(8)) for i in range(4)] for k in range(3)]
        assert all(g == want for g in got)
    finally:
        if comm.value:
            L.vcfxg_comm_destroy(comm)
        for e in es:
            e.close()


@pytest.mark.parametrize("tool,args", [("VCFX_allele_freq_calc", ["-q"]),
                                       ("VCFX_record_filter", ["--filter", "QUAL>=30"])])
def test_sharded_ranks_take_the_walk(tool, args):
    """Each rank's view is the header bytes [0, H) then its records: the load-time hints come
    from the first ingested chunk that holds data lines, so every rank of a GT-only input of
    >= 512 B records takes the walk schedule (VCFXG_SCHEDULE_LOG lists each region call's)."""
    d = tempfile.mkdtemp(prefix="vcfx_walkrank_")
    p, log = os.path.join(d, "gt.vcf"), os.path.join(d, "sched.log")
    try:
        open(p, "wb").write(synth.generate(3000, 300, 85, 1, 0.0, 0, 0.0, 0))
        exe = tool_binary(tool)
        want = subprocess.run([exe] + args + ["-i", p], capture_output=True, timeout=120,
                              env=dict(os.environ, VCFXG_SCHEDULE_LOG=log))
        single = open(log).read().split()
        os.unlink(log)
        got = subprocess.run([exe] + args + ["-i", p], capture_output=True, timeout=120,
                             env=dict(os.environ, VCFX_NGPU="4", VCFXG_SCHEDULE_LOG=log))
        ranks = open(log).read().split()
        assert (got.stdout, got.stderr, got.returncode) == (want.stdout, want.stderr, want.returncode)
        walk = "af_walk" if tool == "VCFX_allele_freq_calc" else "fq_walk"
        assert single == [walk], single
        assert ranks == [walk] * 4, ranks
    finally:
        for f in (p, log):
            if os.path.exists(f):
                os.unlink(f)
        os.rmdir(d)
