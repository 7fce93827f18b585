"""CPU coverage of the record-sharded multi-GPU path (vcfx_amd/shard.py):
world_size-2, 3 and 8 gloo process groups over 127.0.0.1 run the sharded orchestration with
the C oracle standing in for each rank's per-shard GPU run; the merged rank-0 output must
equal the oracle's whole-file output byte for byte, and every case meant to shard must have
reached every rank as a view of its own records.  The stand-in runner applies the view the
tools take from VCFX_INPUT_VIEW (header + record range) by writing it to a file, and the
VCFX_VIEW_SKIP_HEADER rule by stripping the header-only run's output.  The cut logic and the
getopt-style operand detection are checked directly."""
import gzip
import os
import socket
import struct
import tempfile
import zlib

import numpy as np
import pytest

from tests._golden import Oracle
from vcfx_amd import shard, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def oracle_view_runner(o, calls):
    """the C oracle as a rank's tool, honouring the shard view like the drop-ins do"""
    def run(argv, stdin, view=None, skip_header=False):
        calls.append((list(argv), view, skip_header))
        if view is None:
            return o.run(argv, stdin)
        tool = os.path.basename(argv[0])
        path = shard.input_path(tool, argv)
        with open(path, "rb") as f:
            data = f.read()
        if len(view) > 3:  # a BGZF file's view: offsets into its inflated bytes
            assert view[3] == "bgzf"
            data = gzip.decompress(data)
        h, lo, hi = view[:3]
        with tempfile.NamedTemporaryFile(suffix=".vcf") as fv, tempfile.NamedTemporaryFile(suffix=".vcf") as fh:
            fv.write(data[:h] + data[lo:hi])
            fv.flush()
            out, err, rc = o.run([fv.name if a == path else a for a in argv], stdin)
            if skip_header:
                fh.write(data[:h])
                fh.flush()
                H, E, _ = o.run([fh.name if a == path else a for a in argv], stdin)
                assert out.startswith(H)
                out = out[len(H):]
                if err.startswith(E):
                    err = err[len(E):]
        return out, err, rc
    return run


def _worker(rank, world, port, cases, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle()
    try:
        for argv in cases:
            calls = []
            res = shard.run_sharded(argv, b"", dist, runner=oracle_view_runner(o, calls))
            q.put((rank, argv, res, calls))
    finally:
        dist.destroy_process_group()


def _run_world(world, cases):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(len(cases) * world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def _bgzf_member(data):
    """one BGZF member (RFC 1952 + the 'BC' extra subfield holding the member size - 1)"""
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    body = co.compress(data) + co.flush()
    bsize = 18 + len(body) + 8
    hdr = b"\x1f\x8b\x08\x04" + bytes(4) + b"\x00\xff" + struct.pack("<H", 6) + b"BC" + struct.pack("<HH", 2, bsize - 1)
    return hdr + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)


def _files(tmp):
    paths = {}
    head = b"##fileformat=VCFv4.2\n"
    paths["synth"] = synth.generate(700, 37, 61, 1, 0.05, 0, 0.3, 0)
    paths["crlf"] = synth.generate(300, 5, 62, 0, 0.0, 0, 0.2, 1)
    bad = (head + b"1\t1\t.\tA\tG\t.\t.\t.\tGT\t0|1\n"  # data before #CHROM
           + b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n"
           + b"".join(b"1\t%d\t.\tA\tG\t.\t.\t.\tGT\t%d|1\n" % (i, i % 2) for i in range(60))
           + b"1\t99\t.\tA\n"  # short line
           + b"".join(b"2\t%d\t.\tC\tT\t.\t.\t.\tGT\t1/1\n" % i for i in range(40))
           + b"3\t5\tonly\tseven\tcols\t.\t.\n\n")
    paths["bad"] = bad
    paths["tiny"] = head + b"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tS1\n1\t1\t.\tA\tG\t.\t.\t.\tGT\t0|1\n"
    # compressed copies (byte cuts of a gzip file are not record cuts): one gzip
    # member, and BGZF-style 64 KiB members with the BC extra field
    paths["synth.gz"] = gzip.compress(paths["synth"], mtime=0)
    raw = paths["synth"]
    paths["synth.bgz"] = b"".join(_bgzf_member(raw[o:o + 65280]) for o in range(0, len(raw), 65280)) + \
        _bgzf_member(b"")
    out = {}
    for k, b in paths.items():
        p = os.path.join(tmp, k if k.endswith("gz") or k.endswith(".bgz") else k + ".vcf")
        open(p, "wb").write(b)
        out[k] = p
    return out


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    return _files(str(tmp_path_factory.mktemp("shard")))


def _cases(files):
    cases = []
    for k, p in files.items():
        cases += [["VCFX_allele_freq_calc", "-i", p], ["VCFX_allele_freq_calc", "-q", "-i", p],
                  ["VCFX_allele_freq_calc", p], ["VCFX_variant_counter", p]]
        cases += [["VCFX_record_filter", "--filter", "QUAL>=30;AF>=0.05", "-i", p],
                  ["VCFX_genotype_query", "-g", "0/1", "-i", p], ["VCFX_genotype_query", "-g", "1|1", "--strict", p],
                  ["VCFX_nonref_filter", "-i", p], ["VCFX_nonref_filter", p],
                  ["VCFX_dosage_calculator", "-i", p], ["VCFX_dosage_calculator", "-q", p]]
    cases.append(["VCFX_variant_counter", "--strict", files["bad"]])
    return cases


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_runs_match_whole_file(files, world):
    cases = _cases(files)
    o = Oracle()
    got = _run_world(world, cases)
    views = {}
    for rank, argv, res, calls in got:
        views.setdefault(tuple(argv), {})[rank] = calls
        if rank == 0 and argv[-1].endswith(".bgz") and argv[0] != "VCFX_variant_counter":
            # a BGZF chain shards in its inflated bytes: the oracle's output on those bytes (the
            # reference reads compressed bytes as text; inflating is the drop-ins' extension)
            plain = argv[-1][:-len(".bgz")] + ".vcf"
            want = o.run([plain if a == argv[-1] else a for a in argv], b"")
            keep = lambda e: [x for x in e.split(b"\n") if not x.startswith(b"Processing ")]
            assert (res[0], res[2]) == (want[0], want[2]) and keep(res[1]) == keep(want[1]), (argv, world)
        elif rank == 0:
            want = o.run(argv, b"")
            assert res == want, (argv, world)
        else:
            assert res == (b"", b"", 0)
    for argv in cases:
        by_rank = views[tuple(argv)]
        assert set(by_rank) == set(range(world))
        if argv[-1].endswith(".gz") or (argv[-1].endswith(".bgz") and argv[0] == "VCFX_variant_counter"):
            # one gzip member (and variant_counter's own gzip handling): whole on rank 0 (no view),
            # the other ranks run nothing
            assert shard.plan(argv) is None or shard.bgzf_cuts(argv, world) is None, argv
            assert [c[1] for c in by_rank[0]] == [None] and all(not by_rank[r] for r in range(1, world)), argv
            continue
        if argv[-1].endswith(".bgz"):
            # a BGZF member chain: every rank a view of its share of the inflated records
            spans = []
            for r in range(world):
                calls = [c for c in by_rank[r] if c[1] is not None]
                assert len(calls) == 1 and calls[0][1][3] == "bgzf", (argv, r, by_rank[r])
                spans.append(calls[0][1][1:3])
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:])), argv
            continue
        meant = shard.plan(argv) in ("af", "vc", "filter") and not (
            argv[0] in ("VCFX_record_filter", "VCFX_genotype_query", "VCFX_nonref_filter", "VCFX_dosage_calculator")
            and "bad" in argv[-1])
        if not meant:
            continue
        # every rank ran its own view (no silent fallback to an unsharded rank-0 run)
        spans = []
        for r in range(world):
            calls = [c for c in by_rank[r] if c[1] is not None]
            assert len(calls) == 1, (argv, r, by_rank[r])
            _, (h, lo, hi), skip = calls[0]
            assert skip == (r > 0) or argv[0] == "VCFX_variant_counter"
            spans.append((lo, hi))
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))  # contiguous, in rank order


def test_record_cuts_cover_region_at_line_starts():
    rng = np.random.default_rng(5)
    for trial in range(30):
        lines = [b"x" * int(rng.integers(0, 40)) for _ in range(int(rng.integers(0, 50)))]
        buf = b"#H\n#CHROM\n" + b"\n".join(lines) + (b"\n" if rng.integers(0, 2) else b"")
        ds = shard.header_end(buf)
        assert ds == len(b"#H\n#CHROM\n") or ds == len(buf)
        for world in range(1, 9):
            cuts = shard.record_cuts(buf, ds, world)
            assert len(cuts) == world + 1 and cuts[0] == ds and cuts[-1] == len(buf)
            assert all(a <= b for a, b in zip(cuts, cuts[1:]))
            for c in cuts[1:-1]:
                assert c == ds or c == len(buf) or buf[c - 1:c] == b"\n"
            # the shards' lines are exactly the region's lines, each once
            region = buf[ds:]
            joined = b"".join(buf[a:b] for a, b in zip(cuts, cuts[1:]))
            assert joined == region


def test_single_process_passthrough(files):
    o = Oracle()
    argv = ["VCFX_allele_freq_calc", "-i", files["synth"]]
    assert shard.run_sharded(argv, b"", None, runner=oracle_view_runner(o, [])) == o.run(argv, b"")


def test_input_operand_found_like_getopt(files):
    """option values are never taken for the input operand (`-g 1|1 --strict in.vcf`)"""
    p = files["synth"]
    ip = shard.input_path
    assert ip("VCFX_genotype_query", ["VCFX_genotype_query", "-g", "1|1", "--strict", p]) == p
    assert ip("VCFX_genotype_query", ["VCFX_genotype_query", "-g", p, "--strict"]) is None  # p is the query
    assert ip("VCFX_genotype_query", ["VCFX_genotype_query", "--genotype-query=0/1", p]) == p
    assert ip("VCFX_record_filter", ["VCFX_record_filter", "--filter", p, "-l", "or"]) is None
    assert ip("VCFX_record_filter", ["VCFX_record_filter", "-fQUAL>1", p]) == p
    assert ip("VCFX_record_filter", ["VCFX_record_filter", "-f", "QUAL>1", "-i", p]) == p
    assert ip("VCFX_allele_freq_calc", ["VCFX_allele_freq_calc", "-q", p]) == p
    assert ip("VCFX_allele_freq_calc", ["VCFX_allele_freq_calc", "-i" + p]) == p
    assert ip("VCFX_allele_freq_calc", ["VCFX_allele_freq_calc", "--input=" + p]) == p
    assert ip("VCFX_nonref_filter", ["VCFX_nonref_filter", "--", p]) == p
    assert ip("VCFX_ld_calculator", ["VCFX_ld_calculator", "-w", "10", p]) is None  # LD takes -i only
    assert ip("VCFX_ld_calculator", ["VCFX_ld_calculator", "-w", "10", "-i", p]) == p
    assert ip("VCFX_variant_counter", ["VCFX_variant_counter", "-s", p]) == p
    assert shard.plan(["VCFX_genotype_query", "-g", "1|1", "--strict", p]) == "filter"
    assert shard.plan(["VCFX_allele_freq_calc", "-h", p]) is None
    assert shard.plan(["VCFX_ld_calculator", "-m", "-i", p]) is None
