"""Parity at BASELINE scale (configs 2, 3 and 5 at their full sizes).

The drop-in binaries run on the deterministic synthetic inputs of BASELINE.json (427,409 x
2,504 chr21-like and annotated shards, LD at N = 2,504 over complete and knocked-out
256-variant groups, the first 3,000 variants of the bench's LD shard) and their stdout must
hash to the digests the REFERENCE binaries produced on the same bytes
(tests/golden/full_digests.json, made by tests/golden/make_full_digests.py, where the C
oracle was checked against the reference on the same inputs).  These exercise what the
small cases cannot: walker line capacity at 32 K walkers, the compaction, the text
re-format path, the streaming stdin ingest (pipes of > 128 MiB), the FP4 LD ring wrapping
over 20 k-slices across many tiles.  The region API's kept-record bitmaps (the bench's own
calls) are checked against the reference's kept records as well.
"""
import hashlib
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

from tests._golden import GOLDEN
from vcfx_amd import engine, synth, tool_binary

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

with open(os.path.join(GOLDEN, "full_digests.json")) as _f:
    DIG = json.load(_f)


class Inputs:
    """Synthetic inputs written once per module to a temp dir (page-cache warm)."""

    def __init__(self):
        self.dir = tempfile.mkdtemp(prefix="vcfx_scale_")
        self.files = {}

    def path(self, name):
        if name not in self.files:
            arr = synth.generate_array(**DIG["inputs"][name])
            p = os.path.join(self.dir, name + ".vcf")
            arr.tofile(p)
            self.files[name] = (p, arr)
        return self.files[name][0]

    def array(self, name):
        self.path(name)
        return self.files[name][1]

    def drop(self, name):
        if name in self.files:
            p = self.files.pop(name)[0]
            os.unlink(p)
            if os.path.exists(p + ".bgz"):
                os.unlink(p + ".bgz")

    def close(self):
        for n in list(self.files):
            self.drop(n)
        os.rmdir(self.dir)


@pytest.fixture(scope="module")
def inputs():
    i = Inputs()
    yield i
    i.close()


def _hash_cmd(cmd, stdin_path=None):
    """Run a shell pipeline; sha256/len/lines of its stdout, streamed (outputs reach ~4 GB)."""
    h = hashlib.sha256()
    n = lines = 0
    fin = open(stdin_path, "rb") if stdin_path else subprocess.DEVNULL
    try:
        p = subprocess.Popen(["bash", "-o", "pipefail", "-c", cmd], stdin=fin, stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE)
        while True:
            b = p.stdout.read(1 << 24)
            if not b:
                break
            h.update(b)
            n += len(b)
            lines += b.count(b"\n")
        err = p.stderr.read()
        rc = p.wait(timeout=300)
    finally:
        if stdin_path:
            fin.close()
    return {"sha256": h.hexdigest(), "len": n, "lines": lines}, rc, err


def _cmd(stages, path):
    parts = []
    for st in stages:
        argv = [tool_binary(st[0])] + [a.replace("{F}", path) for a in st[1:]]
        parts.append(" ".join("'%s'" % a for a in argv))
    return " | ".join(parts)


def _check(case, inputs, stdin="none"):
    if case not in DIG["cases"]:
        pytest.skip("no reference digest for %s (tests/golden/make_full_digests.py %s)" % (case, case))
    c = DIG["cases"][case]
    path = inputs.path(c["input"])
    cmd = _cmd(c["stages"], path)
    stdin_path = None
    first_reads_stdin = not any("{F}" in a for a in c["stages"][0])
    if stdin == "ngpu8":  # the in-process multi-GPU drop-in: 8 rank contexts on the first stage
        assert not first_reads_stdin
        cmd = "VCFX_NGPU=8 " + cmd
    if first_reads_stdin:
        if stdin == "pipe":
            cmd = "cat '%s' | %s" % (path, cmd)   # a pipe: the streaming ingest path
        else:
            stdin_path = path                     # `< file`: the mapped stdin path
    got, rc, err = _hash_cmd(cmd, stdin_path)
    assert rc == 0, err[-2000:]
    assert got == c["stdout"], (case, got, c["stdout"], err[-2000:])


@pytest.mark.parametrize("case,stdin", [("af_file", "none"), ("af_stdin", "pipe"), ("af_stdin", "file"),
                                        ("nonref_file", "none"), ("pipeline_bench", "none"),
                                        ("nonref_stdin", "pipe"), ("nonref_stdin", "file"),
                                        ("hwe_file", "none"), ("hwe_stdin", "pipe"), ("hwe_stdin", "file"),
                                        ("dose_file", "none"), ("ac_bin_file", "none"), ("ac_agg_file", "none"),
                                        ("ac_sel_file", "none"), ("ac_sel_stdin", "pipe"), ("ac_sel_stdin", "file"),
                                        ("md_file", "none"), ("ph_file", "none"), ("ph_stream_stdin", "pipe")])
def test_chr21_shard_matches_reference(inputs, case, stdin):
    _check(case, inputs, stdin)


@pytest.mark.parametrize("case", ["af_file", "pipeline_bench", "pipeline_annot"])
def test_ngpu8_drop_in_at_full_size(inputs, case):
    """The in-process multi-GPU drop-in (VCFX_NGPU=8 on the first stage: eight rank contexts,
    round robin over the box's devices) on the full 427 K-record shard; stdout must hash to the
    reference's digest (AF: the ranks' rows in order; the RF|GQ pipeline: RF's ranks feeding GQ)."""
    c = DIG["cases"][case]
    path = inputs.path(c["input"])
    cmd = "VCFX_NGPU=8 " + _cmd(c["stages"], path)
    got, rc, err = _hash_cmd(cmd)
    assert rc == 0, err[-2000:]
    assert got == c["stdout"], (case, got, c["stdout"], err[-2000:])


@pytest.mark.parametrize("case,fused", [("pipeline_annot_af", True), ("pipeline_annot_nr_af", True),
                                        ("pipeline_annot", True), ("pipeline_annot_af", False)])
def test_vcfx_pipe_at_full_size(inputs, case, fused):
    """vcfx_pipe (one process, one device context) on the 4.3 GB annotated shard: the fused
    schedule (the input in HBM once, a walk per filter stage, AF rows gathered) and the
    stage-by-stage one, against the reference's digest of the shell pipeline; the same chain
    through the drop-in executables piped by the shell"""
    import shlex
    from vcfx_amd import BUILD
    c = DIG["cases"][case]
    path = inputs.path(c["input"])
    chain = " | ".join(" ".join(shlex.quote(a.replace("{F}", path)) for a in st) for st in c["stages"])
    env = "" if fused else "VCFX_PIPE_FUSED=0 "
    got, rc, err = _hash_cmd(env + shlex.quote(os.path.join(BUILD, "bin", "vcfx_pipe")) + " " + shlex.quote(chain))
    assert rc == 0, err[-2000:]
    assert got == c["stdout"], (case, fused, got, c["stdout"], err[-2000:])
    if not fused:
        _check(case, inputs)


@pytest.mark.parametrize("case,stdin", [("pipeline_annot", "none"), ("rf_stdin_annot", "pipe"),
                                        ("gq_strict_annot", "none")])
def test_annotated_shard_matches_reference(inputs, case, stdin):
    _check(case, inputs, stdin)
    if case == "gq_strict_annot":
        inputs.drop("annot")


@pytest.mark.parametrize("case,stdin", [("md_file_miss", "none"), ("md_stdin_miss", "pipe"),
                                        ("md_stdin_miss", "file")])
def test_missing_shard_matches_reference(inputs, case, stdin):
    """VCFX_missing_detector on the shard with sparse missing calls (most records flagged)"""
    _check(case, inputs, stdin)
    if case == "md_stdin_miss" and stdin == "file":
        inputs.drop("chr21_miss")


@pytest.mark.parametrize("case,stdin", [("af_file_miss", "none"), ("af_file_miss", "ngpu8"), ("af_stdin_miss", "pipe"),
                                        ("af_stdin_miss", "file")])
def test_af_missing_shard_matches_reference(inputs, case, stdin):
    """AF where ~70 % of the records carry a missing call ('.|.'): the walk's fixed-stride
    sweep with missing alleles at BASELINE scale (also as 8 ranks, VCFX_NGPU=8)"""
    _check(case, inputs, stdin)


def test_af_irregular_shard_matches_reference(inputs):
    """AF where 5 % of the records take the general GT path (GT:DP, DP:GT, '/', haploid,
    multi-digit alleles): the walk's leftover lines through gt_first / gt_general"""
    _check("af_file_irreg", inputs)
    inputs.drop("chr21_irreg")


@pytest.mark.parametrize("case,stdin", [("af_file_gtadp", "none"), ("af_file_gtadp", "ngpu8"), ("af_stdin_gtadp", "file")])
def test_af_gtadp_shard_matches_reference(inputs, case, stdin):
    """AF on the 13.2 GB shard with every record GT:AD:DP (the general GT path: the GT-first
    walk) at BASELINE scale (also as 8 ranks, VCFX_NGPU=8)"""
    _check(case, inputs, stdin)
    if stdin == "file":
        inputs.drop("chr21_gtadp")


@pytest.mark.parametrize("case,inp", [("pipeline_annot_miss", "annot_miss"), ("pipeline_annot_gtadp", "annot_gtadp")])
def test_pipeline_general_shards_match_reference(inputs, case, inp):
    """config 3's command (FILTER==PASS;AF>=0.01 | -g 0/1) on the annotated shard with sparse
    missing calls, and on its GT:AD:DP form"""
    _check(case, inputs)
    inputs.drop(inp)


@pytest.mark.parametrize("case,how", [("af_file", "none"), ("af_file", "ngpu8"), ("af_stdin", "pipe"),
                                      ("pipeline_bench", "none"), ("pipeline_bench", "ngpu8"), ("hwe_file", "none"),
                                      ("nonref_file", "none"), ("dose_file", "none"), ("md_file", "none"),
                                      ("md_file", "ngpu8"), ("ac_agg_file", "none"), ("ph_file", "none"),
                                      ("ld20k_bench", "none"), ("ld20k_bench", "ngpu8")])
def test_bgzf_chr21_matches_reference(inputs, case, how):
    """the same shard as BGZF (.vcf.gz, made by build/bin/vcfx_bgzf at level 1): inflated on the
    device (the lane decoder + copy kernels; AF's file form streamed through the pinned file ring,
    a pipe read whole first), then the tool's device path; with VCFX_NGPU=8
    each of the eight rank contexts inflates the members of its share of the inflated bytes (LD:
    every rank the whole file, for its share of the pair rows).  Output identical to the
    reference's on the plain bytes."""
    from vcfx_amd import BUILD
    if case not in DIG["cases"]:
        pytest.skip("no reference digest for %s" % case)
    c = DIG["cases"][case]
    plain = inputs.path(c["input"])
    bgz = plain + ".bgz"
    if not os.path.exists(bgz):
        subprocess.check_call([os.path.join(BUILD, "bin", "vcfx_bgzf"), plain, bgz, "16", "1"])
    cmd = _cmd(c["stages"], bgz)
    if how == "ngpu8":
        cmd = "VCFX_NGPU=8 " + cmd
    elif how == "pipe":
        cmd = "cat '%s' | %s" % (bgz, cmd)
    got, rc, err = _hash_cmd(cmd)
    assert rc == 0, err[-2000:]
    assert got == c["stdout"], (case, got, err[-2000:])


@pytest.mark.parametrize("case", ["ld1500_t02", "ld1500_t0", "ld1500_w300_t0", "ld3000_bench", "ph_ld3000",
                                  "ld20k_bench", "ld20k_miss_bench"])
def test_ld_matches_reference(inputs, case):
    _check(case, inputs)


@pytest.mark.parametrize("case,prefix", [("ld100k_tail_bench", "ld20k_bench"),
                                         ("ld100k_miss_tail_bench", "ld20k_miss_bench")])
def test_ngpu8_ld_at_full_size(case, prefix):
    """Config 5 at 8 ranks (VCFX_NGPU=8: eight rank contexts, each parsing the 100 K shard and
    writing the pair lines of its --shard r/8 share -- equal window-pair counts, row cuts at
    j_k ~ M sqrt(k/8) -- rank 0's stdout first, the others' after it in rank order) on the whole
    100 K x 2,504 bench shard, complete and with 0.1 % missing calls: its first 20 K variants'
    lines against the reference's output on those variants, and its lines with VAR1 >= 80,000
    against the reference's output on that slice (the same digests the one-rank run is held to)"""
    for k in (case, prefix):
        if k not in DIG["cases"]:
            pytest.skip("no reference digest for %s" % k)
    c, cp = DIG["cases"][case], DIG["cases"][prefix]
    params = dict(DIG["inputs"][c["input"]])
    lo, hi = params.pop("slice")
    pin = dict(DIG["inputs"][cp["input"]])
    assert pin.pop("n_records") <= lo and pin == {k: v for k, v in params.items() if k != "n_records"}
    assert c["stages"] == cp["stages"]
    arr, offs = synth.generate_array(rec_offsets=True, **params)
    pos0 = int(bytes(arr[int(offs[lo]):int(offs[lo]) + 64]).split(b"\t")[1])
    d = tempfile.mkdtemp(prefix="vcfx_ld8_")
    path = os.path.join(d, "ld100k.vcf")
    try:
        arr.tofile(path)
        del arr, offs
        argv = [tool_binary("VCFX_ld_calculator")] + [a.replace("{F}", path) for a in c["stages"][0][1:]]
        r = subprocess.run(argv, capture_output=True, timeout=600, env=dict(os.environ, VCFX_NGPU="8"))
        assert r.returncode == 0, r.stderr[-2000:]
        out = r.stdout
        n = cp["stdout"]["len"]
        got = {"sha256": hashlib.sha256(out[:n]).hexdigest(), "len": n, "lines": out[:n].count(b"\n")}
        assert got == cp["stdout"], (prefix, got, cp["stdout"])
        head = out[:out.index(b"\n") + 1]
        tail = head
        for ln in out[len(head):].split(b"\n"):
            if ln and int(ln.split(b"\t", 2)[1]) >= pos0:
                tail += ln + b"\n"
        got = {"sha256": hashlib.sha256(tail).hexdigest(), "len": len(tail), "lines": tail.count(b"\n")}
        assert got == c["stdout"], (case, got, c["stdout"])
    finally:
        if os.path.exists(path):
            os.unlink(path)
        os.rmdir(d)


@pytest.mark.parametrize("case", ["ld100k_tail_bench", "ld100k_miss_tail_bench"])
def test_ld_tail_matches_reference(case):
    """Config 5 past its first 20 K variants.  The reference ran on the header + variants
    [80,000, 100,000) of the bench's 100 K LD shard (complete, and with 0.1 % missing calls);
    the drop-in runs on the WHOLE 100 K shard (every tile row up to 100 K, the count table and
    the row offsets far from the origin) and its lines whose VAR1 is variant >= 80,000 must hash
    to the reference's output: with W = 100 K each variant's pairs stream oldest -> newest, so
    that subsequence is the reference's output on the slice."""
    if case not in DIG["cases"]:
        pytest.skip("no reference digest for %s" % case)
    c = DIG["cases"][case]
    params = dict(DIG["inputs"][c["input"]])
    lo, hi = params.pop("slice")
    assert hi == params["n_records"]
    arr, offs = synth.generate_array(rec_offsets=True, **params)
    pos0 = int(bytes(arr[int(offs[lo]):int(offs[lo]) + 64]).split(b"\t")[1])
    d = tempfile.mkdtemp(prefix="vcfx_ldtail_")
    path = os.path.join(d, "ld100k.vcf")
    try:
        arr.tofile(path)
        del arr, offs
        argv = [tool_binary("VCFX_ld_calculator")] + [a.replace("{F}", path) for a in c["stages"][0][1:]]
        r = subprocess.run(argv, capture_output=True, timeout=600)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = r.stdout.split(b"\n")
        head, keep = lines[0], []
        for ln in lines[1:]:
            if ln and int(ln.split(b"\t", 2)[1]) >= pos0:
                keep.append(ln)
        out = head + b"\n" + b"".join(x + b"\n" for x in keep)
        got = {"sha256": hashlib.sha256(out).hexdigest(), "len": len(out), "lines": out.count(b"\n")}
        assert got == c["stdout"], (case, got, c["stdout"])
    finally:
        if os.path.exists(path):
            os.unlink(path)
        os.rmdir(d)


def _mask_sha(st, n_records):
    keep = (st == 1).astype(np.uint8)  # VCFXG_LINE_ROW: kept
    assert keep.size == n_records
    return hashlib.sha256(np.packbits(keep).tobytes()).hexdigest()


def test_region_api_at_full_size(inputs):
    """The bench's own calls on the full chr21 shard: AF rows text, the fused RF|GQ and the nonref
    walk's per-record decisions against the reference's outputs."""
    arr = inputs.array("chr21")
    n_rec = DIG["inputs"]["chr21"]["n_records"]
    ds = engine.data_start_of(arr[:1 << 20].tobytes())
    eng = engine.Engine(0)
    want_af = DIG["cases"]["af_file"]["stdout"]["sha256"]
    try:
        # the streaming ingest on a fresh context: unequal chunks (records cut mid-line), the
        # device buffer grown from nothing
        cuts = [0, 1000, 77 << 20, 1 << 30, arr.size]
        eng.ingest([arr[a:b] for a, b in zip(cuts, cuts[1:])])
        s = eng.allele_freq_region(ds, engine.MODE_FILE)
        text = b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes)
        assert hashlib.sha256(text).hexdigest() == want_af
        eng.load(arr)
        s = eng.allele_freq_region(ds, engine.MODE_FILE)
        assert s.rows == n_rec and s.general_records == 0
        text = b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes)
        assert hashlib.sha256(text).hexdigest() == want_af
        crits = [(engine.QUAL, engine.GE, 1, 30.0, "QUAL", ""), (engine.FILTER, engine.EQ, 0, 0.0, "FILTER", "PASS")]
        s = eng.filter_query_region(ds, crits, "0|1", and_logic=True, strict=False)
        assert s.n_lines == n_rec
        c = DIG["cases"]["pipeline_bench"]
        assert s.rows == c["kept"]
        assert _mask_sha(eng.statuses(s.n_lines), n_rec) == c["keep_mask_sha256"]
        s = eng.nonref_filter_region(ds, engine.MODE_FILE)
        c = DIG["cases"]["nonref_file"]
        assert s.rows == c["kept"]
        assert _mask_sha(eng.statuses(s.n_lines), n_rec) == c["keep_mask_sha256"]
        s = eng.hwe_region(ds, engine.MODE_FILE)
        c = DIG["cases"]["hwe_file"]
        assert s.rows == c["stdout"]["lines"] - 1 and s.general_records == 0 and not eng.hwe_rechecks()
        text = b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n" + eng.text(s.text_bytes)
        assert hashlib.sha256(text).hexdigest() == c["stdout"]["sha256"]
    finally:
        eng.close()
