#!/usr/bin/env python3
"""bench.py -- the VCFX per-record hot path on MI355X.

Workloads (BASELINE.json configs; the default is the headline one):
  af        configs[1] / configs[3]: VCFX_allele_freq_calc -i on a device-resident
            427,409-record x 2,504-sample chr21-like shard per GPU.  A step =
            vcfxg_allele_freq_region: the walk (af_walk: one wave per chunk walks its lines --
            head from an LDS window, fixed-stride sample sweep, the record's output row composed
            in LDS) and the region tail (rare full-path lines, rows placed in file order); for
            N > 1 ranks also all-reduce the step's global counts over RCCL.
  pipeline  configs[2] as SURVEY §8(d) defines it: VCFX_record_filter --filter
            "FILTER==PASS;AF>=0.01" | VCFX_genotype_query -g 0/1 fused on the device (one walk:
            the filter's INFO key lookup + the genotype query), on the annotated shard
            (INFO=AF=..;DP=.., seed 20251227+rank).
  ld        configs[4]: VCFX_ld_calculator streaming, 100,000-variant window over a
            100,000-variant x 2,504-sample shard (haplotype-block LD structure) with -t 0.5:
            parse + FP4-MFMA pair sums (exact for 0/1/2 dosages; count pass and emit pass) +
            pair text.

value = units processed by all ranks / max-over-ranks wall time of the K timed steps
(inputs already resident in HBM).  One process per GPU (torchrun), record-sharded with
seed = base + rank: weak scaling.  `--gpus N` without a torchrun environment launches the N
ranks itself (torch.distributed.run, 127.0.0.1) before anything touches the GPU.  Rank 0 prints ONE JSON line (contract: DESIGN.md
§Measurement) carrying `roofline` for the dominant kernel (HIP-event timing on the engine's
own stream, algorithmic bytes or ops per launch), `cpu_baseline` (the reference's own tools
compiled from its sources, else the oracle/ C restatement, on a bounded sample, 1 core),
`output_check` (the last step's output against the reference's digests) and `e2e` (the
drop-in CLI end to end: file / pipe / warm context).
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "variant-records/sec (and GB/s vs HBM roofline), 427K var × 2504 samp"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
FP4_PEAK_TOPS = 10000.0  # MI355X_MICROARCH.md: block-scaled FP4 MFMA = 4x the BF16 rate per clock, ~10 PF dense
PMC_FILE = os.path.join(REPO, "profiles", "pmc_traffic.json")
MFMA_FILE = os.path.join(REPO, "profiles", "r02_ld_mfma.json")  # tools/pmc_mfma.py over a --pmc pass


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("af", "pipeline", "ld", "nonref", "hwe", "dose", "ac", "md", "ph"), default="af")
    ap.add_argument("--records", type=int, default=None, help="records per GPU (default per workload)")
    ap.add_argument("--samples", type=int, default=2504)
    ap.add_argument("--window", type=int, default=100000, help="ld: window in variants")
    ap.add_argument("--threshold", type=float, default=0.5, help="ld: r^2 threshold")
    ap.add_argument("--format", choices=("gt", "gt:ad:dp"), default="gt",
                    help="FORMAT of the synthetic records: GT (fixed-stride) or GT:AD:DP (the general GT path)")
    ap.add_argument("--missing-rate", type=float, default=0.0, help="per-sample './.' probability")
    ap.add_argument("--irregular-rate", type=float, default=0.0,
                    help="fraction of records in a general-path shape (GT:DP, DP:GT, '/', haploid, multi-digit)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end CLI timings")
    ap.add_argument("--no-output-check", action="store_true",
                    help="skip the reference-digest check (diagnostic builds whose results are invalid)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) or gloo (rehearsal on one GPU)")
    a = ap.parse_args()
    if a.records is None:
        a.records = 100000 if a.workload == "ld" else 427409
    if a.workload == "ld" and a.steps == 20:
        a.steps = 3
    return a


def input_params(a, rank):
    """vcfx_synth parameters of this rank's shard (the keys of full_digests.json "inputs")"""
    p = dict(n_records=a.records, n_samples=a.samples, seed=20251226 + rank)
    if a.workload == "pipeline":
        p.update(seed=20251227 + rank, info_mode=1)  # the annotated shard: INFO AF=..;DP=..
    if a.workload == "ld":
        p["hap_blocks"] = 1
    if a.missing_rate > 0:
        p["missing_rate"] = a.missing_rate
    if a.irregular_rate > 0:
        p["irregular_rate"] = a.irregular_rate
    if a.format == "gt:ad:dp":
        p["format_mode"] = 1
    return p


_SYNTH_DEFAULTS = dict(seed=20251226, info_mode=0, missing_rate=0.0, hap_blocks=0, irregular_rate=0.0, crlf=0,
                       format_mode=0)


def _same_input(p, q):
    full = lambda d: dict(_SYNTH_DEFAULTS, **d)  # noqa: E731
    return full(p) == full(q)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` from the committed PMC pass (profiles/pmc_traffic.json,
    written by tools/pmc_traffic.py from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs,
    FETCH_SIZE doubled per the gfx950 correction), or None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        return d[workload][kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        return None


REF_DIR = os.path.join(REPO, "oracle", "_ref")
# configs[2] as SURVEY §8(d) states it
PIPE_FILTER, PIPE_QUERY = "FILTER==PASS;AF>=0.01", "0/1"


def _timed_chain(argvs, budget_s, reference):
    """Run a chain of tool invocations (stdout of one = stdin of the next) repeatedly: the
    reference binaries built from /root/reference sources (oracle/_ref, kind "reference") as
    processes, or the C restatement in-process (kind "port")."""
    import subprocess
    o = None
    if not reference:
        from tests._golden import Oracle
        o = Oracle()
    reps, t_total = 0, 0.0
    while t_total < budget_s or reps == 0:
        t0 = time.perf_counter()
        data = b""
        for argv in argvs:
            if reference:
                r = subprocess.run([os.path.join(REF_DIR, argv[0])] + argv[1:], input=data, capture_output=True)
                out, err, rc = r.stdout, r.stderr, r.returncode
            else:
                out, err, rc = o.run(argv, data)
            assert rc == 0, (argv, err[:200])
            data = out
        t_total += time.perf_counter() - t0
        reps += 1
    return reps, t_total


def cpu_baseline(workload, arr, offs, a):
    """The reference's own tools (oracle/_ref, compiled here from /root/reference sources by
    oracle/Makefile.ref; kind "reference"), else the C restatement (oracle/, kind "port"), 1
    thread, over a bounded prefix sample of this rank's synthetic input (the same byte layout
    as the GPU workload)."""
    if workload == "ld":
        nvar = min(a.records, 1500)
    else:
        nvar = min(a.records, 20000)
    sample = arr[:int(offs[nvar])].tobytes()  # header + first nvar records
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else None
    with tempfile.NamedTemporaryFile(suffix=".vcf", dir=shm) as f:
        f.write(sample)
        f.flush()
        if workload == "af":
            argvs = [["VCFX_allele_freq_calc", "-q", "-i", f.name]]
            desc = "VCFX_allele_freq_calc -q -i (file path)"
        elif workload == "nonref":
            argvs = [["VCFX_nonref_filter", "-i", f.name]]
            desc = "VCFX_nonref_filter -i (file path)"
        elif workload == "hwe":
            argvs = [["VCFX_hwe_tester", "-q", "-i", f.name]]
            desc = "VCFX_hwe_tester -q -i (file path)"
        elif workload == "dose":
            argvs = [["VCFX_dosage_calculator", "-q", "-i", f.name]]
            desc = "VCFX_dosage_calculator -q -i (file path)"
        elif workload == "ac":
            argvs = [["VCFX_allele_counter", "-q", "-t", "1", "-i", f.name]]
            desc = "VCFX_allele_counter -q -t 1 -i (file path, one thread)"
        elif workload == "md":
            argvs = [["VCFX_missing_detector", "-q", "-i", f.name]]
            desc = "VCFX_missing_detector -q -i (file path)"
        elif workload == "ph":
            argvs = [["VCFX_haplotype_phaser", "-q", "-i", f.name]]
            desc = "VCFX_haplotype_phaser -q -i (file path, default mode, threshold 0.8)"
        elif workload == "pipeline":
            argvs = [["VCFX_record_filter", "--filter", PIPE_FILTER, "-i", f.name],
                     ["VCFX_genotype_query", "-g", PIPE_QUERY]]
            desc = "VCFX_record_filter -i | VCFX_genotype_query (stdin)"
        else:
            argvs = [["VCFX_ld_calculator", "-q", "-w", str(nvar), "-t", str(a.threshold), "-i", f.name]]
            desc = "VCFX_ld_calculator -w %d -t %g -i (file path)" % (nvar, a.threshold)
        reference = all(os.access(os.path.join(REF_DIR, v[0]), os.X_OK) for v in argvs)
        reps, t = _timed_chain(argvs, a.cpu_seconds, reference)
    kind = "reference" if reference else "port"
    if workload == "ld":
        units = nvar * (nvar - 1) // 2
        return {"value": units * reps / t, "unit": "r2-pairs/s", "cores": 1, "kind": kind,
                "sample": "first %d variants (%.1f MB) of the rank-0 shard, all %d window pairs, %s, %d reps, "
                          "%.1f s" % (nvar, len(sample) / 1e6, units, desc, reps, t)}
    return {"value": nvar * reps / t, "unit": "records/s", "cores": 1, "kind": kind,
            "sample": "first %d records (%.1f MB) of the rank-0 shard, %s, %d reps, %.1f s"
                      % (nvar, len(sample) / 1e6, desc, reps, t)}


def _ph_blocks_sha(arr, flags, off, text):
    """sha256 of the phaser's default-mode output: the '#' lines, then the block lines assembled
    from the per-variant flags (bit 0 pair passes, bit 1 same CHROM) and the entries"""
    import hashlib
    h = hashlib.sha256()
    head = arr[:1 << 20].tobytes()
    for line in head.split(b"\n"):
        if not line.startswith(b"#"):
            break
        h.update(line.rstrip(b"\r") + b"\n")
    h.update(b"#HAPLOTYPE_BLOCKS_START\n")
    parts, blk = [], 0
    for v in range(len(flags)):
        if v == 0 or (flags[v] & 3) != 3:
            if v:
                parts.append(b"\n")
            blk += 1
            parts.append(b"Block %d: " % blk)
        else:
            parts.append(b", ")
        parts.append(text[int(off[v]):int(off[v + 1])])
    h.update(b"".join(parts))
    h.update(b"\n#HAPLOTYPE_BLOCKS_END\n")
    return h.hexdigest()


# per workload: the reference cases whose command is the bench step's (the first whose input
# is this rank's shard is checked)
_CHECK_CASES = {
    "af": ("af_file", "af_file_miss", "af_file_irreg", "af_file_gtadp"),
    "pipeline": ("pipeline_annot", "pipeline_annot_miss", "pipeline_annot_gtadp"),
    "nonref": ("nonref_file",), "hwe": ("hwe_file",), "dose": ("dose_file",), "ac": ("ac_bin_file",),
    "md": ("md_file",), "ph": ("ph_file",),
    "ld": ("ld20k_bench", "ld3000_bench", "ld20k_miss_bench"),
}
# LD: the reference's output on the header + variants [a, n) of the shard (a "slice" input) is
# the full run's lines whose VAR1 is variant >= a (W >= n - a: every pair of the slice is in the
# window; each variant's pairs stream oldest -> newest)
_LD_TAIL_CASES = ("ld100k_tail_bench", "ld100k_miss_tail_bench")


def ld_tail_lines(text, pos0):
    """the pair lines of `text` whose VAR1_POS >= pos0 (positions strictly increase in the shard)"""
    out = []
    for ln in text.split(b"\n"):
        if ln and int(ln.split(b"\t", 2)[1]) >= pos0:
            out.append(ln)
    return b"".join(x + b"\n" for x in out)


def record_pos(arr, k):
    """POS of data record k of a synthetic shard (numpy uint8 array of the file bytes)"""
    import numpy as np
    nl = np.flatnonzero(arr == 10)
    # the data records follow the '#' lines: the first data line starts after the last header '\n'
    starts = np.concatenate([[0], nl[:-1] + 1])
    first = int(np.searchsorted(starts, 0, "left"))
    while arr[starts[first]] == ord("#"):
        first += 1
    s0 = int(starts[first + k])
    return int(bytes(arr[s0:s0 + 64]).split(b"\t")[1])


def output_check(workload, eng, s, a, rank, arr=None):
    """The last timed step's output against the REFERENCE's, on rank 0: the digests
    tests/golden/full_digests.json holds for this exact synthetic input (made by running the
    reference binaries on it; every data shape bench.py can generate that has a digest: the
    chr21-like shard, its missing-call, irregular-record and GT:AD:DP forms, the annotated
    shard and its forms).  AF / DOSE / HWE: sha256 of the formatted rows; pipeline / nonref:
    sha256 of the kept-record bitmap; LD: the first 20,000 variants' pairs (the first lines of
    the stream at a window >= 20,000: 2.0e8 window pairs).  A mismatch raises."""
    import hashlib
    import numpy as np
    try:
        with open(os.path.join(REPO, "tests", "golden", "full_digests.json")) as f:
            dig = json.load(f)
    except OSError:
        return {"checked": False, "why": "no tests/golden/full_digests.json"}
    mine = input_params(a, rank)
    case = None
    for nm in _CHECK_CASES[workload]:
        c = dig["cases"].get(nm)
        if c is None:
            continue
        want_in = dict(dig["inputs"][c["input"]])
        if workload == "ld":  # a prefix of the shard: its first n variants' pairs lead the stream
            if want_in["n_records"] > a.records or a.window < want_in["n_records"] or a.threshold != 0.5:
                continue
            want_in["n_records"] = a.records
        if _same_input(mine, want_in):
            case = nm
            break
    if case is None:
        return {"checked": False, "why": "no reference digest for this rank's input %s" % json.dumps(mine)}
    if workload == "md" and case != "md_file":
        return {"checked": False, "why": "md output assembly is host-side"}
    if workload == "af":
        c = dig["cases"][case]
        got = hashlib.sha256(b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n" + eng.text(s.text_bytes)).hexdigest()
        want, what = c["stdout"]["sha256"], "sha256 of the AF rows vs VCFX_allele_freq_calc -q -i (reference)"
    elif workload == "dose":
        c = dig["cases"]["dose_file"]
        got = hashlib.sha256(b"CHROM\tPOS\tID\tREF\tALT\tDosages\n" + eng.text(s.text_bytes)).hexdigest()
        want, what = c["stdout"]["sha256"], "sha256 of the dosage rows vs VCFX_dosage_calculator -q -i (reference)"
    elif workload == "ac":
        # every (record, sample) count of the shard: the binary form of the same call (one
        # untimed extra call; the text rows' formatting is pinned by tests/test_gpu_scale.py)
        c = dig["cases"].get("ac_bin_file")
        if c is None:
            return {"checked": False, "why": "no ac_bin_file digest"}
        names = ["S%05d" % (k + 1) for k in range(a.samples)]
        sb = eng.allele_counter(0, s.n_lines, list(range(a.samples)), names, seq=1, kind=2)
        hdr = b"VCAC" + (1).to_bytes(4, "little") + a.samples.to_bytes(4, "little") + bytes(8)
        h = hashlib.sha256(hdr)
        for o in range(0, sb.text_bytes, 1 << 28):
            h.update(eng.text_range(o, min(1 << 28, sb.text_bytes - o)))
        got = h.hexdigest()
        want, what = c["stdout"]["sha256"], ("sha256 of every (record, sample) REF/ALT count (the -b form of the "
                                             "same call) vs VCFX_allele_counter -q -b -i (reference)")
    elif workload == "md":
        c = dig["cases"].get("md_file")
        if c is None:
            return {"checked": False, "why": "no md_file digest"}
        # no '.' in the shard's samples (device counts): the tool then writes its input unchanged
        got = "flagged %d, lines with a '.' %d" % (s.rows, s.general_records)
        if s.rows == 0 and s.general_records == 0:
            got = hashlib.sha256(arr).hexdigest()
        want, what = c["stdout"]["sha256"], ("no record flagged and no '.' in any sample column, so the output is "
                                             "the input: its sha256 vs VCFX_missing_detector -q -i (reference)")
    elif workload == "ph":
        c = dig["cases"].get("ph_file")
        if c is None:
            return {"checked": False, "why": "no ph_file digest"}
        # the block lines from the device's pair decisions and entries (the tool's assembly)
        flags, _, off = eng.phaser_variants(s.rows)
        text = eng.text(s.text_bytes)
        got = _ph_blocks_sha(arr, flags, off, text)
        want, what = c["stdout"]["sha256"], "sha256 of the header + block lines vs VCFX_haplotype_phaser -q -i (reference)"
    elif workload == "hwe":
        if "hwe_file" not in dig["cases"]:
            return {"checked": False, "why": "no hwe_file digest"}
        c = dig["cases"]["hwe_file"]
        if eng.hwe_rechecks():
            return {"checked": False, "why": "rows left to the host p-value (not in the device text)"}
        got = hashlib.sha256(b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n" + eng.text(s.text_bytes)).hexdigest()
        want, what = c["stdout"]["sha256"], "sha256 of the HWE rows vs VCFX_hwe_tester -q -i (reference)"
    elif workload in ("pipeline", "nonref"):
        c = dig["cases"][case]
        keep = (eng.statuses(s.n_lines) == 1).astype(np.uint8)
        got = hashlib.sha256(np.packbits(keep).tobytes()).hexdigest()
        want = c["keep_mask_sha256"]
        what = "sha256 of the kept-record bitmap vs the reference's kept records (%s)" % " | ".join(
            st[0] for st in c["stages"])
    else:
        c = dig["cases"][case]
        head = b"#VAR1_CHROM\tVAR1_POS\tVAR1_ID\tVAR2_CHROM\tVAR2_POS\tVAR2_ID\tR2\n"
        n = c["stdout"]["len"] - len(head)
        text = eng.text(s[2])
        got = hashlib.sha256(head + text[:n]).hexdigest()
        want = c["stdout"]["sha256"]
        what = "sha256 of the first %d variants' pair lines vs VCFX_ld_calculator -w 100000 -t 0.5 (reference)" % (
            dig["inputs"][c["input"]]["n_records"])
        # and the shard's tail: the lines whose VAR1 is past the slice start
        for nm in _LD_TAIL_CASES:
            t = dig["cases"].get(nm)
            if t is None or got != want:
                continue
            tin = dict(dig["inputs"][t["input"]])
            lo, hi = tin.pop("slice")
            if hi != a.records or a.window < hi - lo or a.threshold != 0.5 or not _same_input(mine, tin) or arr is None:
                continue
            tail = ld_tail_lines(text, record_pos(arr, lo))
            got_t = hashlib.sha256(head + tail).hexdigest()
            case += "+" + nm
            what += "; sha256 of the pair lines with VAR1 >= variant %d vs the reference on variants [%d, %d)" % (
                lo, lo, hi)
            if got_t != t["stdout"]["sha256"]:
                got, want = got_t, t["stdout"]["sha256"]
    if got != want:
        if os.environ.get("VCFX_BENCH_ABLATION"):  # diagnostic builds (results invalid by design)
            return {"checked": True, "match": False, "case": case, "what": what}
        raise AssertionError("bench output differs from the reference: %s (%s != %s)" % (what, got, want))
    return {"checked": True, "match": True, "case": case, "what": what}


def _walls(records, walls, skip=0):
    """an e2e leg: the best wall's rate as `value` and the median wall's beside it"""
    w = sorted(walls[skip:])
    med = w[len(w) // 2] if len(w) % 2 else 0.5 * (w[len(w) // 2 - 1] + w[len(w) // 2])
    return {"value": records / w[0], "value_median": records / med, "wall_s": [round(x, 4) for x in walls[skip:]],
            "wall_median_s": round(med, 4)}


PCIE_H2D_GBS = 56.0  # pinned H2D measured on MI355X (tools/microbench/h2d_ingest.cpp; spec Gen5 x16 63 GB/s)


def e2e_rates(workload, arr, a, offs=None):
    """End-to-end records/s of the drop-in CLI on this rank's synthetic file: page-cache-warm
    file -> mmap -> H2D -> kernels -> rows -> stdout (/dev/null), wall clock of the whole process
    (HIP runtime start included), best of 3; the same through a pipe (`cat F | tool`, the
    streaming stdin ingest); and the in-process tool call with the device context already open
    (libvcfx_tools, a long-running caller).  Never `value`: the device-resident rate is."""
    import subprocess
    from vcfx_amd import tool_binary, tools
    if workload == "af":
        tool, args = "VCFX_allele_freq_calc", ["-q"]
    elif workload == "nonref":
        tool, args = "VCFX_nonref_filter", []
    elif workload == "hwe":
        tool, args = "VCFX_hwe_tester", ["-q"]
    elif workload == "dose":
        tool, args = "VCFX_dosage_calculator", ["-q"]
    elif workload == "md":
        tool, args = "VCFX_missing_detector", ["-q"]
    elif workload == "ph":
        tool, args = "VCFX_haplotype_phaser", ["-q"]
    elif workload == "pipeline":
        tool, args = "VCFX_record_filter", ["--filter", PIPE_FILTER]
    else:
        return None
    fd, path = tempfile.mkstemp(suffix=".vcf")  # TMPDIR: a disk-backed file system, page cache warm
    os.close(fd)
    try:
        arr.tofile(path)
        exe = tool_binary(tool)
        runs = {}
        for name, cmd in (("process_file", [exe] + args + ["-i", path]),
                          ("process_stdin_pipe", ["bash", "-o", "pipefail", "-c",
                                                  "cat '%s' | '%s' %s" % (path, exe, " ".join("'%s'" % x for x in args))])):
            walls = []
            for _ in range(3):
                t0 = time.perf_counter()
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300)
                walls.append(time.perf_counter() - t0)
                assert r.returncode == 0, r.stderr[-500:]
            runs[name] = _walls(a.records, walls)
        # in-process (libvcfx_tools' vcfx_tool_main, stdout -> /dev/null): the first call opens
        # the context and is not counted
        import ctypes
        L = tools.lib()
        argv = [tool] + args + ["-i", path]
        carr = (ctypes.c_char_p * (len(argv) + 1))(*[x.encode() for x in argv], None)
        dn = os.open(os.devnull, os.O_RDWR)
        walls = []
        try:
            for _ in range(4):
                t0 = time.perf_counter()
                rc = L.vcfx_tool_main(tool.encode(), len(argv), carr, dn, dn, dn)
                walls.append(time.perf_counter() - t0)
                assert rc == 0, rc
        finally:
            os.close(dn)
        runs["warm_context_file"] = dict(_walls(a.records, walls, 1),
                                         note="in-process vcfx_tool_main with the device context already open")
        # the BGZF (.vcf.gz) form of the same file: the compressed bytes cross PCIe and every member
        # is inflated on the device (vcfxg_ingest_bgzf); the host-inflate path beside it
        # (VCFX_BGZF_DEVICE=0: members inflated on <= 16 host threads, the text crosses PCIe)
        bgz = path + ".bgz"
        subprocess.check_call([os.path.join(REPO, "build", "bin", "vcfx_bgzf"), path, bgz, "16", "1"])
        try:
            import hashlib
            plain_sha = hashlib.sha256(subprocess.run([exe] + args + ["-i", path], capture_output=True,
                                                      timeout=300).stdout).hexdigest()
            for name, env in (("process_file_bgzf", {}), ("process_file_bgzf_host_inflate", {"VCFX_BGZF_DEVICE": "0"})):
                walls = []
                for _ in range(3):
                    t0 = time.perf_counter()
                    r = subprocess.run([exe] + args + ["-i", bgz], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                       timeout=300, env=dict(os.environ, **env))
                    walls.append(time.perf_counter() - t0)
                    assert r.returncode == 0, r.stderr[-500:]
                out = subprocess.run([exe] + args + ["-i", bgz], capture_output=True, timeout=300,
                                     env=dict(os.environ, **env)).stdout
                runs[name] = {**_walls(a.records, walls), "compressed_bytes": os.path.getsize(bgz),
                              "stdout_equals_plain_input": hashlib.sha256(out).hexdigest() == plain_sha,
                              "note": "BGZF level 1 (build/bin/vcfx_bgzf); " + (
                                  "members inflated on the host (<= 16 threads)" if env else
                                  "members inflated on the device (vcfxg_ingest_bgzf)")}
            argv = [tool] + args + ["-i", bgz]
            carr = (ctypes.c_char_p * (len(argv) + 1))(*[x.encode() for x in argv], None)
            dn = os.open(os.devnull, os.O_RDWR)
            walls = []
            try:
                for _ in range(4):
                    t0 = time.perf_counter()
                    rc = L.vcfx_tool_main(tool.encode(), len(argv), carr, dn, dn, dn)
                    walls.append(time.perf_counter() - t0)
                    assert rc == 0, rc
            finally:
                os.close(dn)
            runs["warm_context_bgzf"] = dict(_walls(a.records, walls, 1),
                                             note="in-process vcfx_tool_main on the BGZF file, device context open")
        finally:
            os.unlink(bgz)
        # per-invocation start-up: the drop-in process on a small input (the first 100 records),
        # the reference's own binary on the same bytes beside it (best of 5 each)
        if offs is not None:
            small = path + ".small.vcf"
            arr[:int(offs[min(100, len(offs) - 1)])].tofile(small)
            try:
                lat = {}
                for name, ex in (("drop_in", exe), ("reference", os.path.join(REF_DIR, tool))):
                    if not os.access(ex, os.X_OK):
                        continue
                    walls = []
                    for _ in range(5):
                        t0 = time.perf_counter()
                        r = subprocess.run([ex] + args + ["-i", small], stdout=subprocess.DEVNULL,
                                           stderr=subprocess.PIPE, timeout=120)
                        walls.append(time.perf_counter() - t0)
                        assert r.returncode == 0, r.stderr[-500:]
                    lat[name + "_s"] = round(min(walls), 4)
                    lat[name + "_median_s"] = round(sorted(walls)[len(walls) // 2], 4)
                lat["input"] = "first 100 records (%.1f MB)" % (os.path.getsize(small) / 1e6)
                runs["small_input_latency"] = lat
            finally:
                os.unlink(small)
        # the pipe-ingest ceiling on this host: `cat F | vcfx_pipe_ceiling`, the drop-in's own
        # stdin reader (Input::read_fd, host_copy = false: pipe size, prefaulted head, pinned
        # 16 x 1 MiB ring) with the device stage stubbed -- what the tool adds on top is the
        # device; best of 3.  (`cat F | vcfx_drain` in the ring's shape, r03-r04's stand-in, is
        # kept beside it for continuity: a bare read loop, no head, no ring hand-off.)
        for name, exe, extra in (("pipe_ceiling", "vcfx_pipe_ceiling", ""),
                                 ("pipe_drain_ring16x1M", "vcfx_drain", " 1048576 16")):
            exe = os.path.join(REPO, "build", "bin", exe)
            if not os.access(exe, os.X_OK):
                continue
            walls = []
            for _ in range(3):
                t0 = time.perf_counter()
                subprocess.run(["bash", "-o", "pipefail", "-c", "cat '%s' | '%s'%s" % (path, exe, extra)],
                               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=300, check=True)
                walls.append(time.perf_counter() - t0)
            runs[name] = _walls(a.records, walls)
        if "pipe_ceiling" in runs:
            runs["pipe_ceiling"]["what"] = "cat F | vcfx_pipe_ceiling (the tool's reader, device stage stubbed)"
            runs["process_stdin_pipe"]["frac_of_pipe_ceiling"] = round(
                runs["process_stdin_pipe"]["value"] / runs["pipe_ceiling"]["value"], 3)
        if "pipe_drain_ring16x1M" in runs:  # (r03-r04's ceiling: a bare read loop, comparable across rounds)
            runs["process_stdin_pipe"]["frac_of_drain_ceiling"] = round(
                runs["process_stdin_pipe"]["value"] / runs["pipe_drain_ring16x1M"]["value"], 3)
        runs["pcie_ceiling"] = a.records / (arr.size / (PCIE_H2D_GBS * 1e9))
        runs["unit"] = "records/s"
        runs["cmd"] = "%s %s -i FILE > /dev/null (page-cache-warm %.2f GB file)" % (tool, " ".join(args), arr.size / 1e9)
        return runs
    finally:
        os.unlink(path)


def launch_ranks(a):
    """`--gpus N` outside torchrun: start the N ranks as children (torch.distributed.run on
    127.0.0.1, one process per GPU) and return their exit code.  Nothing here has touched the
    GPU, and the ranks are children, not an exec of this process."""
    import socket
    import subprocess
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.stderr.write("bench.py: --gpus %d but WORLD_SIZE=%d\n" % (a.gpus, world))
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = torch = None
    if world > 1:
        # torch first: its HIP runtime (same soname) then serves libvcfx_gpu.so too
        import torch
        import torch.distributed as dist
        if a.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # gloo rehearsal: ranks may share a GPU
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
    from vcfx_amd import engine, synth

    ld = a.workload == "ld"
    general = a.format != "gt" or a.missing_rate > 0 or a.irregular_rate > 0
    arr, offs = synth.generate_array(rec_offsets=True, **input_params(a, rank))
    ds = engine.data_start_of(arr[:1 << 20].tobytes(), strip_cr=not ld)
    eng = engine.Engine(local)
    eng.load(arr)
    region_bytes = arr.size - ds

    red = None
    if dist is not None:
        red = torch.zeros(4, dtype=torch.int64, device="cuda" if a.dist_backend == "nccl" else "cpu")

    def allreduce_counts(vals):
        # global allele-count reduction over RCCL (configs[3]); per-rank outputs stay local
        red.copy_(torch.tensor(vals, dtype=torch.int64))
        dist.all_reduce(red)
        return red

    if a.workload == "af":
        def step():
            s = eng.allele_freq_region(ds, engine.MODE_FILE)  # index + counts + rows
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.data_lines, s.text_bytes])
            return s
        kern_names = ("line_count", "line_emit", "line_compact", "af_records", "af_walk", "walk_compact", "af_complex",
                      "af_rows", "af_format")
    elif a.workload == "nonref":
        def step():
            s = eng.nonref_filter_region(ds, engine.MODE_FILE)  # (the walk) per-record "every sample hom-ref"
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.data_lines, s.general_records])
            return s
        kern_names = ("fq_walk", "fq_rest", "line_count", "line_emit", "line_compact", "nr_records")
    elif a.workload == "hwe":
        def step():
            s = eng.hwe_region(ds, engine.MODE_FILE)  # (the walk) genotype classes + row rules + rows
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.text_bytes, s.general_records])
            return s
        kern_names = ("hwe_walk", "walk_compact", "hwe_lines", "hwe_rows", "hwe_format", "line_count", "line_emit",
                      "line_compact")
    elif a.workload == "dose":
        def step():
            s = eng.dosage_region(ds, engine.MODE_FILE)  # index + per-sample dosages + rows
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.text_bytes, s.general_records])
            return s
        kern_names = ("dose_walk", "walk_compact", "line_count", "line_emit", "line_compact", "dose_len", "dose_rows",
                      "dose_fmt")
    elif a.workload == "ac":
        ac_names = ["S%05d" % (k + 1) for k in range(a.samples)]
        ac_idx = list(range(a.samples))

        def step():
            L = eng.index(ds)
            s = eng.allele_counter(0, L, ac_idx, ac_names, seq=0, kind=0)  # every (record, sample) row
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.text_bytes, s.general_records])
            return s
        kern_names = ("line_count", "line_emit", "line_compact", "ac_len", "ac_fmt")
    elif a.workload == "md":
        def step():
            s = eng.missing_region(ds, engine.MODE_FILE)  # index + per-record missing-genotype test
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.data_lines, s.general_records])
            return s
        kern_names = ("line_count", "line_emit", "line_compact", "md_lines", "md_walk", "md_rest")
    elif a.workload == "ph":
        def step():
            s = eng.haplotype_phaser(ds, engine.MODE_FILE, 0.8, a.samples)  # parse + consecutive-variant LD
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.text_bytes, 0])
            return s
        kern_names = ("line_count", "line_emit", "line_compact", "ph_lines", "ph_pairs", "ph_fmt")
    elif a.workload == "pipeline":
        # FILTER==PASS;AF>=0.01 as VCFX_record_filter's parseCriteria compiles it
        crits = [(engine.FILTER, engine.EQ, 0, 0.0, "FILTER", "PASS"), (engine.INFO, engine.GE, 1, 0.01, "AF", "")]

        def step():
            s = eng.filter_query_region(ds, crits, PIPE_QUERY, and_logic=True, strict=False)  # RF + GQ
            if red is not None:
                allreduce_counts([s.n_lines, s.rows, s.data_lines, s.warn_lines])
            return s
        kern_names = ("fq_walk", "fq_rest", "line_count", "line_emit", "line_compact", "rf_records", "gq_records")
    else:
        W = a.window

        def step():
            m = eng.ld_prepare_region(ds, a.samples)  # (the LD walk: no separate index sweep)
            np_, tb = eng.ld_stream_chunk(0, m, W, a.threshold)
            if red is not None:
                allreduce_counts([m, np_, tb, 0])
            return m, np_, tb
        kern_names = ("line_count", "line_emit", "line_compact", "ld_walk", "ld_parse", "ld_compact", "ld_pack", "ld_gather",
                      "ld_sparse_prep", "ld_pack_vq", "ld_count",
                      "ld_emit", "ld_count_sparse", "ld_count_mask", "ld_emit_mask", "ld_count_gen", "ld_emit_gen",
                      "ld_text")

    s = None
    for _ in range(max(a.warmup - 1, 0)):
        s = step()

    def stats():
        out = {}
        for k in kern_names:
            tot, n = eng.kernel_stats(k)
            if n:
                out[k] = tot / n
        return out

    # the last warmup step with every kernel timed (the per-kernel breakdown, untimed): it names
    # the dominant kernel, the only one with HIP events in the timed steps (an event pair per
    # launch, read after the loop)
    kernels, dom_k = {}, None
    if a.warmup > 0:
        eng.set_profiling(True)
        eng.reset_kernel_stats()
        s = step()
        kernels = stats()
        dom_k = max(kernels, key=kernels.get) if kernels else None
        eng.set_profiling_only(dom_k)

    def barrier():
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    eng.set_profiling(True)
    eng.reset_kernel_stats()
    barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s = step()
    barrier()
    dt = time.perf_counter() - t0
    eng.set_profiling(False)
    eng.set_profiling_only(None)
    kernels.update(stats())  # (the dominant kernel: its launches in the timed steps)
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    if ld:
        m, np_, tb = s
        assert m == a.records, (m, a.records)
        W = min(a.window, m)
        pairs = (m * (m - 1) // 2) if W >= m - 1 else (W * (W - 1) // 2 + (m - W) * W)
        units_total = pairs * world
        unit, metric = "r2-pairs/s", "r2-pairs/sec (and MFMA TOP/s vs peak), %dK var window x %d samp" % (
            a.records // 1000, a.samples)
    else:
        assert (s.rows > 0 or a.workload == "md") and s.n_lines == a.records, (s.rows, s.n_lines)
        if a.workload == "af" and not general:
            assert s.rows == a.records and s.general_records == 0
        if a.workload == "hwe" and not general:
            assert s.general_records == 0
        units_total = a.records * world
        unit, metric = "records/s", METRIC
    value = units_total * a.steps / dt

    if rank == 0:
        L = a.records
        if ld:
            # X.X^T over the window pairs (complete genotypes) on the FP4 MFMA: 2 ops per sample
            # per pair, priced against the dense FP4 peak the kernel's instruction runs at
            # the count kernel of the data: k_ld_fast (complete 256-groups, X.X^T) or, with
            # missing calls, k_ld_mask (the six masked sums: 6x the executed MFMA ops); the
            # algorithmic ops are the same 2 N per window pair either way
            # (k_ld_fast<1, true>: sparse-missing 256-groups, one X.X^T product plus the sparse
            # corrections -- executed ops = algorithmic ops)
            dom = max(("ld_count", "ld_count_sparse", "ld_count_mask"), key=lambda k: kernels.get(k, 0))
            algo_ops = 2.0 * a.samples * pairs
            ach = algo_ops / (kernels[dom] * 1e-3) / 1e12
            roof = {"bound": "mfma", "kernel": dom, "achieved": ach, "peak": FP4_PEAK_TOPS, "unit": "TOP/s",
                    "frac": ach / FP4_PEAK_TOPS, "traffic": pmc_traffic("ld", dom),
                    "algorithmic_ops_per_launch": algo_ops, "avg_launch_ms": kernels[dom]}
            if dom == "ld_count_mask":
                # executed: 6 products over the 128 x 128 tiles the kernel ran (whole tiles)
                roof["executed_ops_per_launch"] = 6.0 * algo_ops
                roof["executed_frac"] = 6.0 * algo_ops / (kernels[dom] * 1e-3) / 1e12 / FP4_PEAK_TOPS
            try:  # MFMA-busy fraction of the SIMD cycles (committed PMC pass of k_ld_fast, profiles/)
                if dom != "ld_count":
                    raise KeyError(dom)
                with open(MFMA_FILE) as f:
                    m = json.load(f)["mean"]
                roof["mfma_util_pmc"] = {"util": m["mfma_util"], "clock_ghz": m["clock_ghz"],
                                         "source": os.path.relpath(MFMA_FILE, REPO)}
            except (OSError, KeyError, ValueError):
                pass
        else:
            tb = s.text_bytes
            algo = {   # algorithmic bytes per launch
                "line_count": region_bytes,
                "line_emit": region_bytes + 8 * L,
                "af_records": region_bytes + L * (8 + 13),      # record bytes + line_end + per-line results
                # walk (no index sweep): the record bytes once + per line its region results
                # (line_end 8, counts/prefix/status 13, head record 16); the compaction reads
                # and rewrites them dense; the per-line rest reads head record + status
                "af_walk": region_bytes + L * (8 + 13 + 16),
                # HWE: the same walk with three class counts per line (8 + 17 + 16)
                "hwe_walk": region_bytes + L * (8 + 17 + 16),
                # dosage: pass 1 reads the records (+ line end, status, length, meta per line);
                # pass 2 reads them again and writes the rows (2 bytes per sample)
                "dose_len": region_bytes + L * (8 + 1 + 8 + 24),
                # the dosage walk (records of >= 512 B): the record bytes once + per line its
                # region results (line end 8, samples / NA 8, status 1, head record 16)
                "dose_walk": region_bytes + L * (8 + 8 + 1 + 16),
                "dose_fmt": region_bytes + tb + L * (8 + 1 + 8 + 24),
                # allele counter: pass 1 reads the records (+ line end, status, length, meta per
                # line); pass 2 reads each selected sample's GT (the records again) and writes the rows
                "ac_len": region_bytes + L * (8 + 1 + 8 + 48),
                "ac_fmt": region_bytes + tb + L * (8 + 1 + 8 + 48),
                # missing detector: the records once + line end, status and the INFO span per line
                "md_lines": region_bytes + L * (8 + 1 + 8),
                # its walk (long GT-only records): the record bytes once + line end, status and
                # head record per line; the rest compacts them and reads status + line ends
                "md_walk": region_bytes + L * (8 + 1 + 16),
                # phaser: the records once + a genotype code per sample + line end, status, flag
                # and the per-line record (24 B); the pairs read each code row twice
                "ph_lines": region_bytes + L * (a.samples + 8 + 1 + 4 + 24),
                "ph_pairs": L * (2 * a.samples + 2 * 8 + 2 * 24 + 1 + 8 + 8),
                "walk_compact": L * 2 * (8 + 13 + 16),
                # the per-line rest: its lines' record bytes when the data are off the fixed-stride
                # layout (every line a GT:AD:DP record), else the head record + status per line
                "af_complex": (region_bytes if a.format != "gt" else 0) + L * (16 + 1),
                "af_format": tb + L * (8 + 8 + 13) + s.rows * 40,
                "af_rows": L * (5 + 8 + 8 + 8),
                "rf_records": region_bytes + L * (8 + 1),
                "gq_records": region_bytes + L * (8 + 2),
                # filter / query walk (no index sweep): the record bytes once + per line its
                # region results (line_end 8, status 1, head record 16, tab offsets 16); the rest
                # compacts them (read + write) and reads status + head record + tabs once more
                # (nonref: the walk stops each record's sweep at its first non-hom-ref sample and
                # scans the rest for the '\n' only when its end was predicted, so fq_walk's bytes are
                # counted as the whole region, as for the query walk)
                "fq_walk": region_bytes + L * (8 + 1 + 16 + (16 if a.workload == "pipeline" else 0)),
                "fq_rest": L * (2 * (8 + 1 + 16 + 16) + 16 + 1 + 16),
            }
            dom = max((k for k in kernels if k in algo), key=kernels.get)
            ach = algo[dom] / (kernels[dom] * 1e-3) / 1e9
            roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS,
                    # (the committed PMC pass is of the default data: none for the general-path shapes)
                    "traffic": None if general else pmc_traffic(a.workload, dom),
                    "algorithmic_bytes_per_launch": int(algo[dom]), "avg_launch_ms": kernels[dom]}
        if general:
            extra = " [data: FORMAT=%s, missing rate %g, irregular rate %g: the general GT path]" % (
                a.format.upper(), a.missing_rate, a.irregular_rate)
        else:
            extra = ""
        workload = {
            "af": "VCFX_allele_freq_calc -i (file path) on a device-resident %d x %d VCF shard per GPU: the walk "
                  "(line ends + allele counts + rows composed in LDS) + the rows in file order" % (a.records, a.samples),
            "pipeline": "VCFX_record_filter --filter '%s' | VCFX_genotype_query -g '%s' fused, device-resident "
                        "%d x %d annotated shard per GPU" % (PIPE_FILTER, PIPE_QUERY, a.records, a.samples),
            "nonref": "VCFX_nonref_filter -i (file path) on a device-resident %d x %d shard per GPU: the walk "
                      "with the per-record all-samples-hom-ref test" % (a.records, a.samples),
            "hwe": "VCFX_hwe_tester -i (file path) on a device-resident %d x %d shard per GPU: the walk with the "
                   "genotype-class reducer + HWE chi-square p-value rows" % (a.records, a.samples),
            "dose": "VCFX_dosage_calculator -i (file path) on a device-resident %d x %d shard per GPU: index + "
                    "per-sample dosage rows (2 output bytes per sample)" % (a.records, a.samples),
            "ac": "VCFX_allele_counter -i (file path, per-sample text rows) on a device-resident %d x %d shard per "
                  "GPU: index + per-(record, sample) REF/ALT counts + %d rows per record" % (a.records, a.samples,
                                                                                            a.samples),
            "ph": "VCFX_haplotype_phaser -i (file path, default mode, -l 0.8) on a device-resident %d x %d shard "
                  "per GPU: parse to genotype codes + consecutive-variant r^2 + entries" % (a.records, a.samples),
            "md": "VCFX_missing_detector -i (file path) on a device-resident %d x %d shard per GPU: index + the "
                  "per-record missing-genotype test" % (a.records, a.samples),
            "ld": "VCFX_ld_calculator -w %d -t %g streaming on a device-resident %d x %d shard per GPU: parse + "
                  "FP4-MFMA pair sums (count + emit) + pair text" % (a.window, a.threshold, a.records, a.samples),
        }[a.workload] + extra
        out = {
            "metric": metric,
            "value": value,
            "unit": unit,
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp4(e2m1)->f32" if ld else "u8",
            "data": "synthetic: vcfx_synth seed %d+rank, chr21-like layout (FORMAT=%s, phased a|b, INFO=%s)"
                    % (input_params(a, 0)["seed"], a.format.upper(),
                       "AF=..;DP=.." if a.workload == "pipeline" else ".") + (", founder-haplotype blocks" if ld else ""),
            "config": {"workload": workload, "records_per_gpu": a.records, "samples": a.samples,
                       "bytes_per_gpu": int(arr.size),
                       "parallelism": "record-sharded x%d%s" % (world, ", RCCL all-reduce of global counts"
                                                                if world > 1 else "")},
            "roofline": roof,
            "kernels_ms": kernels,
            "kernels_ms_source": "%s: HIP events on the engine stream over the timed steps; the others: one "
                                 "profiled warmup step" % (dom_k or "every kernel"),
            "pipeline_input_gbps": region_bytes * world * a.steps / dt / 1e9,
        }
        if ld:
            out["pairs_per_gpu"] = pairs
            out["pairs_emitted"] = np_
        out["output_check"] = ({"checked": False, "match": None, "what": "--no-output-check (diagnostic run)"}
                           if a.no_output_check else output_check(a.workload, eng, s, a, rank, arr))
        if world == 1 and not a.no_e2e and not general:
            out["e2e"] = e2e_rates(a.workload, arr, a, offs)
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.workload, arr, offs, a)
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
