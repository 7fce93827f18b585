#!/usr/bin/env python3
"""Golden digests at BASELINE scale (test infrastructure).

Runs the REFERENCE binaries (built from /root/reference sources by oracle/Makefile.ref into
oracle/_ref/) on the deterministic synthetic workloads of BASELINE.json configs 2, 3 and 5
(and the nonref widening), and records, per case, the sha256 / length / line count of the
reference's stdout, its exit code, and -- for the record filters -- the sha256 of the kept-
record bitmap (np.packbits over the data records, in file order).  The C restatement
(oracle/_build/vcfx_oracle) is run on the same inputs and must agree byte for byte, so the
oracle is pinned at full size too.

Output: tests/golden/full_digests.json, read by tests/test_gpu_scale.py and by bench.py's
output check.  The synthetic inputs are regenerated from their parameters (vcfx_synth is
counter-based: the bytes do not depend on thread count or host), so only digests are
committed.  Needs ~10 GB of /tmp and a few minutes of CPU.

    python tests/golden/make_full_digests.py [--out PATH] [case-name ...]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = os.path.join(REPO, "oracle", "_ref")
ORACLE_CLI = os.path.join(REPO, "oracle", "_build", "vcfx_oracle")
OUT = os.path.join(HERE, "full_digests.json")

# synthetic inputs: vcfx_synth parameters (records, samples, seed, info, missing, hap, irregular, crlf)
INPUTS = {
    # configs 2 / 4: the bench's chr21-like shard (rank 0)
    "chr21": dict(n_records=427409, n_samples=2504, seed=20251226),
    # config 3: annotated INFO (AF=..;DP=..) for the INFO predicate
    "annot": dict(n_records=427409, n_samples=2504, seed=20251227, info_mode=1),
    # config 5: LD -- 1,500 variants with founder-haplotype blocks and sparse missing calls:
    # variants 96 and 848 carry a missing call, so the 256-variant groups 0 and 3 are knocked
    # out (int8 kernel) and groups 1, 2, 4, 5 are complete (FP4 kernel, 20 k-slices each)
    "ld1500": dict(n_records=1500, n_samples=2504, seed=79, hap_blocks=1, missing_rate=4e-7),
    # config 5: the first 3,000 variants of the bench's LD shard (seed 20251226, hap blocks);
    # with a 100 K window their pairs are the first pairs of the bench's own output
    "ld3000": dict(n_records=3000, n_samples=2504, seed=20251226, hap_blocks=1),
    # the chr21-like shard with sparse missing calls (".|." at rate 5e-4: about 70 % of the
    # records carry one) for VCFX_missing_detector's flagging path
    "chr21_miss": dict(n_records=427409, n_samples=2504, seed=20251226, missing_rate=5e-4),
    # config 5: the first 20,000 variants of the bench's LD shard (1.9995e8 window pairs, every
    # tile row of the first 20 K rows: the staging and row offsets past 3 K rows, tiles far from
    # the diagonal)
    "ld20k": dict(n_records=20000, n_samples=2504, seed=20251226, hap_blocks=1),
    # config 5 with missing calls (bench.py --workload ld --missing-rate 0.001: ~8 % of the
    # variants complete, so nearly every tile takes the masked FP4 kernel)
    "ld20k_miss": dict(n_records=20000, n_samples=2504, seed=20251226, hap_blocks=1, missing_rate=0.001),
    # the general GT path at BASELINE scale: every record GT:AD:DP (bench.py --format gt:ad:dp)
    "chr21_gtadp": dict(n_records=427409, n_samples=2504, seed=20251226, format_mode=1),
    # 5 % of the records in a general-path shape (bench.py --irregular-rate 0.05)
    "chr21_irreg": dict(n_records=427409, n_samples=2504, seed=20251226, irregular_rate=0.05),
    # config 3's annotated shard with sparse missing calls
    "annot_gtadp": dict(n_records=427409, n_samples=2504, seed=20251227, info_mode=1, format_mode=1),
    "annot_miss": dict(n_records=427409, n_samples=2504, seed=20251227, info_mode=1, missing_rate=5e-4),
    # config 5 past its first 20 K variants: the header + variants [80,000, 100,000) of the bench's
    # 100 K LD shard (complete, and with 0.1 % missing calls).  With W = 100 K every pair of the
    # slice is in the window, and the reference streams each variant's pairs oldest -> newest, so
    # its output on the slice is exactly the full 100 K run's lines whose VAR1 is variant >= 80,000
    # (tests/test_gpu_scale.py filters the GPU's full run by VAR1_POS: positions strictly increase)
    "ld100k_tail": dict(n_records=100000, n_samples=2504, seed=20251226, hap_blocks=1, slice=[80000, 100000]),
    "ld100k_miss_tail": dict(n_records=100000, n_samples=2504, seed=20251226, hap_blocks=1, missing_rate=0.001,
                             slice=[80000, 100000]),
}

AF, RF, GQ, LD, NR, HWE = ("VCFX_allele_freq_calc", "VCFX_record_filter", "VCFX_genotype_query",
                           "VCFX_ld_calculator", "VCFX_nonref_filter", "VCFX_hwe_tester")
DOSE = "VCFX_dosage_calculator"
AC, MD, PH = "VCFX_allele_counter", "VCFX_missing_detector", "VCFX_haplotype_phaser"
# 50 sample names of the synthetic header (S00001..S02504) in a scrambled order: the MT path's
# per-slot lookup and the stream path's forward-only cursor differ on it
SEL50 = " ".join("S%05d" % (1 + (k * 1597) % 2504) for k in range(50))

# name -> (input, [stage argv ...] with "{F}" for the file; the first stage reads stdin when
# it has no {F}), keep-mask flag
CASES = {
    "af_file": ("chr21", [[AF, "-q", "-i", "{F}"]], False),
    "af_stdin": ("chr21", [[AF, "-q"]], False),
    "nonref_file": ("chr21", [[NR, "-i", "{F}"]], True),
    "hwe_file": ("chr21", [[HWE, "-q", "-i", "{F}"]], False),
    "hwe_stdin": ("chr21", [[HWE]], False),
    "dose_file": ("chr21", [[DOSE, "-q", "-i", "{F}"]], False),
    "pipeline_bench": ("chr21", [[RF, "--filter", "QUAL>=30;FILTER==PASS", "-i", "{F}"],
                                 [GQ, "--genotype-query", "0|1"]], True),
    "pipeline_annot": ("annot", [[RF, "--filter", "FILTER==PASS;AF>=0.01", "-i", "{F}"],
                                 [GQ, "-g", "0/1"]], True),
    "gq_strict_annot": ("annot", [[GQ, "-g", "1|1", "--strict", "-i", "{F}"]], True),
    # the stream (stdin) paths of the pass-through tools: fed through a pipe by the tests
    "nonref_stdin": ("chr21", [[NR]], True),
    "rf_stdin_annot": ("annot", [[RF, "--filter", "FILTER==PASS;AF>=0.01"]], True),
    "ld1500_t02": ("ld1500", [[LD, "-q", "-w", "1500", "-t", "0.2", "-i", "{F}"]], False),
    "ld1500_t0": ("ld1500", [[LD, "-q", "-w", "1500", "-t", "0", "-i", "{F}"]], False),
    "ld1500_w300_t0": ("ld1500", [[LD, "-q", "-w", "300", "-t", "0", "-i", "{F}"]], False),
    "ac_bin_file": ("chr21", [[AC, "-q", "-b", "-i", "{F}"]], False),
    "ac_agg_file": ("chr21", [[AC, "-q", "-a", "-i", "{F}"]], False),
    "ac_sel_file": ("chr21", [[AC, "-q", "-s", SEL50, "-i", "{F}"]], False),
    "ac_sel_stdin": ("chr21", [[AC, "-q", "-s", SEL50]], False),
    "md_file": ("chr21", [[MD, "-q", "-i", "{F}"]], False),
    "md_file_miss": ("chr21_miss", [[MD, "-q", "-i", "{F}"]], False),
    "md_stdin_miss": ("chr21_miss", [[MD]], False),
    "ph_file": ("chr21", [[PH, "-q", "-i", "{F}"]], False),
    "ph_stream_stdin": ("chr21", [[PH, "-q", "-s", "-w", "50", "-l", "0.5"]], False),
    "ph_ld3000": ("ld3000", [[PH, "-l", "0.3", "-i", "{F}"]], False),
    "ld3000_bench": ("ld3000", [[LD, "-q", "-w", "100000", "-t", "0.5", "-i", "{F}"]], False),
    "ld20k_bench": ("ld20k", [[LD, "-q", "-w", "100000", "-t", "0.5", "-i", "{F}"]], False),
    "ld20k_miss_bench": ("ld20k_miss", [[LD, "-q", "-w", "100000", "-t", "0.5", "-i", "{F}"]], False),
    # a three-stage chain (vcfx_pipe's fused schedule): config 3's filter and query feeding AF
    "pipeline_annot_af": ("annot", [[RF, "--filter", "FILTER==PASS;AF>=0.01", "-i", "{F}"], [GQ, "-g", "0/1"], [AF]],
                          False),
    "pipeline_annot_nr_af": ("annot", [[GQ, "-g", "0/1", "-i", "{F}"], [NR], [AF, "-q"]], False),
    "ld100k_tail_bench": ("ld100k_tail", [[LD, "-q", "-w", "100000", "-t", "0.5", "-i", "{F}"]], False),
    "ld100k_miss_tail_bench": ("ld100k_miss_tail", [[LD, "-q", "-w", "100000", "-t", "0.5", "-i", "{F}"]], False),
    "af_file_miss": ("chr21_miss", [[AF, "-q", "-i", "{F}"]], False),
    "af_stdin_miss": ("chr21_miss", [[AF, "-q"]], False),
    "af_file_gtadp": ("chr21_gtadp", [[AF, "-q", "-i", "{F}"]], False),
    "af_stdin_gtadp": ("chr21_gtadp", [[AF, "-q"]], False),
    "af_file_irreg": ("chr21_irreg", [[AF, "-q", "-i", "{F}"]], False),
    "pipeline_annot_miss": ("annot_miss", [[RF, "--filter", "FILTER==PASS;AF>=0.01", "-i", "{F}"],
                                           [GQ, "-g", "0/1"]], True),
    "pipeline_annot_gtadp": ("annot_gtadp", [[RF, "--filter", "FILTER==PASS;AF>=0.01", "-i", "{F}"],
                                             [GQ, "-g", "0/1"]], True),
}


def generate(params):
    """(bytes, data-record offsets) of an input; a "slice": [a, b) input is the header of the
    generated file followed by its data records a .. b-1 (offsets rebased to the slice)."""
    from vcfx_amd import synth
    params = dict(params)
    sl = params.pop("slice", None)
    arr, offs = synth.generate_array(rec_offsets=True, **params)
    if sl is None:
        return arr, offs
    a, b = sl
    h = int(offs[0])
    out = np.concatenate([arr[:h], arr[int(offs[a]):int(offs[b])]])
    o2 = offs[a:b + 1] - offs[a] + np.uint64(h)
    return out, o2


def keep_mask(arr, offs, out):
    """Bitmap of the data records that appear (in order, byte-identical) among out's data lines."""
    n = len(offs) - 1
    keep = np.zeros(n, np.uint8)
    mv = memoryview(arr)
    # first data record: the record offsets index data records only
    k = 0
    for line in out.split(b"\n"):
        if not line or line[:1] == b"#":
            continue
        while k < n:
            s, e = int(offs[k]), int(offs[k + 1]) - 1  # without its '\n'
            k += 1
            if e - s == len(line) and mv[s:e] == line:
                keep[k - 1] = 1
                break
        else:
            raise AssertionError("output line not found among the records")
    return keep


def digest(b):
    return {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b), "lines": b.count(b"\n")}


def run_chain(bindir_fn, stages, path):
    data, rc_all = None, []
    for i, st in enumerate(stages):
        argv = [a.replace("{F}", path) for a in st]
        exe = bindir_fn(argv[0])
        if data is None and "{F}" not in " ".join(st):
            with open(path, "rb") as f:
                r = subprocess.run([exe] + argv[1:], stdin=f, capture_output=True)
        else:
            r = subprocess.run([exe] + argv[1:], input=data if data is not None else b"", capture_output=True)
        rc_all.append(r.returncode)
        data = r.stdout
    return data, rc_all


def main(names, out_path=OUT):
    try:
        with open(out_path) as f:
            doc = json.load(f)
    except OSError:
        doc = {"inputs": {}, "cases": {}}
    doc["about"] = ("reference (oracle/_ref, built from /root/reference sources) stdout digests on the synthetic "
                    "BASELINE-scale inputs; generated by tests/golden/make_full_digests.py")
    doc["inputs"] = INPUTS
    names = names or list(CASES)
    by_input = {}
    for nm in names:
        by_input.setdefault(CASES[nm][0], []).append(nm)
    tmpdir = os.environ.get("TMPDIR", "/tmp")
    for inp, nms in by_input.items():
        t0 = time.time()
        arr, offs = generate(INPUTS[inp])
        # record offsets from the generator start at the first data record
        with tempfile.NamedTemporaryFile(suffix=".vcf", dir=tmpdir) as f:
            arr.tofile(f.name)
            print("%s: %d bytes (%.1fs)" % (inp, arr.size, time.time() - t0), flush=True)
            for nm in nms:
                _, stages, want_mask = CASES[nm]
                t0 = time.time()
                # the reference and the oracle run side by side (subprocesses: no GIL contention)
                with ThreadPoolExecutor(2) as ex:
                    fo = ex.submit(run_chain_oracle, stages, f.name)
                    ref_out, ref_rc = run_chain(lambda t: os.path.join(REF, t), stages, f.name)
                    t_ref = time.time() - t0
                    ora_out, ora_rc = fo.result()
                assert ref_rc == ora_rc, (nm, ref_rc, ora_rc)
                assert ref_out == ora_out, "%s: the C oracle differs from the reference at full size" % nm
                c = {"input": inp, "stages": stages, "rc": ref_rc, "stdout": digest(ref_out),
                     "reference_seconds": round(t_ref, 2)}
                if want_mask:
                    m = keep_mask(arr, offs, ref_out)
                    c["kept"] = int(m.sum())
                    c["keep_mask_sha256"] = hashlib.sha256(np.packbits(m).tobytes()).hexdigest()
                doc["cases"][nm] = c
                print("  %s: %s (%.1fs ref)" % (nm, c["stdout"], t_ref), flush=True)
        del arr, offs
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
        f.write("\n")


def run_chain_oracle(stages, path):
    # the C restatement's process form: `vcfx_oracle <tool> args...`
    data, rcs = None, []
    for st in stages:
        argv = [a.replace("{F}", path) for a in st]
        if data is None and "{F}" not in " ".join(st):
            with open(path, "rb") as f:
                r = subprocess.run([ORACLE_CLI] + argv, stdin=f, capture_output=True)
        else:
            r = subprocess.run([ORACLE_CLI] + argv, input=data if data is not None else b"", capture_output=True)
        rcs.append(r.returncode)
        data = r.stdout
    return data, rcs


if __name__ == "__main__":
    # --out PATH: write (and read) another digest file, so long cases can run in parallel
    # processes and be merged into full_digests.json afterwards
    a = sys.argv[1:]
    out = OUT
    if a[:1] == ["--out"]:
        out, a = a[1], a[2:]
    main(a, out)
