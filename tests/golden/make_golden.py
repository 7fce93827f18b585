#!/usr/bin/env python3
"""Generate golden vectors for the five hot-path tools by running the REFERENCE binaries
(built from /root/reference sources by oracle/Makefile.ref into oracle/_ref/) over the
fixtures in tests/golden/data/, in both input modes.

Writes tests/golden/cases.json.gz: the case list, expected exit codes, sha256/length of
stdout and stderr, and (base64) the raw bytes of outputs <= 16 KiB.
Run from anywhere; all tools run with cwd=tests/golden and relative fixture paths so
file names printed by the tools are stable.  argv[0] is the bare tool name.
"""
import base64
import concurrent.futures
import gzip
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")
INLINE_MAX = 16 * 1024

AF, RF, GQ, LD, VC = ("VCFX_allele_freq_calc", "VCFX_record_filter", "VCFX_genotype_query",
                      "VCFX_ld_calculator", "VCFX_variant_counter")
NR = "VCFX_nonref_filter"
HWE = "VCFX_hwe_tester"
DOSE = "VCFX_dosage_calculator"
AC = "VCFX_allele_counter"
MD = "VCFX_missing_detector"
PH = "VCFX_haplotype_phaser"
# the reference's parseGenotypeRaw loops forever on a GT byte other than a digit, '/', '|'
# or '.' (a CRLF line's last sample, for one): such cases are left out (run_case -> None)
HANG_S = 20


def fixtures():
    names = sorted(os.listdir(os.path.join(HERE, "data")))
    out = [os.path.join("data", n) for n in names if n.endswith(".vcf") or n.endswith(".gz")]
    out += [os.path.join("data", "ref", n) for n in sorted(os.listdir(os.path.join(HERE, "data", "ref")))]
    return out


def build_cases():
    cases = []

    def add(tool, args, stdin=None, tag=None):
        name = "%s__%s" % (tool[5:], tag or "_".join(a.replace("/", "-").replace(" ", "") for a in args) or "noargs")
        name = "".join(c if c.isalnum() or c in "._-=+" else "_" for c in name)
        if stdin:
            name += "__stdin_" + os.path.basename(stdin)
        base, k = name, 1
        while any(c["name"] == name for c in cases):
            k += 1
            name = "%s_%d" % (base, k)
        cases.append({"name": name, "tool": tool, "argv": [tool] + list(args), "stdin": stdin})

    fx = fixtures()
    vcfs = [f for f in fx if f.endswith(".vcf")]
    big = {"data/synth_regular.vcf"}
    # ---- allele_freq_calc
    for f in vcfs:
        add(AF, ["-i", f])
        add(AF, [], stdin=f)
        add(AF, ["-q", f])
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"]):
        add(AF, a)
    add(AF, [], stdin="data/empty.vcf", tag="empty_stdin")
    add(AF, ["-q"], stdin="data/ties.vcf")
    # ---- variant_counter
    for f in vcfs + [g for g in fx if g.endswith(".gz")]:
        if not f.endswith(".gz"):
            add(VC, [f])
            add(VC, ["--strict", f])
        add(VC, [], stdin=f)
        add(VC, ["-s"], stdin=f)
    for a in (["-h"], ["-v"], ["--bogus"], ["data/nope.vcf"]):
        add(VC, a)
    # ---- genotype_query
    queries = [["-g", "0/1"], ["-g", "1|1", "--strict"], ["-g", "0|1", "--strict"], ["-g", "1/0"], ["-g", "0/0"],
               ["-g", "1/2"], ["-g", "2|1"], ["-g", "1/x"], ["-g", "x/1"], ["-g", "0"], ["-g", "./."],
               ["-g", "10/1"], ["-g", "0/10"], ["-g", "00/1"], ["--genotype-query=1|1"], ["-g", "1/1", "-q"],
               ["-g", "0/1", "--strict"], ["-g", "./.", "--strict"], ["-g", "1", "--strict"]]
    for f in vcfs:
        qs = queries if f not in big else queries[:4]
        for q in qs:
            add(GQ, q + ["-i", f])
            add(GQ, q, stdin=f)
        add(GQ, ["-g", "0/1", f])
    for a in (["-h"], ["-v"], ["--vers"], [], ["-g"], ["-s", "-g", "0/1"], ["-g", "0/1", "-i", "data/nope.vcf"]):
        add(GQ, a)
    # ---- record_filter
    filters = ["QUAL>=90", "AF>=0.2", "FILTER==PASS", "POS>=30000", "DP>=40", "DP>10", "QUAL<50", "FLAG==FLAG",
               "FLAG>0", "AF!=0.1", "QUAL==0", "FILTER!=PASS", "POS>0x5", "AF>=0.01;DP<=100", "AF<0.05",
               " QUAL > 20 ; FILTER == PASS ", "AF>=0.2;FILTER==PASS", "FILTER>PASS", "AF==nan", "DP==inf",
               "AF>=0.0001", "QUAL>=1e2", "POS<=1500", "AF>.2", "AF>=-0"]
    for f in vcfs:
        fl = filters if f not in big else filters[:3]
        for flt in fl:
            add(RF, ["--filter", flt, "-i", f])
            add(RF, ["-f", flt], stdin=f)
        add(RF, ["--filter", "QUAL>=50;AF>=0.2", "--logic", "or", f])
        add(RF, ["--filter", "QUAL>=50;AF>=0.2", "-l", "or"], stdin=f)
    for a in ([], ["-h"], ["-v"], ["-q"], ["--filter", "QUAL"], ["--filter", "=5"], ["--filter", "QUAL>="],
              ["--filter", "QUAL>1", "--logic", "xor"], ["--filter", ";;"], ["--filter", "QUAL>1", "data/nope.vcf"],
              ["--filter", "QUAL>1", "-"]):
        add(RF, a, stdin="data/ref/record_filter_input.vcf" if a[-1:] == ["-"] else None)
    # ---- ld_calculator
    ldsets = [["-w", "1000"], ["-w", "1"], ["-w", "3"], ["-t", "0.5"], ["-t", "0.2", "-w", "2"], ["-d", "150"],
              ["-r", "1:100-1000"], ["-r", "21:9411239-9420000"], ["-m"], ["-m", "-r", "1:150-500"]]
    for f in vcfs:
        if f in big:
            continue
        for a in ldsets:
            add(LD, a + ["-i", f])
            add(LD, a, stdin=f)
    for a in (["-h"], ["-v"], ["--versi"], ["-w", "x"], ["-t", "y"], ["-r", "bad"], ["-r", "1:9-2"], ["-t", "1e-400"],
              ["-i", "data/empty.vcf"], ["-i", "data/nope.vcf"], ["-w", "-1", "-i", "data/synth_ld.vcf"],
              ["-t", "2", "-i", "data/synth_ld.vcf"], ["-t", "nan", "-i", "data/synth_ld.vcf"], ["-n", "q"],
              ["-d", "-5", "-i", "data/synth_ld.vcf"], ["-w", "0", "-i", "data/synth_ld.vcf"]):
        add(LD, a)
    # ---- nonref_filter: the shared fixtures, the reference's own nonref fixtures and traps
    nr_dir = os.path.join(HERE, "data", "ref_nonref")
    nr_files = vcfs + [os.path.join("data", "ref_nonref", n) for n in sorted(os.listdir(nr_dir))]
    for f in nr_files:
        add(NR, ["-i", f])
        add(NR, [f])
        add(NR, [], stdin=f)
    add(NR, ["-"], stdin="data/ref_nonref/nonref_traps.vcf")
    add(NR, ["--input", "data/ref_nonref/nonref_basic.vcf"])
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"]):
        add(NR, a)
    add(NR, [], stdin="data/empty.vcf", tag="empty_stdin")
    # ---- hwe_tester: the shared fixtures, the reference's own hwe fixtures, the traps
    hwe_dir = os.path.join(HERE, "data", "ref_hwe")
    for f in vcfs + [os.path.join("data", "ref_hwe", n) for n in sorted(os.listdir(hwe_dir))]:
        add(HWE, ["-i", f])
        add(HWE, ["-q", f])
        add(HWE, [], stdin=f)
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"], ["-i", "data/empty.vcf"]):
        add(HWE, a)
    add(HWE, [], stdin="data/empty.vcf", tag="empty_stdin")
    # ---- dosage_calculator: the shared fixtures, the reference test script's fixtures
    # (tests/golden/extract_sh_fixtures.py), the traps
    ddir = os.path.join(HERE, "data", "ref_dosage")
    for f in vcfs + [os.path.join("data", "ref_dosage", n) for n in sorted(os.listdir(ddir)) if n.endswith(".vcf")]:
        add(DOSE, ["-i", f])
        add(DOSE, ["-q", f])
        add(DOSE, [], stdin=f)
        add(DOSE, ["-q"], stdin=f)
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"], ["-i", "data/empty.vcf"]):
        add(DOSE, a)
    add(DOSE, [], stdin="data/empty.vcf", tag="empty_stdin")
    # ---- allele_counter: every mode (the default threaded file path, the unified path of
    # -a / -b / -z / -l, stdin), sample selections, the reference's fixtures and the traps
    adir = os.path.join(HERE, "data", "ref_ac")
    afiles = vcfs + [os.path.join("data", "ref_ac", n) for n in sorted(os.listdir(adir))]
    for f in afiles:
        add(AC, ["-i", f])
        add(AC, ["-q", f])
        add(AC, ["-q", "-a", "-i", f])
        add(AC, ["-q", "-b", "-i", f])
        add(AC, ["-q", "-l", "2", "-i", f])
        add(AC, [], stdin=f)
        add(AC, ["-q"], stdin=f)
        if "ref_ac" in f:
            for a in (["-s", "B"], ["-s", "C A"], ["-s", " B  A "], ["-s", "A A"], ["-s", "Z"], ["-a", "-s", "C A"],
                      ["-l", "1", "-a"], ["-z"], ["-a", "-z"], ["-b", "-l", "3"], ["-t", "3"], ["-l", "0"]):
                add(AC, ["-q"] + a + ["-i", f])
            add(AC, ["-q", "-s", "C A"], stdin=f)
            add(AC, ["-q", "-s", "Z"], stdin=f)
            add(AC, ["-s", "B", "-a", "-l", "1", "-i", f])
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["-s", "-v"], ["-s", "-h"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"], ["-i", "data/empty.vcf"], ["-a", "-i", "data/empty.vcf"], ["--bogus"], ["-"]):
        add(AC, a)
    add(AC, [], stdin="data/empty.vcf", tag="empty_stdin")
    # ---- missing_detector
    mdir = os.path.join(HERE, "data", "ref_md")
    for f in vcfs + [os.path.join("data", "ref_md", n) for n in sorted(os.listdir(mdir))]:
        add(MD, ["-i", f])
        add(MD, ["-q", f])
        add(MD, ["-t", "3", "-i", f])
        add(MD, [], stdin=f)
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"], ["-i", "data/empty.vcf"], ["-t", "0", "-q", "-i", "data/ref_md/md_traps.vcf"]):
        add(MD, a)
    add(MD, [], stdin="data/empty.vcf", tag="empty_stdin")
    # ---- haplotype_phaser: both modes (default / --streaming) in both input forms, the
    # reference test script's fixtures (copied as data) and the traps
    pdir = os.path.join(HERE, "data", "ref_ph")
    for f in vcfs + [os.path.join("data", "ref_ph", n) for n in sorted(os.listdir(pdir))]:
        for a in ([], ["-l", "0.5"], ["-s"], ["-s", "-w", "2"], ["-q"], ["-q", "-s", "-w", "1", "-l", "0.3"]):
            add(PH, a + ["-i", f])
            add(PH, a, stdin=f)
        add(PH, [f])
        if f not in big:
            add(PH, ["-s", "-w", "0", "-i", f])
            add(PH, ["-l", "0", "-i", f])
            add(PH, ["-l", "1", "-s"], stdin=f)
            add(PH, ["-l", "nan", "-i", f])
    for a in (["-h"], ["--help"], ["-v"], ["--version"], ["--bogus"], ["-x"], ["-i"], ["-i", "data/nope.vcf"],
              ["data/nope.vcf"], ["-i", "data/empty.vcf"], ["-l", "x"], ["-l", "1.5"], ["-l", "-0.1"], ["-l", "1e-400"],
              ["-l", " 0.5", "-i", "data/ph_traps.vcf"], ["-w", "x"], ["-w", "-1", "-i", "data/ph_traps.vcf"],
              ["--ld-threshold=0.7", "--window=3", "--streaming", "--input", "data/ph_traps.vcf"], ["-"]):
        add(PH, a, stdin="data/ph_traps.vcf" if a[-1:] == ["-"] else None)
    add(PH, [], stdin="data/empty.vcf", tag="empty_stdin")
    return cases


def run_case(c, exe_dir=REF):
    exe = os.path.join(exe_dir, c["tool"])
    stdin = open(os.path.join(HERE, c["stdin"]), "rb") if c["stdin"] else subprocess.DEVNULL
    try:
        p = subprocess.run(c["argv"], executable=exe, cwd=HERE, stdin=stdin, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, timeout=HANG_S if c["tool"] in (AC, MD) else 300)
    except subprocess.TimeoutExpired:
        return None
    finally:
        if c["stdin"]:
            stdin.close()
    return p.stdout, p.stderr, p.returncode


def digest(b):
    return {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b)}


def main():
    if not os.path.isdir(REF):
        sys.exit("oracle/_ref missing: make -f oracle/Makefile.ref")
    cases, hung = [], []
    allc = build_cases()
    with concurrent.futures.ThreadPoolExecutor(8) as ex:  # (hung reference runs wait out HANG_S)
        results = list(ex.map(run_case, allc))
    for c, r in zip(allc, results):
        if r is None:
            hung.append(c["name"])
            continue
        cases.append(c)
        out, err, rc = r
        c["rc"] = rc
        c["out"] = digest(out)
        c["err"] = digest(err)
        if len(out) <= INLINE_MAX:
            c["out"]["b64"] = base64.b64encode(out).decode()
        if len(err) <= INLINE_MAX:
            c["err"]["b64"] = base64.b64encode(err).decode()
    with gzip.GzipFile(os.path.join(HERE, "cases.json.gz"), "wb", mtime=0) as f:
        f.write(json.dumps({"generator": "tests/golden/make_golden.py (reference binaries, oracle/Makefile.ref)",
                            "cases": cases}, indent=0).encode())
    print("%d cases (%d left out: the reference did not finish: %s)" % (len(cases), len(hung), " ".join(hung)))


if __name__ == "__main__":
    main()
