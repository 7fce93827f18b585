"""The C restatement oracle is pinned to the reference before anything is checked
against it: (1) every golden vector produced by the reference binaries (built from
/root/reference sources, tests/golden/make_golden.py) and (2) the reference's own
committed expected outputs (copied as data into tests/golden/data/ref_expected/)."""
import collections
import os

import pytest

from tests._golden import GOLDEN, Oracle, case_stdin, load_cases, matches

CASES = load_cases()


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_case_count():
    tools = collections.Counter(c["tool"] for c in CASES)
    # the five hot-path tools + nonref_filter, hwe_tester, dosage_calculator, allele_counter and
    # missing_detector (8(f) rank 2), haplotype_phaser (8(f) rank 3)
    assert len(tools) == 11 and min(tools.values()) > 40


# tests/test_haplotype_phaser.sh (jorgeMFS/VCFX): the block lines its tests 1-3 grep for
PH_EXP = [("basic.vcf", "0.8", [b"Block 1: 0:(1:100), 1:(1:150), 2:(1:200)", b"Block 2: 3:(1:250)"]),
          ("basic.vcf", "0.99", [b"Block 1: 0:(1:100), 1:(1:150), 2:(1:200)", b"Block 2: 3:(1:250)"]),
          ("low_ld.vcf", "0.5", [b"Block 1: 0:(1:100), 1:(1:150), 2:(1:200)", b"Block 2: 3:(1:250)",
                                 b"Block 3: 4:(1:300)"])]


@pytest.mark.parametrize("name,thr,want", PH_EXP)
def test_oracle_phaser_reference_script(oracle, name, thr, want):
    with open(os.path.join(GOLDEN, "data", "ref_ph", name), "rb") as f:
        data = f.read()
    out, _, rc = oracle.run(["VCFX_haplotype_phaser", "--ld-threshold", thr], data)
    assert rc == 0
    lines = out.split(b"\n")
    for w in want:
        assert w in lines, (w, out)


@pytest.mark.parametrize("tool", sorted({c["tool"] for c in CASES}))
def test_oracle_matches_reference_goldens(oracle, tool):
    bad = []
    for c in CASES:
        if c["tool"] != tool:
            continue
        out, err, rc = oracle.run(list(c["argv"]), case_stdin(c), cwd=GOLDEN)
        if rc != c["rc"] or not matches(c["out"], out) or not matches(c["err"], err):
            bad.append(c["name"])
    assert not bad, "%d/%d mismatches, first: %s" % (len(bad), len(CASES), bad[:10])


REF_EXP = [
    # (reference test command, expected file) -- tests/test_allele_freq_calc.sh, test_record_filter.sh,
    # test_variant_counter.sh in jorgeMFS/VCFX
    (["VCFX_allele_freq_calc"], "ref/afc_simple.vcf", "afc_simple.tsv"),
    (["VCFX_allele_freq_calc"], "ref/afc_multiallelic.vcf", "afc_multiallelic.tsv"),
    (["VCFX_allele_freq_calc"], "ref/afc_missing.vcf", "afc_missing.tsv"),
    (["VCFX_allele_freq_calc"], "ref/afc_phased.vcf", "afc_phased.tsv"),
    (["VCFX_allele_freq_calc"], "ref/afc_complex.vcf", "afc_complex.tsv"),
    (["VCFX_record_filter", "--filter", "QUAL>=90"], "ref/record_filter_input.vcf", "record_filter_qual.vcf"),
    (["VCFX_record_filter", "--filter", "AF>=0.2"], "ref/record_filter_input.vcf", "record_filter_af.vcf"),
    (["VCFX_record_filter", "--filter", "FILTER==PASS"], "ref/record_filter_input.vcf", "record_filter_pass.vcf"),
    (["VCFX_record_filter", "--filter", "FILTER==PASS;AF>=0.2", "--logic", "and"], "ref/record_filter_input.vcf",
     "record_filter_multiple_and.vcf"),
    (["VCFX_record_filter", "--filter", "QUAL>=50;AF>=0.2", "--logic", "or"], "ref/record_filter_input.vcf",
     "record_filter_multiple_or.vcf"),
    (["VCFX_record_filter", "--filter", "POS>=30000", "data/ref/record_filter_input.vcf"], None,
     "record_filter_pos.vcf"),
    (["VCFX_record_filter", "--filter", "DP>=40", "data/ref/record_filter_input.vcf"], None, "record_filter_dp.vcf"),
    (["VCFX_variant_counter"], "ref/variant_counter_normal.vcf", "variant_counter_normal.txt"),
    (["VCFX_variant_counter"], "ref/variant_counter_large.vcf", "variant_counter_large.txt"),
    (["VCFX_variant_counter"], "ref/variant_counter_empty.vcf", "variant_counter_empty.txt"),
    # tests/test_nonref_filter.sh:31-34 (`$EXEC < input`, compared with `diff -b`)
    (["VCFX_nonref_filter"], "ref_nonref/nonref_basic.vcf", "nonref_basic_out.vcf"),
    (["VCFX_nonref_filter"], "ref_nonref/nonref_complex.vcf", "nonref_complex_out.vcf"),
    (["VCFX_nonref_filter"], "ref_nonref/nonref_malformed.vcf", "nonref_malformed_out.vcf"),
    (["VCFX_nonref_filter"], "ref_nonref/nonref_no_gt.vcf", "nonref_no_gt_out.vcf"),
    # tests/test_allele_counter.sh:37-62 (`-q < A`, `-q --samples "Y" < B`, and the -i / positional forms)
    (["VCFX_allele_counter", "-q"], "ref_ac/allele_counter_A.vcf", "allele_counter_A_out.tsv"),
    (["VCFX_allele_counter", "-q", "--samples", "Y"], "ref_ac/allele_counter_B.vcf", "allele_counter_B_out.tsv"),
    (["VCFX_allele_counter", "-q", "-i", "data/ref_ac/allele_counter_A.vcf"], None, "allele_counter_A_out.tsv"),
    (["VCFX_allele_counter", "-q", "data/ref_ac/allele_counter_A.vcf"], None, "allele_counter_A_out.tsv"),
    (["VCFX_allele_counter", "-q", "-s", "Y", "-i", "data/ref_ac/allele_counter_B.vcf"], None,
     "allele_counter_B_out.tsv"),
    # tests/test_missing_detector.sh:65-87 (`$EXEC < input`, trailing whitespace stripped, diff -w -B)
    (["VCFX_missing_detector"], "ref_md/md_basic.vcf", "md_basic_out.vcf"),
    (["VCFX_missing_detector"], "ref_md/md_malformed.vcf", "md_malformed_out.vcf"),
    (["VCFX_missing_detector"], "ref_md/md_empty.vcf", "md_empty_out.vcf"),
    (["VCFX_missing_detector", "--help"], None, "md_help_message.txt"),
]


@pytest.mark.parametrize("argv,stdin,expected", REF_EXP)
def test_oracle_matches_reference_committed_expected(oracle, argv, stdin, expected):
    data = open(os.path.join(GOLDEN, "data", stdin), "rb").read() if stdin else b""
    out, err, rc = oracle.run(argv, data, cwd=GOLDEN)
    want = open(os.path.join(GOLDEN, "data", "ref_expected", expected), "rb").read()
    if argv[0] in ("VCFX_nonref_filter", "VCFX_missing_detector"):  # the scripts compare with diff -b / -w -B
        assert [l.split() for l in out.splitlines() if l.strip()] == [l.split() for l in want.splitlines() if l.strip()]
    else:
        assert out == want


# tests/test_hwe_tester.sh:46-80: `$EXEC < input` against the inline expected text (echo -e adds
# the final newline); the inputs are the files the script writes (tests/data/hwe_tester/)
HWE_KNOWN = [("basic_hwe", b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n1\t100\trs1\tA\tG\t1.000000\n"),
             ("multi_allelic", b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n"),
             ("missing_genotypes", b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n1\t100\trs1\tA\tG\t1.000000\n"),
             ("genotype_formats", b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n1\t100\trs1\tA\tG\t1.000000\n"),
             ("no_gt_field", b"CHROM\tPOS\tID\tREF\tALT\tHWE_pvalue\n")]


@pytest.mark.parametrize("name,want", HWE_KNOWN)
def test_hwe_known_answers(oracle, name, want):
    data = open(os.path.join(GOLDEN, "data", "ref_hwe", name + ".vcf"), "rb").read()
    out, _, rc = oracle.run(["VCFX_hwe_tester"], data)
    assert (out, rc) == (want, 0)


# tests/test_dosage_calculator.sh: `$DOSAGE_TOOL < X.vcf` (and -i) against the script's expected_X.txt
# (both extracted as data by tests/golden/extract_sh_fixtures.py)
DOSE_KNOWN = ["basic", "multi_allelic", "phased", "missing", "malformed", "missing_gt", "single", "gt_not_first"]


@pytest.mark.parametrize("name", DOSE_KNOWN)
def test_dosage_known_answers(oracle, name):
    d = os.path.join(GOLDEN, "data", "ref_dosage")
    data = open(os.path.join(d, name + ".vcf"), "rb").read()
    want = open(os.path.join(d, "expected_%s.txt" % name), "rb").read()
    assert oracle.run(["VCFX_dosage_calculator"], data)[0] == want
    assert oracle.run(["VCFX_dosage_calculator", "-i", "data/ref_dosage/%s.vcf" % name], cwd=GOLDEN)[0] == want


def test_dosage_missing_header_error(oracle):
    data = open(os.path.join(GOLDEN, "data", "ref_dosage", "missing_header.vcf"), "rb").read()
    out, err, rc = oracle.run(["VCFX_dosage_calculator"], data)
    assert (out, err, rc) == (b"", b"Error: VCF header (#CHROM) not found before variant records.\n", 0)


def test_af_known_answers(oracle):
    # test_allele_freq_calc.sh:219  verify_frequencies simple 0.5000 0.3333 0.3333 0.8333
    data = open(os.path.join(GOLDEN, "data", "ref", "afc_simple.vcf"), "rb").read()
    out, _, _ = oracle.run(["VCFX_allele_freq_calc"], data)
    freqs = [l.split(b"\t")[-1] for l in out.splitlines()[1:]]
    assert freqs == [b"0.5000", b"0.3333", b"0.3333", b"0.8333"]


def test_af_tie_modes_differ(oracle):
    # 1 ALT of 32 prints 0.0313 (mmap writeDouble4) vs 0.0312 (stdin printf)
    data = open(os.path.join(GOLDEN, "data", "ties.vcf"), "rb").read()
    out_s, _, _ = oracle.run(["VCFX_allele_freq_calc"], data)
    out_m, _, _ = oracle.run(["VCFX_allele_freq_calc", "-q", "-i", "data/ties.vcf"], b"", cwd=GOLDEN)
    assert out_s.splitlines()[1].endswith(b"0.0312") and out_m.splitlines()[1].endswith(b"0.0313")


REF_LD_SO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_ref",
                         "libref_ld_rsq.so")


@pytest.mark.skipif(not os.path.exists(REF_LD_SO), reason="oracle/_ref not built (no /root/reference here)")
def test_oracle_rsq_equals_reference_doubles(oracle):
    """The oracle's computeRsqFast restatement against the reference's own function (its source
    compiled into oracle/_ref/libref_ld_rsq.so by oracle/Makefile.ref), bit for bit on the fp64
    value: random dosage vectors with missing calls, monomorphic and all-missing vectors, rare
    variants and the sample counts the GPU tests use."""
    import ctypes

    import numpy as np
    ref = ctypes.CDLL(REF_LD_SO).ref_rsq_fast
    ref.argtypes, ref.restype = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t], ctypes.c_double
    mine = oracle.lib.oracle_ld_rsq_fast
    rng = np.random.default_rng(5)
    checked = nonzero = 0
    for ns in (1, 2, 3, 17, 33, 300, 2504, 16383):
        for _ in range(40 if ns < 5000 else 6):
            p = rng.uniform(0.0, 0.6, 2)
            miss = rng.choice([0.0, 0.001, 0.05, 0.5, 1.0], p=[0.4, 0.25, 0.2, 0.1, 0.05])
            base = rng.binomial(2, p[0], ns)
            g = []
            for k in range(2):
                x = np.where(rng.random(ns) < rng.uniform(0, 1), base, rng.binomial(2, p[k], ns)).astype(np.int8)
                x[rng.random(ns) < miss] = -1
                g.append(np.ascontiguousarray(x))
            a, b = (x.ctypes.data_as(ctypes.c_void_p) for x in g)
            want, got = ref(a, b, ns), mine(a, b, ns)
            assert np.float64(want).view(np.uint64) == np.float64(got).view(np.uint64), (ns, want, got)
            checked += 1
            nonzero += want > 0
    assert checked > 250 and nonzero > 100
