"""Golden CLI cases through the drop-in tool entries (libvcfx_tools.so, in-process).

On a machine without a GPU, cases whose processing needs the device must fail loudly
(no CPU fallback); every case that the host handles alone (usage, help, version, open
errors, header-only input) must match the reference byte for byte.  The GPU run of the
same cases is tests/test_gpu_cli.py."""
import pytest

from tests._golden import GOLDEN, case_stdin, load_cases, matches
from vcfx_amd import tools

IMPLEMENTED = {"VCFX_allele_freq_calc", "VCFX_genotype_query", "VCFX_record_filter", "VCFX_variant_counter", "VCFX_ld_calculator",
               "VCFX_nonref_filter", "VCFX_hwe_tester", "VCFX_dosage_calculator", "VCFX_missing_detector",
               "VCFX_allele_counter", "VCFX_haplotype_phaser"}
CASES = [c for c in load_cases() if c["tool"] in IMPLEMENTED]
NODEV = b"no usable MI355X"


def test_host_only_cases_match_reference():
    checked = failed_loud = 0
    bad = []
    for c in CASES:
        out, err, rc = tools.run(list(c["argv"]), case_stdin(c), cwd=GOLDEN)
        if NODEV in err:
            assert rc != 0
            failed_loud += 1
            continue
        checked += 1
        if rc != c["rc"] or not matches(c["out"], out) or not matches(c["err"], err):
            bad.append(c["name"])
    assert not bad, bad[:10]
    assert checked >= 10
