"""Every golden case (reference binaries' outputs, tests/golden/cases.json.gz) through the
drop-in tool entries on the GPU: stdout, stderr and exit code byte-identical."""
import pytest

from tests._golden import GOLDEN, case_stdin, load_cases, matches
from vcfx_amd import tools

pytestmark = pytest.mark.gpu

IMPLEMENTED = ["VCFX_allele_freq_calc", "VCFX_genotype_query", "VCFX_record_filter", "VCFX_variant_counter", "VCFX_ld_calculator",
               "VCFX_nonref_filter", "VCFX_hwe_tester", "VCFX_dosage_calculator", "VCFX_missing_detector",
               "VCFX_allele_counter", "VCFX_haplotype_phaser"]
CASES = load_cases()


@pytest.mark.parametrize("tool", IMPLEMENTED)
def test_golden_cases(tool):
    bad = []
    n = 0
    for c in CASES:
        if c["tool"] != tool:
            continue
        n += 1
        out, err, rc = tools.run(list(c["argv"]), case_stdin(c), cwd=GOLDEN)
        if rc != c["rc"] or not matches(c["out"], out) or not matches(c["err"], err):
            bad.append((c["name"], rc, c["rc"], matches(c["out"], out), matches(c["err"], err)))
    assert n > 20
    assert not bad, "%d/%d %s cases differ, first: %s" % (len(bad), n, tool, bad[:8])
