"""The streaming stdin paths on every golden stdin case: stdin is a PIPE (read, not mapped) and
the path sizes are shrunk through the environment (VCFX_PREFETCH_BYTES, VCFX_STREAM_CHUNK,
VCFX_RING_SLOT, VCFX_WINDOW_BYTES), so the small fixtures take the paths the 4 GB inputs take:
the GPU context opened while the pipe is read, a device-only stream through the pinned ring
(AF, RF, GQ, NR: only the header kept on the host), the host-copied stream with its chunked
ingest (LD, VC), and the pass-through tools writing kept records back from the device through a
moving window.  stdout, stderr and exit code must stay byte-identical to the reference's."""
import pytest

from tests._golden import GOLDEN, case_stdin, load_cases, matches
from vcfx_amd import tools

pytestmark = pytest.mark.gpu

CASES = load_cases()
KNOBS = [
    # (prefetch, stream chunk, ring slot, window)
    {"VCFX_PREFETCH_BYTES": "64", "VCFX_STREAM_CHUNK": "256", "VCFX_RING_SLOT": "300", "VCFX_WINDOW_BYTES": "1024"},
    {"VCFX_PREFETCH_BYTES": "4096", "VCFX_STREAM_CHUNK": "8192", "VCFX_RING_SLOT": "65536",
     "VCFX_WINDOW_BYTES": "7000"},
]


def _stdin_cases(tool):
    for c in CASES:
        if c["tool"] == tool and c["stdin"] and not any(a in ("-i", "--input") for a in c["argv"][1:]):
            yield c


@pytest.mark.parametrize("knobs", range(len(KNOBS)))
@pytest.mark.parametrize("tool", ["VCFX_allele_freq_calc", "VCFX_record_filter", "VCFX_genotype_query",
                                  "VCFX_nonref_filter", "VCFX_variant_counter", "VCFX_ld_calculator"])
def test_golden_stdin_cases_through_a_pipe(monkeypatch, tool, knobs):
    for k, v in KNOBS[knobs].items():
        monkeypatch.setenv(k, v)
    bad = []
    n = 0
    for c in _stdin_cases(tool):
        n += 1
        out, err, rc = tools.run_pipe(list(c["argv"]), case_stdin(c), cwd=GOLDEN)
        if rc != c["rc"] or not matches(c["out"], out) or not matches(c["err"], err):
            bad.append((c["name"], rc, c["rc"], matches(c["out"], out), matches(c["err"], err)))
    assert n > 20
    assert not bad, "%d/%d %s cases differ, first: %s" % (len(bad), n, tool, bad[:8])


FILE_KNOBS = [
    # (first head read, ring slot, slots): the head grows by doubling until it holds '#CHROM'
    {"VCFX_FILE_STREAM_MIN": "1", "VCFX_FILE_HEAD": "64", "VCFX_FILE_SLOT": "4096", "VCFX_FILE_SLOTS": "4"},
    {"VCFX_FILE_STREAM_MIN": "1", "VCFX_FILE_HEAD": "1000", "VCFX_FILE_SLOT": "777", "VCFX_FILE_SLOTS": "5"},
    {"VCFX_FILE_STREAM_MIN": "1", "VCFX_FILE_HEAD": "4096", "VCFX_FILE_SLOT": "65536", "VCFX_FILE_SLOTS": "12"},
]


@pytest.mark.parametrize("knobs", range(len(FILE_KNOBS)))
def test_golden_af_file_cases_streamed_from_the_file(monkeypatch, knobs):
    """VCFX_allele_freq_calc -i FILE on every golden file case with the device-only file path
    forced on small files (Input::open_file_device: the head read into host memory, the rest
    by reader threads into a pinned ring of tiny slots and copied to the device in order,
    many ring wraps): stdout, stderr and exit code byte-identical to the reference's."""
    for k, v in FILE_KNOBS[knobs].items():
        monkeypatch.setenv(k, v)
    bad = []
    n = 0
    for c in CASES:
        if c["tool"] != "VCFX_allele_freq_calc" or c["stdin"] or not any(a in ("-i", "--input") for a in c["argv"]):
            continue
        n += 1
        out, err, rc = tools.run(list(c["argv"]), b"", cwd=GOLDEN)
        if rc != c["rc"] or not matches(c["out"], out) or not matches(c["err"], err):
            bad.append((c["name"], rc, c["rc"], matches(c["out"], out), matches(c["err"], err)))
    assert n > 20
    assert not bad, "%d/%d cases differ, first: %s" % (len(bad), n, bad[:8])


def test_af_streamed_file_larger_input(monkeypatch, tmp_path):
    """A 40 MB synthetic input through the streamed file path (16 slots of 256 KiB: ~160 chunks,
    ten ring wraps, six reader threads) equals the mapped path's output."""
    from vcfx_amd import synth
    p = str(tmp_path / "s.vcf")
    open(p, "wb").write(synth.generate(6000, 2504, 91, 1, 0.001, 0, 0.02, 0))
    argv = ["VCFX_allele_freq_calc", "-i", p]
    monkeypatch.setenv("VCFX_FILE_STREAM", "0")
    want = tools.run(argv)
    monkeypatch.delenv("VCFX_FILE_STREAM")
    for k, v in {"VCFX_FILE_STREAM_MIN": "1", "VCFX_FILE_SLOT": str(256 << 10), "VCFX_FILE_SLOTS": "16"}.items():
        monkeypatch.setenv(k, v)
    got = tools.run(argv)
    assert want[2] == 0 and got == want
