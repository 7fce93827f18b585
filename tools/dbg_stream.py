"""debugging aid for the streaming stdin paths (measurement/debug tool)"""
import os, sys
sys.path.insert(0, '.')
from tests._golden import GOLDEN, case_stdin, load_cases, expected_bytes, matches
from vcfx_amd import tools, engine
buf = open(os.path.join(GOLDEN, 'data/crlf.vcf'), 'rb').read()
ds = engine.data_start_of(buf, strip_cr=False)
e = engine.Engine(0)
for q, strict in (("0/1", False), ("1|1", True), ("1|1", True)):
    e.ingest([buf[:576], buf[576:]])
    s = e.genotype_query_region(ds, q, strict=strict)
    print('ingest', q, strict, s.n_lines, s.rows, list(map(int, e.statuses(s.n_lines))))
    e.load(buf)
    s = e.genotype_query_region(ds, q, strict=strict)
    print('load  ', q, strict, s.n_lines, s.rows, list(map(int, e.statuses(s.n_lines))))
e.close()
os.environ.update({"VCFX_PREFETCH_BYTES": "64", "VCFX_STREAM_CHUNK": "256", "VCFX_RING_SLOT": "300", "VCFX_WINDOW_BYTES": "1024", "VCFX_TIMING": "1", "VCFX_DEBUG": "1"})
cases = {c['name']: c for c in load_cases()}
for nm in ['genotype_query__-g_0-1__stdin_crlf.vcf', 'genotype_query__-g_1_1_--strict__stdin_crlf.vcf', 'genotype_query__-g_0-1__stdin_crlf.vcf']:
    c = cases[nm]
    out, err, rc = tools.run_pipe(list(c['argv']), case_stdin(c), cwd=GOLDEN)
    print(nm, matches(c['out'], out), len(out), err)
