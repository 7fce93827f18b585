#!/usr/bin/env python3
"""Run golden cases on the GPU through the drop-in tools and write diffs of failures to
gpurun_out/debug/ (developer aid; usage: debug_cases.py TOOL [max])."""
import base64
import difflib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._golden import GOLDEN, case_stdin, load_cases, matches  # noqa: E402
from vcfx_amd import tools  # noqa: E402

tool = sys.argv[1]
mx = int(sys.argv[2]) if len(sys.argv) > 2 else 20
os.makedirs("gpurun_out/debug", exist_ok=True)
n = 0
for c in load_cases():
    if c["tool"] != tool:
        continue
    out, err, rc = tools.run(list(c["argv"]), case_stdin(c), cwd=GOLDEN)
    if rc == c["rc"] and matches(c["out"], out) and matches(c["err"], err):
        continue
    n += 1
    with open("gpurun_out/debug/%03d_%s.txt" % (n, c["name"][:80]), "w") as f:
        f.write("argv %s stdin %s rc %d want %d\n" % (c["argv"], c["stdin"], rc, c["rc"]))
        for what, got, exp in (("out", out, c["out"]), ("err", err, c["err"])):
            if "b64" in exp:
                want = base64.b64decode(exp["b64"])
                if want != got:
                    f.write("--- %s diff\n" % what)
                    f.writelines(difflib.unified_diff(want.decode("latin-1").splitlines(True),
                                                      got.decode("latin-1").splitlines(True), n=1))
            elif not matches(exp, got):
                f.write("--- %s differs (hash), got %d bytes want %d\n" % (what, len(got), exp["len"]))
    if n >= mx:
        break
print("failures written:", n)
