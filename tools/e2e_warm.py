"""In-process (warm context) timing of a drop-in tool run (measurement tool): the first call
opens the device context; the walls of the next calls are printed (and with VCFX_TIMING=1 each
call's phases on stderr).

  [VCFX_TIMING=1] python tools/e2e_warm.py [--torch] [--json] FILE [tool args...]

--torch: import torch and run a CPU and a GPU op first (bench.py's process state); --json: one
line {"walls": [...]} on stdout."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vcfx_amd import tools  # noqa: E402

args = sys.argv[1:]
use_torch = "--torch" in args
as_json = "--json" in args
args = [x for x in args if x not in ("--torch", "--json")]
if use_torch:
    import torch
    torch.randn(2048, 2048).sum().item()
    if torch.cuda.is_available():
        torch.randn(1024, device="cuda").sum().item()
path = args[0]
extra = args[1:] or ["VCFX_allele_freq_calc", "-q"]
L = tools.lib()
argv = extra + ["-i", path]
carr = (ctypes.c_char_p * (len(argv) + 1))(*[x.encode() for x in argv], None)
dn = os.open(os.devnull, os.O_RDWR)
walls = []
for i in range(4):
    os.write(2, b"--- run %d\n" % i)
    t0 = time.perf_counter()
    rc = L.vcfx_tool_main(argv[0].encode(), len(argv), carr, dn, dn, 2)
    walls.append(time.perf_counter() - t0)
    assert rc == 0
if as_json:
    print(json.dumps({"walls": [round(w, 4) for w in walls[1:]]}))
else:
    print("walls (after the first)", " ".join("%.4f" % w for w in walls[1:]))
