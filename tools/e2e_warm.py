"""In-process (warm context) phase breakdown of a drop-in tool run (measurement tool):
VCFX_TIMING=1 python tools/e2e_warm.py FILE [tool args...]"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vcfx_amd import tools  # noqa: E402

path = sys.argv[1]
extra = sys.argv[2:] or ["VCFX_allele_freq_calc", "-q"]
L = tools.lib()
argv = extra + ["-i", path]
carr = (ctypes.c_char_p * (len(argv) + 1))(*[x.encode() for x in argv], None)
dn = os.open(os.devnull, os.O_RDWR)
for i in range(3):
    os.write(2, b"--- run %d\n" % i)
    rc = L.vcfx_tool_main(argv[0].encode(), len(argv), carr, dn, dn, 2)
    assert rc == 0
