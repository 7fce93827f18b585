"""Shared helpers: golden case list, the C-restatement oracle (ctypes), fixture paths.

The oracle under oracle/ is the CHECKER only (see oracle/vcfx_oracle.h)."""
import base64
import ctypes
import gzip
import hashlib
import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "liboracle.so")


def load_cases():
    with gzip.open(os.path.join(GOLDEN, "cases.json.gz"), "rb") as f:
        return json.loads(f.read())["cases"]


def expected_bytes(d):
    return base64.b64decode(d["b64"]) if "b64" in d else None


def matches(d, got):
    if "b64" in d:
        return base64.b64decode(d["b64"]) == got
    return d["len"] == len(got) and d["sha256"] == hashlib.sha256(got).hexdigest()


def ensure_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-f", os.path.join(REPO, "oracle", "Makefile")])
    return ORACLE_SO


class _Res(ctypes.Structure):
    _fields_ = [("out", ctypes.POINTER(ctypes.c_char)), ("out_len", ctypes.c_size_t),
                ("err", ctypes.POINTER(ctypes.c_char)), ("err_len", ctypes.c_size_t), ("rc", ctypes.c_int)]


class Oracle:
    """ctypes view of oracle/_build/liboracle.so (test infrastructure)."""

    def __init__(self):
        self.lib = ctypes.CDLL(ensure_oracle())
        self.lib.oracle_main.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                         ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(_Res)]
        self.lib.oracle_result_free.argtypes = [ctypes.POINTER(_Res)]
        self.lib.oracle_af_counts.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t]
        self.lib.oracle_af_counts.restype = ctypes.c_long
        self.lib.oracle_ld_rsq_fast.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        self.lib.oracle_ld_rsq_fast.restype = ctypes.c_double

    def run(self, argv, stdin=b"", cwd=None):
        """Run a restated tool in-process: returns (stdout, stderr, rc)."""
        old = os.getcwd()
        if cwd:
            os.chdir(cwd)
        try:
            arr = (ctypes.c_char_p * (len(argv) + 1))(*[a.encode() for a in argv], None)
            r = _Res()
            rc = self.lib.oracle_main(argv[0].encode(), len(argv), arr, stdin, len(stdin), ctypes.byref(r))
            assert rc == 0, "unknown tool %s" % argv[0]
            out = ctypes.string_at(r.out, r.out_len)
            err = ctypes.string_at(r.err, r.err_len)
            code = r.rc
            self.lib.oracle_result_free(ctypes.byref(r))
            return out, err, code
        finally:
            os.chdir(old)

    def af_counts(self, buf, stdin_mode=False):
        import numpy as np
        cap = max(16, buf.count(b"\n") + 2)
        alt = np.zeros(cap, np.int32)
        tot = np.zeros(cap, np.int32)
        n = self.lib.oracle_af_counts(buf, len(buf), int(stdin_mode), alt.ctypes.data, tot.ctypes.data, cap)
        assert n >= 0
        return alt[:n], tot[:n]


def case_stdin(c):
    if not c["stdin"]:
        return b""
    with open(os.path.join(GOLDEN, c["stdin"]), "rb") as f:
        return f.read()
