"""ctypes binding of the deterministic synthetic VCF generator (build/libvcfx_synth.so,
vcfx_amd/csrc/synth/vcfx_synth.c).  Used by tests and bench.py."""
import ctypes
import os

import numpy as np

from . import SYNTH_LIB


class Opts(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_records", ctypes.c_int64), ("n_samples", ctypes.c_int32),
                ("info_mode", ctypes.c_int32), ("missing_rate", ctypes.c_double), ("hap_blocks", ctypes.c_int32),
                ("irregular_rate", ctypes.c_double), ("crlf", ctypes.c_int32), ("format_mode", ctypes.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(SYNTH_LIB)
        _lib.vcfx_synth_size.restype = ctypes.c_size_t
        _lib.vcfx_synth_size.argtypes = [ctypes.POINTER(Opts)]
        _lib.vcfx_synth_fill.restype = ctypes.c_size_t
        _lib.vcfx_synth_fill.argtypes = [ctypes.POINTER(Opts), ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_void_p]
    return _lib


def generate_array(n_records, n_samples, seed=20251226, info_mode=0, missing_rate=0.0, hap_blocks=0,
                   irregular_rate=0.0, crlf=0, threads=None, rec_offsets=False, format_mode=0):
    """numpy uint8 array of the VCF bytes (and optionally int64 record offsets).  format_mode 1:
    the regular records carry FORMAT=GT:AD:DP (variable-width samples: the general GT path)."""
    o = Opts(seed, n_records, n_samples, info_mode, missing_rate, hap_blocks, irregular_rate, crlf, format_mode)
    L = lib()
    n = L.vcfx_synth_size(ctypes.byref(o))
    arr = np.empty(n, np.uint8)
    offs = np.empty(n_records + 1, np.uint64) if rec_offsets else None
    threads = threads or min(16, os.cpu_count() or 1)
    got = L.vcfx_synth_fill(ctypes.byref(o), arr.ctypes.data, n, threads,
                            offs.ctypes.data if offs is not None else None)
    assert got == n
    return (arr, offs) if rec_offsets else arr


def generate(*args, **kw):
    """bytes of the VCF (small inputs)."""
    return generate_array(*args, **kw).tobytes()
