"""ctypes binding of the C ABI in include/vcfx_gpu.h (libvcfx_gpu.so).

This is plumbing for tests and bench.py; the CLI drop-ins call the same ABI from C++."""
import ctypes
import os

from . import GPU_LIB

VCFXG_OK = 0
MODE_FILE, MODE_STDIN = 0, 1
STATUS = {0: "skip", 1: "row", 2: "drop", 3: "warn", 4: "header"}


class Summary(ctypes.Structure):
    _fields_ = [("n_lines", ctypes.c_uint64), ("rows", ctypes.c_uint64), ("data_lines", ctypes.c_uint64),
                ("warn_lines", ctypes.c_uint64), ("text_bytes", ctypes.c_uint64),
                ("general_records", ctypes.c_uint64)]


class AcParams(ctypes.Structure):
    _fields_ = [("sample", ctypes.c_void_p), ("m", ctypes.c_uint64), ("names", ctypes.c_char_p),
                ("name_off", ctypes.c_void_p), ("seq", ctypes.c_int), ("kind", ctypes.c_int)]


class Criterion(ctypes.Structure):
    _fields_ = [("target", ctypes.c_int), ("op", ctypes.c_int), ("numeric", ctypes.c_int), ("value", ctypes.c_double),
                ("key", ctypes.c_char_p), ("key_len", ctypes.c_size_t), ("str", ctypes.c_char_p),
                ("str_len", ctypes.c_size_t)]


# record_filter criterion codes (vcfx_gpu.h vcfxg_criterion)
POS, QUAL, FILTER, INFO = 0, 1, 2, 3
GT, GE, LT, LE, EQ, NE = 0, 1, 2, 3, 4, 5


# every exported entry point: name -> (restype, argtypes)
_P, _VP, _S, _U64, _I = ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
SIGNATURES = {
    "vcfxg_version": (_P, []),
    "vcfxg_device_count": (_I, [ctypes.POINTER(_I)]),
    "vcfxg_open": (_I, [_I, ctypes.POINTER(_VP)]),
    "vcfxg_close": (None, [_VP]),
    "vcfxg_last_error": (_P, [_VP]),
    "vcfxg_stream": (_VP, [_VP]),
    "vcfxg_set_profiling": (_I, [_VP, _I]),
    "vcfxg_set_profiling_only": (_I, [_VP, _P]),
    "vcfxg_kernel_ms": (_I, [_VP, _P, ctypes.POINTER(ctypes.c_float)]),
    "vcfxg_kernel_stats": (_I, [_VP, _P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_U64)]),
    "vcfxg_reset_kernel_stats": (_I, [_VP]),
    "vcfxg_load_host": (_I, [_VP, _VP, _S]),
    "vcfxg_ingest_begin": (_I, [_VP, _S]),
    "vcfxg_ingest": (_I, [_VP, _VP, _S, _I]),
    "vcfxg_ingest_wait": (_I, [_VP, _S]),
    "vcfxg_ingest_bgzf": (_I, [_VP, _VP, _S, _VP, _S, _VP, _S, ctypes.POINTER(_U64)]),
    "vcfxg_bgzf_stage": (_I, [_VP, _VP, _S, _S, _S]),
    "vcfxg_bgzf_inflate": (_I, [_VP, _VP, _S]),
    "vcfxg_host_alloc": (_I, [_VP, _S, ctypes.POINTER(_VP)]),
    "vcfxg_host_free": (None, [_VP, _VP]),
    "vcfxg_input_device_ptr": (_VP, [_VP]),
    "vcfxg_input_fetch": (_I, [_VP, _U64, _S, _VP]),
    "vcfxg_index": (_I, [_VP, _S, ctypes.POINTER(_U64)]),
    "vcfxg_line_ends": (_I, [_VP, _U64, _U64, _VP]),
    "vcfxg_allele_freq": (_I, [_VP, _I, ctypes.POINTER(Summary)]),
    "vcfxg_allele_freq_region": (_I, [_VP, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_genotype_query": (_I, [_VP, _P, _S, _I, _I, ctypes.POINTER(Summary)]),
    "vcfxg_record_filter": (_I, [_VP, _VP, _I, _I, ctypes.POINTER(Summary)]),
    "vcfxg_record_filter_ex": (_I, [_VP, _VP, _I, _I, _I, ctypes.POINTER(Summary)]),
    "vcfxg_variant_count": (_I, [_VP, _I, ctypes.POINTER(Summary)]),
    "vcfxg_nonref_filter": (_I, [_VP, _I, ctypes.POINTER(Summary)]),
    "vcfxg_nonref_filter_region": (_I, [_VP, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_hwe_region": (_I, [_VP, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_hwe_rechecks": (_I, [_VP, _VP, _U64, ctypes.POINTER(_U64)]),
    "vcfxg_dosage_region": (_I, [_VP, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_missing_region": (_I, [_VP, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_allele_counter": (_I, [_VP, _U64, _U64, _VP, ctypes.POINTER(Summary)]),
    "vcfxg_fetch_text_range": (_I, [_VP, _U64, _S, _VP]),
    "vcfxg_shard_cuts": (_I, [_VP, _S, _S, _I, _VP]),
    "vcfxg_comm_init": (_I, [_VP, _I, ctypes.POINTER(_VP)]),
    "vcfxg_comm_allreduce_u64": (_I, [_VP, _I, _VP, _S]),
    "vcfxg_comm_uses_rccl": (_I, [_VP]),
    "vcfxg_comm_destroy": (None, [_VP]),
    "vcfxg_comm_rccl_stats": (_I, [_VP, ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    "vcfxg_last_schedule": (_P, [_VP]),
    "vcfxg_bgzf_handed_over": (_U64, [_VP]),
    "vcfxg_count_byte": (_I, [_VP, _U64, _I, ctypes.POINTER(_U64)]),
    "vcfxg_haplotype_phaser": (_I, [_VP, _S, _I, ctypes.c_double, ctypes.c_uint32, ctypes.POINTER(Summary)]),
    "vcfxg_phaser_variants": (_I, [_VP, _VP, _VP, _VP]),
    "vcfxg_ld_prepare": (_I, [_VP, _I, _I, _P, _S, _I, _I, _I, _I, ctypes.POINTER(_U64)]),
    "vcfxg_ld_prepare_region": (_I, [_VP, _S, _I, _I, _P, _S, _I, _I, _I, _I, ctypes.POINTER(_U64)]),
    "vcfxg_ld_prefixes": (_I, [_VP, _VP, _S, _VP]),
    "vcfxg_ld_matrix": (_I, [_VP, _I, _I, ctypes.POINTER(_U64)]),
    "vcfxg_ld_stream_chunk": (_I, [_VP, _U64, _U64, _U64, ctypes.c_double, _I, ctypes.POINTER(_U64),
                                   ctypes.POINTER(_U64)]),
    "vcfxg_ld_fetch_pairs": (_I, [_VP, _U64, _U64, _VP, _VP, _VP]),
    "vcfxg_selftest_mfma_i8": (_I, [_VP, ctypes.POINTER(_I)]),
    "vcfxg_selftest_mfma_fp4": (_I, [_VP, ctypes.POINTER(_I)]),
    "vcfxg_filter_query": (_I, [_VP, _VP, _I, _I, _P, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_record_filter_region": (_I, [_VP, _S, _VP, _I, _I, ctypes.POINTER(Summary)]),
    "vcfxg_genotype_query_region": (_I, [_VP, _S, _P, _S, _I, _I, ctypes.POINTER(Summary)]),
    "vcfxg_filter_query_region": (_I, [_VP, _S, _VP, _I, _I, _P, _S, _I, ctypes.POINTER(Summary)]),
    "vcfxg_fetch_text": (_I, [_VP, _VP, _S]),
    "vcfxg_fetch_lines": (_I, [_VP, _U64, _U64, _VP, _VP, _VP]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(GPU_LIB):
            raise RuntimeError("libvcfx_gpu.so not built (run `make` or __graft_entry__.build())")
        _lib = ctypes.CDLL(GPU_LIB)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("VCFXG_GPU_LIB") and not hasattr(_lib, name):
                continue  # an older experiment build (A/B runs): its missing entries are not called
            f = getattr(_lib, name)
            f.restype = res
            f.argtypes = args
    return _lib


class EngineError(RuntimeError):
    pass


class Engine:
    """One device context (vcfxg_ctx)."""

    def __init__(self, device=0):
        self.L = lib()
        h = ctypes.c_void_p()
        rc = self.L.vcfxg_open(device, ctypes.byref(h))
        if rc != VCFXG_OK:
            raise EngineError("vcfxg_open(%d) failed rc=%d: no usable gfx950 device" % (device, rc))
        self.h = h
        self._buf = None

    def close(self):
        if self.h:
            self.L.vcfxg_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != VCFXG_OK:
            raise EngineError("%s failed rc=%d: %s" % (what, rc, self.L.vcfxg_last_error(self.h).decode()))

    @property
    def stream(self):
        return self.L.vcfxg_stream(self.h)

    def set_profiling(self, on=True):
        self._chk(self.L.vcfxg_set_profiling(self.h, int(on)), "set_profiling")

    def set_profiling_only(self, name=None):
        """time only the named kernel (None: every kernel)"""
        if not hasattr(self.L, "vcfxg_set_profiling_only"):  # (an older experiment build: every kernel)
            return
        self._chk(self.L.vcfxg_set_profiling_only(self.h, name.encode() if name else None), "set_profiling_only")

    def kernel_ms(self, name):
        v = ctypes.c_float()
        rc = self.L.vcfxg_kernel_ms(self.h, name.encode(), ctypes.byref(v))
        return v.value if rc == VCFXG_OK else None

    def kernel_stats(self, name):
        """(total ms, launches) accumulated since reset_kernel_stats()."""
        t = ctypes.c_double()
        n = ctypes.c_uint64()
        self._chk(self.L.vcfxg_kernel_stats(self.h, name.encode(), ctypes.byref(t), ctypes.byref(n)), "kernel_stats")
        return t.value, n.value

    def reset_kernel_stats(self):
        self._chk(self.L.vcfxg_reset_kernel_stats(self.h), "reset_kernel_stats")

    def load(self, data):
        """data: bytes / bytearray / numpy uint8 array (kept alive until the next load)."""
        import numpy as np
        arr = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data
        self._buf = arr
        self._chk(self.L.vcfxg_load_host(self.h, arr.ctypes.data, arr.size), "load_host")

    def ingest(self, chunks):
        """Streaming load: vcfxg_ingest_begin + one vcfxg_ingest per chunk (the last is final)."""
        import numpy as np
        arrs = [np.frombuffer(c, np.uint8) if not isinstance(c, np.ndarray) else c for c in chunks]
        self._buf = arrs
        self._chk(self.L.vcfxg_ingest_begin(self.h, 0), "ingest_begin")
        if not arrs:
            self._chk(self.L.vcfxg_ingest(self.h, None, 0, 1), "ingest")
        for i, a in enumerate(arrs):
            self._chk(self.L.vcfxg_ingest(self.h, a.ctypes.data, a.size, int(i == len(arrs) - 1)), "ingest")

    def load_bgzf(self, comp, members=None, head=b""):
        """vcfxg_ingest_begin + vcfxg_ingest_bgzf + the final vcfxg_ingest: the BGZF members of
        `comp` inflated on the device into the input.  members: bgzf_members(comp) by default.
        Returns None, or (first bad member, error text) when the device refused a member (the
        input is then not loaded)."""
        import numpy as np
        arr = np.frombuffer(comp, np.uint8) if not isinstance(comp, np.ndarray) else comp
        mem = bgzf_members(arr) if members is None else members
        hd = np.frombuffer(head, np.uint8) if head else None
        self._buf = (arr, mem, hd)
        total = int(mem["out_len"].sum()) if len(mem) else 0
        self._chk(self.L.vcfxg_ingest_begin(self.h, total), "ingest_begin")
        bad = ctypes.c_uint64()
        rc = self.L.vcfxg_ingest_bgzf(self.h, arr.ctypes.data, arr.size, mem.ctypes.data if len(mem) else None,
                                      len(mem), hd.ctypes.data if hd is not None else None,
                                      0 if hd is None else hd.size, ctypes.byref(bad))
        if rc == -7:  # VCFXG_E_DATA
            return bad.value, self.L.vcfxg_last_error(self.h).decode()
        self._chk(rc, "ingest_bgzf")
        self._chk(self.L.vcfxg_ingest(self.h, None, 0, 1), "ingest")
        return None

    def bgzf_handed_over(self):
        """members of the last load_bgzf the lane decoder handed to the wave decoder"""
        return int(self.L.vcfxg_bgzf_handed_over(self.h))

    def input_bytes(self, offset, n):
        """bytes [offset, offset + n) of the loaded device input (vcfxg_input_fetch)"""
        b = ctypes.create_string_buffer(max(1, n))
        self._chk(self.L.vcfxg_input_fetch(self.h, offset, n, b), "input_fetch")
        return b.raw[:n]

    def index(self, data_start):
        n = ctypes.c_uint64()
        self._chk(self.L.vcfxg_index(self.h, data_start, ctypes.byref(n)), "index")
        return n.value

    def allele_freq(self, mode=MODE_FILE):
        s = Summary()
        self._chk(self.L.vcfxg_allele_freq(self.h, mode, ctypes.byref(s)), "allele_freq")
        return s

    def allele_freq_region(self, data_start, mode=MODE_FILE):
        """index + allele counts + rows in one fused device sweep (vcfxg_allele_freq_region)."""
        s = Summary()
        self._chk(self.L.vcfxg_allele_freq_region(self.h, data_start, mode, ctypes.byref(s)), "allele_freq_region")
        return s

    def genotype_query(self, query, strict=False, strip_cr=False):
        q = query.encode() if isinstance(query, str) else query
        s = Summary()
        self._chk(self.L.vcfxg_genotype_query(self.h, q, len(q), int(strict), int(strip_cr), ctypes.byref(s)),
                  "genotype_query")
        return s

    def nonref_filter(self, mode):
        """VCFX_nonref_filter per line over the indexed region (mode MODE_FILE / MODE_STDIN)"""
        s = Summary()
        self._chk(self.L.vcfxg_nonref_filter(self.h, int(mode), ctypes.byref(s)), "nonref_filter")
        return s

    def nonref_filter_region(self, data_start, mode):
        """index + nonref_filter in one call (the walk for long records)"""
        s = Summary()
        self._chk(self.L.vcfxg_nonref_filter_region(self.h, data_start, int(mode), ctypes.byref(s)),
                  "nonref_filter_region")
        return s

    def hwe_region(self, data_start, mode):
        """VCFX_hwe_tester over [data_start, n): counts, row rules and rows (vcfxg_hwe_region)"""
        s = Summary()
        self._chk(self.L.vcfxg_hwe_region(self.h, data_start, int(mode), ctypes.byref(s)), "hwe_region")
        return s

    def dosage_region(self, data_start, mode):
        """VCFX_dosage_calculator rows over the data lines from data_start (vcfxg_dosage_region)"""
        s = Summary()
        self._chk(self.L.vcfxg_dosage_region(self.h, data_start, int(mode), ctypes.byref(s)), "dosage_region")
        return s

    def missing_region(self, data_start, mode):
        """VCFX_missing_detector's per-line test over the lines from data_start (vcfxg_missing_region)"""
        s = Summary()
        self._chk(self.L.vcfxg_missing_region(self.h, data_start, int(mode), ctypes.byref(s)), "missing_region")
        return s

    def allele_counter(self, l0, l1, samples, names, seq=0, kind=0):
        """VCFX_allele_counter rows of indexed lines [l0, l1) for the output slots (sample index,
        name) (vcfxg_allele_counter); seq 0 = the file path's every-slot semantics, 1 = the
        forward cursor; kind 0 text, 1 aggregate, 2 binary"""
        import numpy as np
        idx = np.ascontiguousarray(samples, np.uint32)
        nb = [x.encode() if isinstance(x, str) else bytes(x) for x in names]
        assert len(nb) == len(idx)
        off = np.zeros(len(nb) + 1, np.uint64)
        off[1:] = np.cumsum([len(x) for x in nb])
        p = AcParams(idx.ctypes.data, len(idx), b"".join(nb), off.ctypes.data, int(seq), int(kind))
        s = Summary()
        self._chk(self.L.vcfxg_allele_counter(self.h, l0, l1, ctypes.byref(p), ctypes.byref(s)), "allele_counter")
        return s

    def haplotype_phaser(self, data_start, mode, threshold, n_samples):
        """VCFX_haplotype_phaser's parse + consecutive-variant LD (vcfxg_haplotype_phaser)"""
        s = Summary()
        self._chk(self.L.vcfxg_haplotype_phaser(self.h, data_start, int(mode), float(threshold), int(n_samples),
                                                ctypes.byref(s)), "haplotype_phaser")
        return s

    def phaser_variants(self, n_var):
        """(flags, r2, entry offsets) of the last haplotype_phaser call"""
        import numpy as np
        f = np.zeros(max(n_var, 1), np.uint8)
        r2 = np.zeros(max(n_var, 1), np.float64)
        off = np.zeros(n_var + 1, np.uint64)
        self._chk(self.L.vcfxg_phaser_variants(self.h, f.ctypes.data, r2.ctypes.data, off.ctypes.data),
                  "phaser_variants")
        return f[:n_var], r2[:n_var], off

    def text_range(self, offset, n):
        b = ctypes.create_string_buffer(max(1, n))
        self._chk(self.L.vcfxg_fetch_text_range(self.h, offset, n, b), "fetch_text_range")
        return b.raw[:n]

    def hwe_rechecks(self):
        """the last hwe_region's rows left to the host: [(text_offset, hom_ref, het, hom_alt)]"""
        import numpy as np
        n = ctypes.c_uint64()
        self._chk(self.L.vcfxg_hwe_rechecks(self.h, None, 0, ctypes.byref(n)), "hwe_rechecks")
        a = np.zeros((max(n.value, 1), 3), np.uint64)  # 24 B per vcfxg_hwe_recheck
        self._chk(self.L.vcfxg_hwe_rechecks(self.h, a.ctypes.data, n.value, ctypes.byref(n)), "hwe_rechecks")
        v = a[:n.value].view(np.uint32).reshape(-1, 6)
        return [(int(r[0]) | (int(r[1]) << 32), int(r[2]), int(r[3]), int(r[4])) for r in v]

    def _criteria(self, crits):
        """crits: list of (target, op, numeric, value, key, str) as vcfxg_criterion."""
        arr = (Criterion * max(1, len(crits)))()
        self._keep = []
        for i, (target, op, numeric, value, key, sval) in enumerate(crits):
            k = key.encode() if isinstance(key, str) else key
            s = sval.encode() if isinstance(sval, str) else sval
            self._keep += [k, s]
            arr[i] = Criterion(target, op, int(numeric), float(value), k, len(k), s, len(s))
        return arr

    def record_filter(self, crits, and_logic=True):
        s = Summary()
        arr = self._criteria(crits)
        self._chk(self.L.vcfxg_record_filter(self.h, ctypes.cast(arr, ctypes.c_void_p), len(crits), int(and_logic),
                                             ctypes.byref(s)), "record_filter")
        return s

    def filter_query(self, crits, query, and_logic=True, strict=False):
        s = Summary()
        arr = self._criteria(crits)
        q = query.encode() if isinstance(query, str) else query
        self._chk(self.L.vcfxg_filter_query(self.h, ctypes.cast(arr, ctypes.c_void_p), len(crits), int(and_logic), q,
                                            len(q), int(strict), ctypes.byref(s)), "filter_query")
        return s

    def record_filter_region(self, data_start, crits, and_logic=True):
        """index + record_filter in one call (vcfxg_record_filter_region)."""
        s = Summary()
        arr = self._criteria(crits)
        self._chk(self.L.vcfxg_record_filter_region(self.h, data_start, ctypes.cast(arr, ctypes.c_void_p), len(crits),
                                                    int(and_logic), ctypes.byref(s)), "record_filter_region")
        return s

    def genotype_query_region(self, data_start, query, strict=False, strip_cr=False):
        """index + genotype_query in one call (vcfxg_genotype_query_region)."""
        q = query.encode() if isinstance(query, str) else query
        s = Summary()
        self._chk(self.L.vcfxg_genotype_query_region(self.h, data_start, q, len(q), int(strict), int(strip_cr),
                                                     ctypes.byref(s)), "genotype_query_region")
        return s

    def filter_query_region(self, data_start, crits, query, and_logic=True, strict=False):
        """index + the fused record_filter | genotype_query in one call (vcfxg_filter_query_region)."""
        s = Summary()
        arr = self._criteria(crits)
        q = query.encode() if isinstance(query, str) else query
        self._chk(self.L.vcfxg_filter_query_region(self.h, data_start, ctypes.cast(arr, ctypes.c_void_p), len(crits),
                                                   int(and_logic), q, len(q), int(strict), ctypes.byref(s)),
                  "filter_query_region")
        return s

    def ld_prepare(self, n_samples, id_dot_to_pos=True, region=None):
        n = ctypes.c_uint64()
        rc, rs, re_ = (region[0].encode(), region[1], region[2]) if region else (b"", 0, 0)
        self._chk(self.L.vcfxg_ld_prepare(self.h, n_samples, int(id_dot_to_pos), rc, len(rc), int(bool(region)), rs,
                                          re_, 0, ctypes.byref(n)), "ld_prepare")
        return n.value

    def ld_prepare_region(self, data_start, n_samples, id_dot_to_pos=True, region=None):
        """vcfxg_index + vcfxg_ld_prepare in one call (the LD walk for long records)."""
        n = ctypes.c_uint64()
        rc, rs, re_ = (region[0].encode(), region[1], region[2]) if region else (b"", 0, 0)
        self._chk(self.L.vcfxg_ld_prepare_region(self.h, data_start, n_samples, int(id_dot_to_pos), rc, len(rc),
                                                 int(bool(region)), rs, re_, 0, ctypes.byref(n)), "ld_prepare_region")
        return n.value

    def ld_stream_chunk(self, j0, j1, window, threshold, max_dist=0):
        npairs = ctypes.c_uint64()
        tb = ctypes.c_uint64()
        self._chk(self.L.vcfxg_ld_stream_chunk(self.h, j0, j1, window, threshold, max_dist, ctypes.byref(npairs),
                                               ctypes.byref(tb)), "ld_stream_chunk")
        return npairs.value, tb.value

    def count_byte(self, from_, byte):
        n = ctypes.c_uint64()
        self._chk(self.L.vcfxg_count_byte(self.h, from_, byte, ctypes.byref(n)), "count_byte")
        return n.value

    def ld_prefixes(self, m):
        """The m variants' "CHROM\tPOS\tID" prefixes of the last LD prepare, as a list of bytes."""
        import numpy as np
        offs = np.zeros(m + 1, np.uint64)
        self._chk(self.L.vcfxg_ld_prefixes(self.h, None, 0, offs.ctypes.data) if m == 0 else
                  self.L.vcfxg_ld_prefixes(self.h, None, 1 << 62, offs.ctypes.data), "ld_prefixes")
        text = ctypes.create_string_buffer(int(offs[m]) + 1)
        self._chk(self.L.vcfxg_ld_prefixes(self.h, text, int(offs[m]) + 1, None), "ld_prefixes")
        raw = text.raw
        return [raw[int(offs[k]):int(offs[k + 1])] for k in range(m)]

    def ld_pairs(self, first, count):
        """(i, j, r2) numpy arrays of pairs [first, first + count) of the last ld_stream_chunk."""
        import numpy as np
        vi = np.zeros(count, np.uint32)
        vj = np.zeros(count, np.uint32)
        r2 = np.zeros(count, np.float64)
        self._chk(self.L.vcfxg_ld_fetch_pairs(self.h, first, count, vi.ctypes.data, vj.ctypes.data, r2.ctypes.data),
                  "ld_fetch_pairs")
        return vi, vj, r2

    def selftest_mfma_i8(self):
        m = ctypes.c_int()
        self._chk(self.L.vcfxg_selftest_mfma_i8(self.h, ctypes.byref(m)), "selftest")
        return m.value

    def selftest_mfma_fp4(self):
        m = ctypes.c_int()
        self._chk(self.L.vcfxg_selftest_mfma_fp4(self.h, ctypes.byref(m)), "selftest")
        return m.value

    def text(self, nbytes):
        b = ctypes.create_string_buffer(max(1, nbytes))
        self._chk(self.L.vcfxg_fetch_text(self.h, b, nbytes), "fetch_text")
        return b.raw[:nbytes]

    def lines(self, n):
        import numpy as np
        alt = np.zeros(n, np.int32)
        tot = np.zeros(n, np.int32)
        st = np.zeros(n, np.uint8)
        self._chk(self.L.vcfxg_fetch_lines(self.h, 0, n, alt.ctypes.data, tot.ctypes.data, st.ctypes.data),
                  "fetch_lines")
        return alt, tot, st

    def statuses(self, n):
        """per-line status bytes of the last call (no counts)."""
        import numpy as np
        st = np.zeros(max(n, 1), np.uint8)
        self._chk(self.L.vcfxg_fetch_lines(self.h, 0, n, None, None, st.ctypes.data), "fetch_lines")
        return st[:n]

    def line_ends(self, n):
        import numpy as np
        out = np.zeros(n, np.uint64)
        self._chk(self.L.vcfxg_line_ends(self.h, 0, n, out.ctypes.data), "line_ends")
        return out


BGZF_MEMBER = None


def bgzf_members(buf):
    """The BGZF member table of buf (numpy uint8) for vcfxg_ingest_bgzf: every member a gzip
    member with FLG exactly FEXTRA and a 'BC' subfield (SAM/BAM spec §4.1), ISIZE <= 65536;
    raises ValueError otherwise (not a complete BGZF chain: the host inflates it)."""
    import numpy as np
    global BGZF_MEMBER
    if BGZF_MEMBER is None:
        BGZF_MEMBER = np.dtype([("src_off", "<u8"), ("src_len", "<u4"), ("out_len", "<u4")])
    b = bytes(buf) if not isinstance(buf, (bytes, bytearray)) else buf
    out, p, n = [], 0, len(b)
    while p < n:
        if n - p < 18 or b[p] != 0x1F or b[p + 1] != 0x8B or b[p + 2] != 8 or b[p + 3] != 4:
            raise ValueError("not a BGZF member at %d" % p)
        xlen = b[p + 10] | b[p + 11] << 8
        k, bs = 12, 0
        while k + 4 <= 12 + xlen and p + k + 4 <= n:
            slen = b[p + k + 2] | b[p + k + 3] << 8
            if b[p + k] == 66 and b[p + k + 1] == 67 and slen == 2:
                bs = (b[p + k + 4] | b[p + k + 5] << 8) + 1
            k += 4 + slen
        if not bs or p + bs > n or bs < 12 + xlen + 8:
            raise ValueError("bad BGZF member at %d" % p)
        isize = int.from_bytes(b[p + bs - 4:p + bs], "little")
        if isize > 65536:
            raise ValueError("ISIZE over 64 KiB at %d" % p)
        out.append((p, bs, isize))
        p += bs
    return np.array(out, dtype=BGZF_MEMBER)


def shard_cuts(buf, lo, world):
    """vcfxg_shard_cuts: world + 1 record-aligned cut offsets over [lo, len(buf)) (no device)"""
    import numpy as np
    arr = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    cuts = np.zeros(world + 1, np.uint64)
    rc = lib().vcfxg_shard_cuts(arr.ctypes.data, arr.size, lo, world, cuts.ctypes.data)
    if rc != VCFXG_OK:
        raise EngineError("vcfxg_shard_cuts failed (%d)" % rc)
    return [int(x) for x in cuts]


def data_start_of(buf, strip_cr=True):
    """Byte offset just after the first '#CHROM' line (len(buf) if none)."""
    p = 0
    n = len(buf)
    while p < n:
        e = buf.find(b"\n", p)
        e = n if e < 0 else e
        line = buf[p:e]
        if strip_cr and line.endswith(b"\r"):
            line = line[:-1]
        nxt = e + 1 if e < n else n
        if line[:6] == b"#CHROM":
            return nxt
        p = nxt
    return n
