"""In-process runs of the VCFX_<tool> drop-ins (libvcfx_tools.so).

Mirrors the reference's Python wrapper contract (python/tools/base.py:51-75: argv + stdin
bytes in, stdout/stderr/exit code out) without spawning a process per call, so one GPU
context serves many calls."""
import ctypes
import os
import tempfile

from . import TOOLS_LIB

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(TOOLS_LIB):
            raise RuntimeError("libvcfx_tools.so not built")
        _lib = ctypes.CDLL(TOOLS_LIB)
        _lib.vcfx_tool_main.restype = ctypes.c_int
        _lib.vcfx_tool_main.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib.vcfx_tool_main_sharded.restype = ctypes.c_int
        _lib.vcfx_tool_main_sharded.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib.vcfx_shard_plan.restype = ctypes.c_int
        _lib.vcfx_shard_plan.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int)]
    return _lib


def run(argv, stdin=None, cwd=None, ngpu=1):
    """Run tool argv[0] with argv; returns (stdout bytes, stderr bytes, exit code).  ngpu > 1:
    the in-process multi-GPU run (vcfx_tool_main_sharded, ranks round robin over the devices)."""
    L = lib()
    old = os.getcwd()
    with tempfile.TemporaryFile() as fi, tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
        if stdin:
            fi.write(stdin)
            fi.flush()
            fi.seek(0)
        arr = (ctypes.c_char_p * (len(argv) + 1))(*[a.encode() for a in argv], None)
        if cwd:
            os.chdir(cwd)
        try:
            if ngpu > 1:
                rc = L.vcfx_tool_main_sharded(argv[0].encode(), len(argv), arr, fi.fileno(), fo.fileno(), fe.fileno(),
                                              ngpu)
            else:
                rc = L.vcfx_tool_main(argv[0].encode(), len(argv), arr, fi.fileno(), fo.fileno(), fe.fileno())
        finally:
            os.chdir(old)
        if rc == -100:
            raise NotImplementedError(argv[0])
        fo.seek(0)
        fe.seek(0)
        return fo.read(), fe.read(), rc


def shard_plan(argv, ngpu):
    """(ranks, kind, cuts) of the in-process multi-GPU run of argv at ngpu (host only)"""
    L = lib()
    arr = (ctypes.c_char_p * (len(argv) + 1))(*[a.encode() for a in argv], None)
    cuts = (ctypes.c_uint64 * (ngpu + 1))()
    kind = ctypes.c_int(0)
    w = L.vcfx_shard_plan(argv[0].encode(), len(argv), arr, ngpu, cuts, ctypes.byref(kind))
    return w, kind.value, list(cuts[:w + 1]) if kind.value in (1, 3) else None


def run_pipe(argv, stdin=b"", cwd=None):
    """run() with stdin as a pipe (the tools' streaming stdin path: not a regular file, so it is
    read, not mapped).  A writer thread feeds the pipe while the tool runs."""
    import threading
    L = lib()
    old = os.getcwd()
    rfd, wfd = os.pipe()

    def feed():
        try:
            mv = memoryview(stdin or b"")
            while mv:
                k = os.write(wfd, mv[:1 << 20])
                mv = mv[k:]
        except OSError:
            pass
        finally:
            os.close(wfd)

    th = threading.Thread(target=feed, daemon=True)
    th.start()
    with tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
        arr = (ctypes.c_char_p * (len(argv) + 1))(*[a.encode() for a in argv], None)
        if cwd:
            os.chdir(cwd)
        try:
            rc = L.vcfx_tool_main(argv[0].encode(), len(argv), arr, rfd, fo.fileno(), fe.fileno())
        finally:
            os.chdir(old)
            os.close(rfd)  # a tool that stops early: the writer sees EPIPE
            th.join()
        if rc == -100:
            raise NotImplementedError(argv[0])
        fo.seek(0)
        fe.seek(0)
        return fo.read(), fe.read(), rc


def pipeline_filter_query(filter_, query, input_path=None, stdin=None, logic="and", strict=False, gq_quiet=False,
                          cwd=None):
    """Fused `VCFX_record_filter --filter F --logic L [input] | VCFX_genotype_query -g Q`."""
    L = lib()
    f = L.vcfx_pipeline_filter_query
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                  ctypes.c_int, ctypes.c_int, ctypes.c_int]
    old = os.getcwd()
    with tempfile.TemporaryFile() as fi, tempfile.TemporaryFile() as fo, tempfile.TemporaryFile() as fe:
        if stdin:
            fi.write(stdin)
            fi.flush()
            fi.seek(0)
        if cwd:
            os.chdir(cwd)
        try:
            rc = f(filter_.encode(), logic.encode(), input_path.encode() if input_path else None, query.encode(),
                   int(strict), int(gq_quiet), fi.fileno(), fo.fileno(), fe.fileno())
        finally:
            os.chdir(old)
        fo.seek(0)
        fe.seek(0)
        return fo.read(), fe.read(), rc
