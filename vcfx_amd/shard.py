"""Record-sharded multi-GPU runs of the drop-in tools.

One process per GPU (torchrun); rank r opens the engine on LOCAL_RANK and runs the tool on its
share of ONE input file:

* VCFX_allele_freq_calc -i FILE: the data region (after the '#CHROM' line) is cut at
  i*size/N and each cut advanced past the next '\\n' (the reference's own sharding pattern,
  VCFX_allele_counter.cpp:889-901).  Rank r runs the tool on header + its records; rank 0
  writes the header row and every rank's rows in rank order; the stderr totals
  ("Processed V variants from L data lines") are all-reduced.
* VCFX_variant_counter FILE: the whole file is cut the same way; "Total Variants" is
  all-reduced; warning line numbers are shifted to whole-file numbering; under --strict the
  earliest failing line of any rank wins.
* VCFX_record_filter / VCFX_genotype_query / VCFX_nonref_filter with a file input: the
  records are cut the same way; every rank runs the filter on header + its records, and
  once more on the header alone to learn the header's own output (H, E), which it strips
  from its outputs; rank 0 writes H and E once, then the ranks' kept lines and warnings in
  rank order.  Files with data lines before '#CHROM' run unsharded.
* VCFX_ld_calculator -i FILE (streaming): every rank parses the file and computes the pair
  rows of its `--shard r/N` share (equal window-pair counts); rank 0 writes the header and
  the ranks' pair lines in rank order.  Matrix mode runs on rank 0 only.

Per-rank outputs are gathered to rank 0 (the only writer of stdout/stderr, so pipes work);
the only reductions are the global counts.  Other invocations (stdin input, other tools)
run unsharded on rank 0.  The collectives go through torch.distributed, so the same code
runs over RCCL (nccl backend, device tensors) on MI355X nodes and over gloo in the CPU tests.
"""
import os
import re
import sys
import tempfile

import numpy as np

_SHM = "/dev/shm" if os.path.isdir("/dev/shm") else None


# ---------------------------------------------------------------------------------------
# host-side cut logic
# ---------------------------------------------------------------------------------------
def header_end(buf, strip_cr=True):
    """Offset just after the first '#CHROM' line (len(buf) if none): the tools' '#CHROM'
    gate (engine.data_start_of), searched in growing prefixes of a memory-mapped file."""
    n = len(buf)
    w = min(n, 1 << 20)
    while True:
        pre = bytes(buf[:w])
        p = 0
        while p < w:
            e = pre.find(b"\n", p)
            if e < 0:
                if w < n:
                    break  # the line continues past the window
                e = w
            line = pre[p:e]
            if strip_cr and line.endswith(b"\r"):
                line = line[:-1]
            if line[:6] == b"#CHROM":
                return min(e + 1, n)
            p = e + 1
        if w >= n:
            return n
        w = min(n, w * 4)


def record_cuts(buf, lo, world):
    """world+1 cut offsets over [lo, len(buf)): cut i at lo + i*size/world advanced to the
    first line start at or after it; shard i = [cuts[i], cuts[i+1])."""
    arr = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    n = arr.size
    cuts = [lo]
    for i in range(1, world):
        p = lo + (n - lo) * i // world
        p = max(p, cuts[-1])
        if p > lo and p < n and arr[p - 1] != 10:
            nl = np.flatnonzero(arr[p:min(n, p + (1 << 24))] == 10)
            while nl.size == 0 and p < n:  # a line longer than the probe window
                p += 1 << 24
                nl = np.flatnonzero(arr[p:min(n, p + (1 << 24))] == 10)
            p = n if nl.size == 0 else p + int(nl[0]) + 1
        cuts.append(min(p, n))
    cuts.append(n)
    return cuts


def _write_shard(parts):
    f = tempfile.NamedTemporaryFile(prefix="vcfx_shard_", suffix=".vcf", dir=_SHM, delete=False)
    for p in parts:
        f.write(memoryview(p))
    f.close()
    return f.name


# ---------------------------------------------------------------------------------------
# collectives (torch.distributed; gloo -> CPU tensors, nccl -> device tensors)
# ---------------------------------------------------------------------------------------
class Comm:
    def __init__(self, dist=None):
        self.dist = dist
        if dist is None:
            self.rank, self.world = 0, 1
            return
        import torch
        self.torch = torch
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" \
            else torch.device("cpu")

    def allreduce(self, vals, op="sum"):
        if self.dist is None:
            return list(vals)
        t = self.torch.tensor(list(vals), dtype=self.torch.int64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN if op == "min" else self.dist.ReduceOp.SUM)
        return [int(x) for x in t.cpu().tolist()]

    def gather_bytes(self, b):
        """every rank's bytes, in rank order, on every rank (all_gather of padded tensors)."""
        if self.dist is None:
            return [b]
        torch = self.torch
        n = torch.tensor([len(b)], dtype=torch.int64, device=self.dev)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n)
        sizes = [int(s.item()) for s in sizes]
        m = max(1, max(sizes))
        mine = torch.zeros(m, dtype=torch.uint8)
        if b:
            mine[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        mine = mine.to(self.dev)
        out = [torch.empty(m, dtype=torch.uint8, device=self.dev) for _ in range(self.world)]
        self.dist.all_gather(out, mine)
        return [bytes(o[:s].cpu().numpy().tobytes()) for o, s in zip(out, sizes)]


# ---------------------------------------------------------------------------------------
# per-tool sharded runs; runner(argv, stdin) -> (stdout, stderr, rc)
# ---------------------------------------------------------------------------------------
def _input_path(argv, short="-i", long_="--input", positional=False):
    """the input file named by -i/--input (or, with positional, the first operand); None
    unless it is a regular file"""
    path = None
    i = 1
    while i < len(argv):
        a = argv[i]
        if a in (short, long_) and i + 1 < len(argv):
            path = argv[i + 1]
            break
        if a.startswith(long_ + "="):
            path = a.split("=", 1)[1]
            break
        if positional and not a.startswith("-") and path is None:
            path = a
        i += 1
    return path if path and os.path.isfile(path) else None


_AF_PROCESSED = re.compile(rb"^Processed (\d+) variants from (\d+) data lines\n", re.M)
_AF_HEAD = b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n"
_AF_PRE = b"Warning: Data line encountered before #CHROM header. Skipping.\n"
_AF_FIELDS = b"Warning: Skipping invalid VCF line (fewer than 9 fields).\n"


def run_af(argv, comm, runner):
    path = _input_path(argv, positional=True)
    quiet = "-q" in argv or "--quiet" in argv
    buf = np.memmap(path, np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
    ds = header_end(buf)
    cuts = record_cuts(buf, ds, comm.world)
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    shard = _write_shard([buf[:ds], buf[lo:hi]])
    try:
        sargv = [a if a != path else shard for a in argv]
        out, err, rc = runner(sargv, b"")
    finally:
        os.unlink(shard)
    m = _AF_PROCESSED.search(err)
    v, lines = (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    tot = comm.allreduce([v, lines, rc])
    outs = comm.gather_bytes(out[len(_AF_HEAD):] if out.startswith(_AF_HEAD) else out)
    warns = comm.gather_bytes(_AF_FIELDS * err.count(_AF_FIELDS))
    if comm.rank:
        return b"", b"", 0
    rc = 1 if tot[2] else 0
    stdout = _AF_HEAD + b"".join(outs)
    if quiet:
        return stdout, b"", rc
    size_mb = len(buf) // (1024 * 1024)
    stderr = ("Processing %s (%d MB)\n" % (path, size_mb)).encode() + _AF_PRE * err.count(_AF_PRE) + b"".join(warns)
    stderr += b"Processed %d variants from %d data lines\n" % (tot[0], tot[1])
    return stdout, stderr, rc


_VC_WARN = re.compile(rb"^(Warning: skipping line |Error: line )(\d+)( .*\n)", re.M)


def run_vc(argv, comm, runner):
    path = _input_path(argv, "", "", positional=True)
    buf = np.memmap(path, np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
    if len(buf) >= 2 and buf[0] == 0x1F and buf[1] == 0x8B:
        if comm.rank:
            return b"", b"", 0
        return runner(argv, b"")  # gzip input: not shardable by bytes
    cuts = record_cuts(buf, 0, comm.world)
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    before = int(np.count_nonzero(buf[:lo] == 10))  # lines of earlier shards
    shard = _write_shard([buf[lo:hi]])
    try:
        out, err, rc = runner([a if a != path else shard for a in argv], b"")
    finally:
        os.unlink(shard)
    err = _VC_WARN.sub(lambda m: m.group(1) + str(int(m.group(2)) + before).encode() + m.group(3), err)
    m = re.search(rb"Total Variants: (\d+)", out)
    total = int(m.group(1)) if m else 0
    first_err = int(_VC_WARN.search(err).group(2)) if rc and _VC_WARN.search(err) else (1 << 62)
    red = comm.allreduce([total])
    fe = comm.allreduce([first_err], op="min")[0]
    errs = comm.gather_bytes(err if not rc else b"")
    fails = comm.gather_bytes(err if rc else b"")
    if comm.rank:
        return b"", b"", 0
    if fe < (1 << 62):  # --strict: the earliest failing line of any rank, nothing on stdout
        for r, f in enumerate(fails):
            if f and int(_VC_WARN.search(f).group(2)) == fe:
                return b"", b"".join(errs[:r]) + f, 1
    return b"Total Variants: %d\n" % red[0], b"".join(errs), 0


def _pre_header_data(buf, ds):
    """a data line (not empty, not '#') before the '#CHROM' line"""
    for line in bytes(buf[:ds]).split(b"\n"):
        line = line[:-1] if line.endswith(b"\r") else line
        if line and not line.startswith(b"#"):
            return True
    return False


def run_filter(argv, comm, runner, path):
    buf = np.memmap(path, np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)
    ds = header_end(buf)
    plain = ds < len(buf) and not _pre_header_data(buf, ds)
    ok = comm.allreduce([1 if plain else 0], op="min")[0]
    out = err = b""
    rc = 0
    if ok:
        cuts = record_cuts(buf, ds, comm.world)
        lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
        head = _write_shard([buf[:ds]])
        shard = _write_shard([buf[:ds], buf[lo:hi]])
        try:
            H, E, _ = runner([a if a != path else head for a in argv], b"")
            out, err, rc = runner([a if a != path else shard for a in argv], b"")
        finally:
            os.unlink(head)
            os.unlink(shard)
        good = out.startswith(H) and err.startswith(E)
        ok = comm.allreduce([1 if good else 0], op="min")[0]
        out, err = out[len(H):], err[len(E):]
    if not ok:  # unsharded on rank 0
        if comm.rank:
            return b"", b"", 0
        return runner(argv, b"")
    outs = comm.gather_bytes(out)
    errs = comm.gather_bytes(err)
    rcs = comm.allreduce([rc])
    if comm.rank:
        return b"", b"", 0
    return H + b"".join(outs), E + b"".join(errs), 1 if rcs[0] else 0


def run_ld(argv, comm, runner):
    out, err, rc = runner(argv + ["--shard", "%d/%d" % (comm.rank, comm.world)], b"")
    outs = comm.gather_bytes(out)
    errs = comm.gather_bytes(err)
    rcs = comm.allreduce([rc])
    if comm.rank:
        return b"", b"", 0
    return b"".join(outs), b"".join(errs), 1 if rcs[0] else 0


def run_sharded(argv, stdin=b"", dist=None, runner=None):
    """Run one tool invocation across the ranks of `dist` (None = single process).  Returns
    (stdout, stderr, rc) on rank 0 and empty results on the other ranks."""
    if runner is None:
        from . import tools
        runner = tools.run
    comm = Comm(dist)
    tool = os.path.basename(argv[0])
    if comm.world > 1 and not any(a in ("-h", "--help", "-v", "--version") for a in argv[1:]):
        if tool == "VCFX_allele_freq_calc" and _input_path(argv, positional=True):
            return run_af(argv, comm, runner)
        if tool == "VCFX_variant_counter" and _input_path(argv, "", "", positional=True):
            return run_vc(argv, comm, runner)
        if tool == "VCFX_ld_calculator" and _input_path(argv) and not ("-m" in argv or "--matrix" in argv):
            return run_ld(argv, comm, runner)
        if tool in ("VCFX_record_filter", "VCFX_genotype_query", "VCFX_nonref_filter"):
            path = _input_path(argv, positional=True)
            if path:
                return run_filter(argv, comm, runner, path)
    if comm.rank:
        return b"", b"", 0
    return runner(argv, stdin)


def main():
    """python -m vcfx_amd.shard VCFX_<tool> [args]   (under torchrun: one rank per GPU)"""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        backend = os.environ.get("VCFX_DIST_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        tdist.init_process_group(backend)
        dist = tdist
    argv = sys.argv[1:]
    if "VCFX_DEVICE" not in os.environ:  # the tools open this device (hostio.cpp gpu())
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if os.environ.get("VCFX_DIST_BACKEND", "nccl") != "nccl":  # e.g. a gloo rehearsal on one GPU
            import ctypes
            from . import engine
            n = ctypes.c_int(0)
            engine.lib().vcfxg_device_count(ctypes.byref(n))
            local = local % max(1, n.value)
        os.environ["VCFX_DEVICE"] = str(local)
    stdin = b"" if dist is not None and dist.get_rank() else (sys.stdin.buffer.read() if not sys.stdin.isatty()
                                                              and not _input_path(argv) else b"")
    out, err, rc = run_sharded(argv, stdin, dist)
    if dist is not None:
        dist.destroy_process_group()
    sys.stdout.buffer.write(out)
    sys.stdout.flush()
    sys.stderr.buffer.write(err)
    sys.stderr.flush()
    return rc


if __name__ == "__main__":
    sys.exit(main())
