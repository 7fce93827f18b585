"""Record-sharded multi-GPU runs of the drop-in tools.

One process per GPU (torchrun); rank r opens the engine on LOCAL_RANK and runs the tool on its
share of ONE input file.  A share is a VIEW of the file, not a copy: the tool maps the file
and takes the header bytes [0, H) plus its records [LO, HI) (VCFX_INPUT_VIEW="H:LO:HI",
hostio.cpp Input::apply_view); the device input is ingested straight from those two ranges of
the mapping and kept records are written from the mapping.

* VCFX_allele_freq_calc -i FILE: the data region (after the '#CHROM' line) is cut at
  i*size/N and each cut advanced past the next '\\n' (the reference's own sharding pattern,
  VCFX_allele_counter.cpp:889-901).  Rank r runs the tool on header + its records; ranks > 0
  write no header row (VCFX_VIEW_SKIP_HEADER=1); the stderr totals ("Processed V variants
  from L data lines") are all-reduced.
* VCFX_variant_counter FILE: the whole file is cut the same way; "Total Variants" is
  all-reduced; warning line numbers are shifted to whole-file numbering (each rank counts its
  own shard's lines only when some rank warned); under --strict the earliest failing line of
  any rank wins.
* VCFX_record_filter / VCFX_genotype_query / VCFX_nonref_filter / VCFX_dosage_calculator
  with a file input: the records are cut the same way; rank 0's view writes the header part once, ranks > 0 skip it.
  Files with data lines before '#CHROM' run unsharded.
* VCFX_ld_calculator -i FILE (streaming): every rank parses the file and computes the pair
  rows of its `--shard r/N` share (equal window-pair counts); with a window as large as the
  file (BASELINE config 5) every row range needs every variant, so there is nothing to cut.
  Matrix mode runs on rank 0 only.
* A BGZF file (.vcf.gz as bgzip writes it; the AF and filter tools): the same cuts in the
  inflated bytes' coordinates, planned by the drop-in library (vcfx_shard_plan: the member chain
  parsed, the header and the W - 1 members holding the cuts inflated on the host); rank r's
  view is VCFX_INPUT_VIEW="bgzf:H:LO:HI" and its tool inflates the members inside [LO, HI) on
  its own device (hostio.cpp Input::bgzf_view).  Other gzip files run unsharded on rank 0.

Outputs move to rank 0 only -- the only writer of stdout/stderr, so pipes work -- as chunked
point-to-point sends in rank order (64 MiB per message); rank 0 streams each chunk to the sink
as it arrives, so no rank ever holds another rank's output.  The only reductions are the
global counts.  Other invocations (stdin input, other tools) run unsharded on rank 0.  The
collectives go through torch.distributed: RCCL (nccl backend, device tensors) on MI355X nodes,
gloo in the CPU tests.
"""
import os
import re
import sys

import numpy as np

CHUNK = 64 << 20  # bytes per point-to-point message


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
    first line start at or after it; shard i = [cuts[i], cuts[i+1]).  The engine's C ABI
    (vcfxg_shard_cuts) computes them; record_cuts_py is the same rule in numpy (its test)."""
    from . import engine
    return engine.shard_cuts(buf, lo, world)


def record_cuts_py(buf, lo, world):
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


# ---------------------------------------------------------------------------------------
# argv: the input operand, found as each tool's getopt_long finds it
# ---------------------------------------------------------------------------------------
# options that take a value, per tool (the optstrings / long options of the drop-ins, which
# are the reference's: VCFX_allele_freq_calc.cpp:590-646, VCFX_record_filter.cpp:584-658,
# VCFX_genotype_query.cpp:379-428, VCFX_nonref_filter.cpp:646-652, VCFX_ld_calculator.cpp:
# 1084-1209, VCFX_variant_counter.cpp:154-218)
_VALUE_OPTS = {
    "VCFX_allele_freq_calc": ({"-i"}, {"--input"}),
    "VCFX_record_filter": ({"-f", "-l", "-i"}, {"--filter", "--logic"}),
    "VCFX_genotype_query": ({"-g", "-i"}, {"--genotype-query", "--input"}),
    "VCFX_nonref_filter": ({"-i"}, {"--input"}),
    "VCFX_ld_calculator": ({"-i", "-r", "-w", "-t", "-n", "-d"},
                           {"--input", "--region", "--window", "--threshold", "--threads", "--max-distance",
                            "--shard"}),
    "VCFX_variant_counter": (set(), set()),
    "VCFX_dosage_calculator": ({"-i"}, {"--input"}),
}


def parse_args(tool, argv):
    """(options, operands) of argv[1:] the GNU getopt_long way: options may follow operands,
    "--" ends them, a value-taking option consumes the next argument (or its attached /
    '='-joined value).  options: list of (name, value or None)."""
    short_v, long_v = _VALUE_OPTS.get(tool, (set(), set()))
    opts, operands = [], []
    i, args = 0, argv[1:]
    while i < len(args):
        a = args[i]
        if a == "--":
            operands += args[i + 1:]
            break
        if a.startswith("--") and len(a) > 2:
            name, eq, val = a.partition("=")
            if name in long_v and not eq:
                val = args[i + 1] if i + 1 < len(args) else None
                i += 1
            opts.append((name, val if (eq or name in long_v) else None))
        elif a.startswith("-") and len(a) > 1:
            # a cluster of short options; a value-taking one eats the rest or the next arg
            for k in range(1, len(a)):
                o = "-" + a[k]
                if o in short_v:
                    if k + 1 < len(a):
                        opts.append((o, a[k + 1:]))
                    else:
                        opts.append((o, args[i + 1] if i + 1 < len(args) else None))
                        i += 1
                    break
                opts.append((o, None))
        else:
            operands.append(a)
        i += 1
    return opts, operands


def input_path(tool, argv):
    """The input file the tool reads (-i/--input, else the first operand where the tool takes
    one); None when it reads stdin or the path is not a regular file."""
    opts, operands = parse_args(tool, argv)
    path = None
    for name, val in opts:
        if name in ("-i", "--input"):
            path = val
    if path is None and tool != "VCFX_ld_calculator" and operands:
        path = operands[0]
    if path == "-":
        return None
    return path if path and os.path.isfile(path) else None


def is_gzip(path):
    """the gzip magic (1f 8b) at the start of the file: the tools inflate such input whole"""
    try:
        with open(path, "rb") as f:
            return f.read(2) == b"\x1f\x8b"
    except OSError:
        return False


def bgzf_cuts(argv, world):
    """world + 1 cuts of a BGZF input in its inflated bytes (cuts[0] = the header's end) as the
    drop-in library plans them (vcfx_shard_plan kind 3), or None: not a BGZF member chain, data
    before '#CHROM', no records, or fewer non-empty shares than ranks (then: unsharded)"""
    from . import tools
    w, kind, cuts = tools.shard_plan(argv, world)
    return cuts if kind == 3 and w == world else None


def _has_flag(tool, argv, *names):
    opts, _ = parse_args(tool, argv)
    return any(n in names for n, _ in opts)


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

    def sizes(self, n):
        """every rank's int64 n, in rank order."""
        if self.dist is None:
            return [n]
        t = self.torch.tensor([n], dtype=self.torch.int64, device=self.dev)
        out = [self.torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def to_root(self, b, sink):
        """Rank-ordered concatenation of every rank's bytes `b` into sink (a callable taking
        bytes) on rank 0: rank 0's own first, then each rank's in CHUNK-sized point-to-point
        messages, written as they arrive.  Ranks > 0 only send; nothing is all-gathered."""
        if self.dist is None:
            sink(b)
            return
        torch = self.torch
        sizes = self.sizes(len(b))
        if self.rank == 0:
            sink(b)
            buf = None
            for r in range(1, self.world):
                for off in range(0, sizes[r], CHUNK):
                    k = min(CHUNK, sizes[r] - off)
                    if buf is None or buf.numel() < k:
                        buf = torch.empty(min(CHUNK, max(sizes[1:])), dtype=torch.uint8, device=self.dev)
                    self.dist.recv(buf[:k], src=r)
                    sink(buf[:k].cpu().numpy().tobytes())
        else:
            mv = memoryview(b)
            for off in range(0, len(b), CHUNK):
                piece = torch.frombuffer(bytearray(mv[off:off + CHUNK]), dtype=torch.uint8).to(self.dev)
                self.dist.send(piece, dst=0)


# ---------------------------------------------------------------------------------------
# per-tool sharded runs
#   runner(argv, stdin, view=None, skip_header=False) -> (stdout, stderr, rc):
#   view = (H, LO, HI): the tool's input is the file's bytes [0, H) + [LO, HI)
# ---------------------------------------------------------------------------------------
def tool_runner(argv, stdin, view=None, skip_header=False):
    """The in-process drop-in (libvcfx_tools) with the shard view passed in its environment."""
    from . import tools
    keys = ("VCFX_INPUT_VIEW", "VCFX_VIEW_SKIP_HEADER")
    saved = {k: os.environ.get(k) for k in keys}
    try:
        if view is not None:  # (a 4th item "bgzf": offsets into the inflated bytes)
            os.environ["VCFX_INPUT_VIEW"] = ("bgzf:" if len(view) > 3 else "") + "%d:%d:%d" % tuple(view[:3])
        if skip_header:
            os.environ["VCFX_VIEW_SKIP_HEADER"] = "1"
        return tools.run(argv, stdin)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


_AF_PROCESSED = re.compile(rb"^Processed (\d+) variants from (\d+) data lines\n", re.M)
_AF_PROCESSING = re.compile(rb"^Processing .* \(\d+ MB\)\n", re.M)
_AF_HEAD = b"CHROM\tPOS\tID\tREF\tALT\tAllele_Frequency\n"
_AF_PRE = b"Warning: Data line encountered before #CHROM header. Skipping.\n"


def _memmap(path):
    return np.memmap(path, np.uint8, mode="r") if os.path.getsize(path) else np.zeros(0, np.uint8)


class _Sink:
    """rank 0's stdout: a callable sink, or collected bytes"""

    def __init__(self, write=None):
        self.write = write
        self.parts = []

    def __call__(self, b):
        if not b:
            return
        if self.write is not None:
            self.write(b)
        else:
            self.parts.append(bytes(b))

    def value(self):
        return b"".join(self.parts)


def _unsharded(argv, comm, runner):
    if comm.rank:
        return b"", b"", 0
    return runner(argv, b"")


def run_af(argv, comm, runner, path, sink):
    quiet = _has_flag("VCFX_allele_freq_calc", argv, "-q", "--quiet")
    buf = _memmap(path)
    if is_gzip(path):
        cuts = bgzf_cuts(argv, comm.world)
        if cuts is None:
            return _unsharded(argv, comm, runner)
        tag = ("bgzf",)
    else:
        cuts, tag = record_cuts(buf, header_end(buf), comm.world), ()
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    out, err, rc = runner(argv, b"", view=(cuts[0], lo, hi) + tag, skip_header=comm.rank > 0)
    m = _AF_PROCESSED.search(err)
    v, lines = (int(m.group(1)), int(m.group(2))) if m else (0, 0)
    tot = comm.allreduce([v, lines, rc])
    comm.to_root(out, sink)
    # per-rank stderr without the lines rank 0 rewrites (the header part's warnings are
    # rank 0's: its view holds the header)
    err = _AF_PROCESSED.sub(b"", _AF_PROCESSING.sub(b"", err))
    if comm.rank:
        err = err.replace(_AF_PRE, b"")
    errs = _Sink()
    comm.to_root(err, errs)
    if comm.rank:
        return b"", b"", 0
    rc = 1 if tot[2] else 0
    if quiet:
        return None, errs.value(), rc
    stderr = ("Processing %s (%d MB)\n" % (path, len(buf) // (1024 * 1024))).encode() + errs.value()
    stderr += b"Processed %d variants from %d data lines\n" % (tot[0], tot[1])
    return None, stderr, rc


_VC_WARN = re.compile(rb"^(Warning: skipping line |Error: line )(\d+)( .*\n)", re.M)


def run_vc(argv, comm, runner, path, sink):
    buf = _memmap(path)
    cuts = record_cuts(buf, 0, comm.world)
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    out, err, rc = runner(argv, b"", view=(0, lo, hi))
    if comm.allreduce([1 if _VC_WARN.search(err) else 0])[0]:
        # whole-file line numbers: lines of the earlier shards (each rank counts its own)
        mine = int(np.count_nonzero(buf[lo:hi] == 10)) + (1 if hi > lo and buf[hi - 1] != 10 else 0)
        before = sum(comm.sizes(mine)[:comm.rank])
        err = _VC_WARN.sub(lambda m: m.group(1) + str(int(m.group(2)) + before).encode() + m.group(3), err)
    m = re.search(rb"Total Variants: (\d+)", out)
    total = int(m.group(1)) if m else 0
    first_err = int(_VC_WARN.search(err).group(2)) if rc and _VC_WARN.search(err) else (1 << 62)
    red = comm.allreduce([total])
    fe = comm.allreduce([first_err], op="min")[0]
    # --strict: the earliest failing line of any rank; its rank's stderr ends the output
    fail_rank = comm.allreduce([comm.rank if first_err == fe and fe < (1 << 62) else comm.world], op="min")[0]
    errs = _Sink()
    comm.to_root(err if (fe == (1 << 62) or comm.rank <= fail_rank) else b"", errs)
    if comm.rank:
        return b"", b"", 0
    if fe < (1 << 62):
        return b"", errs.value(), 1
    sink(b"Total Variants: %d\n" % red[0])
    return None, errs.value(), 0


def _pre_header_data(buf, ds):
    """a data line (not empty, not '#') before the '#CHROM' line"""
    for line in bytes(buf[:ds]).split(b"\n"):
        line = line[:-1] if line.endswith(b"\r") else line
        if line and not line.startswith(b"#"):
            return True
    return False


def run_filter(argv, comm, runner, path, sink):
    buf = _memmap(path)
    if is_gzip(path):
        cuts, tag = bgzf_cuts(argv, comm.world), ("bgzf",)
        ok = cuts is not None
    else:
        ds, tag = header_end(buf), ()
        ok = ds < len(buf) and not _pre_header_data(buf, ds)
        cuts = record_cuts(buf, ds, comm.world) if ok else None
    if not comm.allreduce([1 if ok else 0], op="min")[0]:  # unsharded on rank 0
        return _unsharded(argv, comm, runner)
    lo, hi = cuts[comm.rank], cuts[comm.rank + 1]
    out, err, rc = runner(argv, b"", view=(cuts[0], lo, hi) + tag, skip_header=comm.rank > 0)
    comm.to_root(out, sink)
    errs = _Sink()
    comm.to_root(err, errs)
    rcs = comm.allreduce([rc])
    if comm.rank:
        return b"", b"", 0
    return None, errs.value(), 1 if rcs[0] else 0


def run_ld(argv, comm, runner, sink):
    out, err, rc = runner(argv + ["--shard", "%d/%d" % (comm.rank, comm.world)], b"")
    comm.to_root(out, sink)
    errs = _Sink()
    comm.to_root(err, errs)
    rcs = comm.allreduce([rc])
    if comm.rank:
        return b"", b"", 0
    return None, errs.value(), 1 if rcs[0] else 0


SHARDED = ("VCFX_allele_freq_calc", "VCFX_variant_counter", "VCFX_ld_calculator", "VCFX_record_filter",
           "VCFX_genotype_query", "VCFX_nonref_filter", "VCFX_dosage_calculator")


def plan(argv):
    """'af' / 'vc' / 'filter' / 'ld' when argv runs sharded at world > 1, else None (stdin
    input, help/version, LD matrix mode, other tools)."""
    tool = os.path.basename(argv[0])
    if tool not in SHARDED:
        return None
    if _has_flag(tool, argv, "-h", "--help", "-v", "--version"):
        return None
    path = input_path(tool, argv)
    if path is None:
        return None
    if tool == "VCFX_ld_calculator":
        # every rank parses the whole (inflated) input and takes a share of the pair rows
        return None if _has_flag(tool, argv, "-m", "--matrix") else "ld"
    if is_gzip(path) and tool == "VCFX_variant_counter":
        # its gzip input is the reference's own (the first member): unsharded on rank 0
        return None
    # (gzip: a BGZF member chain shards in its inflated bytes, bgzf_cuts; other gzip files
    # then run unsharded on rank 0)
    if tool == "VCFX_allele_freq_calc":
        return "af"
    if tool == "VCFX_variant_counter":
        return "vc"
    return "filter"


def run_sharded(argv, stdin=b"", dist=None, runner=None, write=None):
    """Run one tool invocation across the ranks of `dist` (None = single process).  Returns
    (stdout, stderr, rc) on rank 0 and empty results on the other ranks; with `write` (a
    callable) rank 0's stdout is streamed into it instead and returned as b""."""
    runner = runner or tool_runner
    comm = Comm(dist)
    tool = os.path.basename(argv[0])
    how = plan(argv) if comm.world > 1 else None
    if how is None:
        if comm.rank:
            return b"", b"", 0
        out, err, rc = runner(argv, stdin)
        if write is not None:
            write(out)
            out = b""
        return out, err, rc
    sink = _Sink(write)
    path = input_path(tool, argv)
    if how == "af":
        res = run_af(argv, comm, runner, path, sink)
    elif how == "vc":
        res = run_vc(argv, comm, runner, path, sink)
    elif how == "ld":
        res = run_ld(argv, comm, runner, sink)
    else:
        res = run_filter(argv, comm, runner, path, sink)
    if comm.rank:
        return b"", b"", 0
    out, err, rc = res
    if out is None:  # streamed through the sink
        out = sink.value() if write is None else b""
    elif write is not None:
        write(out)
        out = b""
    return out, err, rc


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
    rank0 = dist is None or dist.get_rank() == 0
    tool = os.path.basename(argv[0]) if argv else ""
    # stdin only when the tool reads it (no input file) -- never under an inherited pipe the
    # tool would not read -- and only on rank 0, which runs such invocations
    stdin = sys.stdin.buffer.read() if rank0 and argv and input_path(tool, argv) is None and \
        not sys.stdin.isatty() and not _has_flag(tool, argv, "-h", "--help", "-v", "--version") else b""
    out, err, rc = run_sharded(argv, stdin, dist, write=sys.stdout.buffer.write if rank0 else None)
    if dist is not None:
        dist.destroy_process_group()
    sys.stdout.buffer.write(out)
    sys.stdout.flush()
    sys.stderr.buffer.write(err)
    sys.stderr.flush()
    return rc


if __name__ == "__main__":
    sys.exit(main())
