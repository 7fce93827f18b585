"""GPU parity of the record-sharded multi-GPU path: two ranks (a gloo group over 127.0.0.1,
both on cuda:0 -- the 1-GPU rehearsal of the torchrun layout) run the real drop-in tools on
their shares and the merged rank-0 output must equal the single-process GPU run (itself
pinned to the oracle by the other GPU tests), for AF (record shards), VC (record shards)
and LD streaming (row shards via --shard r/N)."""
import os
import socket
import tempfile

import pytest

from vcfx_amd import synth

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VCFX_DEVICE="0")
    import torch.distributed as dist
    from vcfx_amd import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for argv in cases:
            res = shard.run_sharded(argv, b"", dist)  # the drop-ins on their shard views
            if rank == 0:
                q.put((argv, res))
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_match_single_gpu(tmp_path):
    import torch.multiprocessing as mp
    from vcfx_amd import tools
    p1 = str(tmp_path / "af.vcf")
    open(p1, "wb").write(synth.generate(3000, 257, 71, 1, 0.02, 0, 0.2, 0))
    p2 = str(tmp_path / "ld.vcf")
    open(p2, "wb").write(synth.generate(1500, 300, 72, 0, 0.01, 1, 0.0, 0))
    cases = [["VCFX_allele_freq_calc", "-i", p1], ["VCFX_allele_freq_calc", "-q", p1],
             ["VCFX_variant_counter", p1],
             ["VCFX_record_filter", "--filter", "QUAL>=30;FILTER==PASS", "-i", p1],
             ["VCFX_genotype_query", "-g", "0|1", "-i", p1], ["VCFX_genotype_query", "-g", "1|1", "--strict", p1],
             ["VCFX_nonref_filter", "-i", p1], ["VCFX_nonref_filter", p1], ["VCFX_dosage_calculator", "-i", p1],
             ["VCFX_ld_calculator", "-i", p2, "-w", "300", "-t", "0.2"],
             ["VCFX_ld_calculator", "-i", p2, "-w", "5000"],
             ["VCFX_ld_calculator", "-i", p2, "-m", "-r", "21:9411239-9430000"]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cases, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=600) for _ in cases]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for argv, res in got:
        want = tools.run(argv, b"")
        assert res == want, argv


def _nccl_worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), VCFX_DEVICE="0")
    import torch
    import torch.distributed as dist
    from vcfx_amd import shard
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        c = shard.Comm(dist)
        got = []
        c.to_root(b"abc" * 1000, got.append)
        q.put((c.dev.type, c.allreduce([3, 4]), c.allreduce([5], op="min"), c.sizes(7), b"".join(got)))
    finally:
        dist.destroy_process_group()


def test_comm_over_rccl_device_tensors():
    """shard.Comm on the nccl (RCCL) backend: device tensors for the count reductions and the
    size exchange (one rank: RCCL does not run two ranks on one GPU)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert res == ("cuda", [3, 4], [5], [7], b"abc" * 1000)
