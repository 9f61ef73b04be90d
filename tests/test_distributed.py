"""Multi-rank host logic of the sampling path on the CPU (gloo, world_size 2).

Each rank takes its shard of the host-generated global batch, runs the DDIM update
(oracle restatement, the CPU checker) on it, and the all-gather reassembles the
global result; it must equal the single-process result bit for bit, and the timing
reduction must return the slowest rank's value."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sd_amd_loader

sd_amd_loader.load()
from sd_amd import distributed as sdd  # noqa: E402
from oracle import schedule as osch  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _pipeline(x, eps_seed):
    """Stand-in per-sample step: DDIM update of x with a deterministic per-row eps."""
    sc = osch.ddim_step_scalars(osch.ddim_tables(50, 0.0), 10)
    g = torch.Generator().manual_seed(eps_seed)
    eps = torch.randn(x.shape, generator=g)
    return torch.from_numpy(osch.ddim_step(x.numpy(), eps.numpy(), sc, None)[0])


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        xg, cg = sdd.global_inputs(2024, world, 3, (4, 8, 8), (5, 16))
        x, c = sdd.shard(xg, rank, world), sdd.shard(cg, rank, world)
        assert x.shape[0] == 3 and c.shape[0] == 3
        # per-row eps seeded by the global row index: shard-independent
        y = torch.cat([_pipeline(x[i:i + 1], 100 + rank * 3 + i) for i in range(3)])
        full = sdd.gather(y, world)
        t = sdd.max_over_ranks(0.5 + rank)
        if rank == 0:
            out_q.put((full, t))
    finally:
        dist.destroy_process_group()


def test_shard_gather_matches_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    xg, _ = sdd.global_inputs(2024, world, 3, (4, 8, 8), (5, 16))
    ref = torch.cat([_pipeline(xg[i:i + 1], 100 + i) for i in range(world * 3)])
    assert torch.equal(full, ref)
    assert t == 1.5


def test_shard_rejects_ragged_batch():
    with pytest.raises(ValueError):
        sdd.shard(torch.zeros(5, 2), 0, 2)
