"""Data-parallel host logic for the sampling path (one process per GPU).

The hot path has no per-step exchange: every latent of a global batch is sampled
independently (reference: ``DDIMSampler.sample`` loops over a batch whose rows never
interact, ``ldm/models/diffusion/ddim.py``), so N GPUs shard the batch and run the
whole 50-step loop + VAE decode locally.  The only collective is one all-gather of
the decoded images (RCCL over xGMI with backend "nccl"; "gloo" in the CPU tests).

* ``global_inputs`` draws the global batch on the host from one seed, so results do
  not depend on the rank count;
* ``shard`` gives rank r rows [r*B, (r+1)*B);
* ``gather`` reassembles the global batch in rank order;
* ``max_over_ranks`` is the bench's timing reduction (slowest rank)."""
from __future__ import annotations

import torch


def world_info():
    import os
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def global_inputs(seed: int, world: int, batch: int, latent_shape, ctx_shape=None):
    """Host-generated global batch: (x_T [world*B, *latent], context [world*B, *ctx] or None)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(world * batch, *latent_shape, generator=g)
    c = torch.randn(world * batch, *ctx_shape, generator=g) if ctx_shape else None
    return x, c


def shard(t, rank: int, world: int):
    if t is None:
        return None
    if t.shape[0] % world:
        raise ValueError(f"global batch {t.shape[0]} is not divisible by world size {world}")
    b = t.shape[0] // world
    return t[rank * b:(rank + 1) * b]


def gather(local, world: int, out=None):
    """All-gather the per-rank results along dim 0 (rank order)."""
    import torch.distributed as dist
    if world == 1:
        return local
    local = local.contiguous()
    if out is None:
        out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    # the same call on both backends (RCCL on the GPU, gloo in the CPU rehearsal), so the tests
    # execute the exact collective the 8-GPU run issues
    dist.all_gather_into_tensor(out, local)
    return out


def max_over_ranks(value: float, device=None) -> float:
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
