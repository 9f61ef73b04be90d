"""Mirror of ``openai_model/utils.py`` (GroupNorm32, conv_nd, linear, zero_module, timestep_embedding).

The nn modules here are parameter holders with the reference's names; the
compute happens in libsdk_amd.so through ``sd_amd.ops``.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .. import ops


class GroupNorm32(nn.GroupNorm):
    """Reference ``openai_model/utils.py:15-22`` (32 groups, eps 1e-5).  ``stats`` returns
    the per-(batch, channel) affine the conv kernel applies in its prologue."""

    def _prepare(self, dev):
        self._g = self.weight.detach().to(dev, torch.float32).contiguous()
        self._b = self.bias.detach().to(dev, torch.float32).contiguous()

    def stats(self, x):
        return ops.group_norm_affine(x, self._g, self._b, self.eps, self.num_groups)

    def scale_shift(self, x):
        """(scale, shift) [B, C] of this GroupNorm of x (from the producers' statistics) for a conv that
        applies it to its own staged input (ops.group_norm_scale_shift)."""
        return ops.group_norm_scale_shift(x, self._g, self._b, self.eps, self.num_groups)

    def norm(self, x, silu=True, pad=0):
        """GroupNorm (+ SiLU) of x materialised (zero-bordered by ``pad``) — one ``sdk_group_norm``."""
        return ops.group_norm(x, self._g, self._b, self.eps, self.num_groups, silu=silu, pad=pad)

    def forward(self, x):
        raise NotImplementedError("sd_amd: GroupNorm32 runs fused inside the HIP conv (use the parent block)")


def normalization(channels):
    return GroupNorm32(32, channels)


def conv_nd(dims, *args, **kwargs):
    if dims == 1:
        return nn.Conv1d(*args, **kwargs)
    if dims == 2:
        return nn.Conv2d(*args, **kwargs)
    raise ValueError(f"sd_amd: unsupported dims: {dims}")


def avg_pool_nd(dims, *args, **kwargs):
    if dims == 2:
        return nn.AvgPool2d(*args, **kwargs)
    raise ValueError(f"sd_amd: unsupported dims: {dims}")


def linear(*args, **kwargs):
    return nn.Linear(*args, **kwargs)


def zero_module(module):
    for p in module.parameters():
        p.detach().zero_()
    return module


def timestep_frequencies(dim: int, max_period: int = 10000) -> torch.Tensor:
    """freqs = exp(-ln(max_period) * k / half) computed once on the host exactly as the
    reference does (``openai_model/utils.py:235-238``); the sin/cos run on the device."""
    half = dim // 2
    return torch.exp(-math.log(max_period) * torch.arange(start=0, end=half, dtype=torch.float32) / half)


def timestep_embedding(timesteps, dim, max_period=10000, repeat_only=False):
    """Device timestep embedding (fp16, as fed to time_embed) — ``openai_model/utils.py:225-245``."""
    if repeat_only:
        raise NotImplementedError("sd_amd: repeat_only timestep embedding is not on the hot path")
    if dim % 2:
        raise ValueError("sd_amd: odd embedding width not supported on the device path")
    freqs = timestep_frequencies(dim, max_period).to(timesteps.device)
    return ops.timestep_embedding(timesteps.long(), freqs, dim)
