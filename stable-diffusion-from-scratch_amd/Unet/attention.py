"""Mirror of ``Unet/attention.py`` — ``make_attention`` / ``FlashAttentionBlock`` (VAE mid-block attention).

Reference ``attention.py:221-264``: GroupNorm(32, C) with torch's default eps
1e-5, q/k/v 1x1 convs, 8 heads x C/8 through flash_attn with
its default scale d^-1/2, proj_out 1x1, + x.  Here: GN folded into ONE fused
q|k|v GEMM, ``sdk_attention``, proj_out GEMM with the residual epilogue.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import ops
from .unet import _gn_prep, gn_act


class FlashAttentionBlock(nn.Module):
    def __init__(self, in_channels, num_heads=8):
        super().__init__()
        self.in_channels = in_channels
        self.num_heads = num_heads
        self.head_dim = in_channels // num_heads
        assert in_channels % num_heads == 0, "in_channels must be divisible by num_heads"
        self.norm = nn.GroupNorm(32, in_channels)
        self.q = nn.Conv2d(in_channels, in_channels, kernel_size=1)
        self.k = nn.Conv2d(in_channels, in_channels, kernel_size=1)
        self.v = nn.Conv2d(in_channels, in_channels, kernel_size=1)
        self.proj_out = nn.Conv2d(in_channels, in_channels, kernel_size=1)

    def _prepare(self, dev):
        _gn_prep(self.norm, dev)
        w = torch.cat([self.q.weight, self.k.weight, self.v.weight], 0)
        b = torch.cat([self.q.bias, self.k.bias, self.v.bias], 0)
        self._pc_qkv = ops.PackedConv([(w, self.in_channels)], b, device=dev)
        self._pc_o = ops.PackedConv([(self.proj_out.weight, self.in_channels)], self.proj_out.bias, device=dev)

    def _run(self, x):
        B, H, W, C = x.shape
        xn = gn_act(self.norm, x, silu=False)
        qkv = ops.conv2d(self._pc_qkv, xn).view(B * H * W, 3 * C)
        o = ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], batch=B, heads=self.num_heads, nq=H * W,
                          nk=H * W, head_dim=self.head_dim, scale=self.head_dim ** -0.5)
        return ops.conv2d(self._pc_o, o.view(B, H, W, C), residual=x, gn_stats=True)   # feeds a GroupNorm


def make_attention(in_channels, attention_type="vanilla"):
    assert attention_type in ["vanilla", "linear", "none"], f"attention_type {attention_type} not found."
    if attention_type == "vanilla":
        return FlashAttentionBlock(in_channels)
    if attention_type == "none":
        return nn.Identity(in_channels)
    raise NotImplementedError("sd_amd: linear attention is not on the SD path")
