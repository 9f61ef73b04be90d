"""C1 pixel-space DDPM UNet — fp32 CPU restatement (TEST INFRASTRUCTURE ONLY).

Follows ``DDPM/models/unet.py:11-80`` and ``DDPM/models/layers.py`` (file:line below) as functional
torch-CPU code over a state_dict with the reference's parameter names:
* positional encoding pe[t] (sin even / cos odd columns, ``layers.py:6-30``) → Linear → GELU → Linear;
* ConvBlock conv3x3 → GroupNorm → SiLU (``:33-48``); ResNetBlock h = block1(x) + Linear(SiLU(temb));
  block2(h) + residual_conv(x) (``:300-338``);
* SelfAttentionBlock: GroupNorm(final_proj(attn(q, k, v)) + x), heads of C/4, scale d^-1/2 (``:135-192``);
* DownsampleBlock conv s2 p1; UpsampleBlock bilinear x2 align_corners=True + conv (``:51-72``).
Pinned by tests/golden/ddpm_unet.npz (the reference UNet itself, synthetic weights).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def _conv(x, sd, p, stride=1):
    w = sd[p + ".weight"]
    return F.conv2d(x, w, sd[p + ".bias"], stride=stride, padding=w.shape[-1] // 2)


def _gn(x, sd, p, groups=32):
    return F.group_norm(x, groups, sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def _lin(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def pe_table(dim=128, max_timesteps=1000):
    pe = torch.zeros(max_timesteps, dim)
    even = torch.arange(0, dim, 2)
    div = torch.exp(even * -(torch.log(torch.tensor(10000.0)) / dim))
    ts = torch.arange(max_timesteps).unsqueeze(1)
    pe[:, 0::2] = torch.sin(ts * div)
    pe[:, 1::2] = torch.cos(ts * div)
    return pe


def _resnet(sd, p, x, temb):
    h = F.silu(_gn(_conv(x, sd, p + ".block1.conv"), sd, p + ".block1.norm"))
    te = _lin(F.silu(temb), sd, p + ".time_embedding_projectile.1")
    h = h + te[:, :, None, None]
    h = F.silu(_gn(_conv(h, sd, p + ".block2.conv"), sd, p + ".block2.norm"))
    r = _conv(x, sd, p + ".residual_conv") if (p + ".residual_conv.weight") in sd else x
    return h + r


def _attn(sd, p, x, heads=4):
    b, c, hh, ww = x.shape
    t = x.view(b, c, hh * ww).transpose(1, 2)
    d = c // heads
    split = lambda y: y.view(b, hh * ww, heads, d).transpose(1, 2)
    q, k, v = (split(_lin(t, sd, p + f".{n}_projection")) for n in ("query", "key", "value"))
    o = torch.softmax(q @ k.transpose(-1, -2) * d ** -0.5, dim=-1) @ v
    o = o.transpose(1, 2).reshape(b, hh * ww, c)
    o = _lin(o, sd, p + ".final_projection").transpose(-1, -2).reshape(b, c, hh, ww)
    return _gn(o + x, sd, p + ".norm")


def _block(sd, p, x, temb, resample):
    i = 0
    while (f"{p}.resnet_blocks.{i}.block1.conv.weight") in sd:
        x = _resnet(sd, f"{p}.resnet_blocks.{i}", x, temb)
        if (f"{p}.attention_blocks.{i}.norm.weight") in sd:
            x = _attn(sd, f"{p}.attention_blocks.{i}", x)
        i += 1
    if resample == "down" and (p + ".downsample.conv.weight") in sd:
        x = _conv(x, sd, p + ".downsample.conv", stride=2)
    if resample == "up" and (p + ".upsample.conv.weight") in sd:
        x = F.interpolate(x, scale_factor=2.0, mode="bilinear", align_corners=True)
        x = _conv(x, sd, p + ".upsample.conv")
    return x


@torch.no_grad()
def unet_forward(sd: dict, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    sd = {k: v.float() for k, v in sd.items()}
    temb = pe_table()[t]
    temb = _lin(F.gelu(_lin(temb, sd, "positional_encoding.1")), sd, "positional_encoding.3")
    x0 = _conv(x.float(), sd, "initial_conv")
    skips, h = [x0], x0
    for i in range(5):
        h = _block(sd, f"downsample_blocks.{i}", h, temb, "down")
        skips.append(h)
    skips = skips[::-1]
    h = _block(sd, "bottleneck", h, temb, None)
    for i in range(5):
        h = _block(sd, f"upsample_blocks.{i}", torch.cat([h, skips[i]], 1), temb, "up")
    h = torch.cat([h, skips[-1]], 1)
    return _conv(F.silu(_gn(h, sd, "output_conv.0")), sd, "output_conv.2")
