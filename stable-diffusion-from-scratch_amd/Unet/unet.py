"""Mirror of ``Unet/unet.py`` VAE building blocks (Normalize, Upsample, Downsample, ResnetBlock), HIP-backed.

Reference semantics kept: GroupNorm eps 1e-6 (``unet.py:9-19``), SiLU after each
norm (``unet.py:23-28``; the reference casts to fp16 first — the device path is
fp16 anyway), nearest-x2 + conv3x3 upsample (``unet.py:34-49``), ResnetBlock with
optional 1x1 ``nin_shortcut`` (``unet.py:74-135``).  The shortcut projection is
fused into conv2 as a second K segment; the identity shortcut is the residual
epilogue of conv2.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import ops


def Normalize(in_channels, num_groups=32):
    return nn.GroupNorm(num_groups=num_groups, num_channels=in_channels, eps=1e-6, affine=True)


def _gn_prep(gn, dev):
    gn._g = gn.weight.detach().to(dev, torch.float32).contiguous()
    gn._b = gn.bias.detach().to(dev, torch.float32).contiguous()


def gn_stats(gn, x):
    return ops.group_norm_affine(x, gn._g, gn._b, gn.eps, gn.num_groups)


def gn_act(gn, x, silu=True, pad=0):
    """Normalize (+ nonlinearity) of x materialised, zero-bordered by ``pad`` (``sdk_group_norm``)."""
    return ops.group_norm(x, gn._g, gn._b, gn.eps, gn.num_groups, silu=silu, pad=pad)


class Upsample(nn.Module):
    def __init__(self, in_channels, with_conv):
        super().__init__()
        self.with_conv = with_conv
        self.in_channels = in_channels
        if not with_conv:
            raise NotImplementedError("sd_amd: conv-less VAE Upsample is not on the SD path")
        self.conv = nn.Conv2d(in_channels, in_channels, kernel_size=3, stride=1, padding=1)

    def _prepare(self, dev):
        self._pc = ops.PackedConv([(self.conv.weight, self.in_channels)], self.conv.bias, device=dev)

    def _run(self, x):
        # the output feeds the next ResnetBlock's norm1: the conv emits its GroupNorm statistics.  As in the UNet's
        # Upsample (openai_model/model.py), the nearest-x2 image is written zero-bordered and the 3x3 conv runs
        # unmasked with pad 0 on the linear A issue, instead of folding the upsample into every DMA address
        # (the folded form ran the 512^2 decoder convs at 730-830 TF/s); SD_AMD_UPSAMPLE_FOLD=1 restores it
        # The materialised image is a temporary of B·(2H+2)·(2W+2)·C·2 bytes beside the input and the output: at C5
        # (B = 8, 384 -> 768, 256 channels) 2.4 GB; above UPSAMPLE_MATERIALISE_MAX_BYTES the folded form runs instead
        from ..openai_model.model import UPSAMPLE_FOLD
        n, h, w, c = x.shape
        big = n * (2 * h + 2) * (2 * w + 2) * c * 2 > UPSAMPLE_MATERIALISE_MAX_BYTES
        if UPSAMPLE_FOLD or c % 8 or big:
            return ops.conv2d(self._pc, x, upsample=True, gn_stats=True)
        return ops.conv2d(self._pc, ops.upsample_nearest2x_padded(x, 1), pad=0, gn_stats=True)


UPSAMPLE_MATERIALISE_MAX_BYTES = 8 << 30   # the VAE Upsample's zero-bordered x2 image


class Downsample(nn.Module):
    """Encoder-side downsample (``unet.py:52-71``): F.pad(x, (0,1,0,1)) + conv3x3 s2 p0, run as one
    implicit-GEMM conv with ``pad_end=1`` (the extra bottom/right zero row and column are taps
    that fall outside the source, read as zeros — no padded copy)."""

    def __init__(self, in_channels, with_conv):
        super().__init__()
        self.with_conv = with_conv
        self.in_channels = in_channels
        if with_conv:
            self.conv = nn.Conv2d(in_channels, in_channels, kernel_size=3, stride=2, padding=0)

    def _prepare(self, dev):
        if not self.with_conv:
            raise NotImplementedError("sd_amd: avg-pool Downsample (with_conv=False) is not on the SD path")
        self._pc = ops.PackedConv([(self.conv.weight, self.in_channels)], self.conv.bias, device=dev)

    def _run(self, x):
        return ops.conv2d(self._pc, x, stride=2, pad=0, pad_end=1, gn_stats=True)


class ResnetBlock(nn.Module):
    def __init__(self, *, in_channels, out_channels=None, conv_shortcut=False, dropout, temb_channels=512):
        super().__init__()
        self.in_channels = in_channels
        out_channels = in_channels if out_channels is None else out_channels
        self.out_channels = out_channels
        self.use_conv_shortcut = conv_shortcut
        self.norm1 = Normalize(in_channels)
        self.conv1 = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=1, padding=1)
        if temb_channels > 0:
            self.temb_proj = nn.Linear(temb_channels, out_channels)
        self.norm2 = Normalize(out_channels)
        self.dropout = nn.Dropout(dropout)
        self.conv2 = nn.Conv2d(out_channels, out_channels, kernel_size=3, stride=1, padding=1)
        if self.in_channels != self.out_channels:
            if self.use_conv_shortcut:
                self.conv_shortcut = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=1, padding=1)
            else:
                self.nin_shortcut = nn.Conv2d(in_channels, out_channels, kernel_size=1, stride=1, padding=0)

    def _prepare(self, dev):
        _gn_prep(self.norm1, dev)
        _gn_prep(self.norm2, dev)
        self._pc1 = ops.PackedConv([(self.conv1.weight, self.in_channels)], self.conv1.bias, device=dev)
        self._mode = "identity"
        if self.in_channels != self.out_channels and not self.use_conv_shortcut:
            self._mode = "fused"
            self._pc2 = ops.PackedConv([(self.conv2.weight, self.out_channels),
                                        (self.nin_shortcut.weight, self.in_channels)],
                                       self.conv2.bias.detach() + self.nin_shortcut.bias.detach(), device=dev)
        else:
            self._pc2 = ops.PackedConv([(self.conv2.weight, self.out_channels)], self.conv2.bias, device=dev)
            if self.in_channels != self.out_channels:
                self._mode = "conv3"
                self._pcs = ops.PackedConv([(self.conv_shortcut.weight, self.in_channels)], self.conv_shortcut.bias,
                                           device=dev)

    def _run(self, x, temb=None):
        if temb is not None:
            raise NotImplementedError("sd_amd: the VAE ResnetBlock path has no timestep embedding")
        # zero-bordered GN+SiLU outputs: both 3x3 convs run with pad 0 (mask-free gather); both outputs
        # feed a GroupNorm (norm2 / the next block's norm1, an attention norm or norm_out), so the convs
        # emit its statistics from their epilogues (no statistics pass over the tensor)
        gp, cp = ops.gn_conv_pad()
        h = ops.conv2d(self._pc1, gn_act(self.norm1, x, silu=True, pad=gp), pad=cp, gn_stats=True)
        ha = gn_act(self.norm2, h, silu=True, pad=gp)
        if self._mode == "identity":
            return ops.conv2d(self._pc2, ha, pad=cp, residual=x, gn_stats=True)
        if self._mode == "fused":
            return ops.conv2d(self._pc2, ha, pad=cp, seg2=(x, None, False), gn_stats=True)
        return ops.conv2d(self._pc2, ha, pad=cp, residual=ops.conv2d(self._pcs, x), gn_stats=True)
