"""Mirror of ``DDPM/models/layers.py`` — the C1 pixel-space DDPM UNet's blocks, HIP-backed.

Parameter names and constructor arguments follow the reference so its state_dicts load.  Semantics
kept (file:line into the reference):
* ``TransformerPositionalEmbedding`` (``layers.py:6-30``): pe[t] with sin on even, cos on odd columns,
  div = exp(-(2i)·ln(1e4)/dim); the table is built with the reference's own fp32 torch expressions.
* ``ConvBlock`` (``:33-48``) conv3x3 → GroupNorm → SiLU (post-activation norm).
* ``DownsampleBlock`` conv3x3 s2 p1 (``:51-58``); ``UpsampleBlock`` bilinear x2 align_corners=True →
  conv3x3 (``:61-72``).
* ``ResNetBlock`` (``:300-338``): h = block1(x); x = Linear(SiLU(temb))[:, :, None, None] + h;
  block2(x) + residual_conv(input) (1x1 when Cin != Cout).
* ``SelfAttentionBlock`` (``:135-192``): q/k/v/out Linear (bias) on the un-normalised tokens, heads of
  C/num_heads channels, scale d^-1/2, then GroupNorm(proj + input) (post-norm, no SiLU).
Device mapping: every conv / Linear is ``sdk_conv2d`` (NHWC fp16, the up-path torch.cat read
zero-copy as a 2-source K range); the GroupNorm + SiLU + time-embedding add + ResNet skip of a
ConvBlock is one ``sdk_group_norm_apply_ex`` pass; attention ``sdk_attention``; bilinear upsample
``sdk_upsample_bilinear2x``.  The time-embedding projections of all ResNetBlocks are one GEMM
(gathered by ``UNet._prepare``).
"""
from __future__ import annotations

import torch
from torch import nn

from ... import ops


def _gn_prep(gn, dev):
    gn._g = gn.weight.detach().to(dev, torch.float32).contiguous()
    gn._b = gn.bias.detach().to(dev, torch.float32).contiguous()


def _stats(gn, x):
    return ops.group_norm_affine(x, gn._g, gn._b, gn.eps, gn.num_groups)


class TransformerPositionalEmbedding(nn.Module):
    def __init__(self, dimension, max_timesteps=1000):
        super().__init__()
        assert dimension % 2 == 0, "Embedding dimension must be even"
        self.dimension = dimension
        self.pe_matrix = torch.zeros(max_timesteps, dimension)
        even_indices = torch.arange(0, self.dimension, 2)
        log_term = torch.log(torch.tensor(10000.0)) / self.dimension
        div_term = torch.exp(even_indices * -log_term)
        timesteps = torch.arange(max_timesteps).unsqueeze(1)
        self.pe_matrix[:, 0::2] = torch.sin(timesteps * div_term)
        self.pe_matrix[:, 1::2] = torch.cos(timesteps * div_term)

    def _prepare(self, dev):
        self._pe = self.pe_matrix.to(dev, torch.float32).contiguous()
        self._zero = torch.zeros(1, self.dimension, device=dev)

    def _run(self, t):
        """t int64 [B] → fp16 [B, dimension] (row gather on the device)."""
        return ops.token_embedding(t.view(-1, 1), self._pe, self._zero).view(t.shape[0], self.dimension)


class ConvBlock(nn.Module):
    def __init__(self, in_channels, out_channels, groups=8):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1)
        self.norm = nn.GroupNorm(groups, out_channels)
        self.act = nn.SiLU()

    def _prepare(self, dev, cin_src=None):
        self._pc = ops.PackedConv([(self.conv.weight, cin_src or self.conv.in_channels)], self.conv.bias, device=dev)
        _gn_prep(self.norm, dev)

    def _run(self, x, post_bias=None, residual=None):
        h = ops.conv2d(self._pc, x)
        return ops.group_norm_apply_ex(h, _stats(self.norm, h), silu=True, post_bias=post_bias, residual=residual)


class DownsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, stride, padding):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, 3, stride=stride, padding=padding)

    def _prepare(self, dev):
        self._pc = ops.PackedConv([(self.conv.weight, self.conv.in_channels)], self.conv.bias, device=dev)

    def _run(self, x):
        return ops.conv2d(self._pc, x, stride=self.conv.stride[0], pad=self.conv.padding[0])


class UpsampleBlock(nn.Module):
    def __init__(self, in_channels, out_channels, scale_factor=2.0):
        super().__init__()
        assert scale_factor == 2.0, "the reference builds x2 upsamplers only"
        self.scale = scale_factor
        self.conv = nn.Conv2d(in_channels, out_channels, 3, padding=1)

    def _prepare(self, dev):
        self._pc = ops.PackedConv([(self.conv.weight, self.conv.in_channels)], self.conv.bias, device=dev)

    def _run(self, x):
        return ops.conv2d(self._pc, ops.upsample_bilinear2x(x))


class ResNetBlock(nn.Module):
    def __init__(self, in_channels, out_channels, *, time_emb_channels=None, num_groups=8):
        super().__init__()
        self.time_embedding_projectile = (nn.Sequential(nn.SiLU(), nn.Linear(time_emb_channels, out_channels))
                                          if time_emb_channels else None)
        self.block1 = ConvBlock(in_channels, out_channels, groups=num_groups)
        self.block2 = ConvBlock(out_channels, out_channels, groups=num_groups)
        self.residual_conv = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else nn.Identity()
        self.in_channels, self.out_channels = in_channels, out_channels

    def _prepare(self, dev):
        self.block1._prepare(dev)
        self.block2._prepare(dev)
        self._pc_res = None
        if isinstance(self.residual_conv, nn.Conv2d):
            self._pc_res = ops.PackedConv([(self.residual_conv.weight, self.in_channels)], self.residual_conv.bias,
                                          device=dev)

    def _run(self, x, emb_all):
        te = emb_all[:, self._emb_off:self._emb_off + self.out_channels] if emb_all is not None else None
        h = self.block1._run(x, post_bias=te)
        r = ops.conv2d(self._pc_res, x, ksize=1, pad=0) if self._pc_res is not None else x
        return self.block2._run(h, residual=r)


class SelfAttentionBlock(nn.Module):
    def __init__(self, num_heads, in_channels, num_groups=32, embedding_dim=256):
        super().__init__()
        self.num_heads = num_heads
        self.d_model = embedding_dim
        self.d_keys = embedding_dim // num_heads
        self.d_values = embedding_dim // num_heads
        self.query_projection = nn.Linear(in_channels, embedding_dim)
        self.key_projection = nn.Linear(in_channels, embedding_dim)
        self.value_projection = nn.Linear(in_channels, embedding_dim)
        self.final_projection = nn.Linear(embedding_dim, embedding_dim)
        self.norm = nn.GroupNorm(num_channels=embedding_dim, num_groups=num_groups)

    def _prepare(self, dev):
        w = torch.cat([self.query_projection.weight, self.key_projection.weight, self.value_projection.weight], 0)
        b = torch.cat([self.query_projection.bias, self.key_projection.bias, self.value_projection.bias], 0)
        self._pc_qkv = ops.PackedConv([(w, self.query_projection.in_features)], b, device=dev)
        self._pc_o = ops.PackedConv([(self.final_projection.weight, self.d_model)], self.final_projection.bias,
                                    device=dev)
        _gn_prep(self.norm, dev)

    def _run(self, x):
        B, H, W, Cc = x.shape
        assert Cc == self.d_model, "the reference adds the projection to its input: in_channels == embedding_dim"
        tok = x.view(B * H * W, Cc)
        qkv = ops.linear(self._pc_qkv, tok)
        D = self.d_model
        o = ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], batch=B, heads=self.num_heads, nq=H * W,
                          nk=H * W, head_dim=self.d_keys, scale=self.d_keys ** -0.5)
        p = ops.linear(self._pc_o, o, residual=tok).view(B, H, W, Cc)
        return ops.group_norm_apply_ex(p, _stats(self.norm, p), silu=False)


class _Block(nn.Module):
    """Shared forward of the four Down/Up block classes (ResNet blocks [+ attention] then resample)."""

    def _run(self, x, emb_all):
        atts = getattr(self, "attention_blocks", None)
        for i, rb in enumerate(self.resnet_blocks):
            x = rb._run(x, emb_all)
            if atts is not None:
                x = atts[i]._run(x)
        rs = getattr(self, "downsample", None) or getattr(self, "upsample", None)
        return rs._run(x) if rs is not None else x


class ConvDownBlock(_Block):
    def __init__(self, in_channels, out_channels, num_layers, time_emb_channels, num_groups, downsample=True):
        super().__init__()
        self.resnet_blocks = nn.ModuleList([
            ResNetBlock(in_channels=in_channels if i == 0 else out_channels, out_channels=out_channels,
                        time_emb_channels=time_emb_channels, num_groups=num_groups) for i in range(num_layers)])
        self.downsample = DownsampleBlock(out_channels, out_channels, stride=2, padding=1) if downsample else None


class ConvUpBlock(_Block):
    def __init__(self, in_channels, out_channels, num_layers, time_emb_channels, num_groups, upsample=True):
        super().__init__()
        self.resnet_blocks = nn.ModuleList([
            ResNetBlock(in_channels=in_channels if i == 0 else out_channels, out_channels=out_channels,
                        time_emb_channels=time_emb_channels, num_groups=num_groups) for i in range(num_layers)])
        self.upsample = UpsampleBlock(out_channels, out_channels) if upsample else None


class AttentionDownBlock(_Block):
    def __init__(self, in_channels, out_channels, num_layers, time_emb_channels, num_groups, num_att_heads,
                 downsample=True):
        super().__init__()
        self.resnet_blocks = nn.ModuleList([
            ResNetBlock(in_channels=in_channels if i == 0 else out_channels, out_channels=out_channels,
                        time_emb_channels=time_emb_channels, num_groups=num_groups) for i in range(num_layers)])
        self.attention_blocks = nn.ModuleList([
            SelfAttentionBlock(in_channels=out_channels, embedding_dim=out_channels, num_heads=num_att_heads,
                               num_groups=num_groups) for _ in range(num_layers)])
        self.downsample = DownsampleBlock(out_channels, out_channels, stride=2, padding=1) if downsample else None


class AttentionUpBlock(_Block):
    def __init__(self, in_channels, out_channels, num_layers, time_emb_channels, num_groups, num_att_heads,
                 upsample=True):
        super().__init__()
        self.resnet_blocks = nn.ModuleList([
            ResNetBlock(in_channels=in_channels if i == 0 else out_channels, out_channels=out_channels,
                        time_emb_channels=time_emb_channels, num_groups=num_groups) for i in range(num_layers)])
        self.attention_blocks = nn.ModuleList([
            SelfAttentionBlock(in_channels=out_channels, embedding_dim=out_channels, num_heads=num_att_heads,
                               num_groups=num_groups) for _ in range(num_layers)])
        self.upsample = UpsampleBlock(out_channels, out_channels) if upsample else None
