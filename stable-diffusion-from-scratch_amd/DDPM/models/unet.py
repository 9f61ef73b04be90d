"""Mirror of ``DDPM/models/unet.py`` — the C1 pixel-space DDPM UNet (58.66 M parameters), HIP-backed.

Structure (``unet.py:11-80``): initial conv3x3 (3→128) → positional MLP (pe → Linear 128→512 → GELU →
Linear 512→512) → 5 down blocks (attention at index 3, each ends with a stride-2 conv) → attention
bottleneck (no downsample) → 5 up blocks on torch.cat([x, skip]) (bilinear x2 + conv) → cat with the
initial conv output → GroupNorm(256) → SiLU → conv3x3 (256→3).  ``forward(input_tensor, time)``
takes NCHW images and int64 timesteps on the GPU and returns NCHW fp32 ε.
"""
from __future__ import annotations

import torch
from torch import nn

from ... import ops
from .layers import (AttentionDownBlock, AttentionUpBlock, ConvDownBlock, ConvUpBlock, ResNetBlock,
                     TransformerPositionalEmbedding, _gn_prep)


class UNet(nn.Module):
    def __init__(self, image_size=256, input_channels=3):
        super().__init__()
        self.input_channels = input_channels
        self.initial_conv = nn.Conv2d(in_channels=input_channels, out_channels=128, kernel_size=3, stride=1,
                                      padding="same")
        self.positional_encoding = nn.Sequential(TransformerPositionalEmbedding(dimension=128),
                                                 nn.Linear(128, 128 * 4), nn.GELU(), nn.Linear(128 * 4, 128 * 4))
        self.downsample_blocks = nn.ModuleList([
            ConvDownBlock(in_channels=128, out_channels=128, num_layers=2, num_groups=32, time_emb_channels=128 * 4),
            ConvDownBlock(in_channels=128, out_channels=128, num_layers=2, num_groups=32, time_emb_channels=128 * 4),
            ConvDownBlock(in_channels=128, out_channels=256, num_layers=2, num_groups=32, time_emb_channels=128 * 4),
            AttentionDownBlock(in_channels=256, out_channels=256, num_layers=2, num_att_heads=4, num_groups=32,
                               time_emb_channels=128 * 4),
            ConvDownBlock(in_channels=256, out_channels=512, num_layers=2, num_groups=32, time_emb_channels=128 * 4)])
        self.bottleneck = AttentionDownBlock(in_channels=512, out_channels=512, num_layers=2, num_att_heads=4,
                                             num_groups=32, time_emb_channels=128 * 4, downsample=False)
        self.upsample_blocks = nn.ModuleList([
            ConvUpBlock(in_channels=512 + 512, out_channels=512, num_layers=2, num_groups=32,
                        time_emb_channels=128 * 4),
            AttentionUpBlock(in_channels=512 + 256, out_channels=256, num_layers=2, num_att_heads=4, num_groups=32,
                             time_emb_channels=128 * 4),
            ConvUpBlock(in_channels=256 + 256, out_channels=256, num_layers=2, num_groups=32,
                        time_emb_channels=128 * 4),
            ConvUpBlock(in_channels=256 + 128, out_channels=128, num_layers=2, num_groups=32,
                        time_emb_channels=128 * 4),
            ConvUpBlock(in_channels=128 + 128, out_channels=128, num_layers=2, num_groups=32,
                        time_emb_channels=128 * 4)])
        self.output_conv = nn.Sequential(nn.GroupNorm(num_channels=256, num_groups=32), nn.SiLU(),
                                         nn.Conv2d(256, 3, 3, padding=1))
        self._prepared_on = None

    def load_state_dict(self, *args, **kwargs):
        self._prepared_on = None
        return super().load_state_dict(*args, **kwargs)

    @torch.no_grad()
    def _prepare(self, dev):
        self._cin_pad = (self.input_channels + 7) // 8 * 8
        self._pc_in = ops.PackedConv([(self.initial_conv.weight, self._cin_pad)], self.initial_conv.bias, device=dev)
        pe, l1, _, l2 = self.positional_encoding
        pe._prepare(dev)
        self._pc_t1 = ops.PackedConv([(l1.weight, 128)], l1.bias, device=dev)
        self._pc_t2 = ops.PackedConv([(l2.weight, 512)], l2.bias, device=dev)
        ws, bs, off = [], [], 0
        for m in self.modules():
            if isinstance(m, ResNetBlock):
                m._prepare(dev)
                lin = m.time_embedding_projectile[1]
                m._emb_off = off
                off += lin.out_features
                ws.append(lin.weight)
                bs.append(lin.bias)
            elif hasattr(m, "_prepare") and m is not self and not isinstance(m, TransformerPositionalEmbedding) \
                    and type(m).__name__ not in ("ConvBlock",):
                m._prepare(dev)
        # every ResNetBlock's Linear(SiLU(temb)) in one GEMM (A-side SiLU, fp32 rows [B, sum(out)])
        self._pc_emb = ops.PackedConv([(torch.cat(ws, 0), 512)], torch.cat(bs, 0), device=dev)
        gn = self.output_conv[0]
        _gn_prep(gn, dev)
        conv = self.output_conv[2]
        self._pc_out = ops.PackedConv([(conv.weight, 256)], conv.bias, device=dev)
        self._prepared_on = dev

    @torch.no_grad()
    def forward(self, input_tensor, time):
        if not input_tensor.is_cuda:
            raise TypeError("sd_amd.DDPM UNet: HIP path only — move inputs to the GPU")
        if self._prepared_on != input_tensor.device:
            self._prepare(input_tensor.device)
        B = input_tensor.shape[0]
        t = torch.as_tensor(time, device=input_tensor.device).to(torch.int64).reshape(-1)
        if t.numel() == 1 and B > 1:
            t = t.expand(B).contiguous()
        pe = self.positional_encoding[0]._run(t)
        e1 = ops.gelu(ops.linear(self._pc_t1, pe))
        temb = ops.linear(self._pc_t2, e1)
        emb_all = ops.linear(self._pc_emb, temb, silu=True, out_mode=ops.OUT_ROWS_F32)
        x = ops.conv2d(self._pc_in, ops.nchw_to_nhwc(input_tensor.float(), self._cin_pad))
        skips = [x]
        for blk in self.downsample_blocks:
            x = blk._run(x, emb_all)
            skips.append(x)
        skips = list(reversed(skips))
        x = self.bottleneck._run(x, emb_all)
        for blk, skip in zip(self.upsample_blocks, skips):
            x = blk._run((x, skip), emb_all)
        gn = self.output_conv[0]
        src = (x, skips[-1])
        xa = ops.group_norm_apply(src, ops.group_norm_affine(src, gn._g, gn._b, gn.eps, gn.num_groups), silu=True)
        return ops.conv2d(self._pc_out, xa, out_mode=ops.OUT_NCHW_F32)
