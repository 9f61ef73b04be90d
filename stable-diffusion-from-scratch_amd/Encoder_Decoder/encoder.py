"""Mirror of ``Encoder_Decoder/encoder.py`` — KL-VAE Encoder and Decoder (HIP-backed).

Encoder walk (``encoder.py:20-103``): conv_in → per level num_res_blocks ResnetBlocks
(attention at ``attn_resolutions``) and a Downsample (asymmetric pad, stride 2) except at
the last level → mid(block_1, attn_1, block_2) → norm_out → SiLU → conv_out.  conv_out is
folded with AutoEncoderKL.quant_conv (1x1, no nonlinearity between them) into one conv that
writes the NCHW fp32 posterior moments directly.

Decoder walk (``encoder.py:106-210``): conv_in → mid(block_1, attn_1, block_2) →
levels reversed (num_res_blocks+1 ResnetBlocks each, attention at
``attn_resolutions``, Upsample except at level 0; ``up.insert(0, ...)`` order) →
norm_out → SiLU → conv_out.  The final GN+SiLU runs inside conv_out's prologue
and conv_out writes the NCHW fp32 image directly.
"""
from __future__ import annotations

import torch
from torch import nn

from .. import ops
from ..Unet.attention import make_attention
from ..Unet.unet import Downsample, Normalize, ResnetBlock, Upsample, _gn_prep, gn_act


class Encoder(nn.Module):
    def __init__(self, *, ch, out_ch, ch_mult=(1, 2, 4, 8), num_res_blocks, attn_resolutions, dropout=0.0,
                 resamp_with_conv=True, in_channels, resolution, z_channels, double_z=True, use_linear_attn=False,
                 attn_type="vanilla", **ignore_kwargs):
        super().__init__()
        if use_linear_attn:
            attn_type = "linear"
        self.ch = ch
        self.temb_ch = 0
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.resolution = resolution
        self.in_channels = in_channels
        self.conv_in = nn.Conv2d(in_channels, self.ch, kernel_size=3, stride=1, padding=1)
        curr_res = resolution
        in_ch_mult = (1,) + tuple(ch_mult)
        self.in_ch_mult = in_ch_mult
        self.down = nn.ModuleList()
        block_in = ch
        for i_level in range(self.num_resolutions):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_in = ch * in_ch_mult[i_level]
            block_out = ch * ch_mult[i_level]
            for _ in range(self.num_res_blocks):
                block.append(ResnetBlock(in_channels=block_in, out_channels=block_out, temb_channels=self.temb_ch,
                                         dropout=dropout))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(make_attention(block_in, attention_type=attn_type))
            down = nn.Module()
            down.block = block
            down.attn = attn
            if i_level != self.num_resolutions - 1:
                down.downsample = Downsample(block_in, resamp_with_conv)
                curr_res = curr_res // 2
            self.down.append(down)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(in_channels=block_in, out_channels=block_in, temb_channels=self.temb_ch,
                                       dropout=dropout)
        self.mid.attn_1 = make_attention(block_in, attention_type=attn_type)
        self.mid.block_2 = ResnetBlock(in_channels=block_in, out_channels=block_in, temb_channels=self.temb_ch,
                                       dropout=dropout)
        self.norm_out = Normalize(block_in)
        self.conv_out = nn.Conv2d(block_in, 2 * z_channels if double_z else z_channels, kernel_size=3, stride=1,
                                  padding=1)

        self._block_out = block_in

    def _prepare(self, dev, in_pad, quant_conv=None):
        """Pack every conv; conv_out is folded with ``quant_conv`` (1x1) when given:
        W = Wq·Wout, b = Wq·b_out + b_q (fp32 on the host, then fp16)."""
        self._in_pad = in_pad
        self._pc_in = ops.PackedConv([(self.conv_in.weight, in_pad)], self.conv_in.bias, device=dev)
        for m in self.modules():
            if m is not self and hasattr(m, "_prepare") and not isinstance(m, (Encoder, Decoder)):
                m._prepare(dev)
        _gn_prep(self.norm_out, dev)
        w, b = self.conv_out.weight.detach().float(), self.conv_out.bias.detach().float()
        if quant_conv is not None:
            wq = quant_conv.weight.detach().float()[:, :, 0, 0]
            w = torch.einsum("nj,jcyx->ncyx", wq, w)
            b = wq @ b + quant_conv.bias.detach().float()
        self._pc_out = ops.PackedConv([(w, self._block_out)], b, device=dev)
        self._prepared_on = (dev, in_pad, quant_conv is not None)

    def _run(self, x_nhwc):
        """x_nhwc: fp16 [B, H, W, in_pad] → fp32 NCHW conv_out (∘ quant_conv) output."""
        h = ops.conv2d(self._pc_in, x_nhwc, gn_stats=True)     # feeds down[0].block[0].norm1
        for i_level in range(self.num_resolutions):
            down = self.down[i_level]
            for i_block in range(self.num_res_blocks):
                h = down.block[i_block]._run(h)
                if len(down.attn) > 0:
                    h = down.attn[i_block]._run(h)
            if i_level != self.num_resolutions - 1:
                h = down.downsample._run(h)
        h = self.mid.block_1._run(h)
        h = self.mid.attn_1._run(h)
        h = self.mid.block_2._run(h)
        gp, cp = ops.gn_conv_pad()
        ha = gn_act(self.norm_out, h, silu=True, pad=gp)
        return ops.conv2d(self._pc_out, ha, pad=cp, out_mode=ops.OUT_NCHW_F32)

    @torch.no_grad()
    def forward(self, x):
        if not x.is_cuda:
            raise TypeError("sd_amd.Encoder: HIP path only — move inputs to the GPU")
        in_pad = (x.shape[1] + 7) // 8 * 8
        if getattr(self, "_prepared_on", None) != (x.device, in_pad, False):
            self._prepare(x.device, in_pad)
        return self._run(ops.nchw_to_nhwc(x.float(), in_pad))


class Decoder(nn.Module):
    def __init__(self, *, ch, out_ch, ch_mult=(1, 2, 4, 8), num_res_blocks, attn_resolutions, dropout=0.0,
                 resamp_with_conv=True, in_channels, resolution, z_channels, give_pre_end=False, tanh_out=False,
                 use_linear_attn=False, attn_type="vanilla", **ignorekwargs):
        super().__init__()
        if use_linear_attn:
            attn_type = "linear"
        self.ch = ch
        self.temb_ch = 0
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.resolution = resolution
        self.in_channels = in_channels
        self.give_pre_end = give_pre_end
        self.tanh_out = tanh_out
        self.z_channels = z_channels
        self.out_ch = out_ch
        block_in = ch * ch_mult[self.num_resolutions - 1]
        curr_res = resolution // 2 ** (self.num_resolutions - 1)
        self.z_shape = (1, z_channels, curr_res, curr_res)
        self.conv_in = nn.Conv2d(in_channels=z_channels, out_channels=block_in, kernel_size=3, stride=1, padding=1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(in_channels=block_in, out_channels=block_in, temb_channels=self.temb_ch,
                                       dropout=dropout)
        self.mid.attn_1 = make_attention(block_in, attention_type=attn_type)
        self.mid.block_2 = ResnetBlock(in_channels=block_in, out_channels=block_in, temb_channels=self.temb_ch,
                                       dropout=dropout)
        self.up = nn.ModuleList()
        for i_level in reversed(range(self.num_resolutions)):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_out = ch * ch_mult[i_level]
            for _ in range(self.num_res_blocks + 1):
                block.append(ResnetBlock(in_channels=block_in, out_channels=block_out, temb_channels=self.temb_ch,
                                         dropout=dropout))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(make_attention(block_in, attention_type=attn_type))
            up = nn.Module()
            up.block = block
            up.attn = attn
            if i_level != 0:
                up.upsample = Upsample(block_in, resamp_with_conv)
                curr_res = curr_res * 2
            self.up.insert(0, up)
        self.norm_out = Normalize(block_in)
        self.conv_out = nn.Conv2d(block_in, out_ch, kernel_size=3, stride=1, padding=1)
        self._block_out = block_in

    def _prepare(self, dev, zc_pad):
        self._zc_pad = zc_pad
        self._pc_in = ops.PackedConv([(self.conv_in.weight, zc_pad)], self.conv_in.bias, device=dev)
        for m in self.modules():
            if m is not self and hasattr(m, "_prepare") and not isinstance(m, Decoder):
                m._prepare(dev)
        _gn_prep(self.norm_out, dev)
        self._pc_out = ops.PackedConv([(self.conv_out.weight, self._block_out)], self.conv_out.bias, device=dev)

    def _run(self, z_nhwc):
        """z_nhwc: fp16 [B, h, w, zc_pad] → fp32 NCHW image."""
        h = ops.conv2d(self._pc_in, z_nhwc, gn_stats=True)     # feeds mid.block_1.norm1
        h = self.mid.block_1._run(h)
        h = self.mid.attn_1._run(h)
        h = self.mid.block_2._run(h)
        for i_level in reversed(range(self.num_resolutions)):
            up = self.up[i_level]
            for i_block in range(self.num_res_blocks + 1):
                h = up.block[i_block]._run(h)
                if len(up.attn) > 0:
                    h = up.attn[i_block]._run(h)
            if i_level != 0:
                h = up.upsample._run(h)
        if self.give_pre_end:
            raise NotImplementedError("sd_amd: give_pre_end is not on the SD path")
        if self.tanh_out:
            raise NotImplementedError("sd_amd: tanh_out is not on the SD path")
        gp, cp = ops.gn_conv_pad()
        ha = gn_act(self.norm_out, h, silu=True, pad=gp)
        return ops.conv2d(self._pc_out, ha, pad=cp, out_mode=ops.OUT_NCHW_F32)

    @torch.no_grad()
    def forward(self, z):
        if not z.is_cuda:
            raise TypeError("sd_amd.Decoder: HIP path only — move inputs to the GPU")
        zc_pad = (z.shape[1] + 7) // 8 * 8
        if getattr(self, "_prepared_on", None) != (z.device, zc_pad):
            self._prepare(z.device, zc_pad)
            self._prepared_on = (z.device, zc_pad)
        return self._run(ops.nchw_to_nhwc(z.float(), zc_pad))
