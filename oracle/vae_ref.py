"""KL-VAE decode — fp32 CPU restatement (TEST INFRASTRUCTURE ONLY).

Follows (file:line into /root/reference):
* ``AutoEncoderKL.decode``: post_quant_conv 1×1 → Decoder — ``VAE/autoencoder.py:126-132``.
* ``Decoder.__init__/forward`` level walk (block_in/out, curr_res, attn at
  ``attn_resolutions``, ``up.insert(0, …)`` ordering) — ``Encoder_Decoder/encoder.py:106-210``.
* ``ResnetBlock`` (GN eps 1e-6, SiLU, conv3×3, no temb in the VAE, nin_shortcut
  1×1 when Cin≠Cout) — ``Unet/unet.py:74-135``; ``Normalize`` — ``Unet/unet.py:9-19``.
  The fp16 cast inside ``nonlinearity`` (``Unet/unet.py:24``) is not restated (fp32 oracle).
* ``Upsample`` nearest×2 + conv3×3 — ``Unet/unet.py:34-49``.
* ``FlashAttentionBlock`` (GN(32) with torch's default eps 1e-5, q/k/v 1×1,
  8 heads × C/8, default scale d^-½, proj_out, + x) — ``Unet/attention.py:221-264``.
* ``decode_first_stage`` scaling z / scale_factor — ``ldm/diffusion/ddpm.py:1095``
  (the ``Diffusion/ddpm.py:728`` variant drops z).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .unet_ref import attention_core


def _gn(x, sd, p, eps):
    return F.group_norm(x, 32, sd[p + ".weight"], sd[p + ".bias"], eps)


def _conv(x, sd, p):
    w = sd[p + ".weight"]
    return F.conv2d(x, w, sd.get(p + ".bias"), padding=w.shape[-1] // 2)


def resnet_block(sd, p, x):
    h = _conv(F.silu(_gn(x, sd, p + ".norm1", 1e-6)), sd, p + ".conv1")
    h = _conv(F.silu(_gn(h, sd, p + ".norm2", 1e-6)), sd, p + ".conv2")
    if (p + ".nin_shortcut.weight") in sd:
        x = _conv(x, sd, p + ".nin_shortcut")
    elif (p + ".conv_shortcut.weight") in sd:
        x = _conv(x, sd, p + ".conv_shortcut")
    return x + h


def flash_attention_block(sd, p, x, num_heads=8):
    b, c, hh, ww = x.shape
    hn = _gn(x, sd, p + ".norm", 1e-5)
    d = c // num_heads
    toks = lambda t: t.reshape(b, num_heads, d, hh * ww).permute(0, 3, 1, 2)
    q, k, v = (toks(_conv(hn, sd, p + "." + n)) for n in ("q", "k", "v"))
    o = attention_core(q, k, v, d ** -0.5)                    # [b, T, H, d]
    o = o.permute(0, 2, 3, 1).reshape(b, c, hh, ww)
    return x + _conv(o, sd, p + ".proj_out")


def decoder_layout(ddconfig: dict) -> dict:
    ch, mult = ddconfig["ch"], list(ddconfig["ch_mult"])
    nrb = ddconfig["num_res_blocks"]
    nres = len(mult)
    block_in = ch * mult[-1]
    curr_res = ddconfig["resolution"] // 2 ** (nres - 1)
    levels = {}
    for i_level in reversed(range(nres)):
        block_out = ch * mult[i_level]
        blocks, attn = [], []
        for _ in range(nrb + 1):
            blocks.append((block_in, block_out))
            block_in = block_out
            if curr_res in ddconfig.get("attn_resolutions", []):
                attn.append(block_in)
        up = i_level != 0
        if up:
            curr_res *= 2
        levels[i_level] = {"blocks": blocks, "attn": attn, "upsample": up}
    return {"mid_ch": ch * mult[-1], "levels": levels, "out_in": block_in}


@torch.no_grad()
def decoder_forward(sd: dict, ddconfig: dict, z: torch.Tensor, prefix="decoder") -> torch.Tensor:
    sd = {k: v.float() for k, v in sd.items()}
    lay = decoder_layout(ddconfig)
    p = prefix
    h = _conv(z.float(), sd, p + ".conv_in")
    h = resnet_block(sd, p + ".mid.block_1", h)
    h = flash_attention_block(sd, p + ".mid.attn_1", h)
    h = resnet_block(sd, p + ".mid.block_2", h)
    for i_level in reversed(range(len(ddconfig["ch_mult"]))):
        lv = lay["levels"][i_level]
        for i_block in range(len(lv["blocks"])):
            h = resnet_block(sd, f"{p}.up.{i_level}.block.{i_block}", h)
            if lv["attn"]:
                h = flash_attention_block(sd, f"{p}.up.{i_level}.attn.{i_block}", h)
        if lv["upsample"]:
            h = F.interpolate(h, scale_factor=2.0, mode="nearest")
            h = _conv(h, sd, f"{p}.up.{i_level}.upsample.conv")
    if ddconfig.get("give_pre_end", False):
        return h
    h = _conv(F.silu(_gn(h, sd, p + ".norm_out", 1e-6)), sd, p + ".conv_out")
    if ddconfig.get("tanh_out", False):
        h = torch.tanh(h)
    return h


@torch.no_grad()
def autoencoder_decode(sd: dict, ddconfig: dict, z: torch.Tensor) -> torch.Tensor:
    sd32 = {k: v.float() for k, v in sd.items()}
    z = F.conv2d(z.float(), sd32["post_quant_conv.weight"], sd32["post_quant_conv.bias"])
    return decoder_forward(sd32, ddconfig, z)


@torch.no_grad()
def decode_first_stage(sd: dict, ddconfig: dict, z: torch.Tensor, scale_factor: float) -> torch.Tensor:
    return autoencoder_decode(sd, ddconfig, 1.0 / scale_factor * z.float())
