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
* Encode: ``Encoder.__init__/forward`` — ``Encoder_Decoder/encoder.py:20-103``
  (conv_in → per level num_res_blocks ResnetBlocks (+attn) and Downsample except at the last
  level → mid → norm_out → SiLU → conv_out), ``Downsample`` F.pad(0,1,0,1) + conv3×3 s2 p0 —
  ``Unet/unet.py:52-71``; ``AutoEncoderKL.encode`` quant_conv 1×1 → posterior —
  ``VAE/autoencoder.py:114-123``; ``DiagonalGaussianDistribution`` (logvar clamp [-30, 20],
  std = exp(logvar/2), sample = mean + std·noise) — ``Distribution/distribution.py:31-50``;
  ``get_first_stage_encoding`` scale_factor·z — ``ldm/diffusion/ddpm.py:795-806``.
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


def encoder_layout(ddconfig: dict) -> list:
    ch, mult = ddconfig["ch"], list(ddconfig["ch_mult"])
    in_mult = (1,) + tuple(mult)
    curr_res = ddconfig["resolution"]
    levels = []
    for i_level in range(len(mult)):
        block_in, block_out = ch * in_mult[i_level], ch * mult[i_level]
        blocks, attn = [], []
        for _ in range(ddconfig["num_res_blocks"]):
            blocks.append((block_in, block_out))
            block_in = block_out
            if curr_res in ddconfig.get("attn_resolutions", []):
                attn.append(block_in)
        down = i_level != len(mult) - 1
        if down:
            curr_res //= 2
        levels.append({"blocks": blocks, "attn": attn, "downsample": down})
    return levels


@torch.no_grad()
def encoder_forward(sd: dict, ddconfig: dict, x: torch.Tensor, prefix="encoder") -> torch.Tensor:
    sd = {k: v.float() for k, v in sd.items()}
    p = prefix
    h = _conv(x.float(), sd, p + ".conv_in")
    for i_level, lv in enumerate(encoder_layout(ddconfig)):
        for i_block in range(len(lv["blocks"])):
            h = resnet_block(sd, f"{p}.down.{i_level}.block.{i_block}", h)
            if lv["attn"]:
                h = flash_attention_block(sd, f"{p}.down.{i_level}.attn.{i_block}", h)
        if lv["downsample"]:
            h = F.pad(h, (0, 1, 0, 1), mode="constant", value=0)
            w = sd[f"{p}.down.{i_level}.downsample.conv.weight"]
            h = F.conv2d(h, w, sd[f"{p}.down.{i_level}.downsample.conv.bias"], stride=2, padding=0)
    h = resnet_block(sd, p + ".mid.block_1", h)
    h = flash_attention_block(sd, p + ".mid.attn_1", h)
    h = resnet_block(sd, p + ".mid.block_2", h)
    return _conv(F.silu(_gn(h, sd, p + ".norm_out", 1e-6)), sd, p + ".conv_out")


@torch.no_grad()
def autoencoder_moments(sd: dict, ddconfig: dict, x: torch.Tensor) -> torch.Tensor:
    """AutoEncoderKL.encode up to the posterior parameters: quant_conv(encoder(x))."""
    sd32 = {k: v.float() for k, v in sd.items()}
    h = encoder_forward(sd32, ddconfig, x)
    return F.conv2d(h, sd32["quant_conv.weight"], sd32["quant_conv.bias"])


def posterior_sample(moments: torch.Tensor, noise=None, scale_factor: float = 1.0) -> torch.Tensor:
    """scale_factor * DiagonalGaussianDistribution(moments).sample() with the given noise (mode if None)."""
    mean, logvar = torch.chunk(moments.float(), 2, dim=1)
    if noise is None:
        return scale_factor * mean
    std = torch.exp(0.5 * torch.clamp(logvar, -30.0, 20.0))
    return scale_factor * (mean + std * noise)


def delta_border(h: int, w: int) -> torch.Tensor:
    """CompVis ``delta_border`` (``ldm/diffusion/ddpm.py:838-859`` with the per-pixel min over the last
    dim; the reference's dim=1 fails in torch.cat for w > 1 — DESIGN.md Q14)."""
    y = torch.arange(0, h).view(h, 1, 1).repeat(1, w, 1)
    x = torch.arange(0, w).view(1, w, 1).repeat(h, 1, 1)
    arr = torch.cat([y, x], dim=-1) / torch.tensor([h - 1, w - 1]).view(1, 1, 2)
    lu = torch.min(arr, dim=-1, keepdim=True)[0]
    rd = torch.min(1 - arr, dim=-1, keepdim=True)[0]
    return torch.min(torch.cat([lu, rd], dim=-1), dim=-1)[0]


@torch.no_grad()
def decode_first_stage_tiled(sd: dict, ddconfig: dict, z: torch.Tensor, scale_factor: float, sp: dict):
    """Patch decode (``ldm/diffusion/ddpm.py:1097-1139``; ``get_fold_unfold`` uf>1 branch ``:894-960``;
    ``get_weighting`` ``:862-891``): Unfold latent patches, decode each, weight, Fold, normalise."""
    ks, stride, uf = tuple(sp["ks"]), tuple(sp["stride"]), int(sp["vqf"])
    z = 1.0 / scale_factor * z.float()
    bs, nc, h, w = z.shape
    Ly, Lx = (h - ks[0]) // stride[0] + 1, (w - ks[1]) // stride[1] + 1
    unfold = torch.nn.Unfold(kernel_size=ks, dilation=1, padding=0, stride=stride)
    fold = torch.nn.Fold(output_size=(h * uf, w * uf), kernel_size=(ks[0] * uf, ks[1] * uf), dilation=1, padding=0,
                         stride=(stride[0] * uf, stride[1] * uf))
    wt = torch.clip(delta_border(ks[0] * uf, ks[1] * uf), sp["clip_min_weight"], sp["clip_max_weight"])
    wt = wt.view(1, ks[0] * uf * ks[1] * uf, 1).repeat(1, 1, Ly * Lx)
    if sp.get("tie_braker", False):
        lw = torch.clip(delta_border(Ly, Lx), sp["clip_min_tie_weight"], sp["clip_max_tie_weight"])
        wt = wt * lw.view(1, 1, Ly * Lx)
    normalization = fold(wt).view(1, 1, h * uf, w * uf)
    wt = wt.view(1, 1, ks[0] * uf, ks[1] * uf, Ly * Lx)
    zp = unfold(z).view(bs, -1, ks[0], ks[1], Ly * Lx)
    o = torch.stack([autoencoder_decode(sd, ddconfig, zp[:, :, :, :, i]) for i in range(Ly * Lx)], dim=-1)
    o = (o * wt).view(bs, -1, Ly * Lx)
    return fold(o) / normalization
