"""SD UNet forward — fp32 CPU restatement (TEST INFRASTRUCTURE ONLY).

A functional re-derivation of ``openai_model`` from its state_dict and its
constructor kwargs; used as the parity oracle for the HIP path.

Semantics followed (file:line into /root/reference):
* timestep_embedding: cat[cos, sin], freqs = exp(-ln(1e4)·k/half) —
  ``openai_model/utils.py:225-245``.
* time_embed MLP Linear→SiLU→Linear — ``openai_model/model.py:352-357,565-566``.
* block construction (channel bookkeeping, heads/dim_head rules incl. the
  mutable ``num_heads`` and ``legacy`` override) — ``openai_model/model.py:362-532``.
* ResBlock (GN32 eps 1e-5 → SiLU → conv3×3; + Linear(SiLU(emb)); GN → SiLU →
  conv3×3; + skip) — ``openai_model/model.py:155-252``.  The reference's
  ``checkpoint(..., flag=False)`` evaluates the block twice
  (``openai_model/utils.py:217-221``); the second result is returned and is
  identical to the first, so it is evaluated once here.
* Downsample conv3×3 s2 p1 / Upsample nearest×2 + conv3×3 — ``model.py:71-131``.
* SpatialTransformer (GN eps 1e-6, proj_in 1×1, BasicTransformerBlock,
  proj_out 1×1, + x_in) — ``openai_model/attention.py:303-363``;
  BasicTransformerBlock — ``attention.py:233-257``; CrossAttention (no-bias
  q/k/v, scale d^-½, flash_attn non-causal) — ``attention.py:24-117``;
  GEGLU FF (Linear C→8C, x·gelu_erf(gate), Linear 4C→C) — ``attention.py:129-172``.
* AttentionBlock + QKVAttentionLegacy (GN32, Conv1d qkv, view [T,3,H,ch],
  softmax scale 1/√√ch — SURVEY quirk Q3) — ``attention.py:490-597``.
* out: GN32 → SiLU → conv3×3 — ``model.py:528-532,595``.
The reference's hard-coded ``.half()`` casts are not restated: the
oracle is pure fp32.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def timestep_embedding(t: torch.Tensor, dim: int, max_period: int = 10000) -> torch.Tensor:
    half = dim // 2
    k = torch.arange(0, half, dtype=torch.float32)
    freqs = torch.exp(-math.log(max_period) * k / half)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def attention_core(q, k, v, scale):
    """flash_attn_func restated: q,k,v [b, n, h, d] → [b, nq, h, d]; softmax(scale·QKᵀ)V, fp32."""
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v.float())


def _gn(x, sd, p, eps):
    return F.group_norm(x, 32, sd[p + ".weight"], sd[p + ".bias"], eps)


def _conv(x, sd, p, stride=1, padding=None):
    w = sd[p + ".weight"]
    if padding is None:
        padding = w.shape[-1] // 2
    return F.conv2d(x, w, sd.get(p + ".bias"), stride=stride, padding=padding)


def _lin(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd.get(p + ".bias"))


# ------------------------------------------------------------------ layout

def unet_layout(cfg: dict) -> dict:
    """Walk the reference constructor (``openai_model/model.py:316-532``) and
    return the block list with channel counts and attention geometry."""
    mc = cfg["model_channels"]
    nrb = cfg["num_res_blocks"]
    mult = list(cfg.get("channel_mult", (1, 2, 4, 8)))
    attn_res = list(cfg["attention_resolutions"])
    num_heads = cfg.get("num_heads", -1)
    nhc = cfg.get("num_head_channels", -1)
    nh_up = cfg.get("num_heads_upsample", -1)
    if nh_up == -1:
        nh_up = num_heads
    legacy = cfg.get("legacy", True)
    use_st = cfg.get("use_spatial_transformer", False)
    depth = cfg.get("transformer_depth", 1)
    conv_resample = cfg.get("conv_resample", True)

    def attn_geom(ch):
        nonlocal num_heads
        if nhc == -1:
            dim_head = ch // num_heads
        else:
            num_heads = ch // nhc
            dim_head = nhc
        if legacy:
            dim_head = ch // num_heads if use_st else nhc
        return num_heads, dim_head

    def attn_desc(ch, heads_for_block, dim_head):
        if use_st:
            return ("st", heads_for_block, dim_head, depth)
        # AttentionBlock(ch, num_heads=..., num_head_channels=dim_head)
        heads = heads_for_block if dim_head == -1 else ch // dim_head
        return ("attn", heads, ch // heads)

    inputs = [[("conv_in", cfg["in_channels"], mc)]]
    chans = [mc]
    ch, ds = mc, 1
    for level, m in enumerate(mult):
        for _ in range(nrb):
            layers = [("res", ch, m * mc)]
            ch = m * mc
            if ds in attn_res:
                nh, dh = attn_geom(ch)
                layers.append(attn_desc(ch, nh, dh))
            inputs.append(layers)
            chans.append(ch)
        if level != len(mult) - 1:
            inputs.append([("down", ch, ch, conv_resample)])
            chans.append(ch)
            ds *= 2
    nh, dh = attn_geom(ch)
    middle = [("res", ch, ch), attn_desc(ch, nh, dh), ("res", ch, ch)]
    outputs = []
    for level, m in list(enumerate(mult))[::-1]:
        for i in range(nrb + 1):
            ich = chans.pop()
            layers = [("res", ch + ich, mc * m, ich)]
            ch = mc * m
            if ds in attn_res:
                nh, dh = attn_geom(ch)
                layers.append(attn_desc(ch, nh_up if not use_st else nh, dh))
            if level and i == nrb:
                layers.append(("up", ch, ch, conv_resample))
                ds //= 2
            outputs.append(layers)
    return {"input_blocks": inputs, "middle_block": middle, "output_blocks": outputs, "out_ch": ch}


# ------------------------------------------------------------------ blocks

def resblock(sd, p, x, emb):
    h = _conv(F.silu(_gn(x, sd, p + ".in_layers.0", 1e-5)), sd, p + ".in_layers.2")
    h = h + _lin(F.silu(emb), sd, p + ".emb_layers.1")[:, :, None, None]
    h = _conv(F.silu(_gn(h, sd, p + ".out_layers.0", 1e-5)), sd, p + ".out_layers.3")
    skip = _conv(x, sd, p + ".skip_connection") if (p + ".skip_connection.weight") in sd else x
    return skip + h


def cross_attention(sd, p, x, context, heads):
    ctx = x if context is None else context
    q = F.linear(x, sd[p + ".to_q.weight"])
    k = F.linear(ctx, sd[p + ".to_k.weight"])
    v = F.linear(ctx, sd[p + ".to_v.weight"])
    b, n, inner = q.shape
    d = inner // heads
    o = attention_core(q.view(b, n, heads, d), k.view(b, -1, heads, d), v.view(b, -1, heads, d), d ** -0.5)
    return _lin(o.reshape(b, n, inner), sd, p + ".to_out.0")


def geglu_ff(sd, p, x):
    hx, gate = _lin(x, sd, p + ".net.0.proj").chunk(2, dim=-1)
    return _lin(hx * F.gelu(gate), sd, p + ".net.2")


def transformer_block(sd, p, x, context, heads):
    C = x.shape[-1]
    ln = lambda t, n: F.layer_norm(t, (C,), sd[f"{p}.{n}.weight"], sd[f"{p}.{n}.bias"], 1e-5)
    x = cross_attention(sd, p + ".attn1", ln(x, "norm1"), None, heads) + x
    x = cross_attention(sd, p + ".attn2", ln(x, "norm2"), context, heads) + x
    x = geglu_ff(sd, p + ".ff", ln(x, "norm3")) + x
    return x


def spatial_transformer(sd, p, x, context, heads, depth):
    b, c, hh, ww = x.shape
    x_in = x
    x = _conv(_gn(x, sd, p + ".norm", 1e-6), sd, p + ".proj_in")
    x = x.permute(0, 2, 3, 1).reshape(b, hh * ww, -1)
    for i in range(depth):
        x = transformer_block(sd, f"{p}.transformer_blocks.{i}", x, context, heads)
    x = x.reshape(b, hh, ww, -1).permute(0, 3, 1, 2)
    return _conv(x, sd, p + ".proj_out") + x_in


def attention_block_legacy(sd, p, x, heads):
    b, c, hh, ww = x.shape
    xf = x.reshape(b, c, -1)
    xn = F.group_norm(xf, 32, sd[p + ".norm.weight"], sd[p + ".norm.bias"], 1e-5)
    qkv = F.conv1d(xn, sd[p + ".qkv.weight"], sd[p + ".qkv.bias"])          # [b, 3c, T]
    T = qkv.shape[-1]
    ch = c // heads
    qkv = qkv.permute(0, 2, 1).reshape(b, T, 3, heads, ch)
    o = attention_core(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], 1.0 / math.sqrt(math.sqrt(ch)))
    o = o.reshape(b, T, c).permute(0, 2, 1)
    h = F.conv1d(o, sd[p + ".proj_out.weight"], sd[p + ".proj_out.bias"])
    return (xf + h).reshape(b, c, hh, ww)


def _run_block(sd, prefix, layers, h, emb, context):
    for j, desc in enumerate(layers):
        p = f"{prefix}.{j}"
        kind = desc[0]
        if kind == "conv_in":
            h = _conv(h, sd, p)
        elif kind == "res":
            h = resblock(sd, p, h, emb)
        elif kind == "st":
            h = spatial_transformer(sd, p, h, context, desc[1], desc[3])
        elif kind == "attn":
            h = attention_block_legacy(sd, p, h, desc[1])
        elif kind == "down":
            h = _conv(h, sd, p + ".op", stride=2, padding=1) if desc[3] else F.avg_pool2d(h, 2, 2)
        elif kind == "up":
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            if desc[3]:
                h = _conv(h, sd, p + ".conv")
        else:
            raise ValueError(kind)
    return h


@torch.no_grad()
def unet_forward(sd: dict, cfg: dict, x: torch.Tensor, timesteps: torch.Tensor, context=None) -> torch.Tensor:
    """UNetModel.forward (``openai_model/model.py:550-595``) in fp32 on the CPU."""
    sd = {k: v.float() for k, v in sd.items()}
    lay = unet_layout(cfg)
    emb = timestep_embedding(timesteps, cfg["model_channels"])
    emb = _lin(F.silu(_lin(emb, sd, "time_embed.0")), sd, "time_embed.2")
    h = x.float()
    ctx = None if context is None else context.float()
    hs = []
    for i, layers in enumerate(lay["input_blocks"]):
        if i == 0:
            h = _conv(h, sd, "input_blocks.0.0")
        else:
            h = _run_block(sd, f"input_blocks.{i}", layers, h, emb, ctx)
        hs.append(h)
    h = _run_block(sd, "middle_block", lay["middle_block"], h, emb, ctx)
    for i, layers in enumerate(lay["output_blocks"]):
        h = torch.cat([h, hs.pop()], dim=1)
        h = _run_block(sd, f"output_blocks.{i}", layers, h, emb, ctx)
    h = F.silu(_gn(h, sd, "out.0", 1e-5))
    return _conv(h, sd, "out.2")
