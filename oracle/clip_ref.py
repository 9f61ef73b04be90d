"""CLIP text transformer — fp32 CPU restatement (TEST INFRASTRUCTURE ONLY).

The reference's text conditioner ``FrozenCLIPEmbedder.forward`` (``clip_encoder/modules.py:212-257``)
tokenizes to 77 ids and returns ``CLIPTextModel(input_ids).last_hidden_state``.  CLIPTextModel is the
third-party ``transformers`` package (``req.txt:11``, unpinned; the version installed here is 5.15.0),
absent from /root/reference; this restates its published algorithm:

* ``CLIPTextEmbeddings``: token_embedding[ids] + position_embedding[arange(T)];
* ``CLIPEncoderLayer`` (pre-LN): x += out_proj(attn(LN1(x))), causal mask, heads of
  hidden/num_heads, scale head_dim^-1/2, q/k/v/out projections with bias;
  x += fc2(quick_gelu(fc1(LN2(x)))), quick_gelu(x) = x·sigmoid(1.702x); LayerNorm eps 1e-5;
* ``final_layer_norm``.
Pinned by tests/golden/clip_tiny.npz (made by tests/golden/make_golden_clip.py from the installed
transformers CLIPTextModel with the same synthetic weights).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _ln(x, sd, p, eps):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], eps)


def _lin(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


@torch.no_grad()
def clip_text_forward(sd: dict, ids: torch.Tensor, num_heads: int, eps: float = 1e-5,
                      prefix: str = "text_model") -> torch.Tensor:
    """ids int64 [B, T] → last_hidden_state fp32 [B, T, D]."""
    sd = {k: v.float() for k, v in sd.items()}
    p = prefix + "." if prefix else ""
    B, T = ids.shape
    x = sd[p + "embeddings.token_embedding.weight"][ids] + sd[p + "embeddings.position_embedding.weight"][:T]
    D = x.shape[-1]
    d = D // num_heads
    mask = torch.full((T, T), float("-inf")).triu(1)
    i = 0
    while (p + f"encoder.layers.{i}.layer_norm1.weight") in sd:
        lp = p + f"encoder.layers.{i}."
        h = _ln(x, sd, lp + "layer_norm1", eps)
        q, k, v = (_lin(h, sd, lp + f"self_attn.{n}_proj").view(B, T, num_heads, d).transpose(1, 2)
                   for n in ("q", "k", "v"))
        att = (q @ k.transpose(-1, -2)) * d ** -0.5 + mask
        o = (att.softmax(-1) @ v).transpose(1, 2).reshape(B, T, D)
        x = x + _lin(o, sd, lp + "self_attn.out_proj")
        h = _ln(x, sd, lp + "layer_norm2", eps)
        f = _lin(h, sd, lp + "mlp.fc1")
        f = f * torch.sigmoid(1.702 * f)
        x = x + _lin(f, sd, lp + "mlp.fc2")
        i += 1
    return _ln(x, sd, p + "final_layer_norm", eps)
