"""Mirror of ``clip_encoder/modules.py`` — FrozenCLIPEmbedder, HIP-backed.

The reference (``modules.py:212-257``) tokenizes a prompt batch to 77 ids and returns
``CLIPTextModel(input_ids).last_hidden_state`` (transformers, ViT-L/14 text tower: 12 pre-LN
layers, width 768, 12 heads, causal self-attention, quick_gelu MLP, final LayerNorm).  Here the
text tower runs on the library's kernels: token + position embedding (``sdk_token_embedding``),
per layer LayerNorm → one q|k|v GEMM (bias) → causal flash attention (``sdk_attention`` with
``causal``) → out_proj GEMM + residual → LayerNorm → fc1 GEMM with the quick_gelu epilogue
(``SDK_ACT_QUICK_GELU``) → fc2 GEMM + residual, then the final LayerNorm.  The residual stream
is fp16, accumulation fp32.  The output is fp16 [B, 77, 768] — the UNet consumes it as context
directly.

Weights: module names follow transformers' checkpoint layout (``transformer.text_model.…``, the
same keys an SD-1 checkpoint holds under ``cond_stage_model.``), so a local
``model.safetensors`` loads with ``load_state_dict``.  ``from_pretrained`` by hub name needs the
network, which this build never has: ``version`` may be a LOCAL directory (config.json,
model.safetensors, vocab.json + merges.txt); otherwise the ViT-L/14 text configuration is built
with uninitialised weights and ``forward(text)`` needs a local tokenizer — ``encode_tokens(ids)``
takes ids directly.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from .. import ops

VIT_L14_TEXT = dict(vocab_size=49408, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                    num_attention_heads=12, max_position_embeddings=77, layer_norm_eps=1e-5,
                    hidden_act="quick_gelu")


class AbstractEncoder(nn.Module):
    def __init__(self):
        super().__init__()

    def encode(self, *args, **kwargs):
        raise NotImplementedError


class _Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg["vocab_size"], cfg["hidden_size"])
        self.position_embedding = nn.Embedding(cfg["max_position_embeddings"], cfg["hidden_size"])


class _Attention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        D = cfg["hidden_size"]
        self.k_proj, self.v_proj, self.q_proj, self.out_proj = (nn.Linear(D, D) for _ in range(4))


class _MLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.fc1 = nn.Linear(cfg["hidden_size"], cfg["intermediate_size"])
        self.fc2 = nn.Linear(cfg["intermediate_size"], cfg["hidden_size"])


class _EncoderLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        D, eps = cfg["hidden_size"], cfg["layer_norm_eps"]
        self.self_attn = _Attention(cfg)
        self.layer_norm1 = nn.LayerNorm(D, eps=eps)
        self.mlp = _MLP(cfg)
        self.layer_norm2 = nn.LayerNorm(D, eps=eps)

    def _prepare(self, dev):
        a = self.self_attn
        w = torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight], 0)
        b = torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias], 0)
        D = a.q_proj.in_features
        self._pc_qkv = ops.PackedConv([(w, D)], b, device=dev)
        self._pc_o = ops.PackedConv([(a.out_proj.weight, D)], a.out_proj.bias, device=dev)
        self._pc_fc1 = ops.PackedConv([(self.mlp.fc1.weight, D)], self.mlp.fc1.bias, device=dev)
        self._pc_fc2 = ops.PackedConv([(self.mlp.fc2.weight, self.mlp.fc1.out_features)], self.mlp.fc2.bias,
                                      device=dev)
        self._ln = [(ln.weight.detach().to(dev, torch.float32).contiguous(),
                     ln.bias.detach().to(dev, torch.float32).contiguous(), ln.eps)
                    for ln in (self.layer_norm1, self.layer_norm2)]

    def _run(self, x, B, T, heads):
        D = x.shape[1]
        (g1, b1, e1), (g2, b2, e2) = self._ln
        qkv = ops.linear(self._pc_qkv, ops.layer_norm(x, g1, b1, e1))
        d = D // heads
        o = ops.attention(qkv[:, :D], qkv[:, D:2 * D], qkv[:, 2 * D:], batch=B, heads=heads, nq=T, nk=T,
                          head_dim=d, scale=d ** -0.5, causal=True)
        x = ops.linear(self._pc_o, o, residual=x)
        f = ops.linear(self._pc_fc1, ops.layer_norm(x, g2, b2, e2), act=ops.ACT_QUICK_GELU)
        return ops.linear(self._pc_fc2, f, residual=x)


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([_EncoderLayer(cfg) for _ in range(cfg["num_hidden_layers"])])


class CLIPTextTransformer(nn.Module):
    """transformers' CLIPTextTransformer parameter layout; HIP forward (``_run``)."""

    def __init__(self, cfg):
        super().__init__()
        self.cfg = dict(cfg)
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = nn.LayerNorm(cfg["hidden_size"], eps=cfg["layer_norm_eps"])
        self._prepared_on = None

    def _prepare(self, dev):
        for layer in self.encoder.layers:
            layer._prepare(dev)
        self._tok = self.embeddings.token_embedding.weight.detach().to(dev, torch.float32).contiguous()
        self._pos = self.embeddings.position_embedding.weight.detach().to(dev, torch.float32).contiguous()
        ln = self.final_layer_norm
        self._lnf = (ln.weight.detach().to(dev, torch.float32).contiguous(),
                     ln.bias.detach().to(dev, torch.float32).contiguous(), ln.eps)
        self._prepared_on = dev

    @torch.no_grad()
    def _run(self, ids):
        if not ids.is_cuda:
            raise TypeError("sd_amd.CLIPTextTransformer: HIP path only — move the ids to the GPU")
        if self._prepared_on != ids.device:
            self._prepare(ids.device)
        ids = ids.to(torch.int64)
        B, T = ids.shape
        if int(ids.min()) < 0 or int(ids.max()) >= self._tok.shape[0]:
            raise ValueError("sd_amd.CLIPTextTransformer: token id outside the vocabulary")
        x = ops.token_embedding(ids, self._tok, self._pos).view(B * T, -1)
        for layer in self.encoder.layers:
            x = layer._run(x, B, T, self.cfg["num_attention_heads"])
        g, b, e = self._lnf
        return ops.layer_norm(x, g, b, e).view(B, T, -1)


class CLIPTextModel(nn.Module):
    """Holder named like transformers' CLIPTextModel (``.text_model``)."""

    def __init__(self, cfg):
        super().__init__()
        self.text_model = CLIPTextTransformer(cfg)

    def load_state_dict(self, state_dict, strict=True, assign=False):
        # transformers >= 5 saves without the "text_model." prefix; older files and SD checkpoints with it
        sd = {(k if k.startswith("text_model.") else "text_model." + k): v for k, v in state_dict.items()
              if not k.endswith("position_ids")}
        self.text_model._prepared_on = None
        return super().load_state_dict(sd, strict=strict, assign=assign)


class FrozenCLIPEmbedder(AbstractEncoder):
    """Uses the CLIP transformer encoder for text (reference ``clip_encoder/modules.py:212-257``)."""

    def __init__(self, version="openai/clip-vit-large-patch14", device="cuda", max_length=77, config=None):
        super().__init__()
        cfg = dict(VIT_L14_TEXT if config is None else config)
        local = isinstance(version, str) and os.path.isdir(version)
        if local and config is None and os.path.exists(os.path.join(version, "config.json")):
            import json
            with open(os.path.join(version, "config.json")) as f:
                c = json.load(f)
            c = c.get("text_config", c)
            cfg.update({k: c[k] for k in VIT_L14_TEXT if k in c})
        self.transformer = CLIPTextModel(cfg)
        self.tokenizer = None
        if local:
            st = os.path.join(version, "model.safetensors")
            if os.path.exists(st):
                from safetensors.torch import load_file
                sd = {k: v for k, v in load_file(st).items() if not k.startswith("vision_model.")}
                self.transformer.load_state_dict(sd, strict=False)
            if os.path.exists(os.path.join(version, "vocab.json")):
                from transformers import CLIPTokenizer
                self.tokenizer = CLIPTokenizer.from_pretrained(version, local_files_only=True)
        self.device = device
        self.max_length = max_length
        self.freeze()

    def freeze(self):
        self.transformer = self.transformer.eval()
        for param in self.parameters():
            param.requires_grad = False

    def encode_tokens(self, input_ids):
        """ids int64 [B, max_length] → last_hidden_state fp16 [B, max_length, hidden]."""
        return self.transformer.text_model._run(input_ids.to(self.device))

    def forward(self, text):
        if torch.is_tensor(text):
            return self.encode_tokens(text)
        if self.tokenizer is None:
            raise RuntimeError("sd_amd.FrozenCLIPEmbedder: no local tokenizer (vocab.json/merges.txt) — "
                               "the hub download of the reference is unavailable offline; pass token ids")
        batch_encoding = self.tokenizer(text, truncation=True, max_length=self.max_length, return_length=True,
                                        return_overflowing_tokens=False, padding="max_length", return_tensors="pt")
        return self.encode_tokens(batch_encoding["input_ids"])

    def encode(self, text):
        return self(text)
