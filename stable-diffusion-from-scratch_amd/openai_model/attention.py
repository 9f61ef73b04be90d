"""Mirror of ``openai_model/attention.py`` — SpatialTransformer / BasicTransformerBlock /
CrossAttention / GEGLU FeedForward / AttentionBlock (+ QKVAttentionLegacy), HIP-backed.

Parameter names and constructor signatures follow the reference so SD
checkpoints and ``Diffusion/config.yaml`` params load unchanged.  Execution
(``_run``) works on NHWC fp16 token matrices:

* q/k/v projections are one fused GEMM for self-attention (concatenated
  weights), the context K/V of cross-attention is one GEMM computed once per
  conditioning tensor (step-invariant across the sampler loop);
* the softmax(QK^T)V core is ``sdk_attention`` (flash-style, fp32 softmax);
* to_out / FF-out / proj_out GEMMs fuse the residual add in their epilogue, the
  GEGLU projection fuses ``x * gelu(gate)`` in its epilogue;
* the SpatialTransformer GroupNorm is one ``sdk_group_norm`` call (its statistics merged from the
  producing conv's epilogue partials, then one apply pass) in front of the proj_in GEMM;
* at the 320-channel (and small 640-channel) levels the cross-attention block — norm2, to_q, the
  attention over the cached context K/V, to_out + residual, norm3 — is one kernel (xattn.hip).
"""
from __future__ import annotations

import os
import math

import torch
from torch import nn

from .. import ops
from .utils import conv_nd, normalization, zero_module


def Normalize(in_channels):
    return torch.nn.GroupNorm(num_groups=32, num_channels=in_channels, eps=1e-6, affine=True)


def _gn_prep(gn: nn.GroupNorm, dev):
    gn._g = gn.weight.detach().to(dev, torch.float32).contiguous()
    gn._b = gn.bias.detach().to(dev, torch.float32).contiguous()


def _gn_stats(gn: nn.GroupNorm, x):
    return ops.group_norm_affine(x, gn._g, gn._b, gn.eps, gn.num_groups)


def _gn(gn: nn.GroupNorm, x, silu=False):
    return ops.group_norm(x, gn._g, gn._b, gn.eps, gn.num_groups, silu=silu)


def _ln_prep(ln: nn.LayerNorm, dev):
    ln._g = ln.weight.detach().to(dev, torch.float32).contiguous()
    ln._b = ln.bias.detach().to(dev, torch.float32).contiguous()


# fused to_q + attention + to_out kernel for cross-attention on the cached context (xattn.hip),
# routed where it measured faster than the three launches (tools/bench_xattn.py, MI355X: 320
# channels at >= 65536 query rows — the 64x64 level at B=16: 1.07-1.11x, its CFG batch of 2 x 16:
# 1.21x; 640 channels only up to 16384 rows, where one workgroup per CU is resident and larger
# grids run two waves); SD_AMD_FUSED_XATTN=0 / 1 forces it off / on
_FUSED_ENV = os.environ.get("SD_AMD_FUSED_XATTN")
FUSED_CROSS_ATTENTION = _FUSED_ENV != "0"
FUSED_XATTN_MIN_ROWS = 0 if _FUSED_ENV == "1" else 65536
FUSED_XATTN_640_MAX_ROWS = 16384
# norm2 / norm3 folded into that kernel (its prologue / epilogue) instead of two layer_norm launches;
# SD_AMD_XATTN_NORMS=0 keeps the separate launches (A/B only: the bits are the same)
FUSED_XATTN_NORMS = os.environ.get("SD_AMD_XATTN_NORMS") != "0"


def _use_fused_xattn(channels, head_dim, nk, n_img, batch):
    if not FUSED_CROSS_ATTENTION or n_img % 64:
        return False
    rows = batch * n_img
    if _FUSED_ENV != "1":
        # measured wins (profiles/r2_xattn_fused_norms.txt, norms folded): 320 channels from 65,536 rows
        # (1.12-1.23x); 640 channels up to 16,384 rows (1.02-1.06x; one 139 KiB group per CU, so the
        # two-wave grids of the 640-channel CFG batches lose: 0.85-0.93x)
        if channels == 320:
            if rows < FUSED_XATTN_MIN_ROWS:
                return False
        elif channels != 640 or rows > FUSED_XATTN_640_MAX_ROWS:
            return False
    return ops.cross_attention_block_supported(channels, head_dim, nk, n_img)


# Reassociated cross-attention where the heads x context columns are fewer than the channels (SD-1's
# 1280-channel levels: 8 x 77 = 616 -> 640 vs 1280): per prompt b and head h, K_h Wq_h (77 x C) and
# Wo_h V_h^T (C x 77) are precomputed with the context K|V, so the per-step block is
#   s = t [K_h Wq_h]_h^T (one GEMM, N = H*77) -> p = segment softmax(scale s) -> out = p [Wo_h V_h^T]_h^T + b + x
# — 4*M*C*H*77 FLOP instead of 4*M*C*(C + 77) (2.1x fewer at 1280), the same math as
# softmax(q K^T) V Wo^T with q = t Wq^T (reference attention.py:96-117).  SD_AMD_XATTN_REASSOC=0 keeps
# the three launches.
XATTN_REASSOC = os.environ.get("SD_AMD_XATTN_REASSOC") != "0"

# The 320-channel GEGLU FeedForward as one kernel (ops.feed_forward: the 4C intermediate stays in
# registers); SD_AMD_FUSED_FF=0 keeps the two GEMMs.
FUSED_FF = os.environ.get("SD_AMD_FUSED_FF") != "0"
# 320 -> 320 token projections (self-attention to_out + residual, SpatialTransformer proj_in with the
# first block's norm1 emitted from the same tile) on the register-resident-weight kernel (csrc/token.hip);
# same-box A/B: UNet step 19.58 -> 19.44 ms (profiles/r4_token_linear_ab.txt).  SD_AMD_TOKEN_LINEAR=0
# keeps the tiled GEMM + separate LayerNorm
TOKEN_LINEAR = os.environ.get("SD_AMD_TOKEN_LINEAR", "1") != "0"


class ReassocContext:
    """A prompt batch's cross-attention operands: the K|V projection (the three-launch path) and the
    per-prompt reassociated GEMM weights, built on first use by a block whose token count takes the
    reassociated path (N % 128 == 0) — the 8x8 middle block of SD-1 at 512^2 never builds them.
    Built outside any graph capture: GraphedUNet runs one eager evaluation before it captures."""
    __slots__ = ("kv", "w1", "w2", "heads", "nk", "batch", "_build")

    def __init__(self, kv, heads, nk, batch, build):
        self.kv, self.heads, self.nk, self.batch, self._build = kv, heads, nk, batch, build
        self.w1 = self.w2 = None

    def weights(self):
        if self.w1 is None:
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                # the build would be recorded into the caller's graph (re-run on every replay, its
                # matrices allocated from that graph's private pool and cached here for other graphs)
                raise RuntimeError("ReassocContext: per-prompt weights are built eagerly — run one eager "
                                   "step with this context before capturing a graph")
            self.w1, self.w2 = self._build()
            self._build = None
        return self.w1, self.w2


def reassoc_weights(k, v, wq, wo):
    """The per-prompt matrices of the reassociated block as math (the CPU statement the tests check the
    regrouping with; the device path computes the same products per head on sdk_conv2d, see
    CrossAttention.context_kv): k, v [B, L, H, d] (the context K / V), wq [H*d, C] (to_q.weight),
    wo [Co, H*d] (to_out.weight) -> w1 [B, H*L, C] with w1[b, h*L + j] = K[b, j, h] Wq_h, and
    w2 [B, Co, H*L] with w2[b, :, h*L + j] = Wo_h V[b, j, h]^T."""
    B, L, H, d = k.shape
    w1 = torch.einsum("bjhe,hec->bhjc", k, wq.view(H, d, -1)).reshape(B, H * L, -1)
    w2 = torch.einsum("che,bjhe->bchj", wo.view(wo.shape[0], H, d), v).reshape(B, wo.shape[0], H * L)
    return w1, w2


def _reassoc_applies(inner, heads, nk):
    kr = (heads * nk + ops.BK - 1) // ops.BK * ops.BK
    return XATTN_REASSOC and 2 * kr <= inner


class CrossAttention(nn.Module):
    """Reference ``attention.py:24-117``: no-bias q/k/v, to_out Linear+Dropout, scale d^-1/2.
    At the 1280-channel levels with a cached context the per-step block runs reassociated
    (``ReassocContext``)."""

    def __init__(self, query_dim, context_dim=None, heads=8, dim_head=64, dropout=0.):
        super().__init__()
        inner_dim = dim_head * heads
        self.self_attn = context_dim is None
        context_dim = query_dim if context_dim is None else context_dim
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.dim_head = dim_head
        self.to_q = nn.Linear(query_dim, inner_dim, bias=False)
        self.to_k = nn.Linear(context_dim, inner_dim, bias=False)
        self.to_v = nn.Linear(context_dim, inner_dim, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner_dim, query_dim), nn.Dropout(dropout))

    def _prepare(self, dev):
        qd = self.to_q.in_features
        cd = self.to_k.in_features
        if self.self_attn:
            w = torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], 0)
            self._pc_qkv = ops.PackedConv([(w, qd)], None, device=dev)
        self._pc_q = ops.PackedConv([(self.to_q.weight, qd)], None, device=dev)
        self._pc_kv = ops.PackedConv([(torch.cat([self.to_k.weight, self.to_v.weight], 0), cd)], None, device=dev)
        self._pc_o = ops.PackedConv([(self.to_out[0].weight, self.heads * self.dim_head)], self.to_out[0].bias,
                                    device=dev)
        inner = self.heads * self.dim_head
        self._ptl_o = (ops.PackedTokenLinear(self.to_out[0].weight, self.to_out[0].bias, dev)
                       if self.self_attn and ops.token_linear_supported(inner, self.to_out[0].out_features) else None)
        if not self.self_attn:
            self._bo32 = self.to_out[0].bias.detach().to(dev, torch.float32).contiguous()
            self._pc_reassoc = None    # per-head GEMM weights of the reassociated per-prompt matrices (lazy)

    def context_kv(self, ctx2d, L=None):
        """K|V of the conditioning, [B*L, 2*inner] — computed once per conditioning tensor; with ``L``
        (context tokens) and a shape where it pays, wrapped with the reassociated per-prompt weights."""
        kv = ops.linear(self._pc_kv, ctx2d)
        inner = self.heads * self.dim_head
        if L is None or self.self_attn or not _reassoc_applies(inner, self.heads, L):
            return kv
        B, H, d = ctx2d.shape[0] // L, self.heads, self.dim_head
        C = self.to_q.in_features
        Co = self.to_out[0].out_features

        def build():
            # per head h, on the library GEMM (sdk_conv2d, fp32 accumulation, fp16 out like the stored
            # matrices): K_h Wq_h = K_h [B*L, d] x (Wq_h^T as an [C, d] weight) and
            # (Wo_h V_h^T)^T = V_h [B*L, d] x (Wo_h as a [Co, d] weight); reassoc_weights is the same math
            dev = kv.device
            if self._pc_reassoc is None:
                wq, wo = self.to_q.weight.detach(), self.to_out[0].weight.detach()
                self._pc_reassoc = (
                    [ops.PackedConv([(wq[h * d:(h + 1) * d].t().contiguous(), d)], None, device=dev) for h in range(H)],
                    [ops.PackedConv([(wo[:, h * d:(h + 1) * d].contiguous(), d)], None, device=dev) for h in range(H)])
            pq, po = self._pc_reassoc
            kr = (H * L + ops.BK - 1) // ops.BK * ops.BK
            w1 = torch.zeros(B, (kr + ops.BN - 1) // ops.BN * ops.BN, C, dtype=torch.float16, device=dev)
            w2 = torch.zeros(B, (Co + ops.BN - 1) // ops.BN * ops.BN, kr, dtype=torch.float16, device=dev)
            w1h = w1[:, :H * L].view(B, H, L, C)
            for h in range(H):
                w1h[:, h] = ops.linear(pq[h], kv[:, h * d:(h + 1) * d]).view(B, L, C)
                w2[:, :Co, h * L:(h + 1) * L] = ops.linear(po[h], kv[:, inner + h * d:inner + (h + 1) * d]).view(
                    B, L, Co).transpose(1, 2)
            return ops.PerImageWeights(w1, H * L), ops.PerImageWeights(w2, Co, self._bo32)
        return ReassocContext(kv, H, L, B, build)

    def _run(self, t, residual, B, N, kv=None, Lc=None):
        inner = self.heads * self.dim_head
        if kv is None:
            if self.self_attn:
                qkv = ops.linear(self._pc_qkv, t)
                q, k, v, nk = qkv[:, :inner], qkv[:, inner:2 * inner], qkv[:, 2 * inner:], N
            else:   # context defaults to x (reference: default(context, x)) — only legal if dims match
                q = ops.linear(self._pc_q, t)
                kvx = ops.linear(self._pc_kv, t)
                k, v, nk = kvx[:, :inner], kvx[:, inner:], N
        else:
            # cross-attention on the cached context K|V: to_q, the attention core and to_out are
            # the per-step block the bench reports (``cross_attention_block``); one fused kernel
            # where the shape is supported, else the three launches
            ops.PROFILER.region = "cross_attention"
            if isinstance(kv, ReassocContext):
                if t.stride(-1) == 1 and N % 128 == 0 and kv.batch == B:
                    w1, w2 = kv.weights()
                    s = ops.linear(w1, t, out_mode=ops.OUT_ROWS_F32, n_img=N)
                    p = ops.segment_softmax(s, kv.heads, kv.nk, self.scale, ld_p=w2.k_total)
                    out = ops.linear(w2, p, residual=residual, n_img=N)
                    ops.PROFILER.region = None
                    return out
                kv = kv.kv
            if t.stride(-1) == 1 and _use_fused_xattn(inner, self.dim_head, Lc, N, B):
                out = ops.cross_attention_block(t, kv, self._pc_q, self._pc_o, batch=B, n_img=N, nk=Lc,
                                                heads=self.heads, head_dim=self.dim_head, scale=self.scale,
                                                residual=residual)
                ops.PROFILER.region = None
                return out
            q = ops.linear(self._pc_q, t)
            k, v, nk = kv[:, :inner], kv[:, inner:], Lc
        o = ops.attention(q, k, v, batch=B, heads=self.heads, nq=N, nk=nk, head_dim=self.dim_head, scale=self.scale)
        if TOKEN_LINEAR and self._ptl_o is not None and o.stride(-1) == 1 and \
                (residual is None or residual.is_contiguous()):
            out = ops.token_linear(self._ptl_o, o, residual=residual)
        else:
            out = ops.linear(self._pc_o, o, residual=residual)
        ops.PROFILER.region = None
        return out


class GELU(nn.Module):
    """GEGLU projection (reference ``attention.py:129-141``): Linear(dim_in, 2*dim_out); x*gelu(gate)."""

    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)


class FeedForward(nn.Module):
    """Reference ``attention.py:146-172`` (glu=True path: GELU → Dropout → Linear)."""

    def __init__(self, dim, dim_out=None, mult=4, glu=False, dropout=0.):
        super().__init__()
        inner_dim = int(dim * mult)
        dim_out = dim if dim_out is None else dim_out
        if not glu:
            raise NotImplementedError("sd_amd: only the gated (GEGLU) feed-forward is on the SD path")
        self.net = nn.Sequential(GELU(dim, inner_dim), nn.Dropout(dropout), nn.Linear(inner_dim, dim_out))

    def _prepare(self, dev):
        p = self.net[0].proj
        self._pc1 = ops.PackedConv([(p.weight, p.in_features)], p.bias, geglu=True, device=dev)
        self._pc2 = ops.PackedConv([(self.net[2].weight, self.net[2].in_features)], self.net[2].bias, device=dev)
        self._pff = None
        if FUSED_FF and ops.ff_supported(p.in_features, p.out_features // 2):
            self._pff = ops.PackedFF(p.weight, p.bias, self.net[2].weight, self.net[2].bias, dev)

    def _run(self, t, residual):
        if self._pff is not None and t.stride(-1) == 1:
            # GEGLU GEMM -> GEGLU -> output GEMM -> + residual in one kernel (320 channels)
            return ops.feed_forward(self._pff, t, residual=residual)
        g = ops.linear(self._pc1, t, out_mode=ops.OUT_GEGLU_F16)
        return ops.linear(self._pc2, g, residual=residual)


class BasicTransformerBlock(nn.Module):
    """Reference ``attention.py:187-257``: x += attn1(LN x); x += attn2(LN x, ctx); x += FF(LN x)."""

    def __init__(self, dim, n_heads, d_head, dropout=0., context_dim=None, gated_ff=True, checkpoint=True):
        super().__init__()
        self.attn1 = CrossAttention(query_dim=dim, heads=n_heads, dim_head=d_head, dropout=dropout)
        self.ff = FeedForward(dim=dim, dropout=dropout, glu=gated_ff)
        self.attn2 = CrossAttention(query_dim=dim, context_dim=context_dim, heads=n_heads, dim_head=d_head,
                                    dropout=dropout)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.norm3 = nn.LayerNorm(dim)
        self.checkpoint = checkpoint

    def _prepare(self, dev):
        for m in (self.attn1, self.attn2, self.ff):
            m._prepare(dev)
        for n in (self.norm1, self.norm2, self.norm3):
            _ln_prep(n, dev)

    def _run(self, tok, B, N, kv=None, Lc=None, t=None):
        """``t``: norm1(tok) when the producer of ``tok`` emitted it (token_linear with a norm)."""
        if t is None:
            t = ops.layer_norm(tok, self.norm1._g, self.norm1._b, self.norm1.eps)
        tok = self.attn1._run(t, tok, B, N)
        a2 = self.attn2
        if (kv is not None and FUSED_XATTN_NORMS and tok.stride(-1) == 1
                and _use_fused_xattn(a2.heads * a2.dim_head, a2.dim_head, Lc, N, B)):
            # norm2 -> cross-attention -> + residual -> norm3 in one kernel
            ops.PROFILER.region = "cross_attention"
            tok, t = ops.cross_attention_block(
                tok, kv, a2._pc_q, a2._pc_o, batch=B, n_img=N, nk=Lc, heads=a2.heads, head_dim=a2.dim_head,
                scale=a2.scale, residual=tok, norm_in=(self.norm2._g, self.norm2._b, self.norm2.eps),
                norm_out=(self.norm3._g, self.norm3._b, self.norm3.eps))
            ops.PROFILER.region = None
            return self.ff._run(t, tok)
        t = ops.layer_norm(tok, self.norm2._g, self.norm2._b, self.norm2.eps)
        tok = self.attn2._run(t, tok, B, N, kv, Lc)
        t = ops.layer_norm(tok, self.norm3._g, self.norm3._b, self.norm3.eps)
        return self.ff._run(t, tok)


class SpatialTransformer(nn.Module):
    """Reference ``attention.py:303-363``: GN(eps 1e-6) → proj_in 1x1 → blocks → proj_out 1x1 → + x."""

    def __init__(self, in_channels, n_heads, d_head, depth=1, dropout=0., context_dim=None):
        super().__init__()
        self.in_channels = in_channels
        inner_dim = n_heads * d_head
        self.inner_dim = inner_dim
        self.norm = Normalize(in_channels)
        self.proj_in = nn.Conv2d(in_channels, inner_dim, kernel_size=1, stride=1, padding=0)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner_dim, n_heads, d_head, dropout=dropout, context_dim=context_dim)
             for _ in range(depth)])
        self.proj_out = zero_module(nn.Conv2d(inner_dim, in_channels, kernel_size=1, stride=1, padding=0))

    def _prepare(self, dev):
        _gn_prep(self.norm, dev)
        self._pc_in = ops.PackedConv([(self.proj_in.weight, self.in_channels)], self.proj_in.bias, device=dev)
        self._ptl_in = (ops.PackedTokenLinear(self.proj_in.weight, self.proj_in.bias, dev)
                        if ops.token_linear_supported(self.in_channels, self.inner_dim) else None)
        self._pc_out = ops.PackedConv([(self.proj_out.weight, self.inner_dim)], self.proj_out.bias, device=dev)
        for blk in self.transformer_blocks:
            blk._prepare(dev)

    def context_kv(self, ctx2d, L=None):
        return [blk.attn2.context_kv(ctx2d, L) for blk in self.transformer_blocks]

    def _run(self, x, kvs=None, Lc=None):
        B, H, W, Cc = x.shape
        # GN materialised by one streaming pass, then the LDS-DMA GEMM (a GN prologue forces the
        # register-staged kernel: 150-190 TF/s on these shapes vs 330-650 for apply + DMA GEMM)
        xn = _gn(self.norm, x)
        t1 = None
        if TOKEN_LINEAR and self._ptl_in is not None and xn.is_contiguous():
            # proj_in + the first block's norm1 in one launch (the LayerNorm rows from the same tile)
            n1 = self.transformer_blocks[0].norm1 if len(self.transformer_blocks) else None
            if n1 is not None:
                tok, t1 = ops.token_linear(self._ptl_in, xn.view(B * H * W, Cc), norm=(n1._g, n1._b, n1.eps))
            else:
                tok = ops.token_linear(self._ptl_in, xn.view(B * H * W, Cc))
        else:
            tok = ops.conv2d(self._pc_in, xn).view(B * H * W, self.inner_dim)
        for i, blk in enumerate(self.transformer_blocks):
            tok = blk._run(tok, B, H * W, None if kvs is None else kvs[i], Lc, t=t1 if i == 0 else None)
        return ops.conv2d(self._pc_out, tok.view(B, H, W, self.inner_dim), residual=x, gn_stats=True)


class QKVAttentionLegacy(nn.Module):
    """Reference ``attention.py:490-526``: qkv viewed [T, 3, H, ch]; softmax scale 1/sqrt(sqrt(ch))
    (SURVEY quirk Q3 — reproduced for parity)."""

    def __init__(self, n_heads):
        super().__init__()
        self.n_heads = n_heads

    def scale(self, ch):
        return 1.0 / math.sqrt(math.sqrt(ch))


class FlashAttention(nn.Module):
    """Reference ``attention.py:369-404`` (use_new_attention_order): same [T, 3, H, d] view, scale d^-1/2."""

    def __init__(self, n_heads):
        super().__init__()
        self.n_heads = n_heads

    def scale(self, ch):
        return 1.0 / math.sqrt(ch)


class AttentionBlock(nn.Module):
    """Reference ``attention.py:539-597``: GN32 → Conv1d qkv → attention → Conv1d proj_out → + x."""

    def __init__(self, channels, num_heads=1, num_head_channels=-1, use_checkpoint=False,
                 use_new_attention_order=False):
        super().__init__()
        self.channels = channels
        if num_head_channels == -1:
            self.num_heads = num_heads
        else:
            assert channels % num_head_channels == 0
            self.num_heads = channels // num_head_channels
        self.use_checkpoint = use_checkpoint
        self.norm = normalization(channels)
        self.qkv = conv_nd(1, channels, channels * 3, 1)
        self.attention = FlashAttention(self.num_heads) if use_new_attention_order else \
            QKVAttentionLegacy(self.num_heads)
        self.proj_out = zero_module(conv_nd(1, channels, channels, 1))

    def _prepare(self, dev):
        self.norm._prepare(dev)
        self._pc_qkv = ops.PackedConv([(self.qkv.weight, self.channels)], self.qkv.bias, device=dev)
        self._pc_proj = ops.PackedConv([(self.proj_out.weight, self.channels)], self.proj_out.bias, device=dev)

    def _run(self, x):
        B, H, W, Cc = x.shape
        xn = self.norm.norm(x, silu=False)
        qkv = ops.conv2d(self._pc_qkv, xn).view(B * H * W, 3 * Cc)
        ch = Cc // self.num_heads
        o = ops.attention(qkv[:, :Cc], qkv[:, Cc:2 * Cc], qkv[:, 2 * Cc:], batch=B, heads=self.num_heads,
                          nq=H * W, nk=H * W, head_dim=ch, scale=self.attention.scale(ch))
        return ops.conv2d(self._pc_proj, o.view(B, H, W, Cc), residual=x, gn_stats=True)
