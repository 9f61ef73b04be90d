"""Mirror of ``openai_model/model.py`` — UNetModel / ResBlock / Down- / Upsample, HIP-backed.

Drop-in contract: same constructor kwargs, same state_dict keys (SD-1.x: 686
keys) and ``UNetModel.forward(x, timesteps=None, context=None, y=None)`` →
``[N, out_ch, H, W]`` in ``x.dtype``.  Internally activations are NHWC fp16,
every conv/linear/norm/attention runs in libsdk_amd.so:

* ResBlock = GN stats → GN-apply+SiLU (one streaming pass) → conv3x3 (bias +
  timestep-embedding broadcast epilogue) → GN stats → GN-apply+SiLU → conv3x3
  (+ skip): the 1x1 skip projection is fused as a second K segment of the same
  GEMM, the identity skip as the residual epilogue.  Each ResBlock runs ONCE (the reference's
  ``checkpoint(..., flag=False)`` evaluates it twice, ``openai_model/utils.py:217-221``).
* The skip concat ``torch.cat([h, hs.pop()], 1)`` is never materialised: the
  next block reads both tensors as one K range.
* Upsample's nearest-x2 is folded into its conv's address generation.
* All 22 ResBlock ``emb_layers`` projections run as ONE GEMM per step.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
from torch import nn

from .. import ops
from .attention import AttentionBlock, SpatialTransformer
from .utils import conv_nd, linear, normalization, timestep_frequencies, zero_module


class TimestepBlock(nn.Module):
    """Any module whose forward takes timestep embeddings as a second argument."""


class TimestepEmbedSequential(nn.Sequential, TimestepBlock):
    """Reference ``model.py:37-67``: dispatch emb / context to the children that take them."""

    def _run(self, x, st):
        for layer in self:
            if isinstance(layer, ResBlock):
                x = layer._run(x, st["emb"], layer._emb_off)
            elif isinstance(layer, SpatialTransformer):
                x = layer._run(x, st["kv"].get(id(layer)) if st["kv"] is not None else None, st["Lc"])
            elif isinstance(layer, (AttentionBlock, Downsample, Upsample)):
                x = layer._run(x)
            elif isinstance(layer, nn.Conv2d):
                x = ops.conv2d(layer._pc, x, gn_stats=True)
            else:
                raise NotImplementedError(f"sd_amd: layer {type(layer).__name__} has no HIP path")
        return x


class Downsample(nn.Module):
    """Reference ``model.py:71-97``: conv3x3 stride 2 pad 1 (``use_conv``)."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None, padding=1):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.dims = dims
        self.padding = padding
        if not use_conv:
            raise NotImplementedError("sd_amd: avg-pool Downsample (conv_resample=False) is not on the SD path")
        self.op = conv_nd(dims, self.channels, self.out_channels, 3, stride=2, padding=padding)

    def _prepare(self, dev):
        self._pc = ops.PackedConv([(self.op.weight, self.channels)], self.op.bias, device=dev)

    def _run(self, x):
        return ops.conv2d(self._pc, x, stride=2, pad=self.padding, gn_stats=True)


# the UNet Upsample materialises the nearest-x2 image zero-bordered and runs its 3x3 conv unmasked (the linear A
# issue of the LDS-DMA kernels) instead of folding the upsample into every DMA address; SD_AMD_UPSAMPLE_FOLD=1
# restores the folded form
UPSAMPLE_FOLD = __import__("os").environ.get("SD_AMD_UPSAMPLE_FOLD", "0") == "1"


class Upsample(nn.Module):
    """Reference ``model.py:100-131``: nearest x2 + conv3x3 (the upsample materialised zero-bordered, or folded
    into the conv's loads)."""

    def __init__(self, channels, use_conv, dims=2, out_channels=None, padding=1):
        super().__init__()
        self.channels = channels
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.dims = dims
        self.padding = padding
        if not use_conv:
            raise NotImplementedError("sd_amd: conv-less Upsample (conv_resample=False) is not on the SD path")
        self.conv = conv_nd(dims, self.channels, self.out_channels, 3, padding=padding)

    def _prepare(self, dev):
        self._pc = ops.PackedConv([(self.conv.weight, self.channels)], self.conv.bias, device=dev)

    def _run(self, x):
        if UPSAMPLE_FOLD or isinstance(x, tuple) or x.shape[-1] % 8:
            return ops.conv2d(self._pc, x, upsample=True, pad=self.padding, gn_stats=True)
        return ops.conv2d(self._pc, ops.upsample_nearest2x_padded(x, self.padding), pad=0, gn_stats=True)


class ResBlock(TimestepBlock):
    """Reference ``model.py:139-252`` (use_scale_shift_norm / up / down are not on the SD path)."""

    def __init__(self, channels, emb_channels, dropout, out_channels=None, use_conv=False,
                 use_scale_shift_norm=False, dims=2, use_checkpoint=False, up=False, down=False):
        super().__init__()
        if use_scale_shift_norm or up or down:
            raise NotImplementedError("sd_amd: use_scale_shift_norm / resblock_updown are not on the SD path")
        self.channels = channels
        self.emb_channels = emb_channels
        self.dropout = dropout
        self.out_channels = out_channels or channels
        self.use_conv = use_conv
        self.use_checkpoint = use_checkpoint
        self.use_scale_shift_norm = use_scale_shift_norm
        self.in_layers = nn.Sequential(normalization(channels), nn.SiLU(),
                                       conv_nd(dims, channels, self.out_channels, 3, padding=1))
        self.updown = False
        self.h_upd = self.x_upd = nn.Identity()
        self.emb_layers = nn.Sequential(nn.SiLU(), linear(emb_channels, self.out_channels))
        self.out_layers = nn.Sequential(normalization(self.out_channels), nn.SiLU(), nn.Dropout(p=dropout),
                                        zero_module(conv_nd(dims, self.out_channels, self.out_channels, 3,
                                                            padding=1)))
        if self.out_channels == channels:
            self.skip_connection = nn.Identity()
        elif use_conv:
            self.skip_connection = conv_nd(dims, channels, self.out_channels, 3, padding=1)
        else:
            self.skip_connection = conv_nd(dims, channels, self.out_channels, 1)
        self._emb_off = 0

    def _prepare(self, dev):
        self.in_layers[0]._prepare(dev)
        self.out_layers[0]._prepare(dev)
        c1, c2 = self.in_layers[2], self.out_layers[3]
        self._pc1 = ops.PackedConv([(c1.weight, self.channels)], c1.bias, device=dev)
        sk = self.skip_connection
        self._skip_mode = "identity"
        if isinstance(sk, nn.Conv2d) and sk.kernel_size[0] == 1:
            self._skip_mode = "fused"
            self._pc2 = ops.PackedConv([(c2.weight, self.out_channels), (sk.weight, self.channels)],
                                       c2.bias.detach() + sk.bias.detach(), device=dev)
        else:
            self._pc2 = ops.PackedConv([(c2.weight, self.out_channels)], c2.bias, device=dev)
            if isinstance(sk, nn.Conv2d):
                self._skip_mode = "conv3"
                self._pc_skip = ops.PackedConv([(sk.weight, self.channels)], sk.bias, device=dev)

    def _run(self, x, emb_all, emb_off):
        B, H, W, _ = ops.src_shape(x)
        c0 = (x[0] if isinstance(x, tuple) else x).shape[-1]
        c1 = x[1].shape[-1] if isinstance(x, tuple) else 0
        # GN+SiLU outputs are written zero-bordered: both 3x3 convs run with pad 0 (mask-free gather)
        gp, cp = ops.gn_conv_pad()
        xa = self.in_layers[0].norm(x, silu=True, pad=gp)
        h = ops.conv2d(self._pc1, xa, pad=cp, row_bias=(emb_all, emb_off), gn_stats=True)
        ha = self.out_layers[0].norm(h, silu=True, pad=gp)
        if self._skip_mode == "identity":
            return ops.conv2d(self._pc2, ha, pad=cp, residual=x, gn_stats=True)
        if self._skip_mode == "fused":
            return ops.conv2d(self._pc2, ha, pad=cp, seg2=(x, None, False), gn_stats=True)
        skip = ops.conv2d(self._pc_skip, x)
        return ops.conv2d(self._pc2, ha, pad=cp, residual=skip, gn_stats=True)


class UNetModel(nn.Module):
    """Reference ``model.py:259-595``.  See the module docstring for the execution plan."""

    def __init__(self, image_size, in_channels, model_channels, out_channels, num_res_blocks,
                 attention_resolutions, dropout=0, channel_mult=(1, 2, 4, 8), conv_resample=True, dims=2,
                 num_classes=None, use_checkpoint=False, use_fp16=False, num_heads=-1, num_head_channels=-1,
                 num_heads_upsample=-1, use_scale_shift_norm=False, resblock_updown=False,
                 use_new_attention_order=False, use_spatial_transformer=False, transformer_depth=1,
                 context_dim=None, n_embed=None, legacy=True):
        super().__init__()
        if use_spatial_transformer:
            assert context_dim is not None, "use_spatial_transformer needs context_dim"
        if context_dim is not None:
            assert use_spatial_transformer, "context_dim needs use_spatial_transformer"
            context_dim = list(context_dim) if isinstance(context_dim, (list, tuple)) else context_dim
        if num_classes is not None or n_embed is not None:
            raise NotImplementedError("sd_amd: class-conditional / codebook heads are not on the SD path")
        if num_heads_upsample == -1:
            num_heads_upsample = num_heads
        if num_heads == -1:
            assert num_head_channels != -1, "Either num_heads or num_head_channels has to be set"
        if num_head_channels == -1:
            assert num_heads != -1, "Either num_heads or num_head_channels has to be set"
        self.image_size = image_size
        self.in_channels = in_channels
        self.model_channels = model_channels
        self.out_channels = out_channels
        self.num_res_blocks = num_res_blocks
        self.attention_resolutions = attention_resolutions
        self.dropout = dropout
        self.channel_mult = channel_mult
        self.conv_resample = conv_resample
        self.num_classes = num_classes
        self.use_checkpoint = use_checkpoint
        self.dtype = torch.float16 if use_fp16 else torch.float32
        self.num_heads = num_heads
        self.num_head_channels = num_head_channels
        self.num_heads_upsample = num_heads_upsample
        self.predict_codebook_ids = False

        def geom(ch):
            nonlocal num_heads
            if num_head_channels == -1:
                dim_head = ch // num_heads
            else:
                num_heads = ch // num_head_channels
                dim_head = num_head_channels
            if legacy:
                dim_head = ch // num_heads if use_spatial_transformer else num_head_channels
            return dim_head

        def attn_layer(ch, heads_for_attnblock):
            dim_head = geom(ch)
            if use_spatial_transformer:
                return SpatialTransformer(ch, num_heads, dim_head, depth=transformer_depth, context_dim=context_dim)
            return AttentionBlock(ch, use_checkpoint=use_checkpoint,
                                  num_heads=num_heads if heads_for_attnblock is None else heads_for_attnblock,
                                  num_head_channels=dim_head, use_new_attention_order=use_new_attention_order)

        time_embed_dim = model_channels * 4
        self.time_embed = nn.Sequential(linear(model_channels, time_embed_dim), nn.SiLU(),
                                        linear(time_embed_dim, time_embed_dim))
        self.input_blocks = nn.ModuleList(
            [TimestepEmbedSequential(conv_nd(dims, in_channels, model_channels, 3, padding=1))])
        input_block_chans = [model_channels]
        ch, ds = model_channels, 1
        for level, mult in enumerate(channel_mult):
            for _ in range(num_res_blocks):
                layers = [ResBlock(ch, time_embed_dim, dropout, out_channels=mult * model_channels, dims=dims,
                                   use_checkpoint=use_checkpoint, use_scale_shift_norm=use_scale_shift_norm)]
                ch = mult * model_channels
                if ds in attention_resolutions:
                    layers.append(attn_layer(ch, None))
                self.input_blocks.append(TimestepEmbedSequential(*layers))
                input_block_chans.append(ch)
            if level != len(channel_mult) - 1:
                if resblock_updown:
                    raise NotImplementedError("sd_amd: resblock_updown is not on the SD path")
                self.input_blocks.append(TimestepEmbedSequential(
                    Downsample(ch, conv_resample, dims=dims, out_channels=ch)))
                input_block_chans.append(ch)
                ds *= 2
        self.middle_block = TimestepEmbedSequential(
            ResBlock(ch, time_embed_dim, dropout, dims=dims, use_checkpoint=use_checkpoint,
                     use_scale_shift_norm=use_scale_shift_norm),
            attn_layer(ch, None),
            ResBlock(ch, time_embed_dim, dropout, dims=dims, use_checkpoint=use_checkpoint,
                     use_scale_shift_norm=use_scale_shift_norm))
        self.output_blocks = nn.ModuleList([])
        for level, mult in list(enumerate(channel_mult))[::-1]:
            for i in range(num_res_blocks + 1):
                ich = input_block_chans.pop()
                layers = [ResBlock(ch + ich, time_embed_dim, dropout, out_channels=model_channels * mult,
                                   dims=dims, use_checkpoint=use_checkpoint,
                                   use_scale_shift_norm=use_scale_shift_norm)]
                ch = model_channels * mult
                if ds in attention_resolutions:
                    layers.append(attn_layer(ch, num_heads_upsample))
                if level and i == num_res_blocks:
                    layers.append(Upsample(ch, conv_resample, dims=dims, out_channels=ch))
                    ds //= 2
                self.output_blocks.append(TimestepEmbedSequential(*layers))
        self.out = nn.Sequential(normalization(ch), nn.SiLU(),
                                 zero_module(conv_nd(dims, model_channels, out_channels, 3, padding=1)))
        self._prepared_on = None
        self._ctx_cache = None

    # ------------------------------------------------------------------ packing
    def load_state_dict(self, *args, **kwargs):
        self._prepared_on = None
        self._ctx_cache = None
        return super().load_state_dict(*args, **kwargs)

    @torch.no_grad()
    def prepare(self, device):
        """Pack weights (NHWC fp16, fused segments) on ``device``.  Called lazily by forward;
        call again after modifying parameters in place."""
        dev = torch.device(device)
        resblocks = [m for m in self.modules() if isinstance(m, ResBlock)]
        off = 0
        ws, bs = [], []
        for rb in resblocks:
            rb._prepare(dev)
            rb._emb_off = off
            off += rb.out_channels
            ws.append(rb.emb_layers[1].weight)
            bs.append(rb.emb_layers[1].bias)
        self._emb_total = off
        te = self.model_channels * 4
        self._pc_emb = ops.PackedConv([(torch.cat(ws, 0), te)], torch.cat(bs, 0), device=dev)
        self._pc_te0 = ops.PackedConv([(self.time_embed[0].weight, self.model_channels)], self.time_embed[0].bias,
                                      device=dev)
        self._pc_te2 = ops.PackedConv([(self.time_embed[2].weight, te)], self.time_embed[2].bias, device=dev)
        for m in self.modules():
            if isinstance(m, (SpatialTransformer, AttentionBlock, Downsample, Upsample)):
                m._prepare(dev)
        conv_in = self.input_blocks[0][0]
        self._cin_pad = (self.in_channels + 7) // 8 * 8
        conv_in._pc = ops.PackedConv([(conv_in.weight, self._cin_pad)], conv_in.bias, device=dev)
        self.out[0]._prepare(dev)
        self._pc_out = ops.PackedConv([(self.out[2].weight, self.model_channels)], self.out[2].bias, device=dev)
        self._freqs = timestep_frequencies(self.model_channels).to(dev)
        self._sts = [m for m in self.modules() if isinstance(m, SpatialTransformer)]
        self._prepared_on = dev
        self._ctx_cache = None
        # packed weights were replaced: graphs captured on the old ones must be dropped
        self.prepare_generation = getattr(self, "prepare_generation", 0) + 1

    # contexts whose K/V stay resident (cond, uncond, their CFG concat, one spare)
    CONTEXT_CACHE_SIZE = 4

    def _context_kv(self, context):
        """K|V of every cross-attention for ``context``, computed once per conditioning tensor
        (step-invariant across the sampler loop, reference ``ldm/diffusion/ddim.py:168-180``).

        The cache is keyed on tensor IDENTITY: an entry holds a strong reference to its context
        tensor (so neither its memory block nor its ``id`` can be handed to another tensor while
        the entry lives) and the tensor's ``_version`` at projection time (an in-place write
        misses).  A different conditioning therefore never hits another's K/V, whatever address
        the caching allocator gives it.  LRU eviction drops only the oldest entry; a captured
        HIP graph keeps its own reference to the K/V it reads (``graphs.GraphedUNet``)."""
        if context is None:
            return None, None
        if self._ctx_cache is None:
            self._ctx_cache = OrderedDict()
        ent = self._ctx_cache.get(id(context))
        if ent is not None and ent[0] is context and ent[1] == context._version:
            self._ctx_cache.move_to_end(id(context))
            return ent[2], context.shape[1]
        B, L, D = context.shape
        if context.dtype == torch.float16:
            c2 = context.reshape(B * L, D).contiguous()
        else:
            c2 = ops.nchw_to_nhwc(context.reshape(B * L, D, 1, 1).float(), D).view(B * L, D)
        kv = {}
        for st in self._sts:
            kv[id(st)] = st.context_kv(c2, L)
        self._ctx_cache[id(context)] = (context, context._version, kv)
        self._ctx_cache.move_to_end(id(context))
        while len(self._ctx_cache) > self.CONTEXT_CACHE_SIZE:
            self._ctx_cache.popitem(last=False)
        return kv, L

    def clear_context_cache(self):
        self._ctx_cache = None

    # ------------------------------------------------------------------ forward
    @torch.no_grad()
    def forward(self, x, timesteps=None, context=None, y=None, **kwargs):
        assert (y is not None) == (self.num_classes is not None), "y iff class-conditional"
        if not x.is_cuda:
            raise TypeError("sd_amd.UNetModel: HIP path only — move inputs to the GPU")
        if self._prepared_on != x.device:
            self.prepare(x.device)
        B = x.shape[0]
        t = timesteps
        if not torch.is_tensor(t):
            t = torch.tensor(t)
        if t.is_floating_point():
            # the reference embeds timesteps[:, None].float() (openai_model/utils.py:234-242); the
            # embedding kernel takes integer steps, so a fractional step must not be truncated
            if not bool((t == t.round()).all()):
                raise ValueError("sd_amd.UNetModel: fractional timesteps are not supported (integer steps only)")
        t = t.to(device=x.device, dtype=torch.int64).reshape(-1)
        if t.numel() == 1 and B > 1:
            t = t.expand(B).contiguous()
        temb = ops.timestep_embedding(t, self._freqs, self.model_channels)
        e1 = ops.linear(self._pc_te0, temb)
        emb = ops.linear(self._pc_te2, e1, silu=True)
        emb_all = ops.linear(self._pc_emb, emb, silu=True, out_mode=ops.OUT_ROWS_F32)
        kv, Lc = self._context_kv(context)
        st = {"emb": emb_all, "kv": kv, "Lc": Lc}
        h = ops.nchw_to_nhwc(x.float(), self._cin_pad)
        hs = []
        for module in self.input_blocks:
            h = module._run(h, st)
            hs.append(h)
        h = self.middle_block._run(h, st)
        for module in self.output_blocks:
            h = module._run((h, hs.pop()), st)
        gp, cp = ops.gn_conv_pad()
        ha = self.out[0].norm(h, silu=True, pad=gp)
        out = ops.conv2d(self._pc_out, ha, pad=cp, out_mode=ops.OUT_NCHW_F32)
        return out if x.dtype == torch.float32 else out.to(x.dtype)
