"""Mirror of ``VAE/autoencoder.py`` — AutoEncoderKL (encode and decode on the HIP path).

``decode(z)`` = post_quant_conv (1x1) → Decoder (``autoencoder.py:126-132``).
``encode(x)`` = Encoder → quant_conv (folded into the encoder's conv_out) →
DiagonalGaussianDistribution (``autoencoder.py:114-123``); the encoder is packed on the
first encode call.
The 1x1 post_quant_conv runs as a GEMM whose output is zero-padded to 8
channels (the NHWC kernels need 8-channel granularity); the decoder's conv_in
consumes those 8 channels with zero weights on the padding.
``lossconfig`` is accepted and ignored (inference only; the reference's
``lossconfig=None`` path raises AttributeError).
"""
from __future__ import annotations

import importlib

import torch
from torch import nn

from .. import ops
from ..Distribution.distribution import DiagonalGaussianDistribution
from ..Encoder_Decoder.encoder import Decoder, Encoder


class AutoEncoderKL(nn.Module):
    def __init__(self, ddconfig, embed_dim, lossconfig=None, ckpt_path=None, ignore_keys=[], colorize_nlabels=None,
                 monitor=None):
        super().__init__()
        self.encoder = Encoder(**ddconfig)
        self.decoder = Decoder(**ddconfig)
        self.learning_rate = 4.5e-06
        assert ddconfig["double_z"], "make sure `double_z: True`"
        self.quant_conv = nn.Conv2d(2 * ddconfig["z_channels"], 2 * embed_dim, kernel_size=1)
        self.post_quant_conv = nn.Conv2d(embed_dim, ddconfig["z_channels"], kernel_size=1)
        self.embed_dim = embed_dim
        self.z_channels = ddconfig["z_channels"]
        if colorize_nlabels is not None:
            self.register_buffer("colorize", torch.randn(3, colorize_nlabels, 1, 1))
        if monitor is not None:
            self.monitor = monitor
        if ckpt_path is not None:
            self.init_from_ckpt(ckpt_path, ignore_keys=ignore_keys)
        self._prepared_on = None

    def init_from_ckpt(self, path, ignore_keys=list()):
        sd = torch.load(path, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd)
        for k in list(sd.keys()):
            if any(k.startswith(ik) for ik in ignore_keys):
                del sd[k]
        self.load_state_dict(sd, strict=False)

    def load_state_dict(self, *args, **kwargs):
        self._prepared_on = None
        self.encoder._prepared_on = None
        return super().load_state_dict(*args, **kwargs)

    @torch.no_grad()
    def prepare(self, device):
        dev = torch.device(device)
        self._ezp = (self.embed_dim + 7) // 8 * 8
        self._zcp = (self.z_channels + 7) // 8 * 8
        w = torch.zeros(self._zcp, self.embed_dim, 1, 1, device=self.post_quant_conv.weight.device)
        w[: self.z_channels] = self.post_quant_conv.weight.detach()
        b = torch.zeros(self._zcp, device=w.device)
        b[: self.z_channels] = self.post_quant_conv.bias.detach()
        self._pc_pq = ops.PackedConv([(w, self._ezp)], b, device=dev)
        self.decoder._prepare(dev, self._zcp)
        self.decoder._prepared_on = (dev, self._zcp)
        self._prepared_on = dev

    @torch.no_grad()
    def encode(self, x):
        """x: NCHW image [B, in_channels, H, W] (any float dtype) → DiagonalGaussianDistribution."""
        if not x.is_cuda:
            raise TypeError("sd_amd.AutoEncoderKL: HIP path only — move inputs to the GPU")
        in_pad = (x.shape[1] + 7) // 8 * 8
        if getattr(self.encoder, "_prepared_on", None) != (x.device, in_pad, True):
            self.encoder._prepare(x.device, in_pad, quant_conv=self.quant_conv)
        moments = self.encoder._run(ops.nchw_to_nhwc(x.float(), in_pad))
        return DiagonalGaussianDistribution(moments)

    @torch.no_grad()
    def decode(self, z, pre_scale: float = 1.0):
        """z: [B, embed_dim, h, w] → [B, out_ch, 8h, 8w] fp32.  ``pre_scale`` fuses
        decode_first_stage's ``1/scale_factor * z`` into the layout conversion."""
        if not z.is_cuda:
            raise TypeError("sd_amd.AutoEncoderKL: HIP path only — move inputs to the GPU")
        if self._prepared_on != z.device:
            self.prepare(z.device)
        zn = ops.nchw_to_nhwc(z.float(), self._ezp, scale=pre_scale)
        zq = ops.conv2d(self._pc_pq, zn)
        return self.decoder._run(zq)

    @torch.no_grad()
    def forward(self, input, sample_posterior=True):
        posterior = self.encode(input)
        z = posterior.sample() if sample_posterior else posterior.mode()
        return self.decode(z), posterior


def instantiate_from_config(config):
    from ..Diffusion.utils import instantiate_from_config as inst
    return inst(config)
