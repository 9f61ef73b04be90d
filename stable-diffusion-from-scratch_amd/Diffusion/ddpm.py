"""Mirror of the inference surface of ``Diffusion/ddpm.py`` — DiffusionWrapper and LatentDiffusion.

Kept: ``register_schedule`` buffers (``ddpm.py:195-253``), ``apply_model``
conditioning wrapping (``ddpm.py:1139-1147,1269-1272`` → ``{'c_crossattn': [c]}``),
``DiffusionWrapper.forward`` dispatch (``ddpm.py:46-73``), ``decode_first_stage``
with the CompVis scaling ``z / scale_factor`` (``ldm/diffusion/ddpm.py:1095``;
``Diffusion/ddpm.py:728`` drops z — SURVEY Q8), ``parameterization``.
Out of scope (training / Lightning / CLIP): losses, EMA, optimisers, data,
logging, ``cond_stage_model`` — the conditioning tensor is passed in directly.
"""
from __future__ import annotations

import torch
from torch import nn

from ..DDIM.diffusion_modules import register_schedule
from .utils import instantiate_from_config


class DiffusionWrapper(nn.Module):
    def __init__(self, diff_model_config, conditioning_key):
        super().__init__()
        self.diffusion_model = instantiate_from_config(diff_model_config)
        self.conditioning_key = conditioning_key
        assert self.conditioning_key in [None, "concat", "crossattn", "hybrid", "adm"]

    def forward(self, x, t, c_concat: list = None, c_crossattn: list = None):
        if self.conditioning_key is None:
            return self.diffusion_model(x, t)
        if self.conditioning_key == "crossattn":
            cc = c_crossattn[0] if len(c_crossattn) == 1 else torch.cat(c_crossattn, 1)
            return self.diffusion_model(x, t, context=cc)
        raise NotImplementedError(f"sd_amd: conditioning_key={self.conditioning_key} is not on the txt2img path")


class LatentDiffusion(nn.Module):
    def __init__(self, first_stage_config, cond_stage_config=None, unet_config=None, num_timesteps_cond=None,
                 cond_stage_key="image", cond_stage_trainable=False, concat_mode=True, cond_stage_forward=None,
                 conditioning_key=None, scale_factor=1.0, scale_by_std=False, timesteps=1000,
                 beta_schedule="linear", linear_start=1e-4, linear_end=2e-2, cosine_s=8e-3, given_betas=None,
                 parameterization="eps", image_size=256, channels=3, first_stage_key="image", log_every_t=100,
                 **ignored):
        super().__init__()
        assert parameterization in ["eps", "x0", "v"], "eps / x0 (reference) or v (extension, SURVEY Q9)"
        if parameterization == "x0":
            raise NotImplementedError("sd_amd: x0-parameterised DDIM is not on the txt2img path")
        self.parameterization = parameterization
        if conditioning_key is None:
            conditioning_key = "concat" if concat_mode else "crossattn"
        if cond_stage_config == "__is_unconditional__":
            conditioning_key = None
        self.conditioning_key = conditioning_key
        self.model = DiffusionWrapper(unet_config, conditioning_key)
        self.first_stage_model = instantiate_from_config(first_stage_config)
        self.cond_stage_model = None     # CLIP text encoder: outside the hot path (synthetic context)
        self.scale_factor = scale_factor
        self.image_size = image_size
        self.channels = channels
        self.log_every_t = log_every_t
        sch = register_schedule(timesteps, linear_start, linear_end, beta_schedule, given_betas, cosine_s)
        self.num_timesteps = sch.pop("num_timesteps")
        for k, v in sch.items():
            self.register_buffer(k, v)

    @property
    def device(self):
        return next(self.model.parameters()).device

    def apply_model(self, x_noisy, t, cond, return_ids=False):
        if isinstance(cond, dict):
            pass
        else:
            if not isinstance(cond, list):
                cond = [cond]
            key = "c_concat" if self.model.conditioning_key == "concat" else "c_crossattn"
            cond = {key: cond}
        if self.model.conditioning_key is None:
            return self.model(x_noisy, t)
        return self.model(x_noisy, t, **cond)

    @torch.no_grad()
    def encode_first_stage(self, x):
        """``ldm/diffusion/ddpm.py:1237-1279`` (non-split branch): the first stage's posterior."""
        return self.first_stage_model.encode(x)

    def get_first_stage_encoding(self, encoder_posterior, noise=None):
        """``ldm/diffusion/ddpm.py:795-806``: scale_factor * posterior sample (fused on the device)."""
        from ..Distribution.distribution import DiagonalGaussianDistribution
        if isinstance(encoder_posterior, DiagonalGaussianDistribution):
            return encoder_posterior.sample_scaled(self.scale_factor, noise=noise)
        if isinstance(encoder_posterior, torch.Tensor):
            return self.scale_factor * encoder_posterior
        raise NotImplementedError(f"encoder_posterior of type '{type(encoder_posterior)}' not yet implemented")

    @torch.no_grad()
    def decode_first_stage(self, z, predict_cids=False, force_not_quantize=False):
        return self.first_stage_model.decode(z, pre_scale=1.0 / self.scale_factor)
