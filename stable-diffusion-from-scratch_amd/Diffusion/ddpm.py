"""Mirror of the inference surface of ``Diffusion/ddpm.py`` — DiffusionWrapper and LatentDiffusion.

Kept: ``register_schedule`` buffers (``ddpm.py:195-253``), ``apply_model``
conditioning wrapping (``ddpm.py:1139-1147,1269-1272`` → ``{'c_crossattn': [c]}``),
``DiffusionWrapper.forward`` dispatch (``ddpm.py:46-73``), ``decode_first_stage``
with the CompVis scaling ``z / scale_factor`` (``ldm/diffusion/ddpm.py:1095``;
``Diffusion/ddpm.py:728`` drops z — SURVEY Q8), ``parameterization``.
``cond_stage_config`` is instantiated as the reference does (``ddpm.py:568-587``:
``__is_first_stage__`` / ``__is_unconditional__`` / a target, frozen), so the reference YAML's
``clip_encoder.modules.FrozenCLIPEmbedder`` resolves to the HIP-backed text tower;
``get_learned_conditioning`` (``ddpm.py:1031-1051``) encodes through it.
``use_graphs(True)`` makes ``DiffusionWrapper.forward`` replay one HIP graph per UNet call
(``graphs.GraphedUNet``) — same chain apply_model → DiffusionWrapper.forward → UNetModel,
one hipGraphLaunch per step instead of ~600 kernel launches.
Out of scope (training / Lightning): losses, EMA, optimisers, data, logging.
"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn

from .. import ops
from ..DDIM.diffusion_modules import register_schedule
from .utils import instantiate_from_config


class DiffusionWrapper(nn.Module):
    def __init__(self, diff_model_config, conditioning_key):
        super().__init__()
        self.diffusion_model = instantiate_from_config(diff_model_config)
        self.conditioning_key = conditioning_key
        assert self.conditioning_key in [None, "concat", "crossattn", "hybrid", "adm"]
        self._graphed = None
        self._graphs_on = False

    def use_graphs(self, on=True):
        """Route the UNet call through one captured HIP graph per (shape, context) key (the
        captured graphs are kept while switched off, e.g. for an eager profiling pass)."""
        from ..graphs import GraphedUNet
        if on and self._graphed is None:
            self._graphed = GraphedUNet(self.diffusion_model)
        self._graphs_on = bool(on)

    @staticmethod
    def _int_timesteps(t, device):
        """Timesteps as int64 on the device, the same check on both paths: fractional values raise
        (the UNet's sinusoidal table is indexed by integer steps); only a floating-point t is
        checked, so the sampler's int64 timesteps never cost a host sync."""
        if not torch.is_tensor(t):
            t = torch.as_tensor(t)
        if t.is_floating_point():
            if not bool((t == t.round()).all()):
                raise ValueError("sd_amd: timesteps must be integral")
        return t.to(device=device, dtype=torch.long)

    def _unet(self, x, t, context=None):
        t = self._int_timesteps(t, x.device)
        if self._graphs_on:
            return self._graphed(x, t.reshape(-1).expand(x.shape[0]), context)
        return self.diffusion_model(x, t, context=context)

    def forward(self, x, t, c_concat: list = None, c_crossattn: list = None):
        if self.conditioning_key is None:
            return self._unet(x, t)
        if self.conditioning_key == "crossattn":
            cc = c_crossattn[0] if len(c_crossattn) == 1 else torch.cat(c_crossattn, 1)
            return self._unet(x, t, context=cc)
        raise NotImplementedError(f"sd_amd: conditioning_key={self.conditioning_key} is not on the txt2img path")


class LatentDiffusion(nn.Module):
    def __init__(self, first_stage_config, cond_stage_config=None, unet_config=None, num_timesteps_cond=None,
                 cond_stage_key="txt", cond_stage_trainable=False, concat_mode=True, cond_stage_forward=None,
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
        self.cond_stage_trainable = cond_stage_trainable
        self.cond_stage_key = cond_stage_key
        self.cond_stage_forward = cond_stage_forward
        self.instantiate_cond_stage(cond_stage_config)
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

    def use_graphs(self, on=True):
        self.model.use_graphs(on)

    def instantiate_cond_stage(self, config):
        """Reference ``Diffusion/ddpm.py:568-587`` (inference: the stage is always frozen)."""
        if config is None or config == "__is_unconditional__":
            self.cond_stage_model = None
        elif config == "__is_first_stage__":
            self.cond_stage_model = self.first_stage_model
        else:
            model = instantiate_from_config(config)
            self.cond_stage_model = model.eval()
            for param in self.cond_stage_model.parameters():
                param.requires_grad = False

    @torch.no_grad()
    def get_learned_conditioning(self, c):
        """Reference ``Diffusion/ddpm.py:1031-1051``: encode prompts (or token ids) with the cond stage."""
        if self.cond_stage_forward is None:
            if hasattr(self.cond_stage_model, "encode") and callable(self.cond_stage_model.encode):
                c = self.cond_stage_model.encode(c)
                from ..Distribution.distribution import DiagonalGaussianDistribution
                if isinstance(c, DiagonalGaussianDistribution):
                    c = c.mode()
            else:
                c = self.cond_stage_model(c)
        else:
            assert hasattr(self.cond_stage_model, self.cond_stage_forward)
            c = getattr(self.cond_stage_model, self.cond_stage_forward)(c)
        return c

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
        """``ldm/diffusion/ddpm.py:1083-1156``: z / scale_factor → first-stage decode; with
        ``split_input_params['patch_distributed_vq']`` the tiled (patch) decode."""
        sp = getattr(self, "split_input_params", None)
        if sp and sp.get("patch_distributed_vq"):
            return self._decode_tiled(z, sp)
        return self.first_stage_model.decode(z, pre_scale=1.0 / self.scale_factor)

    # ------------------------------------------------------------------ tiled decode
    @staticmethod
    def delta_border(h, w):
        """Normalised distance of each pixel to the nearest border (0 at the border, 0.5 at the
        centre): min(y/(h-1), x/(w-1), 1-y/(h-1), 1-x/(w-1)) in fp32 — the CompVis semantics of
        ``ldm/diffusion/ddpm.py:838-859``; the reference takes its first min over dim=1 and then
        fails in torch.cat for any w > 1."""
        f32 = np.float32
        y = np.arange(h, dtype=np.int64)[:, None].astype(f32) / f32(h - 1)
        x = np.arange(w, dtype=np.int64)[None, :].astype(f32) / f32(w - 1)
        y, x = np.broadcast_to(y, (h, w)), np.broadcast_to(x, (h, w))
        lu = np.minimum(y, x)
        rd = np.minimum(f32(1.0) - y, f32(1.0) - x)
        return np.minimum(lu, rd).astype(f32)

    def get_weighting(self, h, w, Ly, Lx, sp):
        """Pixel weights [h, w] and (tie-breaker) patch weights [Ly*Lx] or None
        (``ldm/diffusion/ddpm.py:862-891``; weighting = pixel ⊗ patch, kept separable)."""
        pix = np.clip(self.delta_border(h, w), sp["clip_min_weight"], sp["clip_max_weight"]).astype(np.float32)
        lw = None
        if sp.get("tie_braker", False):
            lo = sp.get("clip_min_tie_weight", sp.get("clip_min_the_weight"))
            hi = sp.get("clip_max_tie_weight", sp.get("clip_max_the_weight"))
            lw = np.clip(self.delta_border(Ly, Lx), lo, hi).astype(np.float32).reshape(-1)
        return pix, lw

    def _decode_tiled(self, z, sp):
        """Patch decode (``ldm/diffusion/ddpm.py:1097-1139`` + ``get_fold_unfold`` uf branch
        ``:894-960``): latent patches of ``ks`` every ``stride`` are decoded as one batch
        (chunks of ``sp.get('max_batch', 16)`` patches·images), weighted and overlap-added at
        uf = vqf on the device (``sdk_extract_patches`` / ``sdk_fold_patches``)."""
        ks, stride, uf = tuple(sp["ks"]), tuple(sp["stride"]), int(sp["vqf"])
        B, Cz, h, w = z.shape
        ks = (min(ks[0], h), min(ks[1], w))
        stride = (min(stride[0], h), min(stride[1], w))
        Ly, Lx = (h - ks[0]) // stride[0] + 1, (w - ks[1]) // stride[1] + 1
        key = (ks, stride, uf, Ly, Lx, z.device)
        cache = getattr(self, "_tile_w", None)
        if cache is None or cache[0] != key:
            pix, lw = self.get_weighting(ks[0] * uf, ks[1] * uf, Ly, Lx, sp)
            cache = (key, torch.from_numpy(pix).to(z.device),
                     torch.from_numpy(lw).to(z.device) if lw is not None else None)
            self._tile_w = cache
        _, pix_w, l_w = cache
        patches = ops.extract_patches(z.float(), ks[0], ks[1], stride[0], stride[1])   # [L, B, C, kh, kw]
        flat = patches.view(Ly * Lx * B, Cz, ks[0], ks[1])
        chunk = int(sp.get("max_batch", 16))
        dec = [self.first_stage_model.decode(flat[i:i + chunk], pre_scale=1.0 / self.scale_factor)
               for i in range(0, flat.shape[0], chunk)]
        dec = torch.cat(dec, 0) if len(dec) > 1 else dec[0]
        dec = dec.view(Ly * Lx, B, dec.shape[1], dec.shape[2], dec.shape[3])
        return ops.fold_patches(dec, pix_w, l_w, h * uf, w * uf, stride[0] * uf, stride[1] * uf, Ly, Lx)
