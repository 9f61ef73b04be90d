"""Mirror of ``DDIM/ddim.py`` (≡ ``ldm/diffusion/ddim.py``, the working CompVis sampler) — DDIMSampler.

Host loop over ``np.flip(ddim_timesteps)`` exactly as the reference
(``ddim.py:114-163``); per step the model call and ONE fused HIP update
(``sdk_ddim_step``: classifier-free-guidance combine + v→ε conversion + DDIM
update, fp32, no contraction → bit-identical to the reference expression on
the same inputs).  Per-step scalars are the fp32 values ``torch.full(...)``
would hold (``ddim.py:189-192``), derived with torch's CPU fp32 ops.

Extensions (documented, not in the reference): ``parameterization == "v"``
on the model and an optional ``noise_fn(i, shape)`` hook
so η>0 runs can be reproduced bit-for-bit.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops
from .diffusion_modules import make_ddim_sampling_parameters, make_ddim_timesteps, noise_like, sqrt_one_minus


class DDIMSampler(object):
    def __init__(self, model, schedule="linear", **kwargs):
        super().__init__()
        self.model = model
        self.ddpm_num_timesteps = model.num_timesteps
        self.schedule = schedule

    def register_buffer(self, name, attr):
        setattr(self, name, attr)

    def make_schedule(self, ddim_num_steps, ddim_discretize="uniform", ddim_eta=0., verbose=True):
        self.ddim_timesteps = make_ddim_timesteps(ddim_discretize, ddim_num_steps, self.ddpm_num_timesteps,
                                                  verbose=verbose)
        alphas_cumprod = self.model.alphas_cumprod
        assert alphas_cumprod.shape[0] == self.ddpm_num_timesteps, "alphas have to be defined for each timestep"
        ac = alphas_cumprod.detach().to("cpu", torch.float32)
        self.register_buffer("alphas_cumprod", ac)
        sig, a, ap = make_ddim_sampling_parameters(ac, self.ddim_timesteps, ddim_eta, verbose=verbose)
        self.register_buffer("ddim_sigmas", sig)
        self.register_buffer("ddim_alphas", a)
        self.register_buffer("ddim_alphas_prev", ap)
        self.register_buffer("ddim_sqrt_one_minus_alphas", sqrt_one_minus(a))
        self.ddim_eta = ddim_eta

    def step_scalars(self, index):
        """fp32 scalars of p_sample_ddim at ``index`` (``ddim.py:189-203``): the values
        ``torch.full((b,1,1,1), table[index])`` holds and the fp32 coefficients torch
        derives from them, evaluated with IEEE numpy fp32 scalars on the host."""
        f32 = np.float32
        a_t = f32(self.ddim_alphas[index].item())
        a_prev = f32(float(self.ddim_alphas_prev[index]))
        sigma = f32(float(self.ddim_sigmas[index]))
        s1m = f32(self.ddim_sqrt_one_minus_alphas[index].item())
        return {"a_t": float(a_t), "sqrt_one_minus_at": float(s1m), "sqrt_at": float(np.sqrt(a_t)),
                "dir_coef": float(np.sqrt(f32(f32(f32(1.0) - a_prev) - f32(sigma * sigma)))),
                "sqrt_a_prev": float(np.sqrt(a_prev)), "sigma": float(sigma),
                "v_sqrt_a": float(np.sqrt(a_t)), "v_sqrt_1ma": float(np.sqrt(f32(f32(1.0) - a_t)))}

    @torch.no_grad()
    def sample(self, S, batch_size, shape, conditioning=None, callback=None, normals_sequence=None, img_callback=None,
               quantize_x0=False, eta=0., mask=None, x0=None, temperature=1., noise_dropout=0., score_corrector=None,
               corrector_kwargs=None, verbose=True, x_T=None, log_every_t=100, unconditional_guidance_scale=1.,
               unconditional_conditioning=None, noise_fn=None, **kwargs):
        if conditioning is not None:
            cbs = conditioning[list(conditioning.keys())[0]].shape[0] if isinstance(conditioning, dict) \
                else conditioning.shape[0]
            if cbs != batch_size:
                print(f"Warning: Got {cbs} conditionings but batch-size is {batch_size}")
        self.make_schedule(ddim_num_steps=S, ddim_eta=eta, verbose=verbose)
        C, H, W = shape
        size = (batch_size, C, H, W)
        if verbose:
            print(f"Data shape for DDIM sampling is {size}, eta {eta}")
        return self.ddim_sampling(conditioning, size, callback=callback, img_callback=img_callback,
                                  quantize_denoised=quantize_x0, mask=mask, x0=x0, noise_dropout=noise_dropout,
                                  temperature=temperature, score_corrector=score_corrector,
                                  corrector_kwargs=corrector_kwargs, x_T=x_T, log_every_t=log_every_t,
                                  unconditional_guidance_scale=unconditional_guidance_scale,
                                  unconditional_conditioning=unconditional_conditioning, noise_fn=noise_fn)

    @torch.no_grad()
    def ddim_sampling(self, cond, shape, x_T=None, ddim_use_original_steps=False, callback=None, timesteps=None,
                      quantize_denoised=False, mask=None, x0=None, img_callback=None, log_every_t=100,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None, noise_fn=None):
        if ddim_use_original_steps or mask is not None or quantize_denoised or score_corrector is not None \
                or noise_dropout > 0:
            raise NotImplementedError("sd_amd: original-steps / masking / quantize / score_corrector / "
                                      "noise_dropout are not on the txt2img hot path")
        device = self.model.device
        b = shape[0]
        img = torch.randn(shape, device=device) if x_T is None else x_T.to(device=device, dtype=torch.float32)
        img = img.contiguous()
        ts_all = self.ddim_timesteps if timesteps is None else \
            self.ddim_timesteps[:int(min(timesteps / self.ddim_timesteps.shape[0], 1) * self.ddim_timesteps.shape[0]) - 1]
        intermediates = {"x_inter": [img], "pred_x0": [img]}
        time_range = np.flip(ts_all)
        total_steps = ts_all.shape[0]
        for i, step in enumerate(time_range):
            index = total_steps - i - 1
            ts = torch.full((b,), int(step), device=device, dtype=torch.long)
            img, pred_x0 = self.p_sample_ddim(img, cond, ts, index=index, temperature=temperature,
                                              unconditional_guidance_scale=unconditional_guidance_scale,
                                              unconditional_conditioning=unconditional_conditioning,
                                              noise=(noise_fn(i, img.shape) if noise_fn is not None else None))
            if callback:
                callback(i)
            if img_callback:
                img_callback(pred_x0, i)
            if index % log_every_t == 0 or index == total_steps - 1:
                intermediates["x_inter"].append(img)
                intermediates["pred_x0"].append(pred_x0)
        return img, intermediates

    def _cfg_context(self, uc, c):
        """``torch.cat([uc, c])`` (``ddim.py:177``), built ONCE per conditioning pair rather than once
        per step: the same tensor object every step lets the UNet's context K/V cache and the
        graph cache (both keyed on tensor identity) hit across the 50 steps.  The cached pair is
        held by reference and checked by identity + version, so new prompts rebuild it."""
        ent = getattr(self, "_cfg_cache", None)
        if ent is not None and ent[0] is uc and ent[1] is c and ent[2] == (uc._version, c._version):
            return ent[3]
        c_in = torch.cat([uc, c])
        self._cfg_cache = (uc, c, (uc._version, c._version), c_in)
        return c_in

    @torch.no_grad()
    def p_sample_ddim(self, x, c, t, index, repeat_noise=False, use_original_steps=False, quantize_denoised=False,
                      temperature=1., noise_dropout=0., score_corrector=None, corrector_kwargs=None,
                      unconditional_guidance_scale=1., unconditional_conditioning=None, noise=None):
        b = x.shape[0]
        sc = self.step_scalars(index)
        e_u = None
        if unconditional_conditioning is None or unconditional_guidance_scale == 1.:
            e_t = self.model.apply_model(x, t, c)
        else:
            x_in = torch.cat([x] * 2)
            t_in = torch.cat([t] * 2)
            c_in = self._cfg_context(unconditional_conditioning, c)
            both = self.model.apply_model(x_in, t_in, c_in)
            e_u, e_t = both[:b], both[b:]
        e_t = e_t.float().contiguous()
        if e_u is not None:
            e_u = e_u.float().contiguous()
        if sc["sigma"] != 0.0 and noise is None:
            noise = noise_like(x.shape, x.device, repeat_noise)
        v = (sc["v_sqrt_a"], sc["v_sqrt_1ma"]) if getattr(self.model, "parameterization", "eps") == "v" else None
        return ops.ddim_step(x.float().contiguous(), e_t, sc, noise=noise if sc["sigma"] != 0.0 else None,
                             e_uncond=e_u, guidance=unconditional_guidance_scale, v_param=v,
                             temperature=temperature)

    # ------------------------------------------------------------------ img2img
    @torch.no_grad()
    def stochastic_encode(self, x0, t, use_original_steps=False, noise=None):
        """q(x_t | x0) at DDIM index t (``ddim.py:207-220``): sqrt(a_t)·x0 + sqrt(1-a_t)·noise, fp32 op
        by op on the device (``sdk_stochastic_encode``) — bit-identical to the reference expression.
        ``t`` holds DDIM indices per sample (original 1000-step indices with ``use_original_steps``)."""
        if use_original_steps:
            ac = self.model.alphas_cumprod.detach().to("cpu", torch.float32).numpy()
            sa_tab = np.sqrt(ac)
            s1m_tab = np.sqrt((np.float32(1.0) - ac).astype(np.float32))
        else:
            sa_tab = np.sqrt(self.ddim_alphas.numpy().astype(np.float32))
            s1m_tab = self.ddim_sqrt_one_minus_alphas.numpy().astype(np.float32)
        x0 = x0.float().contiguous()
        if noise is None:
            noise = torch.randn_like(x0)
        noise = noise.to(device=x0.device, dtype=torch.float32).contiguous()
        tt = torch.as_tensor(t).reshape(-1).to("cpu", torch.long)
        if tt.numel() == 1:
            tt = tt.expand(x0.shape[0])
        out = torch.empty_like(x0)
        vals = tt.unique()
        if vals.numel() == 1:
            i = int(vals[0])
            return ops.stochastic_encode(x0, noise, float(sa_tab[i]), float(s1m_tab[i]), out=out)
        for b in range(x0.shape[0]):                 # per-sample timesteps: one launch per sample
            i = int(tt[b])
            ops.stochastic_encode(x0[b], noise[b], float(sa_tab[i]), float(s1m_tab[i]), out=out[b])
        return out

    @torch.no_grad()
    def decode(self, x_latent, cond, t_start, unconditional_guidance_scale=1.0, unconditional_conditioning=None,
               use_original_steps=False):
        """Denoise from DDIM index ``t_start`` (``ddim.py:222-240``): timesteps[:t_start] walked in
        reverse, index = total_steps - i - 1, one fused HIP update per step."""
        if use_original_steps:
            raise NotImplementedError("sd_amd: original-steps decoding is not on the img2img path")
        timesteps = self.ddim_timesteps[:t_start]
        time_range = np.flip(timesteps)
        total_steps = timesteps.shape[0]
        x_dec = x_latent.float().contiguous()
        for i, step in enumerate(time_range):
            index = total_steps - i - 1
            ts = torch.full((x_latent.shape[0],), int(step), device=x_latent.device, dtype=torch.long)
            x_dec, _ = self.p_sample_ddim(x_dec, cond, ts, index=index, use_original_steps=use_original_steps,
                                          unconditional_guidance_scale=unconditional_guidance_scale,
                                          unconditional_conditioning=unconditional_conditioning)
        return x_dec
