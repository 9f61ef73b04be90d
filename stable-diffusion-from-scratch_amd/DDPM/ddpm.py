"""Mirror of ``DDPM/ddpm.py`` — DDPMPipeline (config C1), HIP-backed.

Tables (``ddpm.py:17-28``): betas = torch.linspace(start, end, T) in fp32, alphas = 1 - betas,
alphas_hat = cumprod (torch's CPU cumprod accumulates in double) — evaluated with numpy IEEE
arithmetic so they are bit-identical to the reference on any host CPU.
``sampling`` (``ddpm.py:53-89``, Algorithm 2 as written): for t = T-1 … 0, ε = model(x, t), then
x = α_t^-½ (x − β_t / √(1 − ᾱ_{t−1}) ε) + √β̃_t · z with ᾱ_{t−1} taken as ``alphas_hat[t-1]`` (which
wraps to ᾱ_{T−1} at t = 0) — one fused ``sdk_ddpm_step`` per step, fp32, no contraction.
``forward_diffusion`` (``ddpm.py:30-48``): √ᾱ_t x + √(1−ᾱ_t) z (``sdk_stochastic_encode``).
``noise_fn(i, shape)`` (extension) supplies the per-step noise so runs are reproducible.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops

F32, F64 = np.float32, np.float64


def _linspace32(start, end, n):
    """torch.linspace(start, end, n) in fp32 (two-sided evaluation, as torch's CPU kernel)."""
    if n == 1:
        return np.array([start], dtype=F32)
    s, e = F32(start), F32(end)
    step = (e - s) / F32(n - 1)
    idx = np.arange(n, dtype=F32)
    half = n // 2
    out = np.empty(n, dtype=F32)
    out[:half] = s + step * idx[:half]
    out[half:] = e - step * (F32(n - 1) - idx[half:])
    return out


def broadcast(values, broadcast_to):
    values = values.flatten()
    while len(values.shape) < len(broadcast_to.shape):
        values = values.unsqueeze(-1)
    return values


class DDPMPipeline:
    def __init__(self, beta_start=1e-4, beta_end=1e-2, num_timesteps=1000):
        b = _linspace32(beta_start, beta_end, num_timesteps)
        a = (F32(1.0) - b).astype(F32)
        ah = np.empty_like(a)
        acc = F64(1.0)
        for i, v in enumerate(a):
            acc = acc * F64(v)
            ah[i] = F32(acc)
        self._b, self._a, self._ah = b, a, ah
        self.betas = torch.from_numpy(b.copy())
        self.alphas = torch.from_numpy(a.copy())
        self.alphas_hat = torch.from_numpy(ah.copy())
        self.num_timesteps = num_timesteps

    def step_scalars(self, t):
        """The fp32 scalars of one ``sampling`` step (``ddpm.py:72-86``)."""
        beta_t, alpha_t, ah = self._b[t], self._a[t], self._ah[t]
        ah_prev = self._ah[t - 1]                         # t = 0 wraps to [-1] as in the reference
        beta_hat = F32(F32(F32(F32(1.0) - ah_prev) / F32(F32(1.0) - ah)) * beta_t)
        return {"inv_sqrt_alpha": float(F32(np.power(alpha_t, F32(-0.5), dtype=F32))),
                "coef": float(F32(beta_t / np.sqrt(F32(F32(1.0) - ah_prev), dtype=F32))),
                "sigma": float(np.sqrt(beta_hat, dtype=F32)) if t > 0 else 0.0}

    def forward_diffusion(self, images, timesteps, noise=None):
        images = images.float().contiguous()
        if noise is None:
            noise = torch.randn(images.shape, device=images.device)
        noise = noise.to(images.device, torch.float32).contiguous()
        ts = torch.as_tensor(timesteps).reshape(-1).to("cpu", torch.long)
        if ts.numel() == 1:
            ts = ts.expand(images.shape[0])
        out = torch.empty_like(images)
        for b in range(images.shape[0]):
            ah = self._ah[int(ts[b])]
            ops.stochastic_encode(images[b], noise[b], float(np.sqrt(ah, dtype=F32)),
                                  float(np.sqrt(F32(F32(1.0) - ah), dtype=F32)), out=out[b])
        return out, noise

    def reverse_diffusion(self, model, noisy_images, timesteps):
        return model(noisy_images, timesteps)

    @torch.no_grad()
    def sampling(self, model, initial_noise, device, save_all_steps=False, noise_fn=None):
        image = initial_noise.to(device, torch.float32).contiguous()
        images = []
        for i, timestep in enumerate(range(self.num_timesteps - 1, -1, -1)):
            ts = timestep * torch.ones(image.shape[0], dtype=torch.long, device=device)
            eps = model(image, ts).float().contiguous()
            sc = self.step_scalars(timestep)
            noise = None
            if timestep > 0:
                noise = noise_fn(i, image.shape) if noise_fn is not None else torch.randn(image.shape, device=device)
                noise = noise.to(device, torch.float32).contiguous()
            image = ops.ddpm_step(image, eps, noise, sc["inv_sqrt_alpha"], sc["coef"], sc["sigma"])
            if save_all_steps:
                images.append(image.cpu())
        return images if save_all_steps else image
