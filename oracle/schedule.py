"""Diffusion schedule bookkeeping and sampler update rules — CPU oracle (test-only).

Restates, in numpy, the dtype chain the reference uses so that the timestep,
alpha and sigma tables can be compared BIT-EXACTLY:

* ``linspace64``            torch.linspace (float64) as used by
  ``make_beta_schedule`` — ``DDIM/diffusion_modules.py:21-25`` (≡
  ``ldm/modules/diffusionmodules/util.py:21-25``).  torch's CPU kernel fills the
  first half as ``start + step*i`` and the second half as
  ``end - step*(n-1-i)``; numpy's linspace does not, so it is restated here.
* ``register_schedule``     ``Diffusion/ddpm.py:195-253`` (fp64 cumprod, fp32
  buffers via ``torch.tensor(dtype=float32)``).
* ``make_ddim_timesteps``   ``DDIM/diffusion_modules.py:46-60``.
* ``make_ddim_sampling_parameters`` ``DDIM/diffusion_modules.py:63-74`` plus the
  conversions of ``DDIM/ddim.py:25-54``: ``ddim_alphas`` fp32,
  ``ddim_alphas_prev`` fp64 holding fp32 values, ``ddim_sigmas`` fp64 with the
  ``1/(1 - alphas)`` factor formed in fp32 (``ndarray / Tensor`` becomes
  ``Tensor.reciprocal() * ndarray``), ``ddim_sqrt_one_minus_alphas`` fp32.
* ``ddim_step``             ``DDIM/ddim.py:184-204`` (``p_sample_ddim``) in fp32,
  op by op, as torch's CPU kernels evaluate it (no fused multiply-add).
* ``ddpm_tables``/``ddpm_step`` ``DDPM/ddpm.py:17-89`` (C1 pixel-space DDPM),
  including the ``alphas_hat[t-1]`` wrap at t = 0.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


def linspace64(start: float, end: float, n: int) -> np.ndarray:
    """torch.linspace(start, end, n, dtype=float64) restated (CPU kernel)."""
    if n == 1:
        return np.array([start], dtype=F64)
    step = (F64(end) - F64(start)) / F64(n - 1)
    idx = np.arange(n, dtype=F64)
    half = n // 2
    out = np.empty(n, dtype=F64)
    out[:half] = F64(start) + step * idx[:half]
    out[half:] = F64(end) - step * (F64(n - 1) - idx[half:])
    return out


def linspace32(start: float, end: float, n: int) -> np.ndarray:
    """torch.linspace(start, end, n) in the default fp32 (``DDPM/ddpm.py:21``)."""
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


def make_beta_schedule(schedule: str, n_timestep: int, linear_start=1e-4, linear_end=2e-2) -> np.ndarray:
    """``DDIM/diffusion_modules.py:21-43`` — only the schedules SD uses."""
    if schedule == "linear":
        return linspace64(linear_start ** 0.5, linear_end ** 0.5, n_timestep) ** 2
    if schedule == "sqrt_linear":
        return linspace64(linear_start, linear_end, n_timestep)
    if schedule == "sqrt":
        return linspace64(linear_start, linear_end, n_timestep) ** 0.5
    raise ValueError(f"schedule '{schedule}' not restated")


def register_schedule(timesteps=1000, linear_start=0.00085, linear_end=0.012, beta_schedule="linear") -> dict:
    """``Diffusion/ddpm.py:195-253``: fp64 math, fp32 buffers."""
    betas = make_beta_schedule(beta_schedule, timesteps, linear_start, linear_end)
    alphas = 1.0 - betas
    ac = np.cumprod(alphas, axis=0)
    ac_prev = np.append(1.0, ac[:-1])
    return {
        "betas64": betas,
        "alphas_cumprod64": ac,
        "betas": betas.astype(F32),
        "alphas_cumprod": ac.astype(F32),
        "alphas_cumprod_prev": ac_prev.astype(F32),
        "sqrt_alphas_cumprod": np.sqrt(ac).astype(F32),
        "sqrt_one_minus_alphas_cumprod": np.sqrt(1.0 - ac).astype(F32),
        "num_timesteps": int(betas.shape[0]),
    }


def make_ddim_timesteps(method: str, num_ddim_timesteps: int, num_ddpm_timesteps: int) -> np.ndarray:
    """``DDIM/diffusion_modules.py:46-60`` (int64 result, +1 shift)."""
    if method == "uniform":
        c = num_ddpm_timesteps // num_ddim_timesteps
        ts = np.asarray(list(range(0, num_ddpm_timesteps, c)))
    elif method == "quad":
        ts = ((np.linspace(0, np.sqrt(num_ddpm_timesteps * 0.8), num_ddim_timesteps)) ** 2).astype(int)
    else:
        raise NotImplementedError(method)
    return (ts + 1).astype(np.int64)


def make_ddim_sampling_parameters(alphacums32: np.ndarray, ddim_timesteps: np.ndarray, eta: float) -> dict:
    """``DDIM/diffusion_modules.py:63-74`` with the dtypes ``DDIM/ddim.py:44-50`` ends up holding."""
    a = alphacums32[ddim_timesteps].astype(F32)
    a_prev = np.asarray([alphacums32[0]] + alphacums32[ddim_timesteps[:-1]].tolist(), dtype=F64)
    one_minus_a = (F32(1.0) - a).astype(F32)            # fp32 tensor op
    # ndarray / Tensor dispatches to Tensor.__rtruediv__ = reciprocal() * other:
    # the reciprocal is taken in fp32, the product in fp64.
    recip = (F32(1.0) / one_minus_a).astype(F32)
    ratio = recip.astype(F64) * (1.0 - a_prev)
    inner = 1.0 - a.astype(F64) / a_prev
    sig = F64(eta) * np.sqrt(ratio * inner)
    return {
        "ddim_timesteps": ddim_timesteps,
        "ddim_alphas": a,
        "ddim_alphas_prev": a_prev,
        "ddim_sigmas": sig.astype(F64),
        "ddim_sqrt_one_minus_alphas": np.sqrt(one_minus_a).astype(F32),
    }


def ddim_tables(S: int, eta: float = 0.0, method="uniform", **sched_kw) -> dict:
    """``DDIMSampler.make_schedule`` (``DDIM/ddim.py:25-54``)."""
    sch = register_schedule(**sched_kw)
    ts = make_ddim_timesteps(method, S, sch["num_timesteps"])
    out = make_ddim_sampling_parameters(sch["alphas_cumprod"], ts, eta)
    out["schedule"] = sch
    return out


def ddim_step_scalars(tab: dict, index: int) -> dict:
    """The four ``torch.full((b,1,1,1), table[index])`` fp32 scalars (``DDIM/ddim.py:189-192``)
    and the fp32 derived coefficients torch forms from them (``:195-203``)."""
    a_t = F32(tab["ddim_alphas"][index])
    a_prev = F32(tab["ddim_alphas_prev"][index])
    sigma = F32(tab["ddim_sigmas"][index])
    s1m = F32(tab["ddim_sqrt_one_minus_alphas"][index])
    sqrt_at = np.sqrt(a_t, dtype=F32)
    dir_coef = np.sqrt(F32(F32(F32(1.0) - a_prev) - F32(sigma * sigma)), dtype=F32)
    sqrt_aprev = np.sqrt(a_prev, dtype=F32)
    return dict(a_t=a_t, a_prev=a_prev, sigma=sigma, sqrt_one_minus_at=s1m, sqrt_at=sqrt_at,
                dir_coef=dir_coef, sqrt_a_prev=sqrt_aprev)


def ddim_step(x: np.ndarray, e_t: np.ndarray, sc: dict, noise: np.ndarray | None = None,
              temperature: float = 1.0):
    """``p_sample_ddim`` update (``DDIM/ddim.py:194-204``), fp32 op by op."""
    x = x.astype(F32)
    e_t = e_t.astype(F32)
    pred_x0 = (x - sc["sqrt_one_minus_at"] * e_t) / sc["sqrt_at"]
    dir_xt = sc["dir_coef"] * e_t
    if noise is None:
        noise = np.zeros_like(x)
    nz = (sc["sigma"] * noise.astype(F32)) * F32(temperature)
    x_prev = (sc["sqrt_a_prev"] * pred_x0 + dir_xt) + nz
    return x_prev.astype(F32), pred_x0.astype(F32)


def v_to_eps(x: np.ndarray, v: np.ndarray, a_t: np.float32) -> np.ndarray:
    """v-prediction → ε (extension for config C5; the reference has no v-pred,
    SURVEY Q9 — parity unpinned): ε = √ᾱ·v + √(1-ᾱ)·x."""
    sa = np.sqrt(F32(a_t), dtype=F32)
    s1m = np.sqrt(F32(F32(1.0) - F32(a_t)), dtype=F32)
    return (sa * v.astype(F32) + s1m * x.astype(F32)).astype(F32)


# ---------------------------------------------------------------- C1 DDPM (pixel space)

def ddpm_tables(beta_start=1e-4, beta_end=1e-2, num_timesteps=1000) -> dict:
    """``DDPMPipeline.__init__`` (``DDPM/ddpm.py:17-28``): fp32 linspace + fp32 cumprod."""
    betas = linspace32(beta_start, beta_end, num_timesteps)
    alphas = (F32(1.0) - betas).astype(F32)
    ah = np.empty_like(alphas)
    acc = F64(1.0)
    for i, a in enumerate(alphas):       # torch's CPU cumprod accumulates in double (acc_type)
        acc = acc * F64(a)
        ah[i] = F32(acc)
    return {"betas": betas, "alphas": alphas, "alphas_hat": ah, "num_timesteps": num_timesteps}


def ddpm_step_scalars(tab: dict, timestep: int) -> dict:
    """Per-step fp32 scalars of ``DDPMPipeline.sampling`` (``DDPM/ddpm.py:72-86``)."""
    beta_t = tab["betas"][timestep]
    alpha_t = tab["alphas"][timestep]
    ah = tab["alphas_hat"][timestep]
    ah_prev = tab["alphas_hat"][timestep - 1]      # wraps to [-1] at t=0 (Q12)
    beta_hat = F32(F32(F32(F32(1.0) - ah_prev) / F32(F32(1.0) - ah)) * beta_t)
    return dict(inv_sqrt_alpha=F32(np.power(alpha_t, F32(-0.5), dtype=F32)),
                coef=F32(beta_t / np.sqrt(F32(F32(1.0) - ah_prev), dtype=F32)),
                sigma=np.sqrt(beta_hat, dtype=F32) if timestep > 0 else F32(0.0))


def ddpm_step(image: np.ndarray, eps: np.ndarray, sc: dict, noise: np.ndarray | None) -> np.ndarray:
    """``image = α_t^-½ (image − β_t/√(1−ᾱ_{t−1}) ε) + √β̃_t·z`` (``DDPM/ddpm.py:84-86``)."""
    out = sc["inv_sqrt_alpha"] * (image.astype(F32) - sc["coef"] * eps.astype(F32))
    if noise is not None and sc["sigma"] != 0:
        out = out + sc["sigma"] * noise.astype(F32)
    return out.astype(F32)


def stochastic_encode(x0: np.ndarray, noise: np.ndarray, tab: dict, index: int) -> np.ndarray:
    """DDIMSampler.stochastic_encode at DDIM index t (``ldm/diffusion/ddim.py:209-222``):
    sqrt(ddim_alphas)[t] * x0 + ddim_sqrt_one_minus_alphas[t] * noise, fp32, op by op."""
    f32 = np.float32
    sa = np.sqrt(f32(tab["ddim_alphas"][index]), dtype=f32)
    s1m = f32(tab["ddim_sqrt_one_minus_alphas"][index])
    return (sa * x0.astype(f32)).astype(f32) + (s1m * noise.astype(f32)).astype(f32)


def ddim_decode(x_latent: np.ndarray, eps_fn, tab: dict, t_start: int) -> np.ndarray:
    """DDIMSampler.decode (``ldm/diffusion/ddim.py:224-241``): the first ``t_start`` DDIM
    timesteps walked in reverse, index = t_start - i - 1, one p_sample_ddim update each."""
    ts = tab["ddim_timesteps"][:t_start]
    x = x_latent.astype(F32)
    for i, step in enumerate(np.flip(ts)):
        index = t_start - i - 1
        e = eps_fn(x, np.full((x.shape[0],), int(step), dtype=np.int64))
        x, _ = ddim_step(x, e, ddim_step_scalars(tab, index))
    return x
