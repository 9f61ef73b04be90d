"""Host-side schedule bookkeeping — mirror of ``DDIM/diffusion_modules.py`` (≡
``ldm/modules/diffusionmodules/util.py``) and ``DDPM.register_schedule``
(``Diffusion/ddpm.py:195-253``).

These are one-time host constants (the reference computes them on the host
too).  They are evaluated with the same torch/numpy dtype chain as the reference
so the tables are bit-identical (tests/test_sampler_tables.py checks them
against the golden vectors): fp64 betas/cumprod, fp32 buffers, ``ddim_alphas``
fp32, ``ddim_alphas_prev`` fp64 holding fp32 values, ``ddim_sigmas`` fp64 whose
``1/(1-alphas)`` factor is an fp32 reciprocal.
"""
from __future__ import annotations

import numpy as np
import torch


def make_beta_schedule(schedule, n_timestep, linear_start=1e-4, linear_end=2e-2, cosine_s=8e-3):
    with torch.device("cpu"):        # host constants, also inside a torch.device("meta") build
        return _beta_schedule(schedule, n_timestep, linear_start, linear_end, cosine_s)


def _beta_schedule(schedule, n_timestep, linear_start, linear_end, cosine_s):
    if schedule == "linear":
        betas = torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n_timestep, dtype=torch.float64) ** 2
    elif schedule == "sqrt_linear":
        betas = torch.linspace(linear_start, linear_end, n_timestep, dtype=torch.float64)
    elif schedule == "sqrt":
        betas = torch.linspace(linear_start, linear_end, n_timestep, dtype=torch.float64) ** 0.5
    elif schedule == "cosine":
        ts = torch.arange(n_timestep + 1, dtype=torch.float64) / n_timestep + cosine_s
        al = torch.cos(ts / (1 + cosine_s) * np.pi / 2).pow(2)
        al = al / al[0]
        betas = torch.clamp(1 - al[1:] / al[:-1], 0, 0.999)
    else:
        raise ValueError(f"schedule '{schedule}' unknown.")
    return betas.numpy()


def register_schedule(timesteps=1000, linear_start=1e-4, linear_end=2e-2, beta_schedule="linear",
                      given_betas=None, cosine_s=8e-3):
    """fp32 buffers of ``DDPM.register_schedule`` (fp64 math)."""
    betas = np.asarray(given_betas, dtype=np.float64) if given_betas is not None else \
        make_beta_schedule(beta_schedule, timesteps, linear_start, linear_end, cosine_s)
    alphas_cumprod = np.cumprod(1.0 - betas, axis=0)
    alphas_cumprod_prev = np.append(1.0, alphas_cumprod[:-1])
    # host constants: always CPU tensors, also when a model is built under torch.device("meta")
    f = lambda a: torch.tensor(a, dtype=torch.float32, device="cpu")
    return {"betas": f(betas), "alphas_cumprod": f(alphas_cumprod), "alphas_cumprod_prev": f(alphas_cumprod_prev),
            "sqrt_alphas_cumprod": f(np.sqrt(alphas_cumprod)),
            "sqrt_one_minus_alphas_cumprod": f(np.sqrt(1.0 - alphas_cumprod)),
            "num_timesteps": int(betas.shape[0])}


def make_ddim_timesteps(ddim_discr_method, num_ddim_timesteps, num_ddpm_timesteps, verbose=True):
    if ddim_discr_method == "uniform":
        stride = num_ddpm_timesteps // num_ddim_timesteps
        base = np.arange(0, num_ddpm_timesteps, stride)
    elif ddim_discr_method == "quad":
        base = ((np.linspace(0, np.sqrt(num_ddpm_timesteps * .8), num_ddim_timesteps)) ** 2).astype(int)
    else:
        raise NotImplementedError(f'There is no ddim discretization method called "{ddim_discr_method}"')
    steps = (base + 1).astype(np.int64)
    if steps[-1] >= num_ddpm_timesteps:
        raise IndexError(f"DDIM timestep {steps[-1]} out of range for {num_ddpm_timesteps} DDPM steps "
                         f"(the reference fails the same way for S={num_ddim_timesteps})")
    if verbose:
        print(f"Selected timesteps for ddim sampler: {steps}")
    return steps


def make_ddim_sampling_parameters(alphacums, ddim_timesteps, eta, verbose=True):
    """Returns (sigmas fp64 tensor, alphas fp32 tensor, alphas_prev fp64 ndarray).

    Evaluated with numpy IEEE fp32/fp64 arithmetic (torch's vectorised CPU kernels
    were seen to differ by 1 ulp across host CPUs)."""
    ac = (alphacums.detach().cpu().numpy() if torch.is_tensor(alphacums) else np.asarray(alphacums))
    ac = ac.astype(np.float32)
    idx = np.asarray(ddim_timesteps, dtype=np.int64)
    alphas = ac[idx]
    alphas_prev = np.asarray([ac[0]] + ac[idx[:-1]].tolist(), dtype=np.float64)
    recip = (np.float32(1.0) / (np.float32(1.0) - alphas)).astype(np.float32)   # Tensor.__rtruediv__: fp32
    ratio = recip.astype(np.float64) * (1.0 - alphas_prev)
    inner = 1.0 - alphas.astype(np.float64) / alphas_prev
    sigmas = np.float64(eta) * np.sqrt(ratio * inner)
    if verbose:
        print(f"Selected alphas for ddim sampler: a_t: {alphas}; a_(t-1): {alphas_prev}")
    return torch.from_numpy(sigmas), torch.from_numpy(alphas), alphas_prev


def sqrt_one_minus(alphas):
    a = alphas.numpy() if torch.is_tensor(alphas) else np.asarray(alphas)
    return torch.from_numpy(np.sqrt(np.float32(1.0) - a.astype(np.float32)).astype(np.float32))


def noise_like(shape, device, repeat=False):
    if repeat:
        return torch.randn((1, *shape[1:]), device=device).repeat(shape[0], *((1,) * (len(shape) - 1)))
    return torch.randn(shape, device=device)
