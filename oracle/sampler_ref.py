"""DDIM sampling loop — CPU oracle (TEST INFRASTRUCTURE ONLY).

``DDIMSampler.sample``/``ddim_sampling``/``p_sample_ddim``
(``DDIM/ddim.py:57-204`` ≡ ``ldm/diffusion/ddim.py:57-206``): iterate
``np.flip(ddim_timesteps)`` with ``index = S - i - 1``, call the model with
``ts = full((B,), step)``, apply the fp32 update.  Classifier-free guidance as in
``DDIM/ddim.py:171-178``.
"""
from __future__ import annotations

import numpy as np
import torch

from . import schedule as sch


@torch.no_grad()
def ddim_sample(model_fn, x_T: torch.Tensor, S: int, eta: float = 0.0, noise_fn=None,
                guidance_scale: float = 1.0, uncond_fn=None, parameterization: str = "eps", **sched_kw):
    tab = sch.ddim_tables(S, eta, **sched_kw)
    ts_all = tab["ddim_timesteps"]
    img = x_T.float().clone()
    b = img.shape[0]
    pred_x0 = img
    for i, step in enumerate(np.flip(ts_all)):
        index = S - i - 1
        ts = torch.full((b,), int(step), dtype=torch.long)
        e_t = model_fn(img, ts).float()
        if uncond_fn is not None and guidance_scale != 1.0:
            e_u = uncond_fn(img, ts).float()
            e_t = e_u + guidance_scale * (e_t - e_u)
        sc = sch.ddim_step_scalars(tab, index)
        if parameterization == "v":
            e_np = sch.v_to_eps(img.numpy(), e_t.numpy(), sc["a_t"])
        else:
            e_np = e_t.numpy()
        noise = noise_fn(i, img.shape).numpy() if (noise_fn is not None and eta > 0) else None
        xp, p0 = sch.ddim_step(img.numpy(), e_np, sc, noise)
        img, pred_x0 = torch.from_numpy(xp), torch.from_numpy(p0)
    return img, pred_x0
