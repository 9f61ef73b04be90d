"""Mirror of ``Diffusion/utils.py`` config helpers (``instantiate_from_config``, ``Diffusion/utils.py:223-253``).

Drop-in resolution: a ``target:`` naming one of the reference's module paths
(``openai_model.model.UNetModel``, ``VAE.autoencoder.AutoEncoderKL``,
``Diffusion.ddpm.LatentDiffusion`` …) resolves to the HIP-backed mirror inside
this package first, so the reference's ``Diffusion/config.yaml`` instantiates
unchanged.  Targets with no mirror (e.g. ``torch.nn.Identity``) import as given.
"""
from __future__ import annotations

import importlib

_PKG = __name__.rsplit(".", 2)[0]      # "sd_amd"
MIRRORED = ("openai_model", "Unet", "Encoder_Decoder", "VAE", "DDIM", "Diffusion", "DDPM", "clip_encoder",
            "Distribution")


def get_obj_from_str(string, reload=False):
    module, cls = string.rsplit(".", 1)
    if module.split(".")[0] in MIRRORED:
        module = f"{_PKG}.{module}"
    mod = importlib.import_module(module)
    if reload:
        mod = importlib.reload(mod)
    return getattr(mod, cls)


def instantiate_from_config(config):
    if "target" not in config:
        if config in ("__is_first_stage__", "__is_unconditional__"):
            return None
        raise KeyError("Expected key `target` to instantiate.")
    return get_obj_from_str(config["target"])(**config.get("params", dict()))


def exists(x):
    return x is not None


def default(val, d):
    if exists(val):
        return val
    return d() if callable(d) else d


def count_params(model, verbose=False):
    total = sum(p.numel() for p in model.parameters())
    if verbose:
        print(f"{model.__class__.__name__} has {total * 1.e-6:.2f} M params.")
    return total
