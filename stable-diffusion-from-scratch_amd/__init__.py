"""sd_amd — MI355X (gfx950) native latent-diffusion hot path.

Host-side mirror of the reference's module API (``openai_model``, ``Unet``,
``Encoder_Decoder``, ``VAE``, ``DDIM``, ``Diffusion``, ``DDPM``) whose compute
runs in hand-written HIP kernels (libsdk_amd.so, C ABI in include/sdk_amd.h).
"""
from . import _lib  # noqa: F401

__version__ = "0.1.0"


def library():
    """Load (and validate the exports of) libsdk_amd.so; raises if it is missing."""
    return _lib.lib()
