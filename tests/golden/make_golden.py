"""Generate the golden fixtures by importing the REFERENCE itself (build container only).

Run from the repo root:  python tests/golden/make_golden.py
Needs /root/reference (read-only).  Everything below the shim block is plain
use of the reference's own modules; the shims are test-only stand-ins for
packages that are absent here:

* ``flash_attn`` (un-vendored, ``req.txt:1``): exact fp32 softmax(scale·QKᵀ)V;
* ``omegaconf.listconfig.ListConfig`` (ctor isinstance only, ``openai_model/model.py:322``);
* ``pytorch_lightning``, ``torchvision``, ``vqvae.autoencoder``, ``Ema.ema``,
  ``Dataset.lsun`` — import-time names only, never called on this path;
* ``Tensor.half``/``Module.half`` → identity so the reference runs in pure fp32
  on the CPU (it cannot run on the CPU as written), and the
  fp16 cast inside ``Unet.unet.nonlinearity`` removed (item 6);
* zero-initialised output layers re-initialised with seeded values (item 7),
  otherwise the UNet output is identically zero;
* ``DDIMSampler.register_buffer`` keeps tensors on the CPU (item 8).

Outputs (inputs AND expected outputs; weights rounded to fp16 so they are
stored exactly in half the bytes) go to tests/golden/*.npz.
"""
from __future__ import annotations

import contextlib
import io
import json
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- shims
def install_shims():
    sys.path.insert(0, REF)
    fa = types.ModuleType("flash_attn")

    def flash_attn_func(q, k, v, dropout_p=0.0, softmax_scale=None, causal=False, **kw):
        assert not causal and dropout_p == 0.0
        d = q.shape[-1]
        s = softmax_scale if softmax_scale is not None else d ** -0.5
        att = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * s
        return torch.einsum("bhqk,bkhd->bqhd", att.softmax(-1), v.float()).to(q.dtype)

    def flash_attn_qkvpacked_func(qkv, dropout_p=0.0, softmax_scale=None, causal=False, **kw):
        q, k, v = qkv.unbind(2)
        return flash_attn_func(q, k, v, dropout_p, softmax_scale, causal)

    fa.flash_attn_func = flash_attn_func
    fa.flash_attn_qkvpacked_func = flash_attn_qkvpacked_func
    sys.modules["flash_attn"] = fa

    om = types.ModuleType("omegaconf")
    oml = types.ModuleType("omegaconf.listconfig")

    class ListConfig(list):
        pass

    oml.ListConfig = ListConfig
    om.listconfig = oml
    sys.modules["omegaconf"] = om
    sys.modules["omegaconf.listconfig"] = oml

    pl = types.ModuleType("pytorch_lightning")
    pl.LightningModule = torch.nn.Module
    plu = types.ModuleType("pytorch_lightning.utilities")
    plr = types.ModuleType("pytorch_lightning.utilities.rank_zero")
    plr.rank_zero_only = lambda f: f
    sys.modules.update({"pytorch_lightning": pl, "pytorch_lightning.utilities": plu,
                        "pytorch_lightning.utilities.rank_zero": plr})
    tv = types.ModuleType("torchvision")
    tvu = types.ModuleType("torchvision.utils")
    tvu.make_grid = lambda *a, **k: None
    tv.utils = tvu
    sys.modules.update({"torchvision": tv, "torchvision.utils": tvu})
    for name, attrs in {"vqvae.autoencoder": {"VQModelInterface": object},
                        "Ema.ema": {"LitEma": object},
                        "Dataset.lsun": {"LSUNBase": object}}.items():
        m = types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m

    torch.Tensor.half = lambda self, *a, **k: self
    torch.nn.Module.half = lambda self: self


@contextlib.contextmanager
def quiet():
    with contextlib.redirect_stdout(io.StringIO()):
        yield


def reinit_(module: torch.nn.Module, seed: int):
    """Deterministic, non-degenerate weights (incl. the zero-initialised output
    layers) regenerated from tests/golden/synth.py — not stored in the fixture."""
    sys.path.insert(0, OUT)
    from synth import synth_weights, keys_shapes_of
    sd = module.state_dict()
    new = synth_weights(keys_shapes_of(sd), seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in new.items()})


def sd_keys(module) -> dict:
    """Key order + shapes (JSON) so the tests can regenerate the same weights."""
    ks = [[k, list(v.shape)] for k, v in module.state_dict().items()]
    return {"keys": np.frombuffer(json.dumps(ks).encode(), dtype=np.uint8)}


# ----------------------------------------------------------------------------- fixtures
def gen_schedule():
    sys.path.insert(0, os.path.join(REF, "DDIM"))
    with quiet():
        import diffusion_modules as dm
        from Diffusion.ddpm import DDPM
        from openai_model.utils import timestep_embedding

    class FakeDDPM:
        v_posterior = 0.0
        parameterization = "eps"

        def register_buffer(self, name, t, persistent=True):
            setattr(self, name, t)

    fake = FakeDDPM()
    DDPM.register_schedule(fake, beta_schedule="linear", timesteps=1000, linear_start=0.00085, linear_end=0.012)
    out = {"betas": fake.betas.numpy(), "alphas_cumprod": fake.alphas_cumprod.numpy(),
           "alphas_cumprod_prev": fake.alphas_cumprod_prev.numpy(),
           "sqrt_one_minus_alphas_cumprod": fake.sqrt_one_minus_alphas_cumprod.numpy()}
    for S in (10, 50, 250):
        for eta in (0.0, 1.0):
            with quiet():
                ts = dm.make_ddim_timesteps("uniform", S, 1000, verbose=False)
                sig, a, ap = dm.make_ddim_sampling_parameters(fake.alphas_cumprod.cpu(), ts, eta, verbose=False)
            tag = f"S{S}_eta{int(eta)}"
            out[f"{tag}_ts"] = np.asarray(ts, dtype=np.int64)
            out[f"{tag}_alphas"] = np.asarray(a, dtype=np.float32)
            out[f"{tag}_alphas_prev"] = np.asarray(ap, dtype=np.float64)
            out[f"{tag}_sigmas"] = np.asarray(sig, dtype=np.float64)
            out[f"{tag}_sqrt_one_minus"] = np.asarray(np.sqrt(1.0 - a), dtype=np.float32)
    # timestep embedding (openai_model/utils.py:225-245) at the SD width
    t = torch.tensor([1, 21, 481, 961, 981, 999], dtype=torch.long)
    out["temb_t"] = t.numpy()
    out["temb_320"] = timestep_embedding(t, 320).numpy()
    out["temb_33"] = timestep_embedding(t, 33).numpy()
    np.savez_compressed(os.path.join(OUT, "schedule.npz"), **out)
    return fake


def make_ddim_sampler(fake_model):
    sys.path.insert(0, os.path.join(REF, "DDIM"))
    with quiet():
        import ddim as ddim_mod
    ddim_mod.DDIMSampler.register_buffer = lambda self, name, attr: setattr(self, name, attr)
    return ddim_mod


def gen_ddim_step(fake):
    """One p_sample_ddim update at several indices, η=0 and η=1 (noise recorded)."""
    ddim_mod = make_ddim_sampler(fake)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 4, 8, 8, generator=g)
    e = torch.randn(2, 4, 8, 8, generator=g)
    nz = torch.randn(2, 4, 8, 8, generator=g)
    out = {"x": x.numpy(), "e": e.numpy(), "noise": nz.numpy()}

    class M:
        num_timesteps = 1000
        alphas_cumprod = fake.alphas_cumprod
        alphas_cumprod_prev = fake.alphas_cumprod_prev
        betas = fake.betas
        device = torch.device("cpu")
        parameterization = "eps"

        def apply_model(self, x, t, c):
            return e

    ddim_mod.noise_like = lambda shape, device, repeat=False: nz
    for eta in (0.0, 1.0):
        s = ddim_mod.DDIMSampler(M())
        with quiet():
            s.make_schedule(50, ddim_eta=eta, verbose=False)
        for index in (0, 1, 25, 49):
            ts = torch.full((2,), int(s.ddim_timesteps[index]), dtype=torch.long)
            with quiet():
                xp, p0 = s.p_sample_ddim(x, None, ts, index=index)
            out[f"eta{int(eta)}_i{index}_xprev"] = xp.numpy()
            out[f"eta{int(eta)}_i{index}_pred_x0"] = p0.numpy()
    np.savez_compressed(os.path.join(OUT, "ddim_step.npz"), **out)


TINY_UNET = dict(image_size=16, in_channels=4, out_channels=4, model_channels=32, attention_resolutions=[1, 2],
                 num_res_blocks=1, channel_mult=[1, 2], num_heads=4, use_spatial_transformer=True,
                 transformer_depth=1, context_dim=48, use_checkpoint=False, legacy=False)
TINY_UNET_UNCOND = dict(image_size=16, in_channels=4, out_channels=4, model_channels=32, attention_resolutions=[2],
                        num_res_blocks=1, channel_mult=[1, 2], num_heads=2, use_spatial_transformer=False,
                        use_checkpoint=False, legacy=False)
TINY_UNET_HC = dict(image_size=16, in_channels=4, out_channels=4, model_channels=32, attention_resolutions=[1, 2],
                    num_res_blocks=1, channel_mult=[1, 2], num_heads=-1, num_head_channels=16,
                    use_spatial_transformer=True, transformer_depth=1, context_dim=40, use_checkpoint=False,
                    legacy=False)


def gen_unet(name, cfg, seed, with_ctx=True, ddim_steps=0):
    with quiet():
        from openai_model.model import UNetModel
        torch.manual_seed(seed)
        m = UNetModel(**cfg)
    reinit_(m, seed)
    m.eval()
    g = torch.Generator().manual_seed(seed + 1)
    B = 2
    x = torch.randn(B, 4, 16, 16, generator=g)
    t = torch.tensor([981, 1], dtype=torch.long)
    ctx = torch.randn(B, 7, cfg["context_dim"], generator=g) if with_ctx else None
    with quiet(), torch.no_grad():
        y = m(x, t, ctx)
    out = dict(sd_keys(m))
    out['seed'] = np.int64(seed)
    out.update(x=x.numpy(), t=t.numpy(), y=y.numpy(), cfg=np.frombuffer(json.dumps(cfg).encode(), dtype=np.uint8))
    if ctx is not None:
        out["ctx"] = ctx.numpy()
    if ddim_steps:
        fake = gen_schedule.__fake__
        ddim_mod = make_ddim_sampler(fake)

        class LD:   # LatentDiffusion.apply_model → DiffusionWrapper('crossattn') (Diffusion/ddpm.py:55-58,1139-1147)
            num_timesteps = 1000
            alphas_cumprod = fake.alphas_cumprod
            alphas_cumprod_prev = fake.alphas_cumprod_prev
            betas = fake.betas
            device = torch.device("cpu")
            parameterization = "eps"

            def apply_model(self, x_noisy, t, cond):
                cc = torch.cat([cond], 1) if cond is not None else None
                return m(x_noisy, t, context=cc)

        xT = torch.randn(B, 4, 16, 16, generator=g)
        ddim_mod.noise_like = lambda shape, device, repeat=False: torch.zeros(shape)   # η = 0: σ·z = 0
        s = ddim_mod.DDIMSampler(LD())
        with quiet(), torch.no_grad():
            samples, inter = s.sample(S=ddim_steps, batch_size=B, shape=(4, 16, 16), conditioning=ctx,
                                      eta=0.0, x_T=xT, verbose=False, log_every_t=1)
        out.update(ddim_xT=xT.numpy(), ddim_samples=samples.numpy(), ddim_steps=np.int64(ddim_steps),
                   ddim_pred_x0_last=inter["pred_x0"][-1].numpy())
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    return m


TINY_VAE = dict(double_z=True, z_channels=4, resolution=32, in_channels=3, out_ch=3, ch=32, ch_mult=[1, 2],
                num_res_blocks=1, attn_resolutions=[], dropout=0.0)


def gen_vae():
    with quiet():
        import Unet.unet as uu
        import Encoder_Decoder.encoder as ee
        silu = lambda x: x * torch.sigmoid(x)        # no fp16 cast
        uu.nonlinearity = silu
        ee.nonlinearity = silu
        from VAE.autoencoder import AutoEncoderKL
        torch.manual_seed(11)
        vae = AutoEncoderKL(ddconfig=dict(TINY_VAE), embed_dim=4, lossconfig={"target": "torch.nn.Identity"})
    reinit_(vae, 11)
    vae.eval()
    g = torch.Generator().manual_seed(12)
    z = torch.randn(2, 4, 8, 8, generator=g)
    scale_factor = 0.18215
    with quiet(), torch.no_grad():
        dec = vae.decode(1.0 / scale_factor * z)            # ldm/diffusion/ddpm.py:1095 scaling
    np.savez_compressed(os.path.join(OUT, "vae_tiny.npz"), **sd_keys(vae), seed=np.int64(11), z=z.numpy(), dec=dec.numpy(),
                        scale_factor=np.float64(scale_factor),
                        cfg=np.frombuffer(json.dumps(TINY_VAE).encode(), dtype=np.uint8))


def gen_ddim_cfg(m, cfg):
    """SURVEY §8(f) rank 1 — classifier-free guidance: the reference DDIMSampler (DDIM/ddim.py:171-178:
    batch doubled as cat([uc, c]), e = e_u + s·(e_c − e_u)) with the tiny UNet, 4 steps, scale 7.5."""
    fake = gen_schedule.__fake__
    ddim_mod = make_ddim_sampler(fake)

    class LD:
        num_timesteps = 1000
        alphas_cumprod = fake.alphas_cumprod
        alphas_cumprod_prev = fake.alphas_cumprod_prev
        betas = fake.betas
        device = torch.device("cpu")
        parameterization = "eps"

        def apply_model(self, x_noisy, t, cond):
            return m(x_noisy, t, context=torch.cat([cond], 1))

    g = torch.Generator().manual_seed(51)
    B = 2
    xT = torch.randn(B, 4, 16, 16, generator=g)
    c = torch.randn(B, 7, cfg["context_dim"], generator=g)
    uc = torch.randn(B, 7, cfg["context_dim"], generator=g) * 0.1
    ddim_mod.noise_like = lambda shape, device, repeat=False: torch.zeros(shape)
    s = ddim_mod.DDIMSampler(LD())
    with quiet(), torch.no_grad():
        samples, _ = s.sample(S=4, batch_size=B, shape=(4, 16, 16), conditioning=c, eta=0.0, x_T=xT,
                              verbose=False, unconditional_guidance_scale=7.5, unconditional_conditioning=uc)
    np.savez_compressed(os.path.join(OUT, "ddim_cfg.npz"), xT=xT.numpy(), c=c.numpy(), uc=uc.numpy(),
                        samples=samples.numpy(), scale=np.float64(7.5), steps=np.int64(4))


def gen_img2img(fake):
    """SURVEY §8(f) rank 2 — img2img: AutoEncoderKL.encode → posterior (moments, a recorded-noise
    sample; VAE/autoencoder.py:114-123, Distribution/distribution.py:31-50), DDIMSampler.stochastic_encode
    at uniform and per-sample DDIM indices (DDIM/ddim.py:207-220) and DDIMSampler.decode from t_start
    with a deterministic stub ε-model (DDIM/ddim.py:222-240)."""
    with quiet():
        import Unet.unet as uu
        import Encoder_Decoder.encoder as ee
        silu = lambda x: x * torch.sigmoid(x)        # no fp16 cast
        uu.nonlinearity = silu
        ee.nonlinearity = silu
        from VAE.autoencoder import AutoEncoderKL
        vae = AutoEncoderKL(ddconfig=dict(TINY_VAE), embed_dim=4, lossconfig={"target": "torch.nn.Identity"})
    reinit_(vae, 13)
    vae.eval()
    g = torch.Generator().manual_seed(14)
    x = torch.rand(2, 3, 32, 32, generator=g) * 2.0 - 1.0
    real_randn = torch.randn
    rec = []

    def rec_randn(*shape, **kw):
        t = real_randn(*shape, generator=g)
        rec.append(t.clone())
        return t

    with quiet(), torch.no_grad():
        post = vae.encode(x)
        torch.randn = rec_randn
        try:
            smp = post.sample()
        finally:
            torch.randn = real_randn
    out = {"x": x.numpy(), "moments": post.parameters.numpy(), "post_noise": rec[0].numpy(),
           "post_sample": smp.numpy(), "post_mode": post.mean.numpy(), "seed": np.int64(13),
           "cfg": np.frombuffer(json.dumps(TINY_VAE).encode(), dtype=np.uint8)}
    out.update(sd_keys(vae))

    ddim_mod = make_ddim_sampler(fake)

    class M:
        num_timesteps = 1000
        alphas_cumprod = fake.alphas_cumprod
        alphas_cumprod_prev = fake.alphas_cumprod_prev
        betas = fake.betas
        device = torch.device("cpu")
        parameterization = "eps"

        def apply_model(self, x, t, c):
            return 0.5 * x + 0.01 * t.float()[:, None, None, None]

    s = ddim_mod.DDIMSampler(M())
    with quiet():
        s.make_schedule(50, ddim_eta=0.0, verbose=False)
    z0 = 0.18215 * smp
    nz = torch.randn(z0.shape, generator=g)
    out["z0"], out["enc_noise"] = z0.numpy(), nz.numpy()
    with quiet(), torch.no_grad():
        out["enc_t30"] = s.stochastic_encode(z0, torch.full((2,), 30, dtype=torch.long), noise=nz).numpy()
        out["enc_t10_40"] = s.stochastic_encode(z0, torch.tensor([10, 40]), noise=nz).numpy()
        out["dec_t5"] = s.decode(torch.from_numpy(out["enc_t30"]), None, 5).numpy()
    np.savez_compressed(os.path.join(OUT, "img2img.npz"), **out)


def gen_tiled_decode():
    """SURVEY §8(f) rank 4 — patch (split_input_params) decode: the reference's own
    get_fold_unfold / get_weighting / meshgrid (Diffusion/ddpm.py, same code as
    ldm/diffusion/ddpm.py:829-997) on a stand-in object, with delta_border's first min taken
    over the last dim (test-only shim: as written, dim=1 fails in torch.cat for w > 1 — DESIGN.md
    Q14), the tiny reference VAE decoding each patch, composed as ldm/diffusion/ddpm.py:1097-1139."""
    with quiet():
        import Unet.unet as uu
        import Encoder_Decoder.encoder as ee
        silu = lambda x: x * torch.sigmoid(x)
        uu.nonlinearity = silu
        ee.nonlinearity = silu
        from VAE.autoencoder import AutoEncoderKL
        from Diffusion.ddpm import LatentDiffusion as RefLD
        vae = AutoEncoderKL(ddconfig=dict(TINY_VAE), embed_dim=4, lossconfig={"target": "torch.nn.Identity"})
    reinit_(vae, 15)
    vae.eval()
    sp = {"patch_distributed_vq": True, "ks": (8, 8), "stride": (4, 4), "vqf": 2, "clip_min_weight": 0.01,
          "clip_max_weight": 0.5, "tie_braker": True, "clip_min_tie_weight": 0.01, "clip_max_tie_weight": 0.5}

    def delta_border(self, h, w):
        lower_right_corner = torch.tensor([h - 1, w - 1]).view(1, 1, 2)
        arr = self.meshgrid(h, w) / lower_right_corner
        dist_left_up = torch.min(arr, dim=-1, keepdim=True)[0]
        dist_right_down = torch.min(1 - arr, dim=-1, keepdim=True)[0]
        return torch.min(torch.cat([dist_left_up, dist_right_down], dim=-1), dim=-1)[0]

    class Stand:
        split_input_params = sp
        meshgrid = RefLD.meshgrid
        get_weighting = RefLD.get_weighting
        get_fold_unfold = RefLD.get_fold_unfold

    Stand.delta_border = delta_border
    st = Stand()
    g = torch.Generator().manual_seed(16)
    zl = torch.randn(2, 4, 16, 16, generator=g)
    scale_factor = 0.18215
    z = 1.0 / scale_factor * zl
    ks, stride, uf = sp["ks"], sp["stride"], sp["vqf"]
    with quiet(), torch.no_grad():
        fold, unfold, normalization, weighting = st.get_fold_unfold(z, ks, stride, uf=uf)
        zp = unfold(z)
        zp = zp.view((zp.shape[0], -1, ks[0], ks[1], zp.shape[-1]))
        o = torch.stack([vae.decode(zp[:, :, :, :, i]) for i in range(zp.shape[-1])], axis=-1)
        o = o * weighting
        o = o.view((o.shape[0], -1, o.shape[-1]))
        dec = fold(o) / normalization
    np.savez_compressed(os.path.join(OUT, "vae_tiled.npz"), **sd_keys(vae), seed=np.int64(15), z=zl.numpy(),
                        dec=dec.numpy(), scale_factor=np.float64(scale_factor),
                        sp=np.frombuffer(json.dumps(sp).encode(), dtype=np.uint8),
                        cfg=np.frombuffer(json.dumps(TINY_VAE).encode(), dtype=np.uint8))


def gen_ddpm():
    """C1 pipeline: DDPMPipeline tables + a 10-step sampling run with a recorded-ε
    stub model and recorded noise (DDPM/ddpm.py:17-89)."""
    sys.path.insert(0, os.path.join(REF, "DDPM"))
    import importlib
    dd = importlib.import_module("ddpm")
    pipe = dd.DDPMPipeline(beta_start=1e-4, beta_end=1e-2, num_timesteps=10)
    g = torch.Generator().manual_seed(21)
    x0 = torch.randn(4, 3, 8, 8, generator=g)
    noises = []
    real_randn = torch.randn

    def rec_randn(*shape, **kw):
        t = real_randn(*shape, generator=g)
        noises.append(t.clone())
        return t

    def stub(img, ts):   # deterministic ε(x, t)
        return 0.5 * img + 0.01 * ts.float()[:, None, None, None]

    torch.randn = rec_randn
    try:
        with quiet():
            img = pipe.sampling(stub, x0, "cpu")
    finally:
        torch.randn = real_randn
    np.savez_compressed(os.path.join(OUT, "ddpm_c1.npz"), betas=pipe.betas.numpy(), alphas=pipe.alphas.numpy(),
                        alphas_hat=pipe.alphas_hat.numpy(), x0=x0.numpy(), out=img.numpy(),
                        noises=torch.stack(noises).numpy())


def gen_ddpm_unet():
    """C1: the reference's 58.66 M DDPM UNet (DDPM/models/unet.py) with synthetic
    weights — one forward at two timesteps, and a 4-step DDPMPipeline.sampling run with it (noise
    recorded; DDPM/ddpm.py:53-89)."""
    import importlib
    sys.path.insert(0, os.path.join(REF, "DDPM"))
    for k in [k for k in sys.modules if k == "models" or k.startswith("models.")]:
        del sys.modules[k]
    unet_mod = importlib.import_module("models.unet")
    dd = importlib.import_module("ddpm")
    torch.manual_seed(0)
    m = unet_mod.UNet(input_channels=3).eval()
    reinit_(m, 41)
    g = torch.Generator().manual_seed(42)
    x = torch.randn(2, 3, 32, 32, generator=g)
    t = torch.tensor([5, 900])
    with torch.no_grad():
        y = m(x, t)
    pipe = dd.DDPMPipeline(beta_start=1e-4, beta_end=1e-2, num_timesteps=4)
    x0 = torch.randn(2, 3, 32, 32, generator=g)
    noises = []
    real_randn = torch.randn

    def rec_randn(*shape, **kw):
        z = real_randn(*shape, generator=g)
        noises.append(z.clone())
        return z

    torch.randn = rec_randn
    try:
        with quiet(), torch.no_grad():
            img = pipe.sampling(m, x0, "cpu")
    finally:
        torch.randn = real_randn
    np.savez_compressed(os.path.join(OUT, "ddpm_unet.npz"), **sd_keys(m), seed=np.int64(41), x=x.numpy(),
                        t=t.numpy(), y=y.numpy(), x0=x0.numpy(), out=img.numpy(), noises=torch.stack(noises).numpy())


def main():
    install_shims()
    torch.set_num_threads(8)
    fake = gen_schedule()
    gen_schedule.__fake__ = fake
    gen_ddim_step(fake)
    m_tiny = gen_unet("unet_tiny", TINY_UNET, 3, with_ctx=True, ddim_steps=4)
    gen_ddim_cfg(m_tiny, TINY_UNET)
    gen_unet("unet_tiny_uncond", TINY_UNET_UNCOND, 5, with_ctx=False)
    gen_unet("unet_tiny_headch", TINY_UNET_HC, 9, with_ctx=True)
    gen_vae()
    gen_img2img(fake)
    gen_tiled_decode()
    gen_ddpm()
    gen_ddpm_unet()
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))


if __name__ == "__main__":
    main()
