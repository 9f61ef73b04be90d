"""The CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  Schedule/timestep tables must match bit-exactly."""
import numpy as np
import pytest
import torch

from golden_util import load, cfg_of, weights_of
from oracle import schedule as sch
from oracle import unet_ref, vae_ref


def test_register_schedule_bitexact():
    z = load("schedule")
    s = sch.register_schedule()
    for k in ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_one_minus_alphas_cumprod"):
        assert s[k].dtype == z[k].dtype
        assert np.array_equal(s[k].view(np.uint32), z[k].view(np.uint32)), k


@pytest.mark.parametrize("S", [10, 50, 250])
@pytest.mark.parametrize("eta", [0, 1])
def test_ddim_tables_bitexact(S, eta):
    z = load("schedule")
    t = sch.ddim_tables(S, float(eta))
    tag = f"S{S}_eta{eta}"
    assert np.array_equal(t["ddim_timesteps"], z[tag + "_ts"])
    assert t["ddim_timesteps"].dtype == np.int64
    for mine, ref in (("ddim_alphas", "_alphas"), ("ddim_alphas_prev", "_alphas_prev"),
                      ("ddim_sigmas", "_sigmas"), ("ddim_sqrt_one_minus_alphas", "_sqrt_one_minus")):
        a, b = t[mine], z[tag + ref]
        assert a.dtype == b.dtype, mine
        assert np.array_equal(a, b), (mine, np.max(np.abs(a - b)))


def test_ddim_uniform_50_timesteps():
    ts = sch.make_ddim_timesteps("uniform", 50, 1000)
    assert ts[0] == 1 and ts[-1] == 981 and len(ts) == 50 and np.all(np.diff(ts) == 20)


@pytest.mark.parametrize("eta", [0, 1])
@pytest.mark.parametrize("index", [0, 1, 25, 49])
def test_ddim_step_bitexact(eta, index):
    z = load("ddim_step")
    tab = sch.ddim_tables(50, float(eta))
    sc = sch.ddim_step_scalars(tab, index)
    xp, p0 = sch.ddim_step(z["x"], z["e"], sc, noise=z["noise"] if eta else None)
    ref_xp, ref_p0 = z[f"eta{eta}_i{index}_xprev"], z[f"eta{eta}_i{index}_pred_x0"]
    assert np.array_equal(p0, ref_p0)
    assert np.array_equal(xp, ref_xp), np.max(np.abs(xp - ref_xp))


def test_timestep_embedding():
    z = load("schedule")
    t = torch.from_numpy(z["temb_t"])
    assert np.array_equal(unet_ref.timestep_embedding(t, 320).numpy(), z["temb_320"])
    assert np.array_equal(unet_ref.timestep_embedding(t, 33).numpy(), z["temb_33"])


@pytest.mark.parametrize("name", ["unet_tiny", "unet_tiny_uncond", "unet_tiny_headch"])
def test_unet_forward(name):
    z = load(name)
    cfg = cfg_of(z)
    sd = weights_of(z)
    ctx = torch.from_numpy(z["ctx"]) if "ctx" in z.files else None
    y = unet_ref.unet_forward(sd, cfg, torch.from_numpy(z["x"]), torch.from_numpy(z["t"]), ctx)
    ref = torch.from_numpy(z["y"])
    err = (y - ref).abs().max().item()
    assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err


def test_ddim_sampling_run():
    """Full 4-step DDIM loop (ldm/diffusion/ddim.py ≡ DDIM/ddim.py) with the tiny UNet."""
    from oracle.sampler_ref import ddim_sample
    z = load("unet_tiny")
    cfg, sd = cfg_of(z), weights_of(z)
    ctx = torch.from_numpy(z["ctx"])
    fn = lambda x, t: unet_ref.unet_forward(sd, cfg, x, t, ctx)
    out, pred_x0 = ddim_sample(fn, torch.from_numpy(z["ddim_xT"]), int(z["ddim_steps"]), eta=0.0)
    ref = z["ddim_samples"]
    assert np.max(np.abs(out.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


def test_vae_decode():
    z = load("vae_tiny")
    cfg = cfg_of(z)
    sd = weights_of(z)
    dec = vae_ref.decode_first_stage(sd, cfg, torch.from_numpy(z["z"]), float(z["scale_factor"]))
    ref = z["dec"]
    assert np.max(np.abs(dec.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


def test_ddpm_c1_pipeline():
    z = load("ddpm_c1")
    tab = sch.ddpm_tables(1e-4, 1e-2, 10)
    for k in ("betas", "alphas", "alphas_hat"):
        assert np.array_equal(tab[k], z[k]), k
    img = z["x0"]
    noises = list(z["noises"])
    for t in range(9, -1, -1):
        ts = np.full((img.shape[0],), t, dtype=np.float32)
        eps = (np.float32(0.5) * img + np.float32(0.01) * ts[:, None, None, None]).astype(np.float32)
        sc = sch.ddpm_step_scalars(tab, t)
        img = sch.ddpm_step(img, eps, sc, noises.pop(0) if t > 0 else None)
    assert np.max(np.abs(img - z["out"])) <= 1e-5 * max(1.0, np.abs(z["out"]).max())


# ---------------------------------------------------------------- img2img
def test_vae_encode_moments():
    z = load("img2img")
    cfg, sd = cfg_of(z), weights_of(z)
    m = vae_ref.autoencoder_moments(sd, cfg, torch.from_numpy(z["x"]))
    ref = z["moments"]
    assert m.shape == ref.shape
    assert np.max(np.abs(m.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


def test_posterior_sample_and_mode():
    z = load("img2img")
    m = torch.from_numpy(z["moments"])
    s = vae_ref.posterior_sample(m, torch.from_numpy(z["post_noise"]))
    np.testing.assert_allclose(s.numpy(), z["post_sample"], rtol=1e-6, atol=1e-6)
    assert np.array_equal(vae_ref.posterior_sample(m).numpy(), z["post_mode"])


def test_stochastic_encode_bitexact():
    z = load("img2img")
    tab = sch.ddim_tables(50, 0.0)
    got = sch.stochastic_encode(z["z0"], z["enc_noise"], tab, 30)
    assert np.array_equal(got, z["enc_t30"])
    per = np.stack([sch.stochastic_encode(z["z0"][i], z["enc_noise"][i], tab, t) for i, t in enumerate((10, 40))])
    assert np.array_equal(per, z["enc_t10_40"])


def test_ddim_decode_from_t_start_bitexact():
    z = load("img2img")
    tab = sch.ddim_tables(50, 0.0)
    stub = lambda x, t: (np.float32(0.5) * x + np.float32(0.01) * t.astype(np.float32)[:, None, None, None]
                         ).astype(np.float32)
    out = sch.ddim_decode(z["enc_t30"], stub, tab, 5)
    assert np.array_equal(out, z["dec_t5"]), np.max(np.abs(out - z["dec_t5"]))


# ---------------------------------------------------------------- CLIP text encoder
def test_clip_text_vs_transformers():
    import json
    from oracle.clip_ref import clip_text_forward
    z = load("clip_tiny")
    cfg = json.loads(bytes(z["cfg"]).decode())
    sd = {("text_model." + k if not k.startswith("text_model.") else k): v for k, v in weights_of(z).items()}
    y = clip_text_forward(sd, torch.from_numpy(z["ids"]), cfg["num_attention_heads"], cfg["layer_norm_eps"])
    ref = z["y"]
    assert y.shape == ref.shape
    assert np.max(np.abs(y.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


# ---------------------------------------------------------------- tiled decode
def test_tiled_decode_vs_reference():
    import json
    z = load("vae_tiled")
    cfg, sd = cfg_of(z), weights_of(z)
    sp = json.loads(bytes(z["sp"]).decode())
    dec = vae_ref.decode_first_stage_tiled(sd, cfg, torch.from_numpy(z["z"]), float(z["scale_factor"]), sp)
    ref = z["dec"]
    assert dec.shape == ref.shape
    assert np.max(np.abs(dec.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


# ---------------------------------------------------------------- C1 DDPM UNet
def test_ddpm_unet_vs_reference():
    from oracle import ddpm_ref
    z = load("ddpm_unet")
    sd = weights_of(z)
    y = ddpm_ref.unet_forward(sd, torch.from_numpy(z["x"]), torch.from_numpy(z["t"]))
    ref = z["y"]
    assert y.shape == ref.shape
    assert np.max(np.abs(y.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())


def test_ddpm_pipeline_with_unet_vs_reference():
    from oracle import ddpm_ref
    z = load("ddpm_unet")
    sd = weights_of(z)
    tab = sch.ddpm_tables(1e-4, 1e-2, 4)
    img = z["x0"]
    noises = list(z["noises"])
    for t in range(3, -1, -1):
        eps = ddpm_ref.unet_forward(sd, torch.from_numpy(img), torch.full((img.shape[0],), t)).numpy()
        img = sch.ddpm_step(img, eps, sch.ddpm_step_scalars(tab, t), noises.pop(0) if t > 0 else None)
    assert np.max(np.abs(img - z["out"])) <= 1e-4 * max(1.0, np.abs(z["out"]).max())


# ---------------------------------------------------------------- classifier-free guidance
def test_ddim_cfg_sampling_vs_reference():
    from oracle.sampler_ref import ddim_sample
    z = load("ddim_cfg")
    u = load("unet_tiny")
    cfg, sd = cfg_of(u), weights_of(u)
    c, uc = torch.from_numpy(z["c"]), torch.from_numpy(z["uc"])
    model = lambda x, t: unet_ref.unet_forward(sd, cfg, x, t, c)
    uncond = lambda x, t: unet_ref.unet_forward(sd, cfg, x, t, uc)
    out, _ = ddim_sample(model, torch.from_numpy(z["xT"]), int(z["steps"]), guidance_scale=float(z["scale"]),
                         uncond_fn=uncond)
    ref = z["samples"]
    assert np.max(np.abs(out.numpy() - ref)) <= 1e-4 * max(1.0, np.abs(ref).max())
