"""C5 at its own size, the v-prediction update, and the reference's drop-in chain on the GPU
(run with -m gpu).

* C5 (BASELINE configs[4]): the SD-2-shape UNet (``num_head_channels: 64``, context 1024,
  ``openai_model/model.py:289-315``) at a 96x96 latent — 9,216-token self-attention at d = 64 —
  and the 96² → 768² VAE decode, each at B = 1 vs the fp32 CPU oracle (limits per test, ~3x the measured
  errors of profiles/r5_parity_errors.txt).
* v-prediction is an extension (the reference has eps / x0 only, ``Diffusion/ddpm.py:131``;
  SURVEY Q9): ε = √ᾱ·v + √(1-ᾱ)·x inside the fused DDIM update, bit-exact vs the oracle's
  restatement ``oracle.schedule.v_to_eps`` — PARITY UNPINNED (no reference value exists).
* Drop-in chain: ``instantiate_from_config`` on configs/sd-v1-txt2img.yaml (the reference's
  Diffusion/config.yaml model section, widths reduced via params) → ``get_learned_conditioning``
  (HIP CLIP text tower) → ``DDIMSampler.sample`` → ``LatentDiffusion.apply_model`` →
  ``DiffusionWrapper.forward`` → UNetModel (eager and HIP-graph) → ``decode_first_stage``,
  against the reference sampler's golden output and the oracle chain."""
import json
import os

import numpy as np
import pytest
import torch

from golden_util import cfg_of, load, weights_of
from gpu_util import check_golden, check_parity, rel_l2
from synth import synth_weights

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SD2 = dict(image_size=32, in_channels=4, out_channels=4, model_channels=320, attention_resolutions=[4, 2, 1],
           num_res_blocks=2, channel_mult=[1, 2, 4, 4], num_heads=-1, num_head_channels=64,
           use_spatial_transformer=True, transformer_depth=1, context_dim=1024, use_checkpoint=False, legacy=False)
SD_VAE = dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128, ch_mult=[1, 2, 4, 4],
              num_res_blocks=2, attn_resolutions=[], dropout=0.0)


def _synth_module(cls, seed, **kw):
    with torch.device("meta"):
        m = cls(**kw)
    ks = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    sd = {k: torch.from_numpy(v) for k, v in synth_weights(ks, seed).items()}
    m = cls(**kw)
    m.load_state_dict(sd)
    return m, sd


def test_c5_sd2_unet_96_latent_vs_oracle(sdk):
    """SD-2-shape UNet (865.9 M params) at the C5 latent 96x96, B=1: the 64² levels run
    9,216-token self-attention at head_dim 64 (5 heads at 320 channels)."""
    from oracle.unet_ref import unet_forward
    from sd_amd.openai_model.model import UNetModel
    m, sd = _synth_module(UNetModel, 321, **SD2)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(1, 4, 96, 96, generator=g)
    ctx = torch.randn(1, 77, 1024, generator=g)
    t = torch.tensor([641])
    y = m(x.to(DEV), t.to(DEV), ctx.to(DEV))
    torch.set_num_threads(16)
    ref = unet_forward(sd, SD2, x, t, ctx)
    assert y.shape == (1, 4, 96, 96)
    check_parity("C5 SD-2 UNet 96x96", y, ref, 5e-3, 6e-3)   # measured 1.60e-3 / 1.87e-3


def test_c5_vae_decode_96_to_768_vs_oracle(sdk):
    """SD VAE decoder at the C5 size: 4x96x96 → 3x768x768 (mid attention over 9,216 tokens)."""
    from oracle.vae_ref import decode_first_stage
    from sd_amd.VAE.autoencoder import AutoEncoderKL
    vae, sd = _synth_module(AutoEncoderKL, 79, ddconfig=SD_VAE, embed_dim=4)
    g = torch.Generator().manual_seed(13)
    z = torch.randn(1, 4, 96, 96, generator=g)
    dec = vae.decode(z.to(DEV), pre_scale=1.0 / 0.18215)
    torch.set_num_threads(16)
    ref = decode_first_stage(sd, SD_VAE, z, 0.18215)
    assert dec.shape == (1, 3, 768, 768)
    check_parity("C5 VAE decode 96->768", dec, ref, 3.5e-3, 4e-3)   # measured 1.09e-3 / 1.15e-3


@pytest.mark.parametrize("index", [0, 7, 25, 49])
@pytest.mark.parametrize("guidance", [1.0, 7.5])
def test_v_prediction_ddim_step_bitexact(sdk, index, guidance):
    """Fused update with v→ε (and the CFG combine before it) vs the oracle restatement, bitwise.
    Parity unpinned: the reference has no v-prediction."""
    from oracle import schedule as osch
    from sd_amd import ops
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd.DDIM.diffusion_modules import register_schedule
    sch = register_schedule(1000, 0.00085, 0.012)

    class LD:
        num_timesteps = 1000
        alphas_cumprod = sch["alphas_cumprod"]
        device = DEV
        parameterization = "v"

    s = DDIMSampler(LD())
    s.make_schedule(50, ddim_eta=0.0, verbose=False)
    sc = s.step_scalars(index)
    tab = osch.ddim_tables(50, 0.0)
    osc = osch.ddim_step_scalars(tab, index)
    g = torch.Generator().manual_seed(100 + index)
    x = torch.randn(3, 4, 24, 24, generator=g)
    v = torch.randn(3, 4, 24, 24, generator=g)
    vu = torch.randn(3, 4, 24, 24, generator=g)
    eu = vu.to(DEV) if guidance != 1.0 else None
    xp, p0 = ops.ddim_step(x.to(DEV), v.to(DEV), sc, e_uncond=eu, guidance=guidance,
                           v_param=(sc["v_sqrt_a"], sc["v_sqrt_1ma"]))
    vv = v.numpy()
    if guidance != 1.0:
        f32 = np.float32
        vv = (vu.numpy() + f32(guidance) * (v.numpy() - vu.numpy())).astype(f32)
    e_ref = osch.v_to_eps(x.numpy(), vv, osc["a_t"])
    xr, pr = osch.ddim_step(x.numpy(), e_ref, osc)
    assert np.array_equal(xp.cpu().numpy(), xr)
    assert np.array_equal(p0.cpu().numpy(), pr)


def test_v_prediction_sampler_loop_bitexact(sdk):
    """DDIMSampler.sample with parameterization 'v' and a deterministic elementwise stub model vs
    the oracle sampler loop (v branch), 10 steps: bitwise equal (timestep bookkeeping + update)."""
    from oracle.sampler_ref import ddim_sample
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd.DDIM.diffusion_modules import register_schedule
    sch = register_schedule(1000, 0.00085, 0.012)

    class LD:
        num_timesteps = 1000
        alphas_cumprod = sch["alphas_cumprod"]
        device = DEV
        parameterization = "v"

        def apply_model(self, x, t, c):
            return 0.5 * x + 0.01 * t.float()[:, None, None, None]

    g = torch.Generator().manual_seed(77)
    xT = torch.randn(2, 4, 12, 12, generator=g)
    out, _ = DDIMSampler(LD()).sample(S=10, batch_size=2, shape=(4, 12, 12), eta=0.0, x_T=xT.to(DEV), verbose=False)
    ref, _ = ddim_sample(lambda x, t: 0.5 * x + 0.01 * t.float()[:, None, None, None], xT, 10,
                         parameterization="v")
    assert np.array_equal(out.cpu().numpy(), ref.numpy())


# ------------------------------------------------------------------ the reference's drop-in chain
def _yaml_model(unet_cfg, ddconfig, cond_stage):
    import yaml
    y = yaml.safe_load(open(os.path.join(ROOT, "configs", "sd-v1-txt2img.yaml")))["model"]
    y["params"]["unet_config"]["params"] = unet_cfg
    y["params"]["first_stage_config"]["params"]["ddconfig"] = ddconfig
    y["params"]["cond_stage_config"] = cond_stage
    return y


@pytest.mark.parametrize("graphs", [False, True])
def test_dropin_chain_vs_reference_sampler_golden(sdk, graphs):
    """LatentDiffusion from the YAML (reference targets) → DDIMSampler.sample → apply_model →
    DiffusionWrapper → UNet: equals the reference DDIMSampler's own output (golden; limits in gpu_util.GOLDEN_LIMITS);
    decode_first_stage vs the oracle decode."""
    from oracle.vae_ref import decode_first_stage
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd.Diffusion.ddpm import DiffusionWrapper, LatentDiffusion
    from sd_amd.Diffusion.utils import instantiate_from_config
    u, v = load("unet_tiny"), load("vae_tiny")
    ld = instantiate_from_config(_yaml_model(cfg_of(u), cfg_of(v), None))
    assert type(ld) is LatentDiffusion and type(ld.model) is DiffusionWrapper
    assert ld.model.conditioning_key == "crossattn" and ld.scale_factor == 0.18215
    ld.model.diffusion_model.load_state_dict(weights_of(u))
    vsd = weights_of(v)
    ld.first_stage_model.load_state_dict(vsd)
    ld = ld.to(DEV)
    ld.use_graphs(graphs)
    calls = []
    orig = ld.model.forward
    ld.model.forward = lambda *a, **k: (calls.append(1), orig(*a, **k))[1]
    s = DDIMSampler(ld)
    steps = int(u["ddim_steps"])
    z, _ = s.sample(S=steps, batch_size=2, shape=(4, 16, 16), conditioning=torch.from_numpy(u["ctx"]).to(DEV),
                    eta=0.0, x_T=torch.from_numpy(u["ddim_xT"]).to(DEV), verbose=False)
    assert len(calls) == steps                 # every step went through DiffusionWrapper.forward
    check_golden("drop-in chain vs reference sampler", z, torch.from_numpy(u["ddim_samples"]))
    img = ld.decode_first_stage(z)
    ref = decode_first_stage(vsd, cfg_of(v), z.cpu(), 0.18215)
    assert img.shape == (2, 3, 32, 32)
    check_golden("drop-in chain decode vs oracle", img, ref)


def test_dropin_chain_with_text_conditioning_vs_oracle(sdk):
    """Token ids → get_learned_conditioning (HIP CLIP text tower from the YAML's cond stage target)
    → 4-step DDIM with classifier-free guidance through apply_model → decode, vs the oracle chain
    (clip_ref → unet_ref in sampler_ref.ddim_sample → vae_ref)."""
    from oracle.clip_ref import clip_text_forward
    from oracle.sampler_ref import ddim_sample
    from oracle.unet_ref import unet_forward
    from oracle.vae_ref import decode_first_stage
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd.Diffusion.utils import instantiate_from_config
    c, u, v = load("clip_tiny"), load("unet_tiny"), load("vae_tiny")
    ccfg = json.loads(bytes(c["cfg"]).decode())
    ucfg = dict(cfg_of(u), context_dim=ccfg["hidden_size"])
    cond = {"target": "clip_encoder.modules.FrozenCLIPEmbedder", "params": {"config": ccfg, "device": "cuda"}}
    ld = instantiate_from_config(_yaml_model(ucfg, cfg_of(v), cond))
    assert type(ld.cond_stage_model).__module__ == "sd_amd.clip_encoder.modules"
    csd = weights_of(c)
    ld.cond_stage_model.transformer.load_state_dict(csd)
    ks = [(k, tuple(t.shape)) for k, t in ld.model.diffusion_model.state_dict().items()]
    usd = {k: torch.from_numpy(a) for k, a in synth_weights(ks, 606).items()}
    ld.model.diffusion_model.load_state_dict(usd)
    vsd = weights_of(v)
    ld.first_stage_model.load_state_dict(vsd)
    ld = ld.to(DEV)
    ld.use_graphs(True)
    ids = torch.from_numpy(c["ids"])
    ids_u = ids.clone()
    ids_u[:, 1:] = int(ccfg["eos_token_id"])
    cc = ld.get_learned_conditioning(ids.to(DEV))
    uc = ld.get_learned_conditioning(ids_u.to(DEV))
    assert cc.shape == (2, 77, ccfg["hidden_size"])
    g = torch.Generator().manual_seed(31)
    xT = torch.randn(2, 4, 16, 16, generator=g)
    z, _ = DDIMSampler(ld).sample(S=4, batch_size=2, shape=(4, 16, 16), conditioning=cc, eta=0.0, x_T=xT.to(DEV),
                                  verbose=False, unconditional_guidance_scale=7.5, unconditional_conditioning=uc)
    img = ld.decode_first_stage(z)

    heads = ccfg["num_attention_heads"]
    rc = clip_text_forward(csd, ids, heads, prefix="")
    ru = clip_text_forward(csd, ids_u, heads, prefix="")
    check_golden("drop-in text cond vs oracle CLIP", cc, rc)
    zr, _ = ddim_sample(lambda x, t: unet_forward(usd, ucfg, x, t, rc), xT, 4, guidance_scale=7.5,
                        uncond_fn=lambda x, t: unet_forward(usd, ucfg, x, t, ru))
    ir = decode_first_stage(vsd, cfg_of(v), zr, 0.18215)
    check_golden("drop-in text chain latent vs oracle", z, zr)
    check_golden("drop-in text chain image vs oracle", img, ir)
