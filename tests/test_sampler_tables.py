"""Host-side sampler tables of the product (sd_amd.DDIM) vs the reference's golden tables — bit-exact, CPU."""
import numpy as np

from golden_util import load


def test_sampler_tables_bitexact(sdk):
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd.DDIM.diffusion_modules import register_schedule
    z = load("schedule")
    sch = register_schedule(1000, 0.00085, 0.012)
    assert np.array_equal(sch["alphas_cumprod"].numpy(), z["alphas_cumprod"])

    class M:
        num_timesteps = 1000
        alphas_cumprod = sch["alphas_cumprod"]

    for S in (10, 50, 250):
        for eta in (0, 1):
            s = DDIMSampler(M())
            s.make_schedule(S, ddim_eta=float(eta), verbose=False)
            tag = f"S{S}_eta{eta}"
            assert np.array_equal(s.ddim_timesteps, z[tag + "_ts"])
            assert np.array_equal(s.ddim_alphas.numpy(), z[tag + "_alphas"])
            assert np.array_equal(np.asarray(s.ddim_alphas_prev), z[tag + "_alphas_prev"])
            assert np.array_equal(s.ddim_sigmas.numpy(), z[tag + "_sigmas"])
            assert np.array_equal(s.ddim_sqrt_one_minus_alphas.numpy(), z[tag + "_sqrt_one_minus"])
