"""Locate a non-determinism of the C3 bench step: UNet eager vs eager, eager vs graph replay, graph vs graph,
sampler twice (z), decode twice — bitwise comparisons at the bench batch with the committed table."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sd_amd import ops
    from sd_amd.DDIM.ddim import DDIMSampler
    cfg = bench.CONFIGS["c3"]
    ops.AUTOTUNE.load(os.path.join(ROOT, "configs", "conv_tuning_mi355x.json"))
    ops.AUTOTUNE.enable(False)
    dev = torch.device("cuda", 0)
    unet, vae, ld = bench.build_models(cfg, dev, graph=False)
    B, L = cfg["batch"], cfg["latent"]
    xT, ctx = bench.rank_inputs(2024, 1, 0, B, (4, L, L), cfg["ctx"], dev)
    t = torch.full((B,), 501, dtype=torch.long, device=dev)

    def eps():
        return ld.apply_model(xT, t, ctx).float().clone()
    e1, e2 = eps(), eps()
    print("eager vs eager", torch.equal(e1, e2), (e1 - e2).abs().max().item(), flush=True)
    ld.use_graphs(True)
    g1 = eps()          # warm-up / capture call
    g2, g3 = eps(), eps()
    print("eager vs graph(first)", torch.equal(e1, g1), (e1 - g1).abs().max().item(), flush=True)
    print("eager vs graph(replay)", torch.equal(e1, g2), (e1 - g2).abs().max().item(), flush=True)
    print("graph vs graph", torch.equal(g2, g3), flush=True)
    s = DDIMSampler(ld)

    def run(graphs, steps=50):
        ld.use_graphs(graphs)
        z, inter = s.sample(S=steps, batch_size=B, shape=(4, L, L), conditioning=ctx, eta=0.0, x_T=xT,
                            verbose=False, log_every_t=1)
        return [x.float().clone() for x in inter["x_inter"]]

    def cmp(tag, a, b):
        first = next((i for i, (u, v) in enumerate(zip(a, b)) if not torch.equal(u, v)), None)
        print(f"{tag}: first differing state {first} of {len(a)}; last max |diff| "
              f"{(a[-1] - b[-1]).abs().max().item():.3e}", flush=True)
    xt0 = xT.clone()
    e_a, e_b = run(False), run(False)
    cmp("eager sample vs eager sample", e_a, e_b)
    print("x_T unchanged", torch.equal(xt0, xT), flush=True)
    g_a, g_b = run(True), run(True)
    cmp("graph sample vs graph sample", g_a, g_b)
    cmp("eager sample vs graph sample", e_a, g_a)
    z1 = g_a[-1]
    d1 = ld.decode_first_stage(z1).float().clone()
    d2 = ld.decode_first_stage(z1).float().clone()
    print("decode vs decode", torch.equal(d1, d2), (d1 - d2).abs().max().item(), flush=True)


if __name__ == "__main__":
    main()
