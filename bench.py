"""Headline benchmark: SD-1.x txt2img, 512x512, 50-step DDIM + VAE decode (BASELINE.json config C3/C4).

One "step" = one full pass of the hot path over one batch: DDIM sampling (50
UNet evaluations + 50 fused DDIM updates) of B latents 4x64x64 with a 77x768
context, then the KL-VAE decode to B images 3x512x512.  Weights are seeded
random (SD-1.x architecture, 860M UNet + 83.7M VAE); inputs are synthetic.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU; the latents of a global batch N*B are generated on the
host from one seed and sliced per rank (weak scaling: B per GPU); no per-step
collective; one RCCL all_gather_into_tensor of the decoded images at the end of
every step.  Timing: barrier + synchronize on both sides of the K timed steps,
max over ranks.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_F16_TFLOPS = 2500.0        # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_HBM_GBS = 8000.0

SD1_UNET = dict(image_size=32, in_channels=4, out_channels=4, model_channels=320, attention_resolutions=[4, 2, 1],
                num_res_blocks=2, channel_mult=[1, 2, 4, 4], num_heads=8, use_spatial_transformer=True,
                transformer_depth=1, context_dim=768, use_checkpoint=False, legacy=False)
SD_VAE = dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128, ch_mult=[1, 2, 4, 4],
              num_res_blocks=2, attn_resolutions=[], dropout=0.0)
CONFIGS = {
    "c3": dict(workload="sd1-txt2img-512-ddim50", unet=SD1_UNET, latent=64, ctx=(77, 768), batch=16),
    "c2": dict(workload="ldm-uncond-256-ddim50", unet=dict(SD1_UNET, use_spatial_transformer=False,
                                                           context_dim=None), latent=32, ctx=None, batch=8),
    "c1": dict(workload="ddpm-pixel-32-10step", ddpm=True, image=32, batch=4, timesteps=10),
    "c5": dict(workload="sd2shape-768-vpred-ddim50", unet=dict(SD1_UNET, num_heads=-1, num_head_channels=64,
                                                               context_dim=1024), latent=96, ctx=(77, 1024),
               batch=8, v=True),
}


def synth_init_(module, seed, device):
    """Seeded N(0, 0.02^2) conv/linear weights (zero-init layers included), zero biases,
    GN/LN gamma=1 beta=0 — SURVEY §8(d) synthetic weights, materialised on the device."""
    g = torch.Generator(device=device).manual_seed(seed)
    for name, p in module.named_parameters():
        if p.dim() >= 2:
            p.data = torch.randn(p.shape, generator=g, device=device) * 0.02
        elif name.endswith("bias"):
            p.data = torch.zeros(p.shape, device=device)
        else:
            p.data = torch.ones(p.shape, device=device)


def build_models(cfg, device, graph=False):
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd.openai_model.model import UNetModel
    from sd_amd.VAE.autoencoder import AutoEncoderKL
    from sd_amd.DDIM.diffusion_modules import register_schedule
    with torch.device("meta"):
        unet = UNetModel(**cfg["unet"])
        vae = AutoEncoderKL(ddconfig=SD_VAE, embed_dim=4)
    unet = unet.to_empty(device=device)
    vae = vae.to_empty(device=device)
    synth_init_(unet, 1234, device)
    synth_init_(vae, 4321, device)
    unet.prepare(device)
    vae.prepare(device)
    sch = register_schedule(1000, 0.00085, 0.012)
    from sd_amd.graphs import GraphedUNet
    graphed = GraphedUNet(unet)

    class LatentModel:
        """LatentDiffusion.apply_model / decode_first_stage semantics (Diffusion/ddpm.py)."""
        num_timesteps = 1000
        alphas_cumprod = sch["alphas_cumprod"]
        parameterization = "v" if cfg.get("v") else "eps"
        scale_factor = 0.18215

        def __init__(self):
            self.device = device
            self.graph = graph

        def apply_model(self, x, t, c):
            if self.graph:
                return graphed(x, t, c)
            return unet(x, t, context=c)

        def decode_first_stage(self, z):
            return vae.decode(z, pre_scale=1.0 / self.scale_factor)

    return unet, vae, LatentModel()


def unet_gflops_per_image(cfg):
    return {"c3": 803.3, "c2": 125.1, "c5": 2149.1, "c1": 3.275}[cfg]


def vae_gflops_per_image(cfg):
    return {"c3": 2514.5, "c2": 622.2, "c5": 5754.3, "c1": 0.0}[cfg]


def main_ddpm(args, cfg, world, rank, local, dist, device):
    """C1 (BASELINE configs[0]): the pixel-space DDPM pipeline, DDPMPipeline.sampling over T steps with the
    58.66 M DDPM UNet (DDPM/ddpm.py:53-89, DDPM/models/unet.py), one HIP graph per UNet call."""
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    from sd_amd import distributed as sdd
    from sd_amd.DDPM.ddpm import DDPMPipeline
    from sd_amd.DDPM.models.unet import UNet
    from sd_amd.graphs import GraphedUNet
    m = UNet(input_channels=3).to(device)       # (its positional table is a plain tensor: no meta init)
    synth_init_(m, 1234, device)
    B, S, T = args.batch or cfg["batch"], cfg["image"], cfg["timesteps"]
    pipe = DDPMPipeline(beta_start=1e-4, beta_end=1e-2, num_timesteps=T)

    class _Call(torch.nn.Module):       # GraphedUNet's (x, t, context) calling convention
        def forward(self, x, t, context=None):
            return m(x, t)

    graphed = GraphedUNet(_Call())
    model = (lambda x, t: graphed(x, t)) if not args.no_graph else m
    x_all, _ = sdd.global_inputs(2024, world, B, (3, S, S), None)
    x0 = sdd.shard(x_all, rank, world).to(device)
    gen = torch.Generator(device=device).manual_seed(99 + rank)
    noise_fn = lambda i, shape: torch.randn(shape, device=device, generator=gen)
    cached = 0
    if args.tuning_cache and os.path.exists(args.tuning_cache) and not args.no_autotune:
        cached = ops.AUTOTUNE.load(args.tuning_cache)
    ops.AUTOTUNE.enable(not args.no_autotune)
    pipe.sampling(m, x0, device, noise_fn=noise_fn)          # eager: autotune + settle workspaces
    ops.AUTOTUNE.enable(False)
    if args.tuning_out and rank == 0 and len(ops.AUTOTUNE.table) > cached:
        os.makedirs(os.path.dirname(os.path.abspath(args.tuning_out)), exist_ok=True)
        ops.AUTOTUNE.save(args.tuning_out)

    def barrier():
        if dist:
            import torch.distributed as tdist
            tdist.barrier()
        torch.cuda.synchronize()

    for _ in range(max(args.warmup, 1)):
        img = pipe.sampling(model, x0, device, noise_fn=noise_fn)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        img = pipe.sampling(model, x0, device, noise_fn=noise_fn)
    barrier()
    elapsed = sdd.max_over_ranks(time.perf_counter() - t0, device=device)
    value = world * B * args.steps / elapsed
    out = {"metric": METRIC, "value": round(value, 4), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f16",
           "data": "synthetic (seeded random weights, N(0,1) images and noise)",
           "config": {"workload": cfg["workload"], "global_batch": world * B, "batch_per_gpu": B,
                      "image": [3, S, S], "timesteps": T, "parallelism": f"dp{world}", "collective": None},
           "finite": bool(torch.isfinite(img).all().item()), "hip_graph": not args.no_graph,
           "tuning_cache_entries": cached}
    if not args.no_roofline and rank == 0:
        ops.PROFILER.start()
        pipe.sampling(m, x0, device, noise_fn=noise_fn)
        torch.cuda.synchronize()
        ops.PROFILER.stop()
        summ = ops.PROFILER.summary()
        conv = {"launches": 0, "ms": 0.0, "flops": 0.0}
        for k, d in summ.items():
            if k.startswith("conv"):
                for f in conv:
                    conv[f] += d[f]
        if conv["launches"]:
            ach = conv["flops"] / (conv["ms"] / 1000.0) / 1e12
            out["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(ach / PEAK_F16_TFLOPS, 4), "traffic": None,
                               "kernel": "conv family (launch-bound at 32x32, B=4)", "launches": conv["launches"],
                               "avg_launch_us": round(1000 * conv["ms"] / conv["launches"], 2)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from oracle.ddpm_ref import unet_forward
        torch.set_num_threads(args.cpu_threads)
        sd = {k: v.detach().float().cpu() for k, v in m.state_dict().items()}
        xc = torch.randn(1, 3, S, S)
        t0 = time.perf_counter()
        unet_forward(sd, xc, torch.tensor([T - 1]))
        t_unet = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": 1.0 / (T * t_unet), "unit": "images/sec", "cores": args.cpu_threads,
                               "kind": "port", "sample": f"fp32 CPU oracle: 1 DDPM UNet eval ({t_unet:.2f} s) at "
                                                         f"batch 1, extrapolated to {T} steps per image"}
    if rank == 0:
        print(json.dumps(out), flush=True)


def cpu_baseline(cfg_name, cfg, ddim_steps, threads):
    """The fp32 CPU oracle (a port of the reference path) timed on this host: one UNet
    evaluation + one VAE decode at batch 1, extrapolated to a full 50-step image."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from oracle.unet_ref import unet_forward
    from oracle.vae_ref import decode_first_stage
    from sd_amd.openai_model.model import UNetModel
    from sd_amd.VAE.autoencoder import AutoEncoderKL
    torch.set_num_threads(threads)
    with torch.device("meta"):
        um = UNetModel(**cfg["unet"])
        vm = AutoEncoderKL(ddconfig=SD_VAE, embed_dim=4)
    g = torch.Generator().manual_seed(0)
    usd = {k: torch.randn(v.shape, generator=g) * 0.02 if v.dim() >= 2 else torch.zeros(v.shape)
           for k, v in um.state_dict().items()}
    vsd = {k: torch.randn(v.shape, generator=g) * 0.02 if v.dim() >= 2 else torch.ones(v.shape)
           for k, v in vm.state_dict().items()}
    L = cfg["latent"]
    x = torch.randn(1, 4, L, L, generator=g)
    ctx = torch.randn(1, *cfg["ctx"], generator=g) if cfg["ctx"] else None
    t0 = time.perf_counter()
    unet_forward(usd, cfg["unet"], x, torch.tensor([501]), ctx)
    t_unet = time.perf_counter() - t0
    t0 = time.perf_counter()
    decode_first_stage(vsd, SD_VAE, x, 0.18215)
    t_vae = time.perf_counter() - t0
    per_img = ddim_steps * t_unet + t_vae
    return {"value": 1.0 / per_img, "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"fp32 CPU oracle: 1 UNet eval ({t_unet:.2f} s) + 1 VAE decode ({t_vae:.2f} s) at batch 1, "
                      f"{L}x{L} latent, extrapolated to {ddim_steps} DDIM steps + decode per image"}


def pmc_traffic(args):
    """HBM bytes per conv launch from the committed rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE,
    gfx950-corrected, tools/prof_summary.py) of this same workload — only when they were taken
    on the current conv kernel source (else null: counters cannot be read from inside the run)."""
    p = os.path.join(ROOT, "profiles", "conv_traffic.json")
    if args.config != "c3" or args.ddim_steps != 50 or not os.path.exists(p):
        return None
    from sd_amd import ops
    d = json.load(open(p))
    if d.get("conv_source") != ops._conv_source_hash() or "traffic_bytes_per_launch" not in d:
        return None
    return round(d["traffic_bytes_per_launch"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--ddim-steps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-autotune", action="store_true")
    ap.add_argument("--tuning-cache", default=os.path.join(ROOT, "configs", "conv_tuning_mi355x.json"),
                    help="conv tile/split-K table measured on MI355X (loaded if present; missing problems are timed)")
    ap.add_argument("--tuning-out", default=None, help="write the (extended) tuning table here")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one HIP graph per UNet step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local if dist else 0)
    torch.cuda.set_device(device)
    cfg = CONFIGS[args.config]
    if cfg.get("ddpm"):
        main_ddpm(args, cfg, world, rank, local, dist, device)
        if dist:
            import torch.distributed as tdist
            tdist.destroy_process_group()
        return
    B = args.batch or cfg["batch"]
    L = cfg["latent"]

    unet, vae, model = build_models(cfg, device, graph=not args.no_graph)
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd import ops
    sampler = DDIMSampler(model)

    # host-generated global batch, sliced per rank (parity with any rank count)
    from sd_amd import distributed as sdd
    xT_all, ctx_all = sdd.global_inputs(2024, world, B, (4, L, L), cfg["ctx"])
    xT = sdd.shard(xT_all, rank, world).to(device)
    ctx = sdd.shard(ctx_all, rank, world).to(device) if ctx_all is not None else None
    gathered = torch.empty(world * B, 3, 8 * L, 8 * L, dtype=torch.float16, device=device) if dist else None

    def one_step():
        z, _ = sampler.sample(S=args.ddim_steps, batch_size=B, shape=(4, L, L), conditioning=ctx, eta=0.0, x_T=xT,
                              verbose=False, log_every_t=10 ** 9)
        img = model.decode_first_stage(z)
        if dist:
            sdd.gather(img.half(), world, out=gathered)
        return img

    def barrier():
        if dist:
            import torch.distributed as tdist
            tdist.barrier()
        torch.cuda.synchronize()

    # the first warm-up step also autotunes every distinct conv problem (tile config x split-K);
    # the UNet graph is captured on its first graphed call, after the eager autotuning call
    cached = 0
    if args.tuning_cache and os.path.exists(args.tuning_cache) and not args.no_autotune:
        cached = ops.AUTOTUNE.load(args.tuning_cache)
    ops.AUTOTUNE.enable(not args.no_autotune)
    model.graph = False
    one_step()
    ops.AUTOTUNE.enable(False)
    if args.tuning_out and rank == 0 and len(ops.AUTOTUNE.table) > cached:
        os.makedirs(os.path.dirname(os.path.abspath(args.tuning_out)), exist_ok=True)
        ops.AUTOTUNE.save(args.tuning_out)
    model.graph = not args.no_graph
    if model.graph:                      # capture the UNet graph (setup, not a sampling step)
        model.apply_model(xT, torch.full((B,), 999, dtype=torch.long, device=device), ctx)
    for _ in range(max(args.warmup - 1, 0)):
        one_step()
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        img = one_step()
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = sdd.max_over_ranks(elapsed, device=device)
    finite = bool(torch.isfinite(img).all().item())

    # UNet step latency at the config batch (HIP events around replays of the sampler's UNet call)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tts = torch.full((B,), 501, dtype=torch.long, device=device)
    model.apply_model(xT, tts, ctx)
    torch.cuda.synchronize()
    e0.record()
    nrep = 5
    for _ in range(nrep):
        model.apply_model(xT, tts, ctx)
    e1.record()
    torch.cuda.synchronize()
    unet_ms = e0.elapsed_time(e1) / nrep

    # per-kernel breakdown: one extra, untimed, eager step on rank 0 with HIP events
    # around every launch (not part of `value`)
    if not args.no_roofline and rank == 0:
        model.graph = False
        ops.PROFILER.start()
        z, _ = sampler.sample(S=args.ddim_steps, batch_size=B, shape=(4, L, L), conditioning=ctx, eta=0.0, x_T=xT,
                              verbose=False, log_every_t=10 ** 9)
        model.decode_first_stage(z)
        torch.cuda.synchronize()
        ops.PROFILER.stop()
        model.graph = not args.no_graph

    images = world * B * args.steps
    value = images / elapsed
    out = {"metric": METRIC, "value": round(value, 4), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f16", "data": "synthetic (seeded random weights, "
           "N(0,1) latents, N(0,1) 77-token context)",
           "config": {"workload": cfg["workload"], "global_batch": world * B, "batch_per_gpu": B,
                      "latent": [4, L, L], "image": [3, 8 * L, 8 * L], "ddim_steps": args.ddim_steps, "eta": 0.0,
                      "parallelism": f"dp{world}", "collective": "all_gather decoded images (RCCL)" if dist else None},
           "unet_step_ms": round(unet_ms, 3), "finite": finite, "hip_graph": not args.no_graph,
           "autotuned_conv_problems": len(ops.AUTOTUNE.table), "tuning_cache_entries": cached}
    if not args.no_roofline and rank == 0:
        summ = ops.PROFILER.summary()
        conv = {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0}
        for k, d in summ.items():
            if k.startswith("conv"):
                for f in conv:
                    conv[f] += d[f]
        if conv["launches"]:
            avg_s = conv["ms"] / 1000.0 / conv["launches"]
            ach = conv["flops"] / conv["launches"] / avg_s / 1e12
            out["roofline"] = {"bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(ach / PEAK_F16_TFLOPS, 4), "traffic": pmc_traffic(args),
                               "kernel": "conv family: conv_glds_kernel / conv_ph_kernel / conv_igemm_kernel "
                                         "(+splitk_reduce_kernel on split-K launches)",
                               "launches": conv["launches"], "avg_launch_us": round(1e6 * avg_s, 2),
                               "flops_per_launch": conv["flops"] / conv["launches"],
                               "algorithmic_bytes_per_launch": round(conv["bytes"] / conv["launches"]),
                               "traffic_unit": "bytes per launch (PMC, profiles/conv_traffic.json)"}
        out["kernel_time_ms_profiled_step"] = {k: round(v["ms"], 2) for k, v in summ.items()}
        xa = ops.PROFILER.region_summary("cross_attention")
        if xa["launches"]:
            # north-star item: MFMA use of the cross-attention block (to_q + core on the cached
            # context K/V + to_out with its residual), FLOPs / (its device time x dense peak)
            ach = xa["flops"] / (xa["ms"] * 1e-3) / 1e12
            out["cross_attention_block"] = {
                "achieved": round(ach, 2), "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(ach / PEAK_F16_TFLOPS, 4), "ms_per_sample": round(xa["ms"], 2),
                "share_of_profiled_step": round(xa["ms"] / sum(v["ms"] for v in summ.values()), 4),
                "by_kind": {k: {"ms": round(v["ms"], 2), "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
                            for k, v in xa["by_kind"].items()}}
        if os.environ.get("BENCH_SEQ_OUT"):
            # launch sequence of ONE UNet forward (kind, shape, flops) for tools/trace_step.py,
            # which pairs it with a graph-replayed step of a rocprofv3 trace (device times)
            recs = ops.PROFILER.records
            ops.PROFILER.start()
            model.graph = False
            model.apply_model(xT, tts, ctx)
            torch.cuda.synchronize()
            ops.PROFILER.stop()
            model.graph = not args.no_graph
            seq = [[k, v, fl, list(sh) if isinstance(sh, tuple) else sh]
                   for k, v, fl, _, _, sh, _ in ops.PROFILER.records]
            ops.PROFILER.records = recs
            with open(os.environ["BENCH_SEQ_OUT"], "w") as f:
                json.dump(seq, f)
        if os.environ.get("BENCH_SHAPES_OUT"):
            with open(os.environ["BENCH_SHAPES_OUT"], "w") as f:
                for (kind, shape), n, ms, tf in ops.PROFILER.shape_table():
                    f.write(f"{kind:10s} {str(shape):44s} launches={n:5d} ms={ms:9.2f} TFLOP/s={tf:7.1f}\n")
        tot_tf = (unet_gflops_per_image(args.config) * args.ddim_steps + vae_gflops_per_image(args.config)) / 1000
        out["end_to_end_tflops"] = round(tot_tf * value, 1)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.config, cfg, args.ddim_steps, args.cpu_threads)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
