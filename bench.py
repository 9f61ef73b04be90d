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
import sd_amd_loader  # noqa: E402  (registers the package as `sd_amd`; the HIP library loads on first use)

sd_amd_loader.load()

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_F16_TFLOPS = 2500.0        # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md, no sparsity)
PEAK_HBM_GBS = 8000.0

SD1_UNET = dict(image_size=32, in_channels=4, out_channels=4, model_channels=320, attention_resolutions=[4, 2, 1],
                num_res_blocks=2, channel_mult=[1, 2, 4, 4], num_heads=8, use_spatial_transformer=True,
                transformer_depth=1, context_dim=768, use_checkpoint=False, legacy=False)
SD_VAE = dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128, ch_mult=[1, 2, 4, 4],
              num_res_blocks=2, attn_resolutions=[], dropout=0.0)
UNCOND_OVERRIDE = dict(use_spatial_transformer=False, context_dim=None)
SD2_OVERRIDE = dict(num_heads=-1, num_head_channels=64, context_dim=1024)
CONFIGS = {
    "c3": dict(workload="sd1-txt2img-512-ddim50", unet=SD1_UNET, latent=64, ctx=(77, 768), batch=16),
    "c2": dict(workload="ldm-uncond-256-ddim50", unet=dict(SD1_UNET, **UNCOND_OVERRIDE), unet_override=UNCOND_OVERRIDE,
               latent=32, ctx=None, batch=8),
    "c1": dict(workload="ddpm-pixel-32-10step", ddpm=True, image=32, batch=4, timesteps=10),
    "c5": dict(workload="sd2shape-768-vpred-ddim50", unet=dict(SD1_UNET, **SD2_OVERRIDE), unet_override=SD2_OVERRIDE,
               latent=96, ctx=(77, 1024), batch=8, v=True),
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


def model_config(cfg):
    """The LatentDiffusion config of a workload: the reference's Diffusion/config.yaml `model`
    section (configs/sd-v1-txt2img.yaml, same targets/params) with the config's UNet overrides."""
    import copy
    import yaml
    y = yaml.safe_load(open(os.path.join(ROOT, "configs", "sd-v1-txt2img.yaml")))["model"]
    y = copy.deepcopy(y)
    p = y["params"]
    p["unet_config"]["params"].update(cfg.get("unet_override", {}))
    if cfg["ctx"] is None:
        p["cond_stage_config"] = "__is_unconditional__"       # conditioning_key -> None (C2)
    elif cfg.get("v"):
        p["parameterization"] = "v"                           # SD-2 shape (C5): synthetic 1024-wide context
        p["cond_stage_config"] = None
    return y


def build_models(cfg, device, graph=False):
    """LatentDiffusion built through the drop-in chain (instantiate_from_config on the reference's
    YAML targets), seeded random weights materialised on the device.  Sampling calls
    apply_model -> DiffusionWrapper.forward -> UNetModel (HIP graph replay when ``graph``)."""
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd.Diffusion.utils import instantiate_from_config
    with torch.device("meta"):
        ld = instantiate_from_config(model_config(cfg))
    unet = ld.model.diffusion_model.to_empty(device=device)
    vae = ld.first_stage_model.to_empty(device=device)
    synth_init_(unet, 1234, device)
    synth_init_(vae, 4321, device)
    unet.prepare(device)
    vae.prepare(device)
    ld.use_graphs(graph)
    return unet, vae, ld


class GatherTimer:
    """Device time of the all-gather of each step: HIP events on the current stream around the
    collective (all_gather_into_tensor makes the current stream wait for RCCL's stream, so the closing
    event completes after the collective); wall clock on the CPU (gloo is synchronous there)."""

    def __init__(self, device):
        self.cuda = device.type == "cuda"
        self.reset()

    def reset(self):
        self.marks = []

    def run(self, fn):
        if self.cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn()
            e1.record()
            self.marks.append((e0, e1))
        else:
            t0 = time.perf_counter()
            out = fn()
            self.marks.append(1000.0 * (time.perf_counter() - t0))
        return out

    def mean_ms(self):
        if not self.marks:
            return None
        if self.cuda:
            torch.cuda.synchronize()
            ms = [a.elapsed_time(b) for a, b in self.marks]
        else:
            ms = self.marks
        return sum(ms) / len(ms)


def make_one_step(sampler, ld, xT, ctx, ddim_steps, world, gathered, gather_timer=None):
    """One bench step on one rank: 50-step DDIM over the rank's shard (x_T and context already in
    HBM), the VAE decode, and — for N > 1 ranks — the one collective of the path, an all-gather of
    the decoded images into ``gathered`` (rank-major, all_gather_into_tensor: RCCL over xGMI), timed by
    ``gather_timer`` when given."""
    from sd_amd import distributed as sdd
    B, shape = xT.shape[0], tuple(xT.shape[1:])

    def one_step():
        z, _ = sampler.sample(S=ddim_steps, batch_size=B, shape=shape, conditioning=ctx, eta=0.0, x_T=xT,
                              verbose=False, log_every_t=10 ** 9)
        img = ld.decode_first_stage(z)
        if world > 1:
            gat = lambda: sdd.gather(img.half(), world, out=gathered)   # noqa: E731
            gather_timer.run(gat) if gather_timer is not None else gat()
        return img
    return one_step


def timed_steps(one_step, steps, warmup, barrier, device, gather_timer=None):
    """W untimed warm-up steps, then exactly K steps between barrier + synchronize pairs; the
    elapsed time is the MAX over ranks.  ``gather_timer`` keeps the timed steps' all-gathers only."""
    from sd_amd import distributed as sdd
    img = None
    for _ in range(warmup):
        img = one_step()
    barrier()
    if gather_timer is not None:
        gather_timer.reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        img = one_step()
    barrier()
    return img, sdd.max_over_ranks(time.perf_counter() - t0, device=device)


def dp_report(img, gathered, rank, world, device, gather_timer):
    """Evidence of the N-rank run, for the bench line (every rank calls it: it holds collectives):
    the world size and backend the process group reports, the mean device time of the timed steps'
    all-gathers (max over ranks), and a bitwise check that slice r of the gathered batch is rank r's own
    fp16 image batch of the last step (mismatching ranks counted by an all-reduce)."""
    import torch.distributed as tdist
    from sd_amd import distributed as sdd
    B = img.shape[0]
    ok = torch.equal(gathered[rank * B:(rank + 1) * B], img.half())
    bad = torch.tensor([0 if ok else 1], dtype=torch.int64, device=device)
    tdist.all_reduce(bad, op=tdist.ReduceOp.SUM)
    ag = gather_timer.mean_ms() if gather_timer is not None else None
    return {"ranks_seen": tdist.get_world_size(), "backend": tdist.get_backend(),
            "allgather_ms": None if ag is None else round(sdd.max_over_ranks(ag, device=device), 3),
            "allgather_bytes_per_rank": img[:1].numel() * B * 2,
            "gather_slices_bitwise_equal": int(bad.item()) == 0, "gather_mismatched_ranks": int(bad.item())}


def make_barrier(dist, device):
    def barrier():
        if dist:
            import torch.distributed as tdist
            tdist.barrier()
        if device.type == "cuda":
            torch.cuda.synchronize(device)
    return barrier


def rank_inputs(seed, world, rank, batch, latent_shape, ctx_shape, device):
    """The rank's shard of the host-generated global batch (results independent of N)."""
    from sd_amd import distributed as sdd
    xT_all, ctx_all = sdd.global_inputs(seed, world, batch, latent_shape, ctx_shape)
    xT = sdd.shard(xT_all, rank, world).to(device)
    ctx = sdd.shard(ctx_all, rank, world).to(device) if ctx_all is not None else None
    return xT, ctx


# The reference itself timed as written on the survey container's CPU (BASELINE.md:22-25):
# not re-run here (/root/reference does not exist on the GPU box), carried beside the port's figure
REFERENCE_AS_WRITTEN = {
    "c3": {"value": 0.00516, "unit": "images/sec", "cores": 8, "kind": "reference",
           "sample": "reference path as written, B=1 full 50-step run + decode, 193.8 s/img, 8-vCPU Xeon "
                     "(survey container, BASELINE.md:22)"},
    "c2": {"value": 0.0466, "unit": "images/sec", "cores": 8, "kind": "reference",
           "sample": "reference path as written, B=8 UNet step 3.22 s + decode 10.3 s, extrapolated to 50 steps, "
                     "8-vCPU Xeon (BASELINE.md:24)"},
    "c5": {"value": 0.00273, "unit": "images/sec", "cores": 8, "kind": "reference",
           "sample": "reference path as written (eps-pred), B=8 UNet step 56.9 s + decode 90.3 s, extrapolated, "
                     "8-vCPU Xeon (BASELINE.md:25)"},
}


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


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(n, entry=None):
    """``bench.py --gpus N`` (N > 1) started without a launcher: this GPU-free parent checks that N
    devices are visible (device_count does not initialise the GPU on this image) and starts one
    rank per GPU with torch.distributed.run as a CHILD process (no exec), exiting with its code.
    ``entry``: the per-rank script (default this file; tests/bench_rank_stub.py in the CPU rehearsal)."""
    import subprocess
    have = torch.cuda.device_count()
    if have < n and not _rehearsal():
        print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have}; refusing to report a "
              f"{have}-GPU number as an {n}-GPU one", file=sys.stderr, flush=True)
        sys.exit(3)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(entry or __file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.exit(subprocess.call(cmd, env=env))


def _rehearsal():
    """SD_AMD_BENCH_REHEARSAL=cpu: the launcher and rank plumbing on the CPU (gloo, no GPU) — the
    tests' rehearsal of the 8-GPU launch; never set for a measured run."""
    return os.environ.get("SD_AMD_BENCH_REHEARSAL") == "cpu"


def setup_ranks(args):
    """(world, rank, local, dist, device) — one process per GPU, checked against --gpus."""
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            launch_ranks(args.gpus)                  # does not return
        world, rank, local = 1, 0, 0
    else:
        world = int(os.environ["WORLD_SIZE"])
        rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(3)
    dist = world > 1
    if _rehearsal():
        if dist:
            import torch.distributed as tdist
            tdist.init_process_group("gloo")
            assert tdist.get_world_size() == args.gpus
        return world, rank, local, dist, torch.device("cpu")
    if torch.cuda.device_count() <= local:
        print(f"bench.py: rank {rank} has no GPU of its own (local rank {local}, "
              f"{torch.cuda.device_count()} visible)", file=sys.stderr, flush=True)
        sys.exit(3)
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=device)
        assert tdist.get_world_size() == args.gpus
    return world, rank, local, dist, device


def make_parser():
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
    return ap


def main():
    args = make_parser().parse_args()

    world, rank, local, dist, device = setup_ranks(args)
    cfg = CONFIGS[args.config]
    if cfg.get("ddpm"):
        main_ddpm(args, cfg, world, rank, local, dist, device)
        if dist:
            import torch.distributed as tdist
            tdist.destroy_process_group()
        return
    B = args.batch or cfg["batch"]
    L = cfg["latent"]

    unet, vae, model = build_models(cfg, device, graph=False)
    from sd_amd.DDIM.ddim import DDIMSampler
    from sd_amd import ops
    sampler = DDIMSampler(model)

    xT, ctx = rank_inputs(2024, world, rank, B, (4, L, L), cfg["ctx"], device)
    gathered = torch.empty(world * B, 3, 8 * L, 8 * L, dtype=torch.float16, device=device) if dist else None
    gtimer = GatherTimer(device) if dist else None
    one_step = make_one_step(sampler, model, xT, ctx, args.ddim_steps, world, gathered, gtimer)
    barrier = make_barrier(dist, device)

    # the first warm-up step (eager) also autotunes every distinct conv problem missing from the
    # tuning table (tile config x split-K); the UNet graph is captured on the first graphed call
    cached = 0
    if args.tuning_cache and os.path.exists(args.tuning_cache) and not args.no_autotune:
        cached = ops.AUTOTUNE.load(args.tuning_cache)
    ops.AUTOTUNE.enable(not args.no_autotune)
    one_step()
    ops.AUTOTUNE.enable(False)
    if args.tuning_out and rank == 0 and len(ops.AUTOTUNE.table) > cached:
        os.makedirs(os.path.dirname(os.path.abspath(args.tuning_out)), exist_ok=True)
        ops.AUTOTUNE.save(args.tuning_out)
    model.use_graphs(not args.no_graph)
    if not args.no_graph:                # capture the UNet graph (setup, not a sampling step)
        model.apply_model(xT, torch.full((B,), 999, dtype=torch.long, device=device), ctx)
    img, elapsed = timed_steps(one_step, args.steps, max(args.warmup - 1, 0), barrier, device, gtimer)
    finite = bool(torch.isfinite(img).all().item())
    dp = dp_report(img, gathered, rank, world, device, gtimer) if dist else None

    # UNet step latency at the config batch (HIP events around replays of the sampler's UNet call,
    # through apply_model -> DiffusionWrapper -> graph replay)
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
        model.use_graphs(False)
        ops.PROFILER.start()
        z, _ = sampler.sample(S=args.ddim_steps, batch_size=B, shape=(4, L, L), conditioning=ctx, eta=0.0, x_T=xT,
                              verbose=False, log_every_t=10 ** 9)
        model.decode_first_stage(z)
        torch.cuda.synchronize()
        ops.PROFILER.stop()
        model.use_graphs(not args.no_graph)

    images = world * B * args.steps
    value = images / elapsed
    out = {"metric": METRIC, "value": round(value, 4), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f16", "data": "synthetic (seeded random weights, "
           "N(0,1) latents, N(0,1) 77-token context)",
           "config": {"workload": cfg["workload"], "global_batch": world * B, "batch_per_gpu": B,
                      "latent": [4, L, L], "image": [3, 8 * L, 8 * L], "ddim_steps": args.ddim_steps, "eta": 0.0,
                      "parallelism": f"dp{world}", "collective": "all_gather decoded images (RCCL)" if dist else None,
                      "entry": "LatentDiffusion (configs/sd-v1-txt2img.yaml) -> DDIMSampler.sample -> "
                               "decode_first_stage"},
           "unet_step_ms": round(unet_ms, 3), "finite": finite, "hip_graph": not args.no_graph,
           "autotuned_conv_problems": len(ops.AUTOTUNE.table), "tuning_cache_entries": cached}
    if dp is not None:
        out.update(dp)
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
                               "kernel": "conv family: conv_glds_kernel / conv_ph_kernel / "
                                         "conv_igemm_kernel / conv_direct_kernel / conv_skinny_kernel "
                                         "(+splitk_reduce_kernel on split-K launches)",
                               "launches": conv["launches"], "avg_launch_us": round(1e6 * avg_s, 2),
                               "flops_per_launch": conv["flops"] / conv["launches"],
                               "algorithmic_bytes_per_launch": round(conv["bytes"] / conv["launches"]),
                               "traffic_unit": "bytes per launch (PMC, profiles/conv_traffic.json)"}
            # the achievable ceilings of THIS device (random-operand MFMA loops, HBM copy; sdk_probe_*),
            # next to the spec peak `frac` is quoted against
            probe = ops.probe_peaks()
            out["roofline"]["peak_measured"] = probe
            out["roofline"]["frac_of_measured_peak"] = round(
                ach / max(probe["mfma_16x16x32_f16_tflops"], probe["mfma_32x32x16_f16_tflops"]), 4)
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
            model.use_graphs(False)
            model.apply_model(xT, tts, ctx)
            torch.cuda.synchronize()
            ops.PROFILER.stop()
            model.use_graphs(not args.no_graph)
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
        if args.config in REFERENCE_AS_WRITTEN:
            out["cpu_baseline"]["reference_as_written"] = REFERENCE_AS_WRITTEN[args.config]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
