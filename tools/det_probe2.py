"""Repeat one UNet evaluation of the C3 bench batch (eager) many times on the same input and count the
distinct results, under routing variants (bisecting a run-to-run difference):
  default | no halo conv (tuning entries choosing variants 36 / 37 sent to the planner) |
  no fused cross-attention block | both."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sd_amd import ops
    from sd_amd.openai_model import attention as att
    cfg = bench.CONFIGS["c3"]
    ops.AUTOTUNE.load(os.path.join(ROOT, "configs", "conv_tuning_mi355x.json"))
    ops.AUTOTUNE.enable(False)
    table0 = dict(ops.AUTOTUNE.table)
    dev = torch.device("cuda", 0)
    unet, vae, ld = bench.build_models(cfg, dev, graph=False)
    B, L = cfg["batch"], cfg["latent"]
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(B, 4, L, L, generator=g) * 3.0).to(dev)
    ctx = (torch.randn(B, 77, 768, generator=g)).to(dev)
    reps = int(os.environ.get("REPS", "24"))

    def trial(tag):
        outs = []
        for t in [int(v) for v in os.environ.get("TS", "981,501,21").split(",")]:
            tt = torch.full((B,), t, dtype=torch.long, device=dev)
            ref = ld.apply_model(x, tt, ctx).float().clone()
            bad = 0
            for _ in range(reps):
                y = ld.apply_model(x, tt, ctx).float()
                if not torch.equal(y, ref):
                    bad += 1
                    outs.append((t, (y - ref).abs().max().item()))
            print(f"{tag}: t={t}: {bad}/{reps} runs differ", flush=True)
        if outs:
            print(f"   max diffs {outs[:6]}", flush=True)

    modes = os.environ.get("MODES", "default,nohalo,noxattn").split(",")
    for mode in modes:
        ops.AUTOTUNE.table.clear()
        ops.AUTOTUNE.table.update(table0)
        att.FUSED_CROSS_ATTENTION, att.FUSED_XATTN_NORMS = True, True
        att.FUSED_XATTN_MIN_ROWS, att.FUSED_XATTN_640_MAX_ROWS = 65536, 16384
        if mode == "nohalo":
            ops.AUTOTUNE.table.clear()
            ops.AUTOTUNE.table.update({k: ((0, 0) if v[0] in (37, 38) else v) for k, v in table0.items()})
        elif mode == "noxattn":
            att.FUSED_CROSS_ATTENTION = False
        elif mode == "only320":
            att.FUSED_XATTN_640_MAX_ROWS = 0
        elif mode == "only640":
            att.FUSED_XATTN_MIN_ROWS = 1 << 30
        elif mode == "nonorms":
            att.FUSED_XATTN_NORMS = False
        trial(mode)


if __name__ == "__main__":
    main()
