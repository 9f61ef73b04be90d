"""Determinism stress on the MI355X: (1) the C3 bench step (B=16, tuning table, graphs, 50 DDIM steps +
decode) repeated, bitwise vs the first run; (2) every LDS-DMA tile conv problem of the C3 UNet step launched
repeatedly (eager and graph-replayed), bitwise vs its first output.  A mismatch means a race."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def main():
    import bench
    from sd_amd import ops
    from sd_amd.DDIM.ddim import DDIMSampler
    reps_step = int(os.environ.get("STRESS_STEPS", "4"))
    reps_conv = int(os.environ.get("STRESS_CONV", "100"))
    cfg = bench.CONFIGS["c3"]
    import json
    d = json.load(open(os.path.join(ROOT, "configs", "conv_tuning_mi355x.json")))
    for k, v in d["entries"]:            # tile choices as tuned, even if the kernel source moved since
        ops.AUTOTUNE.table[tuple(k)] = tuple(v)
    ops.AUTOTUNE.enable(False)
    dev = torch.device("cuda", 0)
    unet, vae, ld = bench.build_models(cfg, dev, graph=True)
    xT, ctx = bench.rank_inputs(2024, 1, 0, 16, (4, 64, 64), cfg["ctx"], dev)
    step = bench.make_one_step(DDIMSampler(ld), ld, xT, ctx, 50, 1, None)
    first = step().clone()
    bad = 0
    for r in range(reps_step):
        img = step()
        eq = torch.equal(img, first)
        bad += not eq
        d = (img.float() - first.float()).abs().max().item()
        print(f"step rep {r}: bitwise {'equal' if eq else 'DIFFERENT'} (max |d| {d:.3e})", flush=True)
    # the LDS-DMA tile conv problems of one UNet step (the one-barrier interleaved K loop), replayed
    calls = []
    orig = ops.conv2d

    def spy(pc, x, **kw):
        y = orig(pc, x, **kw)
        calls.append((pc, x, dict(kw)))
        return y
    ops.conv2d = spy
    ld.use_graphs(False)
    ld.apply_model(xT, torch.full((16,), 501, dtype=torch.long, device=dev), ctx)
    ops.conv2d = orig
    torch.cuda.synchronize()
    seen = 0
    for pc, x, kw in calls:
        ops.PROFILER.start()
        y0 = ops.conv2d(pc, x, **kw).clone()
        ops.PROFILER.stop()
        v = ops.PROFILER.records[-1][1]
        if v not in (22, 23, 24, 2, 3, 6, 7):
            continue
        seen += 1
        nbad = 0
        for _ in range(reps_conv):
            y = ops.conv2d(pc, x, **kw)
            nbad += not torch.equal(y, y0)
        bad += nbad
        shp = tuple(x[0].shape) if isinstance(x, tuple) else tuple(x.shape)
        print(f"conv v{v} {shp} -> {pc.N}: {reps_conv} launches, {nbad} differ", flush=True)
    print(f"STRESS {'OK' if bad == 0 else 'FAILED'}: {seen} tile-conv problems, {bad} mismatches", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
