"""Probe (not product code): one SD-1 UNet evaluation at B=16 as one graph on one stream vs the
same batch as two B=8 halves captured as two concurrent branches (fork/join on two streams,
separate workspace lanes) in one graph.  Device time from HIP events around graph replays."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(f, reps=10):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    import bench
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS["c3"]
    unet, _, _ = bench.build_models(cfg, dev)
    B = int(os.environ.get("B", "16"))
    lanes = int(os.environ.get("LANES", "2"))
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(B, 4, 64, 64, generator=g).to(dev)
    ctx = torch.randn(B, 77, 768, generator=g).to(dev).half()
    t = torch.full((B,), 501, dtype=torch.long, device=dev)
    tune = os.path.join(ROOT, "configs", "conv_tuning_mi355x.json")
    if os.path.exists(tune):
        ops.AUTOTUNE.load(tune)
    ops.AUTOTUNE.enable(True)
    hb = B // lanes
    parts = [(x[i * hb:(i + 1) * hb].contiguous(), t[i * hb:(i + 1) * hb].contiguous(),
              ctx[i * hb:(i + 1) * hb].contiguous()) for i in range(lanes)]
    unet(x, t, context=ctx)
    for i, (xi, ti, ci) in enumerate(parts):
        with ops.WORKSPACE.use_lane(i):
            unet(xi, ti, context=ci)
    ops.AUTOTUNE.enable(False)
    torch.cuda.synchronize()

    # (a) whole batch, one stream
    ga = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        unet(x, t, context=ctx)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(ga):
        ya = unet(x, t, context=ctx)
    ta = timeit(ga.replay)

    # (b) halves sequential on one stream
    gb = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gb):
        yb = []
        for i, (xi, ti, ci) in enumerate(parts):
            with ops.WORKSPACE.use_lane(i):
                yb.append(unet(xi, ti, context=ci))
    tb = timeit(gb.replay)

    # (c) halves as concurrent branches
    streams = [torch.cuda.Stream() for _ in range(lanes)]
    gc = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gc):
        cur = torch.cuda.current_stream()
        yc = []
        for i, (xi, ti, ci) in enumerate(parts):
            streams[i].wait_stream(cur)
            with torch.cuda.stream(streams[i]), ops.WORKSPACE.use_lane(i):
                yc.append(unet(xi, ti, context=ci))
        for i in range(lanes):
            cur.wait_stream(streams[i])
    tc = timeit(gc.replay)
    gc.replay()
    torch.cuda.synchronize()
    ref = ya.float()
    got = torch.cat([y.float() for y in yc], 0)
    rel = ((got - ref).norm() / ref.norm()).item()
    print(f"B={B} lanes={lanes}: one-stream {ta:.3f} ms | halves sequential {tb:.3f} ms | "
          f"halves concurrent {tc:.3f} ms | rel diff {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
