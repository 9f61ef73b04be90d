"""A/B (not product code): SD-1 UNet step at B=16, graph-replayed, with ops settings toggled inside
ONE process on ONE device (device-to-device spread on the pool is ~10%, so cross-run numbers
cannot rank small kernel changes).  usage: python tools/ab_unet.py PREPAD=0 PREPAD=1 ..."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    dev = torch.device("cuda:0")
    unet, _, _ = bench.build_models(bench.CONFIGS["c3"], dev)
    g = torch.Generator().manual_seed(1234)
    B = int(os.environ.get("B", "16"))
    x = torch.randn(B, 4, 64, 64, generator=g).to(dev)
    ctx = torch.randn(B, 77, 768, generator=g).to(dev).half()
    t = torch.full((B,), 501, dtype=torch.long, device=dev)
    tune = os.environ.get("TUNE", os.path.join(ROOT, "configs", "conv_tuning_mi355x.json"))
    if os.path.exists(tune):
        ops.AUTOTUNE.load(tune)
    arms = [dict(kv.split("=") for kv in a.split(",")) for a in sys.argv[1:]]
    graphs = []
    import importlib
    for arm in arms:
        for k, v in arm.items():
            mod, _, name = k.rpartition(".")   # "attention.FUSED_XATTN_640_MAX_ROWS" -> sd_amd.openai_model.attention
            target = importlib.import_module(f"sd_amd.openai_model.{mod}") if mod else ops
            setattr(target, name, int(v))
        ops.AUTOTUNE.enable(True)
        unet(x, t, context=ctx)
        ops.AUTOTUNE.enable(False)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            y = unet(x, t, context=ctx)
        graphs.append((arm, gr, y))
    if os.environ.get("SAVE_TUNE"):           # the next process of a cross-process A/B loads this table
        ops.AUTOTUNE.save(os.environ["SAVE_TUNE"])
    res = {i: [] for i in range(len(graphs))}
    for rep in range(5):                      # interleaved: drift affects every arm alike
        for i, (arm, gr, _) in enumerate(graphs):
            gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                gr.replay()
            e1.record()
            torch.cuda.synchronize()
            res[i].append(e0.elapsed_time(e1) / 10)
    base = graphs[0][2].float()
    for i, (arm, _, y) in enumerate(graphs):
        ts = sorted(res[i])
        rel = ((y.float() - base).norm() / base.norm()).item()
        print(f"{arm}: UNet step median {ts[2]:.3f} ms (min {ts[0]:.3f})  rel-diff vs arm 0 {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
