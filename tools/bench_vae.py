"""VAE decode (C3: B=16 64x64 latents -> 512x512) device time, median of reps (HIP events), with the
bench's seeded weights and tuning table.  A/B knobs are environment variables of the process."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from sd_amd import ops
    dev = torch.device("cuda:0")
    _, vae, ld = bench.build_models(bench.CONFIGS["c3"], dev)
    tune = os.environ.get("TUNE", os.path.join(ROOT, "configs", "conv_tuning_mi355x.json"))
    if os.path.exists(tune):
        ops.AUTOTUNE.load(tune)
    ops.AUTOTUNE.enable(os.environ.get("AUTOTUNE", "1") == "1")
    z = torch.randn(16, 4, 64, 64, generator=torch.Generator().manual_seed(3)).to(dev)
    img = ld.decode_first_stage(z)
    torch.cuda.synchronize()
    ts = []
    for _ in range(int(os.environ.get("REPS", "7"))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        img = ld.decode_first_stage(z)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(f"VAE decode B=16 512x512: median {ts[len(ts) // 2]:.2f} ms (min {ts[0]:.2f})  "
          f"chunk_limit={ops.BUF_LIMIT}  checksum {img.float().abs().mean().item():.6f}", flush=True)


if __name__ == "__main__":
    main()
