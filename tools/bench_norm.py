"""GroupNorm statistics / apply and LayerNorm microbenchmark on SD-1 shapes (B=16)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for (H, C) in [(64, 320), (64, 640), (32, 640), (32, 960), (16, 1280), (8, 2560), (128, 512), (512, 128)]:
    B = 16
    x = torch.randn(B, H, H, C, device="cuda").half()
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    us = timeit(lambda: ops.group_norm_affine(x, g, b, 1e-5))
    sc, sh = ops.group_norm_affine(x, g, b, 1e-5)
    y = torch.empty_like(x)
    ua = timeit(lambda: ops.group_norm_apply(x, (sc, sh), silu=True, out=y))
    gb = x.numel() * 2 / 1e9
    print(f"GN {H}x{H}x{C}: stats {us:7.1f} us ({gb / us * 1e6 / 1e3:5.2f} TB/s)  apply {ua:7.1f} us ({2 * gb / ua * 1e6 / 1e3:5.2f} TB/s)")
for (M, C) in [(65536, 320), (16384, 640), (4096, 1280)]:
    x = torch.randn(M, C, device="cuda").half()
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    us = timeit(lambda: ops.layer_norm(x, g, b))
    gb = 2 * x.numel() * 2 / 1e9
    print(f"LN {M}x{C}: {us:7.1f} us ({gb / us * 1e6 / 1e3:5.2f} TB/s)")
