"""GroupNorm statistics / apply and LayerNorm microbenchmark on SD-1 shapes (B=16)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops


def timeit(f, reps=20):
    """Per-call device time of `reps` back-to-back calls replayed from one HIP graph (no host launch
    overhead in the measurement: these kernels run 5-30 us)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1e3


for (H, C) in [(64, 320), (64, 640), (32, 640), (32, 960), (16, 1280), (8, 2560), (128, 512), (512, 128)]:
    B = 16
    x = torch.randn(B, H, H, C, device="cuda").half()
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    us = timeit(lambda: ops.group_norm_affine(x, g, b, 1e-5))
    sc, sh = ops.group_norm_affine(x, g, b, 1e-5)
    y = torch.empty_like(x)
    ua = timeit(lambda: ops.group_norm_apply(x, (sc, sh), silu=True, out=y))
    gb = x.numel() * 2 / 1e9
    yp = torch.empty(B, H + 2, H + 2, C, device="cuda").half()
    uf = timeit(lambda: ops.group_norm(x, g, b, 1e-5, 32, silu=True, pad=1, out=yp))
    print(f"GN {H}x{H}x{C}: stats {us:7.1f} us ({gb / us * 1e6 / 1e3:5.2f} TB/s)  apply {ua:7.1f} us ({2 * gb / ua * 1e6 / 1e3:5.2f} TB/s)"
          f"  group_norm (one call, padded) {uf:7.1f} us")
for (M, C) in [(65536, 320), (16384, 640), (4096, 1280)]:
    x = torch.randn(M, C, device="cuda").half()
    g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    us = timeit(lambda: ops.layer_norm(x, g, b))
    gb = 2 * x.numel() * 2 / 1e9
    print(f"LN {M}x{C}: {us:7.1f} us ({gb / us * 1e6 / 1e3:5.2f} TB/s)")
