"""Skinny token GEMMs (M = batch rows): variant 35 vs the tiled kernels on the time-embedding MLP
shapes of the SD-1 UNet at the bench batch.  HIP events, median of reps; prints us per launch."""
import math, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

DEV = "cuda"
SHAPES = [(16, 320, 1280, False, "nhwc"), (16, 1280, 1280, True, "nhwc"), (16, 1280, 20160, True, "rows"),
          (32, 1280, 20160, True, "rows")]


def t_us(fn, reps=10, per=20):
    """device time per launch: a HIP graph of `per` back-to-back launches, median over replays
    (a Python-side loop would time the host's argument marshalling, not the kernel)"""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        fn()
        s.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(per):
                fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); g.replay(); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / per)
    return sorted(ts)[len(ts) // 2]


for M, K, N, silu, mode in SHAPES:
    x = torch.randn(M, K, device=DEV).half()
    pc = ops.PackedConv([(torch.randn(N, K) / math.sqrt(K), K)], torch.randn(N) * 0.1, device=DEV)
    om = {"nhwc": ops.OUT_NHWC_F16, "rows": ops.OUT_ROWS_F32}[mode]
    x4 = x.view(1, M, 1, K)
    row = [f"M={M} K={K} N={N}"]
    for v, sp in ((35, None), (0, None), (4, None), (4, 2), (31, None), (31, 4)):
        try:
            us = t_us(lambda: ops.conv2d(pc, x4, ksize=1, pad=0, silu=silu and v in (0, 35), out_mode=om,
                                         variant=v, split_k=sp))
            row.append(f"v{v}{'' if sp is None else '/s' + str(sp)} {us:7.1f}us")
        except RuntimeError as e:
            row.append(f"v{v} n/a")
    wb = N * K * 2
    row.append(f"(weight {wb / 1e6:.1f} MB)")
    print("  ".join(row), flush=True)
