"""Attention kernel microbenchmark on the SD-1 / SD-2 / VAE shapes (random data, HIP events)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

SHAPES = [  # name, B, heads, nq, nk, d
    ("sd1_self_64x64_d40", 16, 8, 4096, 4096, 40),
    ("sd1_cross_64x64_d40", 16, 8, 4096, 77, 40),
    ("sd1_self_32x32_d80", 16, 8, 1024, 1024, 80),
    ("sd1_self_16x16_d160", 16, 8, 256, 256, 160),
    ("sd2_self_96x96_d64", 8, 5, 9216, 9216, 64),
    ("vae_mid_64x64_d64", 16, 8, 4096, 4096, 64),
]
ONLY = sys.argv[1:]          # optional shape-name filter (profiling one kernel)
REPS = int(os.environ.get("BENCH_REPS", "5"))
for name, B, H, nq, nk, d in SHAPES:
    if ONLY and name not in ONLY:
        continue
    q = torch.randn(B * nq, H * d, device="cuda").half()
    k = torch.randn(B * nk, H * d, device="cuda").half()
    v = torch.randn(B * nk, H * d, device="cuda").half()
    f = lambda: ops.attention(q, k, v, batch=B, heads=H, nq=nq, nk=nk, head_dim=d, scale=d ** -0.5)
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(REPS):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 5)
    ms = sorted(ts)[len(ts) // 2]
    fl = 4.0 * B * H * nq * nk * d
    byt = 2.0 * (B * nq * H * d * 2 + 2 * B * nk * H * d)
    print(f"{name:24s} {ms*1000:9.1f} us  {fl/ms/1e9:8.1f} TFLOP/s  {byt/ms/1e6:8.1f} GB/s")
