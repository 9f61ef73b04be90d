"""Split-K conv shapes of the SD-1 16x16 / 8x8 levels (B=16): best time over (variant, split) per
shape, HIP events, random data — for A/B of the work-item order (SD_AMD_LIB selects the library)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

SHAPES = [  # name, B, H, W, Cin, Cout (3x3, zero-bordered input: pad 0)
    ("u8_1280x1280", 16, 10, 10, 1280, 1280), ("u8_2560x1280", 16, 10, 10, 2560, 1280),
    ("u16_1280x1280", 16, 18, 18, 1280, 1280), ("u16_2560x1280", 16, 18, 18, 2560, 1280),
    ("u16_1920x1280", 16, 18, 18, 1920, 1280), ("u32_640x640", 16, 34, 34, 640, 640),
]
VARIANTS = (5, 7, 19, 22, 23, 8, 20)
SPLITS = (1, 2, 4, 8, 16)


def t_of(f, reps=5, inner=4):
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(inner):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / inner)
    return sorted(ts)[len(ts) // 2]


for name, B, H, W, Ci, Co in SHAPES:
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, 3, 3, device="cuda") / (Ci * 9) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), device="cuda")
    fl = 2.0 * B * (H - 2) * (W - 2) * Co * Ci * 9
    best = (1e9, None)
    res = []
    for v in VARIANTS:
        for sp in SPLITS:
            try:
                t = t_of(lambda: ops.conv2d(pc, x, pad=0, variant=v, split_k=sp))
            except RuntimeError:
                continue
            res.append((t, v, sp))
            best = min(best, (t, (v, sp)))
    res.sort()
    top = " ".join(f"v{v}/s{sp}:{fl / t / 1e9:.0f}" for t, v, sp in res[:4])
    print(f"{name:16s} best {fl / best[0] / 1e9:7.1f} TF/s {best[0]*1000:8.1f} us  {top}", flush=True)
