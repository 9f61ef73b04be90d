"""Tile visiting order of unsplit conv / GEMM plans (sdk_conv_args.tile_group_m): time per (variant, gm) on
the SD-1 B=16 shapes, HIP events, random data.  gm = M-panels per tile group (1 = M-panel major)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

SHAPES = [  # name, B, H, W, Cin, Cout, ksize, pad, geglu, variants
    ("ff1_32_640x5120", 16, 32, 32, 640, 5120, 1, 0, True, (20, 2, 8)),
    ("ff1_16_1280x10240", 16, 16, 16, 1280, 10240, 1, 0, True, (20, 2, 8)),
    ("ff2_32_2560x640", 16, 32, 32, 2560, 640, 1, 0, False, (23, 22, 5)),
    ("ff2_64_1280x320", 16, 64, 64, 1280, 320, 1, 0, False, (22, 5)),
    ("qkv_64_320x960", 16, 64, 64, 320, 960, 1, 0, False, (22, 5)),
    ("c3_64_320x320", 16, 66, 66, 320, 320, 3, 0, False, (36, 5)),
    ("c3_32_640x640", 16, 34, 34, 640, 640, 3, 0, False, (36, 37, 23)),
    ("c3_64_640x320", 16, 66, 66, 640, 320, 3, 0, False, (36, 5)),
    ("vae_128_512x512", 16, 130, 130, 512, 512, 3, 0, False, (8, 20, 36)),
    ("vae_256_256x256", 8, 258, 258, 256, 256, 3, 0, False, (8, 20, 36)),
]
GMS = tuple(int(g) for g in os.environ.get("GMS", "1,2,4,8,16").split(","))


def t_of(f, reps=5, inner=3):
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


for name, B, H, W, Ci, Co, k, pad, geglu, variants in SHAPES:
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), device="cuda")
    fl = 2.0 * B * (H - k + 1) * (W - k + 1) * Co * Ci * k * k
    mode = ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16
    cells = []
    for v in variants:
        row = []
        for g in GMS:
            ops.TILE_GROUP_M = g
            try:
                t = t_of(lambda: ops.conv2d(pc, x, ksize=k, pad=pad, out_mode=mode, variant=v, split_k=1))
            except RuntimeError:
                row.append("   -  ")
                continue
            row.append(f"{fl / t / 1e9:6.0f}")
        cells.append(f"v{v}: " + " ".join(row))
    ops.TILE_GROUP_M = None
    print(f"{name:18s} TF/s at gm {GMS} | " + " | ".join(cells), flush=True)
