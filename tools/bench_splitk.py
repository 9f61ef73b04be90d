"""Split-K conv / token-GEMM shapes of the SD-1 16x16 / 8x8 levels (B=16): time per (variant, split),
HIP events, random data.  Split -2 = the in-launch combine of two K halves (sdk_conv_args.split_inlaunch).
Per shape: the best overall, then the best per split (slab splits vs in-launch)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

SHAPES = [  # name, B, H, W, Cin, Cout, ksize (3x3: zero-bordered input, pad 0; 1x1: token GEMM M = B*H*W)
    ("u8_1280x1280", 16, 10, 10, 1280, 1280, 3), ("u8_2560x1280", 16, 10, 10, 2560, 1280, 3),
    ("u16_1280x1280", 16, 18, 18, 1280, 1280, 3), ("u16_2560x1280", 16, 18, 18, 2560, 1280, 3),
    ("u16_1920x1280", 16, 18, 18, 1920, 1280, 3), ("u32_640x640", 16, 34, 34, 640, 640, 3),
    ("t16_1280x1280", 16, 16, 16, 1280, 1280, 1), ("t16_1280x640", 16, 16, 16, 1280, 640, 1),
    ("t32_640x640", 16, 32, 32, 640, 640, 1), ("t8_1280x1280", 16, 8, 8, 1280, 1280, 1),
    ("t16_5120x1280", 16, 16, 16, 5120, 1280, 1), ("t32_2560x640", 16, 32, 32, 2560, 640, 1),
]
VARIANTS = (2, 3, 4, 5, 7, 16, 17, 18, 19, 22, 23, 24, 25, 26, 31, 32, 33)
SPLITS = tuple(int(s) for s in os.environ.get("SPLITS", "1,2,4,8,-2").split(","))


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


for name, B, H, W, Ci, Co, k in SHAPES:
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
    r = torch.randn(B, H - k + 1, W - k + 1, Co, device="cuda").half()
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), device="cuda")
    fl = 2.0 * B * (H - k + 1) * (W - k + 1) * Co * Ci * k * k
    res = []
    for v in VARIANTS:
        for sp in SPLITS:
            try:
                t = t_of(lambda: ops.conv2d(pc, x, ksize=k, pad=0, residual=r, variant=v, split_k=sp))
            except RuntimeError:
                continue
            res.append((t, v, sp))
    res.sort()
    per = []
    for sp in SPLITS:
        b = [x for x in res if x[2] == sp]
        if b:
            per.append(f"s{sp}:v{b[0][1]} {b[0][0]*1000:.1f}")
    print(f"{name:16s} best {fl / res[0][0] / 1e9:7.1f} TF/s {res[0][0]*1000:8.1f} us v{res[0][1]}/s{res[0][2]} | "
          + "  ".join(per), flush=True)
