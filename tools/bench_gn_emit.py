"""Cost of emitting GroupNorm statistics from the conv epilogue vs what it saves: per shape and
variant, conv time with / without the emission and GroupNorm (+SiLU, padded) time from the
partials vs with its own statistics pass.  Graph-replayed, B=16, MI355X.
usage: python tools/bench_gn_emit.py [variants]"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops
from tools.bench_norm import timeit

SHAPES = [  # (name, B, H, W, Cin, Cout, k, pad, residual)
    ("64x64 320->320 3x3", 16, 66, 66, 320, 320, 3, 0, True),
    ("32x32 640->640 3x3", 16, 34, 34, 640, 640, 3, 0, True),
    ("16x16 1280->1280 3x3", 16, 18, 18, 1280, 1280, 3, 0, True),
    ("64x64 proj_out 320", 16, 64, 64, 320, 320, 1, 0, True),
    ("32x32 proj_out 640", 16, 32, 32, 640, 640, 1, 0, True),
]
VARIANTS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "5,7,22,23,25,19".split(","))]
for name, B, H, W, Ci, Co, k, pad, res in SHAPES:
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.randn(Co, device="cuda"), device="cuda")
    Ho, Wo = H - 2 * (k // 2 - pad), W - 2 * (k // 2 - pad)
    r = torch.randn(B, Ho, Wo, Co, device="cuda").half() if res else None
    g, bt = torch.ones(Co, device="cuda"), torch.zeros(Co, device="cuda")
    yp = torch.empty(B, Ho + 2, Wo + 2, Co, device="cuda").half()
    fl = 2.0 * B * Ho * Wo * Co * Ci * k * k
    for v in VARIANTS:
        try:
            y0 = ops.conv2d(pc, x, pad=pad, residual=r, variant=v, split_k=1)
            y1 = ops.conv2d(pc, x, pad=pad, residual=r, variant=v, split_k=1, gn_stats=True)
        except RuntimeError as e:
            print(f"{name:24s} v{v}: {e}")
            continue
        emits = getattr(y1, ops.GN_ATTR, None) is not None
        t0 = timeit(lambda: ops.conv2d(pc, x, pad=pad, residual=r, variant=v, split_k=1))
        t1 = timeit(lambda: ops.conv2d(pc, x, pad=pad, residual=r, variant=v, split_k=1, gn_stats=True))
        ga = timeit(lambda: ops.group_norm(y0, g, bt, 1e-5, 32, silu=True, pad=1, out=yp))
        gb = timeit(lambda: ops.group_norm(y1, g, bt, 1e-5, 32, silu=True, pad=1, out=yp))
        print(f"{name:24s} v{v:2d}: conv {t0:7.1f} us ({fl / t0 / 1e6:6.1f} TF/s), +stats {t1:7.1f} us"
              f"{'' if emits else ' (no emission)'};  group_norm with pass {ga:6.1f} us, from partials {gb:6.1f} us;"
              f"  net {t1 + gb - t0 - ga:+6.1f} us", flush=True)
