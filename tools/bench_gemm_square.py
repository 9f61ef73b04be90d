"""Calibration: sd_amd conv kernel variants on plain square GEMMs (token GEMM path, 1x1) vs
hipBLASLt (torch.matmul) — separates the GEMM core's efficiency from the SD shapes' short K,
N quantisation and implicit-conv gather.  Random N(0,1) fp16 operands, HIP events, median."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader
sd_amd_loader.load()
from sd_amd import ops

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (16384, 640, 5760), (65536, 320, 2880), (4096, 1280, 11520),
          (16384, 5120, 640), (65536, 320, 320)]
VARIANTS = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "2,5,8,9,19,20,21,22,23".split(","))]


def timeit(f, reps=7, inner=3):
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


print("M x N x K".ljust(22) + "hipBLASLt".rjust(10) + "".join(f"v{v}".rjust(8) for v in VARIANTS))
for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").half()
    w = torch.randn(N, K, device="cuda").half()
    fl = 2.0 * M * N * K
    row = f"{M}x{N}x{K}".ljust(22)
    t = timeit(lambda: torch.matmul(a, w.t()))
    row += f"{fl / t / 1e9:10.1f}"
    pc = ops.PackedConv([(w.float(), K)], None, device="cuda")
    for v in VARIANTS:
        try:
            t = timeit(lambda: ops.linear_variant(pc, a, v) if hasattr(ops, "linear_variant") else
                       ops.conv2d(pc, a.view(1, M, 1, K), ksize=1, pad=0, variant=v))
            row += f"{fl / t / 1e9:8.1f}"
        except RuntimeError:
            row += "       -"
    print(row, flush=True)
