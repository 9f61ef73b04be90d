"""Microbenchmark: the fused GEGLU feed-forward (ops.feed_forward) vs the two-GEMM path (GEGLU GEMM +
output GEMM with residual, tuned table) at the SD UNet's 320-channel shapes; HIP-event timing on the
launch stream, averaged over --reps launches after a warm-up."""
import argparse
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sd_amd_loader  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--fused-only", action="store_true")
    ap.add_argument("--m", type=int, default=None, help="one row count instead of the three shapes")
    ap.add_argument("--f", type=int, default=1280, help="GEGLU features (SD: 4 x 320)")
    args = ap.parse_args()
    sd_amd_loader.load()
    from sd_amd import ops
    tab = os.path.join(ROOT, "configs", "conv_tuning_mi355x.json")
    if os.path.exists(tab):
        ops.AUTOTUNE.load(tab)
    ops.AUTOTUNE.enable(True)
    dev = torch.device("cuda")
    C, F = 320, args.f
    g = torch.Generator().manual_seed(0)
    w1 = (torch.randn(2 * F, C, generator=g) / math.sqrt(C)).half()
    b1 = torch.randn(2 * F, generator=g) * 0.2
    w2 = (torch.randn(C, F, generator=g) / math.sqrt(F)).half()
    b2 = torch.randn(C, generator=g) * 0.2
    pf = ops.PackedFF(w1, b1, w2, b2, dev)
    pc1 = ops.PackedConv([(w1.float(), C)], b1, geglu=True, device=dev)
    pc2 = ops.PackedConv([(w2.float(), F)], b2, device=dev)
    for M in ((args.m,) if args.m else (65536, 73728, 16384)):
        t = torch.randn(M, C, device=dev).half()
        res = torch.randn(M, C, device=dev).half()
        out = torch.empty_like(res)
        fl = 2.0 * M * C * 3 * F
        tf = timed(lambda: ops.feed_forward(pf, t, residual=res, out=out), args.reps)
        if args.fused_only:
            print(f"M={M} C={C} F={F}: fused {tf:7.1f} us ({fl / tf * 1e-6:6.1f} TF/s)", flush=True)
            continue
        hbuf = torch.empty(M, F, device=dev, dtype=torch.float16)
        t1 = timed(lambda: ops.linear(pc1, t, out_mode=ops.OUT_GEGLU_F16, out=hbuf), args.reps)
        t2 = timed(lambda: ops.linear(pc2, hbuf, residual=res, out=out), args.reps)
        print(f"M={M} C={C} F={F}: fused {tf:7.1f} us ({fl / tf * 1e-6:6.1f} TF/s)   two GEMMs {t1:6.1f} + {t2:6.1f} = "
              f"{t1 + t2:7.1f} us ({fl / (t1 + t2) * 1e-6:6.1f} TF/s)   speedup {(t1 + t2) / tf:.2f}x", flush=True)


if __name__ == "__main__":
    main()
