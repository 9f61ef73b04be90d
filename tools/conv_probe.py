"""Time one conv configuration (for rocprofv3 counter passes and A/B runs).
usage: [GM=<tile_group_m>] [GN=1] python tools/conv_probe.py <shape> <variant> <split> [iters]
shape: a tools/bench_conv.py SHAPES name, or B,H,W,Cin,Cout,k,up"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import SHAPES


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    if os.environ.get("GM"):          # tile group (sdk_conv_args.tile_group_m)
        ops.TILE_GROUP_M = int(os.environ["GM"])
    name, variant, split = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    spec = {s[0]: s[1:] for s in SHAPES}.get(name)
    if spec is None:
        B, H, W, Ci, Co, k, up = (int(v) for v in name.split(","))
        st, geglu = 1, 0
    else:
        B, H, W, Ci, Co, k, st, up, geglu = spec
    torch.manual_seed(0)
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), geglu=bool(geglu), device="cuda")
    kw = dict(stride=st, pad=0 if name.endswith("_prepad") else k // 2, upsample=bool(up),
              variant=None if variant < 0 else variant,
              split_k=None if split == 0 else split,   # -2: in-launch split-K
              out_mode=ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16,
              gn_stats=os.environ.get("GN") == "1")   # GN=1: the epilogue emits GroupNorm statistics
    y = ops.conv2d(pc, x, **kw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ops.conv2d(pc, x, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    Ho, Wo = y.shape[1], y.shape[2]
    tf = 2.0 * B * Ho * Wo * Co * Ci * k * k / (ms * 1e-3) / 1e12
    print(f"{name} v{variant} split{split}: {ms * 1e3:.1f} us/call  {tf:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
