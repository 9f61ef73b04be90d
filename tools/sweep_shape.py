"""Sweep every conv tile variant x split-K on one shape, device time per launch from a HIP graph of
back-to-back launches (host marshalling excluded).  usage: python tools/sweep_shape.py B,H,W,Ci,Co,k[,geglu] ..."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def graph_us(fn, per=20, reps=7):
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


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    for spec in sys.argv[1:]:
        v = [int(t) for t in spec.split(",")]
        B, H, W, Ci, Co, k = v[:6]
        geglu = len(v) > 6 and v[6]
        torch.manual_seed(0)
        x = torch.randn(B, H, W, Ci, device="cuda").half()
        w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
        pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), geglu=bool(geglu), device="cuda")
        om = ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16
        flop = 2.0 * B * H * W * Co * Ci * k * k
        res = []
        vs = [int(t) for t in os.environ["SWEEP_VARIANTS"].split(",")] if os.environ.get("SWEEP_VARIANTS") else ops.AUTOTUNE.VARIANTS
        sps = [int(t) for t in os.environ.get("SWEEP_SPLITS", "1,2,4,8").split(",")]
        for var in vs:
            for sp in sps:
                try:
                    us = graph_us(lambda: ops.conv2d(pc, x, pad=k // 2, variant=var, split_k=sp, out_mode=om))
                except RuntimeError:
                    continue
                res.append((us, var, sp))
        res.sort()
        print(f"{spec}: " + "  ".join(f"v{v_}/s{s_} {u:.1f}us {flop / u / 1e6:.0f}TF" for u, v_, s_ in res[:8]),
              flush=True)


if __name__ == "__main__":
    main()
