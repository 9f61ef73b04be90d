"""Time conv / GEMM cases on the device (graph-replayed launches, median of reps, random data) — the
per-kernel A/B driver: run once per library (SD_AMD_LIB selects an A/B build) and compare the lines.
usage: python tools/ab_cases.py [case ...]; case = name:B,H,W,Ci,Co,k,pad,variant,split[,geglu[,residual[,gn_stats[,emb]]]]
(no cases: the default SD-1 list below).  Prints '<name> v<variant> s<split> <us> us <TF/s>'."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEFAULT = [
    "u64_3x3_320:16,66,66,320,320,3,0,22,1",
    "u64_3x3_640to320:16,66,66,640,320,3,0,22,1",
    "u64_qkv:16,64,64,320,960,1,0,22,1",
    "u64_proj:16,64,64,320,320,1,0,22,1",
    "u32_proj_v23:16,32,32,640,640,1,0,23,1",
    "u32_proj_v7:16,32,32,640,640,1,0,7,1",
    "u32_3x3_640:16,34,34,640,640,3,0,24,1",
    "u32_qkv_v20:16,32,32,640,1920,1,0,20,1",
    "u32_ff1_v20:16,32,32,640,5120,1,0,20,1,1",
    "u32_ff1_v2:16,32,32,640,5120,1,0,2,1,1",
    "u32_ff2_v8:16,32,32,2560,640,1,0,8,1",
    "u32_ff2_v2:16,32,32,2560,640,1,0,2,1",
    "u16_proj_v31:16,16,16,1280,1280,1,0,31,1",
    "u16_proj_v32:16,16,16,1280,1280,1,0,32,1",
    "u16_3x3_v20:16,18,18,1280,1280,3,0,20,2",
    "u16_3x3_v25:16,18,18,1280,1280,3,0,25,2",
    "u16_ff1_v20:16,16,16,1280,10240,1,0,20,1,1",
    "u16_ff1_v2:16,16,16,1280,10240,1,0,2,1,1",
    "u16_ff2_v8:16,16,16,5120,1280,1,0,8,2",
    "u16_ff2_v19:16,16,16,5120,1280,1,0,19,2",
    "u8_3x3_v20:16,10,10,1280,1280,3,0,20,12",
    "u8_3x3_v26:16,10,10,1280,1280,3,0,26,12",
    "vae128_v8:16,130,130,512,512,3,0,8,1",
    "vae128_v2:16,130,130,512,512,3,0,2,1",
]


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    cases = sys.argv[1:] or DEFAULT
    reps = int(os.environ.get("AB_REPS", "5"))
    # the clock under sustained load (MI355X_MICROARCH.md 'DVFS give-back'): short bursts after idle run below it —
    # round 6 measured the 64x64 3x3 conv at 110-118 us in bursts and 95 us after 2 s of back-to-back launches
    # (tools/conv_stamps.py, profiles/r6_conv_ablation.txt) — so a busy loop of AB_WARM_S seconds comes first
    warm_s = float(os.environ.get("AB_WARM_S", "2"))
    if warm_s > 0:
        import time
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)
        t0 = time.time()
        while time.time() - t0 < warm_s:
            for _ in range(8):
                a @ a
            torch.cuda.synchronize()
        del a
    for c in cases:
        name, spec = c.split(":")
        v = [int(t) for t in spec.split(",")]
        B, H, W, Ci, Co, k, pad, variant, split = v[:9]
        geglu = len(v) > 9 and v[9] == 1
        with_res = len(v) > 10 and v[10] == 1
        with_gn = len(v) > 11 and v[11] == 1      # the epilogue emits GroupNorm statistics (ResBlock convs)
        with_emb = len(v) > 12 and v[12] == 1     # per-(image, channel) embedding row (ResBlock conv1)
        torch.manual_seed(0)
        x = torch.randn(B, H, W, Ci, device="cuda").half()
        w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
        pc = ops.PackedConv([(w, Ci)], torch.randn(Co, device="cuda") * 0.1, geglu=geglu, device="cuda")
        mode = ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16
        kw = dict(pad=pad, variant=variant, split_k=split, out_mode=mode)
        if with_gn:
            kw["gn_stats"] = True
        if with_emb:
            kw["row_bias"] = (torch.randn(B, Co, device="cuda"), 0)
        if with_res:
            Ho, Wo = (H + 2 * pad - k) + 1, (W + 2 * pad - k) + 1
            kw["residual"] = torch.randn(B, Ho, Wo, Co, device="cuda").half()
        try:
            y = ops.conv2d(pc, x, **kw)
        except Exception as e:   # the forced plan does not apply
            print(f"{name} v{variant} s{split} n/a ({str(e)[:60]})", flush=True)
            continue
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    ops.conv2d(pc, x, **kw)
        torch.cuda.current_stream().wait_stream(s)
        g.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 100)   # us per launch
        ts.sort()
        us = ts[len(ts) // 2]
        Ho, Wo = y.shape[1], y.shape[2]
        fl = 2.0 * B * Ho * Wo * Co * Ci * k * k
        print(f"{name} v{variant} s{split} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
        del g


if __name__ == "__main__":
    main()
