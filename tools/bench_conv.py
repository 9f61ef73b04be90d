"""Conv/GEMM kernel microbenchmark on the SD-1 UNet / VAE shapes (B=16), all variants.
Prints TFLOP/s per shape per variant (HIP events, median of reps, random data)."""
import ctypes, json, os, subprocess, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (name, B, H, W, Cin, Cout, k, stride, upsample, geglu)
    ("unet64_320x320_3x3", 16, 64, 64, 320, 320, 3, 1, False, 0),
    ("unet64_320x320_3x3_prepad", 16, 66, 66, 320, 320, 3, 1, False, 0),
    ("unet16_1280x1280_3x3_prepad", 16, 18, 18, 1280, 1280, 3, 1, False, 0),
    ("vae128_512x512_3x3_prepad", 16, 130, 130, 512, 512, 3, 1, False, 0),
    ("unet64_640x320_3x3", 16, 64, 64, 640, 320, 3, 1, False, 0),
    ("unet32_640x640_3x3", 16, 32, 32, 640, 640, 3, 1, False, 0),
    ("unet16_1280x1280_3x3", 16, 16, 16, 1280, 1280, 3, 1, False, 0),
    ("unet8_2560x1280_3x3", 16, 8, 8, 2560, 1280, 3, 1, False, 0),
    ("unet64_ff1_320x2560", 16, 64, 64, 320, 2560, 1, 1, False, 1),
    ("unet64_proj_320x320", 16, 64, 64, 320, 320, 1, 1, False, 0),
    ("unet32_proj_640x640", 16, 32, 32, 640, 640, 1, 1, False, 0),
    ("unet16_proj_1280x1280", 16, 16, 16, 1280, 1280, 1, 1, False, 0),
    ("unet32_ff1_640x5120", 16, 32, 32, 640, 5120, 1, 1, False, 1),
    ("unet64_ff2_1280x320", 16, 64, 64, 1280, 320, 1, 1, False, 0),
    ("unet64_qkv_320x960", 16, 64, 64, 320, 960, 1, 1, False, 0),
    ("unet32_up_640x640", 16, 16, 16, 640, 640, 3, 1, True, 0),
    ("vae512_128x128_3x3", 16, 512, 512, 128, 128, 3, 1, False, 0),
    ("vae256_256x256_3x3", 16, 256, 256, 256, 256, 3, 1, False, 0),
    ("vae128_512x512_3x3", 16, 128, 128, 512, 512, 3, 1, False, 0),
    ("vae256_up_512x512", 16, 128, 128, 512, 512, 3, 1, True, 0),
]


def run(variant):
    env = dict(os.environ, SDK_CONV_VARIANT=str(variant))
    out = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True)
    if out.returncode:
        print(out.stdout, out.stderr)
        raise SystemExit(out.returncode)
    return json.loads(out.stdout.strip().splitlines()[-1])


def child():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    res = {}
    for name, B, H, W, Ci, Co, k, st, up, geglu in SHAPES:
        x = torch.randn(B, H, W, Ci, device="cuda").half()
        w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
        nob = os.environ.get("BENCH_NO_BIAS") == "1"
        pc = ops.PackedConv([(w, Ci)], None if nob else torch.zeros(Co, device="cuda"), geglu=bool(geglu),
                            device="cuda")
        mode = ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16
        pad = 0 if name.endswith("_prepad") else k // 2
        resid = None
        if os.environ.get("BENCH_RESIDUAL") == "1" and not geglu and st == 1 and not up:
            resid = torch.randn(B, H - 2 * (k // 2 - pad), W - 2 * (k // 2 - pad), Co, device="cuda").half()
        f = lambda: ops.conv2d(pc, x, stride=st, pad=pad, upsample=up, out_mode=mode, residual=resid)
        y = f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                f()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        ts.sort()
        Ho, Wo = y.shape[1], y.shape[2]
        flops = 2.0 * B * Ho * Wo * Co * Ci * k * k
        res[name] = round(flops / (ts[len(ts) // 2] * 1e-3) / 1e12, 1)
        del x, w, pc, y
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["2", "3", "4", "5", "6", "7", "8", "-1"])]
        table = {v: run(v) for v in variants}
        names = [s[0] for s in SHAPES]
        print("shape".ljust(24) + "".join(f"v{v}".rjust(9) for v in variants))
        for n in names:
            print(n.ljust(24) + "".join(f"{table[v][n]:9.1f}" for v in variants))
