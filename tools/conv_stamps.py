"""Phase times of one conv configuration from the diagnostics build's workgroup stamps (SDK_CONV_STAMPS=1,
libsdk_amd_diag.so): per workgroup, thread 0's s_memtime at entry / after the prologue / after the K loop /
at the end (conv.hip ph_stamp).  Prints the mean cycles of prologue, K loop and epilogue, the mean workgroup
lifetime, and the kernel span in cycles.
usage: SD_AMD_LIB=.../libsdk_amd_diag.so SDK_CONV_STAMPS=1 python tools/conv_stamps.py <shape> <variant>"""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_conv import SHAPES


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops, _lib
    name, variant = sys.argv[1], int(sys.argv[2])
    B, H, W, Ci, Co, k, st, up, geglu = {s[0]: s[1:] for s in SHAPES}[name]
    x = torch.randn(B, H, W, Ci, device="cuda").half()
    w = torch.randn(Co, Ci, k, k, device="cuda") / (Ci * k * k) ** 0.5
    pc = ops.PackedConv([(w, Ci)], torch.zeros(Co, device="cuda"), geglu=bool(geglu), device="cuda")
    kw = dict(stride=st, pad=k // 2 if "prepad" not in name else 0, upsample=bool(up), variant=variant, split_k=1,
              out_mode=ops.OUT_GEGLU_F16 if geglu else ops.OUT_NHWC_F16)
    for _ in range(3):
        ops.conv2d(pc, x, **kw)
    torch.cuda.synchronize()
    ops.conv2d(pc, x, **kw)
    torch.cuda.synchronize()
    info = ops.ConvPlanInfo()
    n = info.grid_tiles if False else None
    lib = _lib.lib()
    f = lib.sdk_diag_conv_stamps
    f.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    nwg = 65536
    buf = np.zeros(nwg * 8, dtype=np.uint64)
    assert f(buf.ctypes.data, nwg * 8) == 0
    s = buf.reshape(-1, 8).astype(np.int64)
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    live = s[(s[:, 3] >= s[:, 0])]
    pro = (live[:, 1] - live[:, 0]).mean()
    kl = (live[:, 2] - live[:, 1]).mean()
    ep = (live[:, 3] - live[:, 2]).mean()
    print(f"{name} v{variant}: {len(live)} workgroups; mean cycles prologue {pro:.0f}  K loop {kl:.0f}  "
          f"epilogue {ep:.0f}  lifetime {(live[:, 3] - live[:, 0]).mean():.0f}")
    g = live[live[:, 4] > 0]
    if len(g):
        prev = g[:, 2]
        parts = []
        for k in range(4, 8):
            ok = g[:, k] > 0
            if not ok.any():
                break
            parts.append(f"{(g[ok, k] - prev[ok]).mean():.0f}")
            prev = np.where(ok, g[:, k], prev)
        print("   epilogue groups (cycles after the K loop / the previous group):", " ".join(parts))


if __name__ == "__main__":
    main()
