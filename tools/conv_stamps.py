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
    import time
    warm = float(os.environ.get("STAMP_WARM_S", "0"))   # back-to-back launches first: the clock under sustained load
    t0 = time.time()
    while True:
        for _ in range(3):
            ops.conv2d(pc, x, **kw)
        torch.cuda.synchronize()
        if time.time() - t0 >= warm:
            break
    # launch time in this same process and clock state: 20 back-to-back launches between HIP events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.conv2d(pc, x, **kw)
    e1.record()
    e1.synchronize()
    print(f"{name} v{variant}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us per launch (20 back-to-back, HIP events)")
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
    if os.environ.get("SDK_CONV_STAMPS") == "2":   # slots 6 / 7: s_memrealtime (100 MHz) at entry / end
        rt = live[(live[:, 7] > live[:, 6])]
        clk = (rt[:, 3] - rt[:, 0]) / ((rt[:, 7] - rt[:, 6]) / 100e6) / 1e9
        print(f"   shader clock over the workgroup lifetimes: median {np.median(clk):.3f} GHz "
              f"[{clk.min():.3f}-{clk.max():.3f}]; lifetime {np.median((rt[:, 7] - rt[:, 6]) / 100.0):.1f} us (realtime)")
        st, en = (rt[:, 6] - rt[:, 6].min()) / 100.0, (rt[:, 7] - rt[:, 6].min()) / 100.0
        print(f"   realtime span first start -> last end {en.max():.1f} us; starts spread {np.percentile(st, 50):.1f} / "
              f"{np.percentile(st, 90):.1f} / {st.max():.1f} us (p50 / p90 / max), ends {np.percentile(en, 10):.1f} / "
              f"{np.percentile(en, 50):.1f} / {en.max():.1f} us (p10 / p50 / max)")
        return
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
