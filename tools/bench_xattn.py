"""Fused cross-attention block (xattn.hip) vs the three launches it replaces (to_q GEMM,
attention core, to_out GEMM + residual) on the SD-1 / SD-2 shapes at B=16, device time from HIP
events over back-to-back launches."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [("sd1_64x64", 16, 4096, 320, 40), ("sd1_32x32", 16, 1024, 640, 80), ("sd1_16x16", 16, 256, 1280, 160),
          ("sd1_8x8", 16, 64, 1280, 160), ("sd2_64x64", 16, 4096, 320, 64), ("sd2_32x32", 16, 1024, 640, 64),
          ("sd2_96_64x64", 8, 9216, 320, 64), ("sd1_64x64_cfg", 32, 4096, 320, 40),
          ("sd1_32x32_cfg", 32, 1024, 640, 80), ("sd2_96_cfg_96x96", 16, 9216, 320, 64),
          ("sd2_96_cfg_48x48", 16, 2304, 640, 64)]


def timeit(f, reps=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    nk = 77
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    for name, B, N, C, D in SHAPES:
        if only and name not in only:
            continue
        H = C // D
        t = torch.randn(B * N, C, device="cuda").half()
        kv = torch.randn(B * nk, 2 * C, device="cuda").half()
        res = torch.randn(B * N, C, device="cuda").half()
        pcq = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], None, device="cuda")
        pco = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], torch.zeros(C), device="cuda")
        fused = lambda: ops.cross_attention_block(t, kv, pcq, pco, batch=B, n_img=N, nk=nk, heads=H, head_dim=D,
                                                  scale=D ** -0.5, residual=res)

        def three():
            q = ops.linear(pcq, t)
            o = ops.attention(q, kv[:, :C], kv[:, C:], batch=B, heads=H, nq=N, nk=nk, head_dim=D, scale=D ** -0.5)
            return ops.linear(pco, o, residual=res)
        sup = ops.cross_attention_block_supported(C, D, nk, N)
        if "--norms" in sys.argv:
            # norm2 -> block -> norm3: folded into the kernel vs two layer_norm launches around it
            if not sup:
                continue
            g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
            t3 = torch.empty_like(t)
            folded = lambda: ops.cross_attention_block(res, kv, pcq, pco, batch=B, n_img=N, nk=nk, heads=H,
                                                       head_dim=D, scale=D ** -0.5, residual=res, norm_in=(g, b, 1e-5),
                                                       norm_out=(g, b, 1e-5), out_ln=t3)

            def separate():
                t2 = ops.layer_norm(res, g, b, 1e-5, out=t)
                y = ops.cross_attention_block(t2, kv, pcq, pco, batch=B, n_img=N, nk=nk, heads=H, head_dim=D,
                                              scale=D ** -0.5, residual=res)
                return ops.layer_norm(y, g, b, 1e-5, out=t3)
            def separate3():
                t2 = ops.layer_norm(res, g, b, 1e-5, out=t)
                q = ops.linear(pcq, t2)
                o = ops.attention(q, kv[:, :C], kv[:, C:], batch=B, heads=H, nq=N, nk=nk, head_dim=D, scale=D ** -0.5)
                y = ops.linear(pco, o, residual=res)
                return ops.layer_norm(y, g, b, 1e-5, out=t3)
            tn, ts, tb, t3l = timeit(folded), timeit(separate), timeit(fused), timeit(separate3)
            print(f"{name:16s} B={B:3d} N={N:5d} C={C:4d} d={D:3d}  norms folded {tn:8.1f} us   LN + block + LN "
                  f"{ts:8.1f} us (block alone {tb:8.1f})   LN + three launches + LN {t3l:8.1f} us   "
                  f"speedup vs best {min(ts, t3l) / tn:5.2f}x", flush=True)
            continue
        tf = timeit(fused) if sup else float("nan")
        t3 = timeit(three)
        flops = 4.0 * B * N * C * C + 4.0 * B * N * nk * C       # the block as the reference computes it
        hbm = 3 * B * N * C * 2            # t + residual read, out written
        print(f"{name:16s} B={B:3d} N={N:5d} C={C:4d} d={D:3d}  fused {tf:8.1f} us ({flops / tf / 1e6:7.1f} TFLOP/s, "
              f"{hbm / tf / 1e6:6.2f} TB/s)   three launches {t3:8.1f} us ({flops / t3 / 1e6:7.1f} TFLOP/s)   "
              f"speedup {t3 / tf:5.2f}x", flush=True)


def phases():
    """Per-workgroup phase durations of the fused kernel (wall_clock64 stamps, 100 MHz)."""
    import ctypes
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    from sd_amd._lib import lib
    nk = 77
    names = ["t stage", "q proj", "heads", "o proj", "store"]
    for name, B, N, C, D in SHAPES:
        if not ops.cross_attention_block_supported(C, D, nk, N):
            continue
        H = C // D
        t = torch.randn(B * N, C, device="cuda").half()
        kv = torch.randn(B * nk, 2 * C, device="cuda").half()
        res = torch.randn(B * N, C, device="cuda").half()
        pcq = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], None, device="cuda")
        pco = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], torch.zeros(C), device="cuda")
        groups = B * N // 64
        st = torch.zeros(groups * 8, dtype=torch.int64, device="cuda")
        lib().sdk_xattn_debug_stamps(ctypes.c_void_p(st.data_ptr()))
        kw = {}
        if "--norms" in sys.argv:   # norm2 counts into "t stage", norm3 into "store"
            g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
            kw = dict(norm_in=(g, b, 1e-5), norm_out=(g, b, 1e-5))
        ops.cross_attention_block(t, kv, pcq, pco, batch=B, n_img=N, nk=nk, heads=H, head_dim=D, scale=D ** -0.5,
                                  residual=res, **kw)
        torch.cuda.synchronize()
        lib().sdk_xattn_debug_stamps(None)
        s = st.view(groups, 8)[:, :6].double().cpu()
        d = (s[:, 1:] - s[:, :-1]) * 10.0 / 1000.0            # us
        life = (s[:, 5] - s[:, 0]) * 10.0 / 1000.0
        span = (s[:, 5].max() - s[:, 0].min()) * 10.0 / 1000.0
        print(f"{name:16s} groups={groups:5d} span {span:7.1f} us  group life {life.mean():6.1f} us  " +
              "  ".join(f"{n} {v:5.1f}" for n, v in zip(names, d.mean(0).tolist())), flush=True)


def reassoc():
    """The 1280-channel block (sd1_16x16: B=16, 256 tokens; and its CFG batch): reassociated (per-prompt
    K_h Wq_h / Wo_h V_h^T GEMMs around a segment softmax) vs the three launches, through the model's own
    CrossAttention._run, both autotuned; prints the two timings and their rel-L2 difference."""
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    from sd_amd.openai_model.attention import CrossAttention, ReassocContext
    ops.AUTOTUNE.enable(True)
    torch.manual_seed(0)
    for name, B, N in (("sd1_16x16", 16, 256), ("sd1_16x16_cfg", 32, 256)):
        C, D, H, L = 1280, 160, 8, 77
        att = CrossAttention(query_dim=C, context_dim=768, heads=H, dim_head=D).cuda()
        with torch.no_grad():
            for m in (att.to_q, att.to_k, att.to_v, att.to_out[0]):
                m.weight.normal_(0, m.in_features ** -0.5)
        att._prepare(torch.device("cuda"))
        ctx = torch.randn(B * L, 768, device="cuda").half()
        kvr = att.context_kv(ctx, L)
        assert isinstance(kvr, ReassocContext)
        t = torch.randn(B * N, C, device="cuda").half()
        res = torch.randn(B * N, C, device="cuda").half()
        f_re = lambda: att._run(t, res, B, N, kvr, L)
        f_3 = lambda: att._run(t, res, B, N, kvr.kv, L)
        y_re, y_3 = f_re(), f_3()
        err = ((y_re.float() - y_3.float()).norm() / (y_3.float() - res.float()).norm()).item()
        t_re, t_3 = timeit(f_re), timeit(f_3)
        fl3 = 4.0 * B * N * C * C + 4.0 * B * N * L * C
        print(f"{name:16s} B={B:3d} N={N:5d} C={C}  reassociated {t_re:8.1f} us   three launches {t_3:8.1f} us "
              f"({fl3 / t_3 / 1e6:6.1f} TFLOP/s)  speedup {t_3 / t_re:5.2f}x  rel-L2(reassoc - three) of the "
              f"block's update {err:.2e}", flush=True)


def ab_arms(which):
    """The block with the norms folded (the UNet's form), A/B of two kernel settings in one process:
    ``waves640`` = 4 vs 8 waves per workgroup at 640 channels (sdk_xattn_debug_waves640; bitwise equal),
    ``packed`` = projection weights in the row layout vs fragment-packed (ops.XATTN_PACKED_W; bitwise equal).
    5 alternating rounds of 20 launches each, median [min-max] per arm, bitwise check and rel-L2 of the
    block update."""
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    from sd_amd._lib import lib
    nk = 77
    if which == "waves640":
        arms, setter, reset, cw = (4, 8), lib().sdk_xattn_debug_waves640, 8, 640
    else:
        arms, setter, reset, cw = (0, 1), lambda v: setattr(ops, "XATTN_PACKED_W", bool(v)), 1, None
    for name, B, N, C, D in SHAPES:
        if (cw is not None and C != cw) or not ops.cross_attention_block_supported(C, D, nk, N):
            continue
        H = C // D
        tok = torch.randn(B * N, C, device="cuda").half()
        kv = torch.randn(B * nk, 2 * C, device="cuda").half()
        pcq = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], None, device="cuda")
        pco = ops.PackedConv([(torch.randn(C, C) / math.sqrt(C), C)], torch.zeros(C), device="cuda")
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        t3 = torch.empty_like(tok)
        f = lambda: ops.cross_attention_block(tok, kv, pcq, pco, batch=B, n_img=N, nk=nk, heads=H, head_dim=D,
                                              scale=D ** -0.5, residual=tok, norm_in=(g, b, 1e-5),
                                              norm_out=(g, b, 1e-5), out_ln=t3)
        res, outs = {a: [] for a in arms}, {}
        for r in range(5):
            for a in arms:
                setter(a)
                res[a].append(timeit(f))
                if r == 0:
                    y, _ = f()
                    torch.cuda.synchronize()
                    outs[a] = (y.clone(), t3.clone())
        setter(reset)
        same = all(torch.equal(x, y) for x, y in zip(outs[arms[0]], outs[arms[1]]))
        y0, y1 = outs[arms[0]][0].float(), outs[arms[1]][0].float()
        rel = ((y1 - y0).norm() / (y0 - tok.float()).norm()).item()
        flops = 4.0 * B * N * C * C + 4.0 * B * N * nk * C
        line = f"{name:16s} B={B:3d} N={N:5d} C={C} d={D:3d} norms folded"
        for a in arms:
            ts = sorted(res[a])
            line += f"   {which}={a} {ts[2]:7.1f} us [{ts[0]:.1f}-{ts[-1]:.1f}] ({flops / ts[2] / 1e6:6.1f} TFLOP/s)"
        print(line + f"   bitwise equal {same}, rel-L2 of the block update {rel:.1e}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] in ("--waves640", "--packed"):
        ab_arms(sys.argv[1][2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "--phases":
        phases()
    elif len(sys.argv) > 1 and sys.argv[1] == "--reassoc":
        reassoc()
    else:
        main()
