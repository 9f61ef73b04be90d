"""The fused cross-attention block <320, 40> with norm2 / norm3 folded in, in isolation: repeat it on the
same inputs and report which output (out / out_ln) differs from the first run, and where."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    dev = torch.device("cuda")
    B, N, C, D, L = 16, 4096, 320, 40, 77
    g = torch.Generator().manual_seed(1)
    tok = (torch.randn(B * N, C, generator=g) * 2).half().to(dev)
    kv = (torch.randn(B * L, 2 * C, generator=g)).half().to(dev)
    wq = torch.randn(C, C, generator=g) / math.sqrt(C)
    wo = torch.randn(C, C, generator=g) / math.sqrt(C)
    pc_q = ops.PackedConv([(wq, C)], None, device=dev)
    pc_o = ops.PackedConv([(wo, C)], torch.randn(C, generator=g) * 0.1, device=dev)
    gam = [(1 + 0.1 * torch.randn(C, generator=g)).to(dev) for _ in range(2)]
    bet = [(0.1 * torch.randn(C, generator=g)).to(dev) for _ in range(2)]
    mode = os.environ.get("NORMS", "both")
    nin = (gam[0], bet[0], 1e-5) if mode in ("both", "in") else None
    nout = (gam[1], bet[1], 1e-5) if mode in ("both", "out") else None

    def run():
        r = ops.cross_attention_block(tok, kv, pc_q, pc_o, batch=B, n_img=N, nk=L, heads=C // D, head_dim=D,
                                      scale=D ** -0.5, residual=tok, norm_in=nin, norm_out=nout)
        return tuple(x.clone() for x in r) if isinstance(r, tuple) else (r.clone(),)
    ref = run()
    reps = int(os.environ.get("REPS", "300"))
    bad = 0
    for i in range(reps):
        y = run()
        for k, (a, b) in enumerate(zip(y, ref)):
            if not torch.equal(a, b):
                bad += 1
                d = (a.float() - b.float()).abs()
                rows = torch.nonzero(d.amax(1) > 0).flatten()
                cols = torch.nonzero(d.amax(0) > 0).flatten()
                print(f"rep {i} output {k}: {rows.numel()} rows differ (first {rows[:4].tolist()}, blocks "
                      f"{sorted(set((rows // 64).tolist()))[:8]}), {cols.numel()} cols (first {cols[:8].tolist()}), "
                      f"max {d.max().item():.3e}", flush=True)
    print(f"NORMS={mode}: {bad} differing outputs over {reps} reps", flush=True)


if __name__ == "__main__":
    main()
