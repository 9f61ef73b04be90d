"""320-channel token linear (csrc/token.hip) vs the tiled GEMM (ops.linear) at the 64x64-level shapes,
device time per launch from a HIP graph of back-to-back launches."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.sweep_shape import graph_us  # noqa: E402


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd import ops
    ops.AUTOTUNE.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                   "conv_tuning_mi355x.json"))
    dev = torch.device("cuda")
    for M in (65536, 16384):
        w = torch.randn(320, 320, device=dev) / math.sqrt(320)
        b = torch.randn(320, device=dev) * 0.1
        x = torch.randn(M, 320, device=dev).half()
        r = torch.randn(M, 320, device=dev).half()
        pc = ops.PackedConv([(w, 320)], b, device=dev)
        pk = ops.PackedTokenLinear(w, b, dev)
        for tag, res in (("no residual", None), ("residual", r)):
            t0 = graph_us(lambda: ops.linear(pc, x, residual=res))
            t1 = graph_us(lambda: ops.token_linear(pk, x, residual=res))
            nb = M * 320 * 2 * (3 if res is not None else 2)
            print(f"M={M} {tag:12s}: tiled {t0:6.1f} us  token {t1:6.1f} us  ({nb / t1 / 1e3:.0f} GB/s algorithmic)",
                  flush=True)
        g = torch.ones(320, device=dev)
        bt = torch.zeros(320, device=dev)
        t0 = graph_us(lambda: ops.layer_norm(ops.linear(pc, x), g, bt, 1e-5))
        t1 = graph_us(lambda: ops.token_linear(pk, x, norm=(g, bt, 1e-5)))
        nb = M * 320 * 2 * 3
        print(f"M={M} {'+ norm':12s}: tiled+LN {t0:6.1f} us  token_ln {t1:6.1f} us  ({nb / t1 / 1e3:.0f} GB/s algorithmic)",
              flush=True)


if __name__ == "__main__":
    main()
