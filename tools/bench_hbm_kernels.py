"""HBM-bound kernels of the SD-1 C3 step against the measured copy ceiling (profiles/README.md table).

Prints the HBM copy probe per shape (sdk_probe_copy_ex modes; 1 GiB, beyond the 256 MB Infinity Cache), then per
kernel at its C3 shape (B = 16): algorithmic bytes (every tensor read or written once), device time per call
(HIP-graph replay of back-to-back calls: tensors up to ~100 MB stay resident in the Infinity Cache between calls,
so small shapes can read above the HBM rate), GB/s and the fraction of the best copy rate."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sd_amd_loader  # noqa: E402

sd_amd_loader.load()
from sd_amd import ops  # noqa: E402
from sd_amd._lib import lib  # noqa: E402


def timeit(f, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps) * 1e3


def copy_modes():
    nbytes = 1 << 30
    src = torch.empty(nbytes // 2, dtype=torch.float16, device="cuda").normal_()
    dst = torch.empty_like(src)
    best = 0.0
    names = {0: "grid-stride 4 loads", 1: "grid-stride 8 loads", 2: "grid-stride 4 nt", 3: "grid-stride 8 nt",
             1 | (8 << 2): "8 loads, 8 WG/CU", 3 | (8 << 2): "8 nt, 8 WG/CU", 1 | (32 << 2): "8 loads, 32 WG/CU",
             3 | (32 << 2): "8 nt, 32 WG/CU", 256: "flat 4 loads", 257: "flat 8 loads", 258: "flat 4 nt",
             259: "flat 8 nt"}
    for mode, name in names.items():
        f = lambda: lib().sdk_probe_copy_ex(src.data_ptr(), dst.data_ptr(), nbytes, mode, None)  # noqa: E731
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        gbs = 2 * nbytes / (min(ts) * 1e-3) / 1e9
        best = max(best, gbs)
        print(f"copy  {name:22s} 2 GiB moved   {min(ts) * 1e3:9.1f} us  {gbs:8.1f} GB/s", flush=True)
    del src, dst
    return best


def row(name, shape, nbytes, us, ceil):
    gbs = nbytes / (us * 1e-6) / 1e9
    print(f"{name:24s} {shape:22s} {nbytes / 1e6:8.1f} MB {us:8.1f} us {gbs:8.1f} GB/s  {gbs / ceil:5.2f}", flush=True)


def main():
    ceil = copy_modes()
    print(f"# best copy {ceil:.1f} GB/s; columns: kernel, shape, algorithmic bytes, us/call, GB/s, fraction of the copy")
    B = 16
    for H, C in ((64, 320), (64, 640), (32, 640), (32, 1280), (16, 1280), (8, 1280)):
        x = torch.randn(B, H, H, C, device="cuda").half()
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        nch = max(1, H * H // 256)
        part = torch.zeros(B, nch, C, 2, device="cuda")
        part[..., 1] = H * H / nch
        y = torch.empty(B, H + 2, H + 2, C, dtype=torch.float16, device="cuda")
        nb = x.numel() * 2 + y.numel() * 2

        def from_parts():
            setattr(x, ops.GN_ATTR, (part, nch, x._version))
            ops.group_norm(x, g, b, 1e-5, 32, silu=True, pad=1, out=y)
            delattr(x, ops.GN_ATTR)

        row("GN+SiLU from partials", f"{B}x{H}x{H}x{C}", nb, timeit(from_parts), ceil)
    for M, C in ((16384, 640), (4096, 1280), (1024, 1280)):
        x = torch.randn(M, C, device="cuda").half()
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        out = torch.empty_like(x)
        row("layer_norm", f"{M}x{C}", 2 * x.numel() * 2, timeit(lambda: ops.layer_norm(x, g, b, out=out)), ceil)
    M = B * 4096
    w = torch.randn(320, 320, device="cuda") / 320 ** 0.5
    pk = ops.PackedTokenLinear(w.half(), torch.zeros(320, device="cuda"), torch.device("cuda"))
    x = torch.randn(M, 320, device="cuda").half()
    r = torch.randn(M, 320, device="cuda").half()
    o = torch.empty_like(x)
    row("token_linear + residual", f"{M}x320x320", 3 * M * 320 * 2,
        timeit(lambda: ops.token_linear(pk, x, residual=r, out=o)), ceil)


if __name__ == "__main__":
    main()
