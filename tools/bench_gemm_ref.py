"""Calibration only (not product code): torch.matmul (hipBLASLt) vs sd_amd conv/linear on the
SD-1 token GEMM shapes, device time from HIP events over back-to-back launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(65536, 320, 320), (16384, 640, 640), (4096, 1280, 1280), (1024, 1280, 1280), (65536, 2560, 320),
          (16384, 5120, 640), (4096, 10240, 1280), (65536, 320, 1280), (16384, 640, 2560), (4096, 1280, 5120),
          (65536, 960, 320), (65536, 320, 2880), (16384, 640, 5760), (4096, 1280, 11520)]


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
    g = torch.cuda.CUDAGraph
    for M, N, K in SHAPES:
        a = torch.randn(M, K, device="cuda").half()
        w = torch.randn(N, K, device="cuda").half()
        t_ref = timeit(lambda: torch.matmul(a, w.t()))
        pc = ops.PackedConv([(w.float(), K)], None, device="cuda")
        # graph-captured so host launch cost is excluded like in the sampler
        ops.linear(pc, a)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            graph = g()
            with torch.cuda.graph(graph):
                for _ in range(10):
                    ops.linear(pc, a)
        torch.cuda.current_stream().wait_stream(s)
        t_ours = timeit(lambda: graph.replay(), reps=5) / 10
        fl = 2.0 * M * N * K
        print(f"M={M:6d} N={N:6d} K={K:6d}  hipBLASLt {t_ref:8.1f} us {fl / t_ref / 1e6:7.1f} TF/s   "
              f"sd_amd {t_ours:8.1f} us {fl / t_ours / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
