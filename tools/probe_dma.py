"""LDS-DMA / register-staged L2->LDS fill rate per CU on the MI355X (sdk_probe_dma): waves per workgroup
x pieces in flight per wave, from an L2-resident 2 MiB table and from a 1 GiB HBM buffer; 256 and 512
workgroups.  Prints GB/s per CU.  What bounds the GEMM K-loops (40-45 GB/s per CU measured in them)?"""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import sd_amd_loader
    sd_amd_loader.load()
    from sd_amd._lib import lib, check
    L = lib()
    L.sdk_probe_dma.argtypes = [C.c_int32] * 3 + [C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
    big = torch.empty(1 << 29, dtype=torch.float16, device="cuda").normal_()     # 1 GiB
    sink = torch.empty(4096, dtype=torch.float32, device="cuda")
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for src_bytes, name in ((2 << 20, "L2 2MiB"), (1 << 30, "HBM 1GiB")):
        for blocks in (256, 512):
            for nw, inf, mode in ((4, 1, 0), (4, 2, 0), (4, 4, 0), (4, 6, 0), (8, 1, 0), (8, 2, 0), (8, 4, 0),
                                  (8, 6, 0), (16, 1, 0), (16, 2, 0), (16, 4, 0), (16, 6, 0), (8, 2, 1), (8, 4, 1),
                                  (16, 2, 1), (16, 4, 1)):
                pieces = max(64, (256 << 10) // nw)  // 1   # 256 KiB... per wave: scaled so a launch moves ~1 GiB
                pieces = (1 << 30) // (blocks * nw * 1024)
                f = lambda: check(L.sdk_probe_dma(nw, inf, mode, C.c_void_p(big.data_ptr()), src_bytes, pieces, blocks,
                                                  C.c_void_p(sink.data_ptr()), stream), "probe_dma")   # noqa: E731
                f()
                torch.cuda.synchronize()
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    f()
                    e1.record()
                    e1.synchronize()
                    best = min(best, e0.elapsed_time(e1))
                moved = blocks * nw * pieces * 1024
                gbs = moved / (best * 1e-3) / 1e9
                print(f"{name:9s} blocks={blocks} nw={nw:2d} inflight={inf} mode={'dma' if mode == 0 else 'reg'}: "
                      f"{gbs:7.0f} GB/s chip, {gbs / 256:5.1f} GB/s per CU", flush=True)


if __name__ == "__main__":
    main()
