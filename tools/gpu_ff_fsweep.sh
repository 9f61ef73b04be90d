#!/bin/bash
# fused feed-forward launch time vs GEGLU width at M = 65536 (fixed cost = the F = 32 point), product
# build and the no-MFMA / no-DMA diagnostics build (SDK_FF_DBG=3)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for f in 32 64 128 320 640 1280; do timeout -k 10 60 python -u tools/bench_ff.py --fused-only --m 65536 --f $f 2>&1 | grep M=; done
for f in 32 1280; do SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd_diag.so SDK_FF_DBG=3 timeout -k 10 60 python -u tools/bench_ff.py --fused-only --m 65536 --f $f 2>&1 | grep M=; done
