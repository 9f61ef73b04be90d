#!/bin/bash
# fused feed-forward ablations (diagnostics build): no DMA / no MFMA / no GEGLU math, fused kernel time
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/ff
L=gpurun_out/ff/ablate.log
: > $L
for d in 0 1 2 3 4 5; do
  echo "== SDK_FF_DBG=$d" >> $L
  SD_AMD_LIB=$PWD/stable-diffusion-from-scratch_amd/libsdk_amd_diag.so SDK_FF_DBG=$d timeout -k 10 120 python -u tools/bench_ff.py --fused-only >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep -v amdgpu.ids $L
