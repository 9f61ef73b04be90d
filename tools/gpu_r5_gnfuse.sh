#!/bin/bash
# GroupNorm from the producers' partials as ONE launch (gn_apply_part_kernel: per-workgroup statistics merge, the
# first round of image loads issued before it) up to SDK_GN_PART_FUSED_MAX_HW pixels, vs finalize + apply launches:
# GN kernel times per shape and the SD-1 UNet step (B = 16, graph-replayed) at thresholds 256 / 1024 / 4096, then
# the GroupNorm parity tests at the largest threshold.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/gnfuse
mkdir -p $L
for t in 256 1024 4096; do
  SDK_GN_PART_FUSED_MAX_HW=$t timeout -k 10 240 python -u tools/bench_hbm_kernels.py > $L/hbm_$t.txt 2>&1 || { tail -20 $L/hbm_$t.txt; exit 1; }
  grep "GN+SiLU" $L/hbm_$t.txt | sed "s/^/[$t] /"
done
for t in 256 4096 1024 256; do
  SDK_GN_PART_FUSED_MAX_HW=$t timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 > $L/unet_$t.txt 2>&1 || { tail -20 $L/unet_$t.txt; exit 1; }
  sed "s/^/[$t] /" $L/unet_$t.txt | grep "UNet step"
done
SDK_GN_PART_FUSED_MAX_HW=4096 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "group_norm or gn or vae or sd1" --timeout 300 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -2 $L/tests.log
