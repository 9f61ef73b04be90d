#!/bin/bash
# GroupNorm apply (one-pass form): scale / shift staged in LDS (SDK_GN_APPLY_LDSV=1) vs read from global (=0)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/gnldsv
mkdir -p $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "group_norm or gn or vae or sd1" --timeout 300 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -1 $L/tests.log
for f in 0 1; do
  SDK_GN_APPLY_LDSV=$f timeout -k 10 240 python -u tools/bench_hbm_kernels.py > $L/hbm_$f.txt 2>&1 || { tail -20 $L/hbm_$f.txt; exit 1; }
  grep "GN+SiLU\|best copy" $L/hbm_$f.txt | sed "s/^/[ldsv=$f] /"
done
for f in 0 1 0 1; do
  SDK_GN_APPLY_LDSV=$f timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 > $L/unet_$f.txt 2>&1 || { tail -20 $L/unet_$f.txt; exit 1; }
  sed "s/^/[ldsv=$f] /" $L/unet_$f.txt | grep "UNet step"
done
