#!/bin/bash
# One-wave GroupNorm finalize (default) vs the 256-thread form (SDK_GN_FINALIZE_WAVE=0): the full GPU suite with the new
# default, then per-call GN times and the SD-1 UNet step with both, alternated in separate processes on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/gnfinw
mkdir -p $L
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
tail -1 $L/tests.log
for f in 0 1; do
  SDK_GN_FINALIZE_WAVE=$f timeout -k 10 240 python -u tools/bench_hbm_kernels.py > $L/hbm_$f.txt 2>&1 || { tail -20 $L/hbm_$f.txt; exit 1; }
  grep "GN+SiLU" $L/hbm_$f.txt | sed "s/^/[wave=$f] /"
done
for f in 0 1 0 1; do
  SDK_GN_FINALIZE_WAVE=$f timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 > $L/unet_$f.txt 2>&1 || { tail -20 $L/unet_$f.txt; exit 1; }
  sed "s/^/[wave=$f] /" $L/unet_$f.txt | grep "UNet step"
done
