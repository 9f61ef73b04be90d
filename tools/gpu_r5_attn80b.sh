#!/bin/bash
# d = 80 stagger on by default: attention / SD-1 / bench-config parity, then the UNet step with it (default) and without
# (SDK_ATTN_STAG=0: no stagger anywhere, the previous SD-1 routing), alternated in separate processes on one box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/attn80b
mkdir -p $L
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_bench_parity.py -x -q -s -k "attention or attn or sd1 or bench" --timeout 400 --timeout-method thread > $L/tests.log 2>&1 || { tail -30 $L/tests.log; exit 1; }
grep "\[parity\]" $L/tests.log | head -8; tail -1 $L/tests.log
for e in "SDK_ATTN_STAG=0" "SDK_ATTN_DEFAULT=1" "SDK_ATTN_STAG=0" "SDK_ATTN_DEFAULT=1"; do
  env $e timeout -k 10 300 python -u tools/ab_unet.py EMIT_GN_STATS=1 > $L/unet.txt 2>&1 || { tail -20 $L/unet.txt; exit 1; }
  sed "s/^/[$e] /" $L/unet.txt | grep "UNet step"
done
