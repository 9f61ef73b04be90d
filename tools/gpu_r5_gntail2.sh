#!/bin/bash
# GroupNorm group-statistics tail: UNet-step A/B in one process (tail on / off, in-process tuning on the first arm),
# then the HBM-bound kernel table (copy-probe shapes, GroupNorm from partials / groups, LayerNorm, token linear).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
L=gpurun_out/gntail
mkdir -p $L
timeout -k 10 900 python -u tools/ab_unet.py GN_GROUP_TAIL=1 GN_GROUP_TAIL=0 GN_GROUP_TAIL=1 GN_GROUP_TAIL=0 > $L/ab.log 2>&1 || { tail -20 $L/ab.log; exit 1; }
grep "UNet step" $L/ab.log
timeout -k 10 300 python -u tools/bench_hbm_kernels.py > $L/hbm.log 2>&1 || { tail -20 $L/hbm.log; exit 1; }
grep -v amdgpu.ids $L/hbm.log
