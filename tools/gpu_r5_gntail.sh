#!/bin/bash
# GroupNorm group-statistics tail: its tests, the GN / conv kernel tests, then the UNet-step A/B (tail on / off).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/gntail
L=gpurun_out/gntail
timeout -k 10 400 python -u -m pytest tests/test_gpu_gn_tail.py -x -v -s --timeout 120 --timeout-method thread > $L/tests.log 2>&1 || { tail -40 $L/tests.log; exit 1; }
grep -E "passed|failed" $L/tests.log | tail -1
grep "\[gn_tail\]" $L/tests.log | head -20
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_bench_parity.py -x -q --timeout 300 --timeout-method thread > $L/tests2.log 2>&1 || { tail -40 $L/tests2.log; exit 1; }
tail -1 $L/tests2.log
timeout -k 10 400 python -u tools/ab_unet.py GN_GROUP_TAIL=1 GN_GROUP_TAIL=0 GN_GROUP_TAIL=1 GN_GROUP_TAIL=0 > $L/ab.log 2>&1 || { tail -20 $L/ab.log; exit 1; }
grep "UNet step" $L/ab.log
