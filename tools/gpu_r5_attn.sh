#!/bin/bash
# d = 40 attention: pipelined loop parity + A/B (SDK_ATTN_PIPE 0 = one tile at a time, 1 = pipelined with
# sched_group_barrier placement, 2 = pipelined, compiler placement), then the short-K GEMM sweep.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/attn
L=gpurun_out/attn/ab.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k attention -x -v --timeout 120 --timeout-method thread > gpurun_out/attn/tests.log 2>&1 || { tail -30 gpurun_out/attn/tests.log; exit 1; }
grep -c PASSED gpurun_out/attn/tests.log
for rep in 1 2; do
  for v in 0 1 2; do
    echo "== SDK_ATTN_PIPE=$v" >> $L
    SDK_ATTN_PIPE=$v timeout -k 10 120 python -u tools/bench_attn.py sd1_self_64x64_d40 sd1_cross_64x64_d40 >> $L 2>&1 || { tail -30 $L; exit 1; }
  done
done
grep -v "^$" $L | grep "==\|us "
if [ "${SHORTK:-1}" = 1 ]; then bash tools/gpu_r5_shortk.sh && wc -l gpurun_out/shortk/ab.txt; fi
