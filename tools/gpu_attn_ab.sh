#!/bin/bash
# attention variant A/B: parity of the staggered form, then the microbench with and without it
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p gpurun_out/attn
L=gpurun_out/attn/ab.log
SDK_ATTN_STAG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k attention -x -q --timeout 120 --timeout-method thread > $L 2>&1 || { tail -30 $L; exit 1; }
tail -3 $L
for rep in 1; do
  for v in 0 1; do
    echo "== SDK_ATTN_STAG=$v" >> $L
    SDK_ATTN_STAG=$v timeout -k 10 120 python -u tools/bench_attn.py >> $L 2>&1 || { tail -30 $L; exit 1; }
  done
done
grep -v "^$" $L | grep "==\|us " 
